// The PatchGAN's last layer (ir:628-630: nn.Conv2d(512, 1, kernel_size=4, stride=1, padding=1))
// -- one patch logit per output pixel -- and its backward-data / weight gradient.  Each is
// 7.9 GFLOP at B=32 against 31 MB of activations: bandwidth / latency work that the MFMA conv
// kernels ran at 0.00-0.01 of peak (30 / 30 / 38 us forward / backward-data / weight gradient,
// ~0.1 ms of the D step per train step, which is the step's critical path).  Here:
//  * forward (Cout == 1): a block stages the KH input rows of one 16-column output strip in LDS
//    (zero-filled out of range); lane = one 8-channel group, wave = four output columns; a
//    pixel is KH*KW v_dot2_f32_bf16 x 4 per lane and one wave reduction;
//  * backward-data (dY with one real channel, 8-padded, onto Cout % 8 output channels): lane =
//    (pixel, 8 channels), the tap weights of its 8 channels stay in registers (fp32), dY rows
//    staged per block; packed fp32 FMAs, one 16-byte store per lane;
//  * weight gradient (Cout == 1): block = (image, output rows), wave = KH*KW/4 taps, lane = 8
//    channels; per (pixel, tap) one 16-byte x load (L1 hits across the waves' taps) and four
//    packed FMAs with the pixel's dY; fixed-order partials through the caller's workspace.
// Entered from the conv dispatch in conv.hip (irgan_conv_fwd / irgan_conv_wgrad_ws).
#include "conv_epilogue.h"

namespace {

typedef __attribute__((ext_vector_type(2))) __bf16 hbf2_t;
typedef __attribute__((ext_vector_type(2))) float hf2_t;

IRGAN_HD float dot8(uint4 a, uint4 b, float acc) {
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(hbf2_t, a.x), __builtin_bit_cast(hbf2_t, b.x), acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(hbf2_t, a.y), __builtin_bit_cast(hbf2_t, b.y), acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(hbf2_t, a.z), __builtin_bit_cast(hbf2_t, b.z), acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(hbf2_t, a.w), __builtin_bit_cast(hbf2_t, b.w), acc, false);
    return acc;
}

IRGAN_HD float wave_sum(float v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    return v;
}

IRGAN_HD hf2_t bf2pair(uint32_t w) { return hf2_t{__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)}; }

constexpr int HT = 256;   // threads per block (4 waves)
constexpr int HCW = 16;   // forward: output columns per block
constexpr int HDW = 1024; // backward-data: dY row span (Wo + KW - 1) staged per block

// ---- forward: y[n][i][j] = act(bias + sum_{ty, tx, c} w[(ty KW + tx) Cin + c] x[n][i + ty + c0y][j + tx + c0x][c])
template <int KH, int KW>
__global__ __launch_bounds__(HT) void head_fwd_kernel(const irgan_conv_desc d, const bf16_t* __restrict__ x,
                                                      const bf16_t* __restrict__ w, const float* __restrict__ bias,
                                                      void* __restrict__ y) {
    constexpr int XC = HCW + KW - 1;
    __shared__ uint4 sx[KH * XC * 64];  // [KH][XC][CG], Cin <= 512
    const int CG = d.Cin / 8;
    const int j0 = blockIdx.x * HCW, i = blockIdx.y, n = blockIdx.z;
    const int total = KH * XC * CG;
    for (int e0 = 0; e0 < total; e0 += 4 * HT) {  // four 16-byte loads in flight per thread
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = e0 + u * HT + threadIdx.x;
            const int g = e % CG, r = e / CG, col = r % XC, ty = r / XC;
            const int iy = i + ty + d.c0y, ix = j0 + col + d.c0x;
            v[u] = make_uint4(0u, 0u, 0u, 0u);
            if (e < total && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W)
                v[u] = *(const uint4*)(x + ((long)(n * d.H + iy) * d.W + ix) * d.ldx + d.xoff + g * 8);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (e0 + u * HT + threadIdx.x < total) sx[e0 + u * HT + threadIdx.x] = v[u];
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint4 wr[KH * KW];
#pragma unroll
    for (int t = 0; t < KH * KW; ++t)
        wr[t] = lane < CG ? *(const uint4*)(w + t * d.Cin + lane * 8) : make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    float acc[HCW / 4];
#pragma unroll
    for (int q = 0; q < HCW / 4; ++q) {
        const int jj = wv + 4 * q;
        float a = 0.f;
        if (lane < CG) {
#pragma unroll
            for (int ty = 0; ty < KH; ++ty)
#pragma unroll
                for (int tx = 0; tx < KW; ++tx) a = dot8(sx[(ty * XC + jj + tx) * CG + lane], wr[ty * KW + tx], a);
        }
        acc[q] = a;
    }
#pragma unroll
    for (int q = 0; q < HCW / 4; ++q) acc[q] = wave_sum(acc[q]);
    if (lane != 0) return;
    const float b = bias ? bias[0] : 0.f;
#pragma unroll
    for (int q = 0; q < HCW / 4; ++q) {
        const int j = j0 + wv + 4 * q;
        if (j >= d.Wo) continue;
        const float v = conv_act(acc[q] + b, d.act);
        const long o = (((long)n * d.OH + i * d.omy + d.ooy) * d.OW + j * d.omx + d.oox) * d.ldy + d.yoff;
        if (d.out_dtype == IRGAN_F32) {
            float* yp = (float*)y + o;
            *yp = d.accumulate ? *yp + v : v;
        } else {
            bf16_t* yp = (bf16_t*)y + o;
            *yp = f2bf(d.accumulate ? bf2f(*yp) + v : v);
        }
    }
}

// ---- backward-data as a forward conv of the one-channel (8-padded, channel 0 real) dY:
// dx[n][i][j][co] = sum_{ty, tx} w[co][(ty KW + tx) 8] dy[n][i + ty + c0y][j + tx + c0x][0]
template <int KH, int KW>
__global__ __launch_bounds__(HT) void head_dgrad_kernel(const irgan_conv_desc d, const bf16_t* __restrict__ dy,
                                                        const bf16_t* __restrict__ w, const float* __restrict__ bias,
                                                        void* __restrict__ dx, int Kw) {
    __shared__ float sd[KH * HDW];  // [KH][Wo + KW - 1] dY channel 0 of the rows this output row reads
    const int i = blockIdx.x, n = blockIdx.y;
    const int XW = d.Wo + KW - 1;
    for (int e = threadIdx.x; e < KH * XW; e += HT) {
        const int col = e % XW, ty = e / XW;
        const int iy = i + ty + d.c0y, ix = col + d.c0x;
        float v = 0.f;
        if ((unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W)
            v = bf2f(dy[((long)(n * d.H + iy) * d.W + ix) * d.ldx + d.xoff]);
        sd[e] = v;
    }
    const int CG = d.Cout / 8;
    const int cg = threadIdx.x % CG;  // HT % CG == 0: a thread keeps its channel group
    const int co = cg * 8;
    hf2_t wr[KH * KW][4];
#pragma unroll
    for (int t = 0; t < KH * KW; ++t)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float a = bf2f(w[(long)(co + 2 * k) * Kw + t * 8]);
            const float b = bf2f(w[(long)(co + 2 * k + 1) * Kw + t * 8]);
            wr[t][k] = hf2_t{a, b};
        }
    float4 b0 = make_float4(0.f, 0.f, 0.f, 0.f), b1 = b0;
    if (bias) {
        b0 = *(const float4*)(bias + co);
        b1 = *(const float4*)(bias + co + 4);
    }
    __syncthreads();
    for (int j = threadIdx.x / CG; j < d.Wo; j += HT / CG) {
        hf2_t acc[4] = {hf2_t{b0.x, b0.y}, hf2_t{b0.z, b0.w}, hf2_t{b1.x, b1.y}, hf2_t{b1.z, b1.w}};
#pragma unroll
        for (int ty = 0; ty < KH; ++ty)
#pragma unroll
            for (int tx = 0; tx < KW; ++tx) {
                const float g = sd[ty * XW + j + tx];
                const hf2_t gg = hf2_t{g, g};
#pragma unroll
                for (int k = 0; k < 4; ++k) acc[k] = __builtin_elementwise_fma(wr[ty * KW + tx][k], gg, acc[k]);
            }
        float v[8] = {acc[0].x, acc[0].y, acc[1].x, acc[1].y, acc[2].x, acc[2].y, acc[3].x, acc[3].y};
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = conv_act(v[k], d.act);
        const long o = (((long)n * d.OH + i * d.omy + d.ooy) * d.OW + j * d.omx + d.oox) * d.ldy + d.yoff + co;
        if (d.out_dtype == IRGAN_F32) {
            float4* yp = (float4*)((float*)dx + o);
            float4 p0 = make_float4(v[0], v[1], v[2], v[3]), p1 = make_float4(v[4], v[5], v[6], v[7]);
            if (d.accumulate) {
                const float4 q0 = yp[0], q1 = yp[1];
                p0.x += q0.x; p0.y += q0.y; p0.z += q0.z; p0.w += q0.w;
                p1.x += q1.x; p1.y += q1.y; p1.z += q1.z; p1.w += q1.w;
            }
            yp[0] = p0;
            yp[1] = p1;
        } else {
            uint4* yp = (uint4*)((bf16_t*)dx + o);
            if (d.accumulate) {
                const uint4 u = *yp;
                const uint32_t q[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    v[2 * k] += __uint_as_float(q[k] << 16);
                    v[2 * k + 1] += __uint_as_float(q[k] & 0xffff0000u);
                }
            }
            *yp = make_uint4(pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3]), pk_bf16(v[4], v[5]), pk_bf16(v[6], v[7]));
        }
    }
}

// ---- weight gradient: part[blk][t][c] = sum over the block's output pixels of dy * x_t[c];
// block = (image, HRG output rows); wave wv takes taps wv, wv + 4, ... (TPW of them); lane = 8
// channels of the Cin (lane < Cin / 8)
constexpr int HRG = 2, HJU = 4;
template <int KH, int KW>
__global__ __launch_bounds__(HT) void head_wgrad_kernel(const irgan_conv_desc d, const bf16_t* __restrict__ x,
                                                        const bf16_t* __restrict__ dy, float* __restrict__ part,
                                                        int nrg) {
    constexpr int TAPS = KH * KW, TPW = (TAPS + 3) / 4;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int rg = blockIdx.x % nrg, n = blockIdx.x / nrg;
    const int CG = d.Cin / 8;
    hf2_t acc[TPW][4];
#pragma unroll
    for (int u = 0; u < TPW; ++u)
#pragma unroll
        for (int k = 0; k < 4; ++k) acc[u][k] = hf2_t{0.f, 0.f};
    const int i1 = min(d.Ho, (rg + 1) * HRG);
    if (lane < CG) {
        for (int i = rg * HRG; i < i1; ++i) {
            const bf16_t* dyr = dy + ((long)(n * d.Ho + i) * d.Wo) * d.ldy + d.yoff;
            // HJU output columns per batch: all their loads in flight before the first FMA
            for (int j0 = 0; j0 < d.Wo; j0 += HJU) {
                float g[HJU];
                uint4 xv[HJU][TPW];
#pragma unroll
                for (int jj = 0; jj < HJU; ++jj) {
                    const int j = j0 + jj;
                    const bool okj = j < d.Wo;
                    g[jj] = okj ? bf2f(dyr[(long)j * d.ldy]) : 0.f;
#pragma unroll
                    for (int u = 0; u < TPW; ++u) {
                        const int t = wv + 4 * u;
                        const int iy = i + t / KW + d.c0y, ix = j + t % KW + d.c0x;
                        xv[jj][u] = (okj && t < TAPS && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W)
                                        ? *(const uint4*)(x + ((long)(n * d.H + iy) * d.W + ix) * d.ldx + d.xoff +
                                                          lane * 8)
                                        : make_uint4(0u, 0u, 0u, 0u);
                    }
                }
#pragma unroll
                for (int jj = 0; jj < HJU; ++jj) {
                    const hf2_t gg = hf2_t{g[jj], g[jj]};
#pragma unroll
                    for (int u = 0; u < TPW; ++u) {
                        acc[u][0] = __builtin_elementwise_fma(bf2pair(xv[jj][u].x), gg, acc[u][0]);
                        acc[u][1] = __builtin_elementwise_fma(bf2pair(xv[jj][u].y), gg, acc[u][1]);
                        acc[u][2] = __builtin_elementwise_fma(bf2pair(xv[jj][u].z), gg, acc[u][2]);
                        acc[u][3] = __builtin_elementwise_fma(bf2pair(xv[jj][u].w), gg, acc[u][3]);
                    }
                }
            }
        }
    }
    if (lane >= CG) return;
    float* pp = part + (long)blockIdx.x * TAPS * d.Cin;
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
        const int t = wv + 4 * u;
        if (t >= TAPS) continue;
        float4* q = (float4*)(pp + t * d.Cin + lane * 8);
        q[0] = make_float4(acc[u][0].x, acc[u][0].y, acc[u][1].x, acc[u][1].y);
        q[1] = make_float4(acc[u][2].x, acc[u][2].y, acc[u][3].x, acc[u][3].y);
    }
}

// dw[e] += sum over the nb partial rows in order (deterministic)
__global__ __launch_bounds__(256) void head_wgrad_reduce(const float* __restrict__ part, int nb, long n,
                                                         float* __restrict__ dw) {
    const long e = blockIdx.x * 256L + threadIdx.x;
    if (e >= n) return;
    float s = 0.f;
    for (int b = 0; b < nb; ++b) s += part[(long)b * n + e];
    dw[e] += s;
}

}  // namespace

// Forward of a stride-1 4x4 conv onto ONE output channel (bf16 operands, Cin % 8 == 0,
// Cin <= 512, ldx / xoff % 8, no mask); any output dtype / activation / accumulate.
extern "C" int irgan_conv_fwd_head(const irgan_conv_desc* d, const void* x, const void* w, const float* bias, void* y,
                                   const void* mask, hipStream_t st) {
    if ((long)d->N * d->Ho * d->Wo <= 0) return 0;
    if (d->dtype != IRGAN_BF16 || d->Cout != 1 || d->KH != 4 || d->KW != 4 || d->sy != 1 || d->sx != 1 ||
        d->Cin % 8 || d->Cin > 512 || d->cin_real || mask || d->ldx % 8 || d->xoff % 8 ||
        (d->out_dtype != IRGAN_F32 && d->out_dtype != IRGAN_BF16))
        return IRGAN_EUNSUPPORTED;
    head_fwd_kernel<4, 4><<<dim3(irgan_cdiv(d->Wo, HCW), d->Ho, d->N), HT, 0, st>>>(*d, (const bf16_t*)x,
                                                                                      (const bf16_t*)w, bias, y);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

// Backward-data of that layer as a forward conv of its dY: one real input channel stored 8-wide
// (Cin == 8, cin_real == 1), 4x4 stride-1 taps onto Cout % 8 == 0, Cout <= 256 * 8 with
// 256 % (Cout / 8) == 0 (a thread keeps one 8-channel group), no mask.
extern "C" int irgan_conv_dgrad_head(const irgan_conv_desc* d, const void* dy, const void* w, const float* bias,
                                     void* dx, const void* mask, hipStream_t st) {
    if ((long)d->N * d->Ho * d->Wo <= 0) return 0;
    const int cg = d->Cout / 8;
    if (d->dtype != IRGAN_BF16 || d->Cin != 8 || d->cin_real != 1 || d->KH != 4 || d->KW != 4 || d->sy != 1 ||
        d->sx != 1 || d->Cout % 8 || cg < 1 || HT % cg || mask || d->ldy % 8 || d->yoff % 8 ||
        (d->out_dtype != IRGAN_F32 && d->out_dtype != IRGAN_BF16) || d->Wo + 3 > HDW)
        return IRGAN_EUNSUPPORTED;
    const int Kw = irgan_cdiv(16 * 8, 64) * 64;
    head_dgrad_kernel<4, 4><<<dim3(d->Ho, d->N), HT, 0, st>>>(*d, (const bf16_t*)dy, (const bf16_t*)w, bias, dx, Kw);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

// Weight gradient of the one-output-channel 4x4 stride-1 layer: dw (fp32 [1][4][4][Cin]) +=
// sum over N x Ho x Wo of dy * x; bf16, Cin % 8 == 0, Cin <= 512, ldx / xoff % 8.  The block
// partials go through ws (fixed-order reduce); IRGAN_EUNSUPPORTED (nothing launched) when ws
// cannot hold them.
extern "C" int irgan_conv_wgrad_head(const irgan_conv_desc* d, const void* x, const void* dy, float* dw, float* ws,
                                     long ws_cap, hipStream_t st) {
    if ((long)d->N * d->Ho * d->Wo <= 0) return 0;
    if (d->dtype != IRGAN_BF16 || d->Cout != 1 || d->KH != 4 || d->KW != 4 || d->sy != 1 || d->sx != 1 ||
        d->Cin % 8 || d->Cin > 512 || d->ldx % 8 || d->xoff % 8 || !ws)
        return IRGAN_EUNSUPPORTED;
    const int nrg = irgan_cdiv(d->Ho, HRG);
    const int nb = d->N * nrg;
    const long n = 16L * d->Cin;
    if ((long)nb * n > ws_cap) return IRGAN_EUNSUPPORTED;
    head_wgrad_kernel<4, 4><<<nb, HT, 0, st>>>(*d, (const bf16_t*)x, (const bf16_t*)dy, ws, nrg);
    head_wgrad_reduce<<<irgan_cdiv(n, 256), 256, 0, st>>>(ws, nb, n, dw);
    IRGAN_LAUNCH_CHECK();
    return 0;
}
