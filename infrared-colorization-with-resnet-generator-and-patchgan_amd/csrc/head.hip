// PatchGAN head: NLayerDiscriminator's last layer, Conv2d(ndf * 8, 1, kernel 4, stride 1, pad 1)
// (ir:625-627), forward, backward-data and weight gradient.  One output channel makes the
// implicit GEMMs 1 wide: on the generic MFMA conv kernels they ran as narrow tiles at 8-16
// TF/s, latency-bound (26-34 us each at B = 32).  Here the 16 taps are the GEMM's narrow side:
//
//  * forward: Z[tap][pixel] = w[tap] . x[pixel] for every input pixel (M = pixels, N = 16
//    taps, K = 512 on v_mfma_f32_16x16x32_bf16; x read once), then y = the 16 shifted taps of
//    Z summed per output pixel in a fixed order;
//  * backward-data: dx[pixel] = sum_tap G[pixel][tap] w[tap] with G the 16 shifted dL/dy
//    values of the pixel (K = 16 taps, run as K = 32 with dL/dy split into bf16 hi + lo, so
//    the fp32 gradient is not rounded to bf16), 16-byte bf16 stores;
//  * weight gradient: dW = G^T x (M = 16 taps, K = pixels): x staged in LDS and read
//    column-wise by ds_read_b64_tr_b16 (pixels are x's non-contiguous axis), G split hi + lo
//    as above; one partial per block, summed in a fixed order by one reduce pass.
//
// Deterministic (fixed summation order, no atomics).  C = 512 channels.
#include "common.h"

namespace {

constexpr int HC = 512;  // channels


IRGAN_HD f32x4 mfma(const uint4 a, const uint4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                   0, 0, 0);
}

// Forward, step 1: Z[tap][p] = sum_c w[tap][c] * x[p][c] for every input pixel p -- a GEMM of
// M = pixels, N = 16 taps, K = 512 on v_mfma_f32_16x16x32_bf16, one 16-pixel tile per wave.
// K step kk takes channels 32 kk ... 32 kk + 31 (lane quarter q: 32 kk + 8 q ... + 7), so a
// load instruction reads 64 contiguous bytes of each of the 16 pixels.
// z is [16][Pp] fp32 (Pp = P rounded up to 16); the D fragment's 4 pixels per lane are one
// 16-byte store.
__global__ __launch_bounds__(256) void head_fwd_z_kernel(const bf16_t* __restrict__ x, int P, int Pp, int ldx,
                                                         int xoff, const bf16_t* __restrict__ w, float* __restrict__ z) {
    const int lane = threadIdx.x & 63, q = lane >> 4, r = lane & 15;
    const int p0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 16;
    if (p0 >= P) return;   // wave-uniform
    uint4 wb[16], xa[16];
    const bf16_t* wr = w + r * HC + q * 8;   // B[k][tap r]
    const bf16_t* xr = x + (long)min(p0 + r, P - 1) * ldx + xoff + q * 8;   // A[pixel r][k]
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) xa[kk] = *(const uint4*)(xr + kk * 32);
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) wb[kk] = *(const uint4*)(wr + kk * 32);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) acc = mfma(xa[kk], wb[kk], acc);
    // D[pixel 4q + e][tap r]; rows past P are never read (Pp pads them)
    *(f32x4*)(z + (long)r * Pp + p0 + 4 * q) = acc;
}

// Forward, step 2: y[n][oy][ox] = bias + sum_{ky, kx} Z[ky * 4 + kx][n][oy + ky - 1][ox + kx - 1]
// (zero outside the input), taps in a fixed order; one thread per output pixel.
__global__ __launch_bounds__(256) void head_fwd_sum_kernel(const float* __restrict__ z, int Pp, int N, int H, int W,
                                                           const float* __restrict__ bias, float* __restrict__ y) {
    const int Ho = H - 1, Wo = W - 1;
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= (long)N * Ho * Wo) return;
    const int ox = i % Wo, oy = (i / Wo) % Ho, n = i / ((long)Wo * Ho);
    // all 16 loads issued at once (clamped addresses, zeroed after): no dependent load chain
    float v[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
        const int iy = min(max(oy + (t >> 2) - 1, 0), H - 1), ix = min(max(ox + (t & 3) - 1, 0), W - 1);
        v[t] = z[(long)t * Pp + ((long)n * H + iy) * W + ix];
    }
    float a = bias ? bias[0] : 0.f;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
        const bool in = (unsigned)(oy + (t >> 2) - 1) < (unsigned)H && (unsigned)(ox + (t & 3) - 1) < (unsigned)W;
        a += in ? v[t] : 0.f;
    }
    y[i] = a;
}

// Backward-data: dx[p][c] = sum_tap G[p][tap] * w[tap][c], G[p][ky * 4 + kx] = g[n][iy + 1 - ky]
// [ix + 1 - kx] (0 outside the output) -- a GEMM of K = 16 taps, run transposed on
// v_mfma_f32_16x16x32_bf16 (A = w^T: 16 channels x K, B = G^T: K x 16 pixels) with K = 32 =
// the taps twice: G split into bf16 hi + lo parts (g = hi + lo to 2^-16), w repeated, so
// the fp32 dL/dy is not rounded to bf16.  Rows of a tile pair are permuted so each lane's D
// fragments of the pair are 8 consecutive channels of one pixel (one 16-byte store).
// block = 4 waves x 128 channels, looping over HD_T 16-pixel tiles; grid ceil(P / (16 HD_T)).
constexpr int HD_T = 2;
__global__ __launch_bounds__(256) void head_dgrad_kernel(const float* __restrict__ g, int ldg,
                                                         const bf16_t* __restrict__ w, bf16_t* __restrict__ dx, int N,
                                                         int H, int W, int lddx, int dxoff) {
    const int lane = threadIdx.x & 63, q = lane >> 4, r = lane & 15, wv = threadIdx.x >> 6;
    const int Ho = H - 1, Wo = W - 1, P = N * H * W;
    const int t0 = (q & 1) * 8;   // this lane's 8 taps of K
    // A operand, 8 tiles (4 pairs x 2 halves): row r of tile (tp, h) is channel
    // wv * 128 + tp * 32 + 8 * (r >> 2) + 4 * h + (r & 3)
    uint4 wa[4][2];
#pragma unroll
    for (int tp = 0; tp < 4; ++tp)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int c = wv * 128 + tp * 32 + 8 * (r >> 2) + 4 * h + (r & 3);
            uint32_t u[4];
#pragma unroll
            for (int j = 0; j < 4; ++j)
                u[j] = (uint32_t)w[(t0 + 2 * j) * HC + c] | ((uint32_t)w[(t0 + 2 * j + 1) * HC + c] << 16);
            wa[tp][h] = make_uint4(u[0], u[1], u[2], u[3]);
        }
    for (int tile = 0; tile < HD_T; ++tile) {
        const int p0 = (blockIdx.x * HD_T + tile) * 16;
        if (p0 >= P) break;   // block-uniform
        // B operand: lane (pixel r, quarter q) holds G[p0 + r][t0 .. t0 + 7], hi (q < 2) or lo part
        const int p = p0 + r;
        const int ix = p % W, iy = (p / W) % H, n = p / (W * H);
        float gv[8];   // clamped loads all in flight, zeroed outside the output after
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int t = t0 + j, oy = min(max(iy + 1 - (t >> 2), 0), Ho - 1), ox = min(max(ix + 1 - (t & 3), 0), Wo - 1);
            gv[j] = g[(((long)min(n, N - 1) * Ho + oy) * Wo + ox) * ldg];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int t = t0 + j;
            if (!(p < P && (unsigned)(iy + 1 - (t >> 2)) < (unsigned)Ho && (unsigned)(ix + 1 - (t & 3)) < (unsigned)Wo))
                gv[j] = 0.f;
        }
        uint32_t gb[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t hi = pk_bf16(gv[2 * j], gv[2 * j + 1]);
            gb[j] = q < 2 ? hi
                          : pk_bf16(gv[2 * j] - __uint_as_float(hi << 16), gv[2 * j + 1] - __uint_as_float(hi & 0xffff0000u));
        }
        const uint4 bop = make_uint4(gb[0], gb[1], gb[2], gb[3]);
        bf16_t* dst = dx + (long)min(p, P - 1) * lddx + dxoff + wv * 128 + 8 * q;
#pragma unroll
        for (int tp = 0; tp < 4; ++tp) {
            const f32x4 z = {0.f, 0.f, 0.f, 0.f};
            const f32x4 d0 = mfma(wa[tp][0], bop, z), d1 = mfma(wa[tp][1], bop, z);
            // D[row 4q + e][pixel r]: channels tp * 32 + 8q + e (d0) and + 4 + e (d1)
            const uint4 st = make_uint4(pk_bf16(d0[0], d0[1]), pk_bf16(d0[2], d0[3]), pk_bf16(d1[0], d1[1]),
                                        pk_bf16(d1[2], d1[3]));
            if (p < P) *(uint4*)(dst + tp * 32) = st;
        }
    }
}

// Weight gradient on MFMA: dW[tap][c] = sum_p G[p][tap] x[p][c], a GEMM of M = 16 taps, N = 512
// channels, K = pixels.  Per 32-pixel chunk the block stages x[32][512] in LDS (one 16-byte
// load per thread and piece, coalesced) and each wave reads its B operands (x, K = pixels x
// 16 channels) column-wise with ds_read_b64_tr_b16 -- the reduction axis is x's non-contiguous
// one; A = G^T (16 taps x 32 pixels) is gathered from the fp32 dL/dy and split into bf16 hi +
// lo (two MFMAs per tile), so dL/dy keeps ~16 bits.  Wave = 128 channels (8 tiles of 16);
// block = chunks blockIdx.x, + gridDim.x, ...; one partial [16][512] per block.
constexpr int WG_PIT = HC * 2 + 32;   // bytes per staged pixel row (pad: rows 8 apart share no banks)
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4_t lds_bf16x4_t;
__global__ __launch_bounds__(256) void head_wgrad_mfma_kernel(const bf16_t* __restrict__ x, int N, int H, int W,
                                                              int ldx, int xoff, const float* __restrict__ g, int ldg,
                                                              int nchunk, float* __restrict__ part) {
    __shared__ __attribute__((aligned(16))) unsigned char sx[32 * WG_PIT];
    const int tid = threadIdx.x, lane = tid & 63, q = lane >> 4, r = lane & 15, wv = tid >> 6;
    const int Ho = H - 1, Wo = W - 1, P = N * H * W;
    f32x4 acc[8];
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    // chunk ch's x pieces and dL/dy gathers; the next chunk's are in flight during this one's MFMAs
    uint4 v[8];   // x[pc0 + row][16-byte piece]: row = e >> 6, piece = e & 63, e = tid + 256 k
    float gv[8];  // A = G^T: lane (tap r, quarter q) holds G[pc0 + 8q + j][r], j = 0..7
    auto load = [&](int ch) {
        const int pc0 = ch * 32;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int e = tid + 256 * k, p = pc0 + (e >> 6);
            v[k] = p < P ? *(const uint4*)(x + (long)p * ldx + xoff + (e & 63) * 8) : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int p = min(pc0 + 8 * q + j, P - 1);
            const int ix = p % W, iy = (p / W) % H, n = p / (W * H);
            const int oy = iy + 1 - (r >> 2), ox = ix + 1 - (r & 3);
            gv[j] = g[(((long)n * Ho + min(max(oy, 0), Ho - 1)) * Wo + min(max(ox, 0), Wo - 1)) * ldg];
            if (pc0 + 8 * q + j >= P || (unsigned)oy >= (unsigned)Ho || (unsigned)ox >= (unsigned)Wo) gv[j] = 0.f;
        }
    };
    if (blockIdx.x < nchunk) load(blockIdx.x);
    for (int ch = blockIdx.x; ch < nchunk; ch += gridDim.x) {   // block-uniform
        uint32_t hw[4], lw[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            hw[j] = pk_bf16(gv[2 * j], gv[2 * j + 1]);
            lw[j] = pk_bf16(gv[2 * j] - __uint_as_float(hw[j] << 16), gv[2 * j + 1] - __uint_as_float(hw[j] & 0xffff0000u));
        }
        const uint4 ahi = make_uint4(hw[0], hw[1], hw[2], hw[3]), alo = make_uint4(lw[0], lw[1], lw[2], lw[3]);
        __syncthreads();   // the previous chunk's reads are done
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int e = tid + 256 * k;
            *(uint4*)(sx + (e >> 6) * WG_PIT + (e & 63) * 16) = v[k];
        }
        __syncthreads();
        if (ch + (int)gridDim.x < nchunk) load(ch + gridDim.x);
        // B = x (K = 32 pixels x 16 channels): group q reads rows 8q .. 8q + 7 of the tile's 16
        // channels in two 4-row transposed reads; lane 4q' + p' addresses row 8q + q',
        // channels c0 + 4p' .. + 3, and receives its column (channel c0 + r) of the 4 rows
        const unsigned char* b1 = sx + (8 * q + (r >> 2)) * WG_PIT + (wv * 128 + 4 * (r & 3)) * 2;
#pragma unroll
        for (int nt = 0; nt < 8; ++nt) {
            const bf16x4_t t0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(b1 + nt * 32));
            const bf16x4_t t1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(b1 + nt * 32 + 4 * WG_PIT));
            const uint2 u0 = __builtin_bit_cast(uint2, t0), u1 = __builtin_bit_cast(uint2, t1);
            const uint4 bop = make_uint4(u0.x, u0.y, u1.x, u1.y);
            acc[nt] = mfma(ahi, bop, acc[nt]);
            acc[nt] = mfma(alo, bop, acc[nt]);
        }
    }
    // D[tap 4q + e][channel wv * 128 + nt * 16 + r]
    float* dst = part + (long)blockIdx.x * 16 * HC + wv * 128 + r;
#pragma unroll
    for (int nt = 0; nt < 8; ++nt)
#pragma unroll
        for (int e = 0; e < 4; ++e) dst[(4 * q + e) * HC + nt * 16] = acc[nt][e];
}

// Ordered sum of the nb (<= 256) block partials (16 * 512 floats each) into dw: block = 16
// float4 outputs x 16 partial groups; thread (column c, group k) adds partials k, k + 16, ...
// with all its loads in flight, then the 16 group sums are added in order onto dw.
constexpr int HW_N = 16 * HC, HW_MAXB = 256;
__global__ __launch_bounds__(256) void head_wgrad_reduce(const float4* __restrict__ part, int nb,
                                                         float4* __restrict__ dw) {
    __shared__ float4 sums[16][16];
    const int c = threadIdx.x & 15, k = threadIdx.x >> 4;
    const int i = blockIdx.x * 16 + c;   // float4 index in [0, HW_N / 4)
    float4 v[HW_MAXB / 16];
#pragma unroll
    for (int m = 0; m < HW_MAXB / 16; ++m) {
        const int b = k + 16 * m;
        v[m] = b < nb ? part[(long)b * (HW_N / 4) + i] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float4 a = v[0];
#pragma unroll
    for (int m = 1; m < HW_MAXB / 16; ++m) {
        a.x += v[m].x; a.y += v[m].y; a.z += v[m].z; a.w += v[m].w;
    }
    sums[k][c] = a;
    __syncthreads();
    if (k == 0) {
        float4 r = dw[i];
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            r.x += sums[m][c].x; r.y += sums[m][c].y; r.z += sums[m][c].z; r.w += sums[m][c].w;
        }
        dw[i] = r;
    }
}

}  // namespace

extern "C" int irgan_patch_head_fwd(const void* x, int32_t N, int32_t H, int32_t W, int32_t C, int32_t ldx,
                                    int32_t xoff, const void* w, const float* bias, float* y, float* ws,
                                    int64_t ws_floats, irgan_stream_t s) {
    if (!x || !w || !y) return IRGAN_EINVAL;
    if (N <= 0 || H < 2 || W < 2) return 0;
    const long P = (long)N * H * W, Pp = (P + 15) / 16 * 16;
    if (C != HC || ldx % 8 || xoff % 8 || P * ldx >= (1L << 31) || !ws || 16 * Pp > ws_floats)
        return IRGAN_EUNSUPPORTED;
    head_fwd_z_kernel<<<irgan_cdiv(P, 64), 256, 0, (hipStream_t)s>>>((const bf16_t*)x, P, Pp, ldx, xoff,
                                                                     (const bf16_t*)w, ws);
    IRGAN_LAUNCH_CHECK();
    head_fwd_sum_kernel<<<irgan_cdiv((long)N * (H - 1) * (W - 1), 256), 256, 0, (hipStream_t)s>>>(ws, Pp, N, H, W,
                                                                                                 bias, y);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_patch_head_dgrad(const float* g, int32_t ldg, const void* w, void* dx, int32_t N, int32_t H,
                                      int32_t W, int32_t C, int32_t lddx, int32_t dxoff, irgan_stream_t s) {
    if (!g || !w || !dx || ldg < 1) return IRGAN_EINVAL;
    if (N <= 0 || H < 2 || W < 2) return 0;
    const long P = (long)N * H * W;
    if (C != HC || lddx % 8 || dxoff % 8 || P * lddx >= (1L << 31)) return IRGAN_EUNSUPPORTED;
    head_dgrad_kernel<<<irgan_cdiv(P, 16 * HD_T), 256, 0, (hipStream_t)s>>>(g, ldg, (const bf16_t*)w, (bf16_t*)dx, N,
                                                                           H, W, lddx, dxoff);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_patch_head_wgrad(const void* x, int32_t N, int32_t H, int32_t W, int32_t C, int32_t ldx,
                                      int32_t xoff, const float* g, int32_t ldg, float* dw, float* ws, int64_t ws_cap,
                                      irgan_stream_t s) {
    if (!x || !g || !dw || ldg < 1) return IRGAN_EINVAL;
    if (N <= 0 || H < 2 || W < 2) return 0;
    static const bool off = getenv("IRGAN_NO_HEAD_WGRAD") != nullptr;   // A/B: the generic wgrad
    const long P = (long)N * H * W;
    if (off || C != HC || ldx % 8 || xoff % 8 || P * ldx >= (1L << 31)) return IRGAN_EUNSUPPORTED;
    const int nchunk = irgan_cdiv(P, 32), nb = min(nchunk, HW_MAXB);
    if (!ws || (long)nb * HW_N > ws_cap) return IRGAN_EUNSUPPORTED;
    head_wgrad_mfma_kernel<<<nb, 256, 0, (hipStream_t)s>>>((const bf16_t*)x, N, H, W, ldx, xoff, g, ldg, nchunk, ws);
    IRGAN_LAUNCH_CHECK();
    head_wgrad_reduce<<<HW_N / 4 / 16, 256, 0, (hipStream_t)s>>>((const float4*)ws, nb, (float4*)dw);
    IRGAN_LAUNCH_CHECK();
    return 0;
}
