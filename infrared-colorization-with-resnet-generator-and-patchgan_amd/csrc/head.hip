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
//  * weight gradient: VALU (the reduction runs over pixels, x's non-contiguous axis): x in
//    registers, dL/dy broadcast by v_readlane into packed fp32 FMAs, block partials summed
//    in a fixed order by one reduce pass.
//
// Deterministic (fixed summation order, no atomics).  C = 512 channels.
#include "common.h"

namespace {

constexpr int HC = 512, HS = 8;  // channels; input columns per wave (weight gradient)

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

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

// dw[ky * 4 + kx][c] += sum_{n, iy, ix} x[n][iy][ix][c] * g[n][iy + 1 - ky][ix + 1 - kx] (g = dL/dy,
// fp32 [N][Ho][Wo], pixel stride ldg; terms outside the output are zero).  The transpose of the
// backward-data product: a wave owns HS input columns of hr input rows, a lane 8 channels and
// the 16 taps' fp32 sums of them (128 registers); per input row the 4 x (HS + 3) dL/dy window
// is loaded one per lane and broadcast by v_readlane into packed fp32 FMAs.  The block's four
// wave sums are added in LDS in wave order and stored as one partial [16][512]; one ordered
// pass (head_wgrad_reduce) adds the partials into dw -- deterministic, no atomics.
// grid (ceil(nstrip / 4), ceil(H / hr), N)
__global__ __launch_bounds__(256) void head_wgrad_kernel(const bf16_t* __restrict__ x, int H, int W, int ldx, int xoff,
                                                         const float* __restrict__ g, int ldg, int hr, int nstrip,
                                                         float* __restrict__ part) {
    constexpr int GC = HS + 3;
    __shared__ float4 red[16 * HC / 4];   // 32 KB: [tap][channel]
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int strip = blockIdx.x * 4 + wv;
    const int iy0 = blockIdx.y * hr, n = blockIdx.z;
    const int Ho = H - 1, Wo = W - 1, ix0 = strip * HS;
    f32x2 a[16][4];
#pragma unroll
    for (int t = 0; t < 16; ++t)
#pragma unroll
        for (int k = 0; k < 4; ++k) a[t][k] = f32x2{0.f, 0.f};
    if (strip < nstrip) {   // wave-uniform; idle waves still take part in the block sum below
        const int iy1 = min(H, iy0 + hr);
        // per input row: lane r * GC + c holds g[n][iy + 1 - r][ix0 - 2 + c] (0 outside the
        // output), r = ky, and xv the row's HS pixels; the next row's load while this one sums
        auto load_row = [&](int iy, float& gl, uint4* xv) {
            gl = 0.f;
            if (lane < 4 * GC) {
                const int r = lane / GC, c = lane - r * GC;
                const int oy = iy + 1 - r, ox = ix0 - 2 + c;
                if ((unsigned)oy < (unsigned)Ho && (unsigned)ox < (unsigned)Wo)
                    gl = g[(((long)n * Ho + oy) * Wo + ox) * ldg];
            }
            const bf16_t* row = x + (long)(n * H + iy) * W * ldx + xoff + lane * 8;
#pragma unroll
            for (int p = 0; p < HS; ++p)
                xv[p] = ix0 + p < W ? *(const uint4*)(row + (long)(ix0 + p) * ldx) : make_uint4(0u, 0u, 0u, 0u);
        };
        float gl, gn = 0.f;
        uint4 xv[HS], xn[HS];
        load_row(iy0, gl, xv);
#pragma unroll 1
        for (int iy = iy0; iy < iy1; ++iy) {
            if (iy + 1 < iy1) load_row(iy + 1, gn, xn);
#pragma unroll
            for (int p = 0; p < HS; ++p) {
                const uint32_t u[4] = {xv[p].x, xv[p].y, xv[p].z, xv[p].w};
                f32x2 xf[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) xf[k] = f32x2{__uint_as_float(u[k] << 16), __uint_as_float(u[k] & 0xffff0000u)};
#pragma unroll
                for (int ky = 0; ky < 4; ++ky)
#pragma unroll
                    for (int kx = 0; kx < 4; ++kx) {
                        const float gv =
                            __int_as_float(__builtin_amdgcn_readlane(__float_as_int(gl), ky * GC + p + 3 - kx));
                        const f32x2 g2 = f32x2{gv, gv};
#pragma unroll
                        for (int k = 0; k < 4; ++k) a[ky * 4 + kx][k] = __builtin_elementwise_fma(xf[k], g2, a[ky * 4 + kx][k]);
                    }
            }
            gl = gn;
#pragma unroll
            for (int p = 0; p < HS; ++p) xv[p] = xn[p];
        }
    }
    for (int w = 0; w < 4; ++w) {   // block sum in wave order
        if (wv == w) {
#pragma unroll
            for (int t = 0; t < 16; ++t)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    float4& r = red[t * (HC / 4) + lane * 2 + h];
                    const f32x2 lo = a[t][2 * h], hi = a[t][2 * h + 1];
                    if (w == 0) r = make_float4(lo.x, lo.y, hi.x, hi.y);
                    else {
                        float4 v = r;
                        v.x += lo.x; v.y += lo.y; v.z += hi.x; v.w += hi.y;
                        r = v;
                    }
                }
        }
        __syncthreads();
    }
    const long b = ((long)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    float4* dst = (float4*)(part + b * 16 * HC);
    for (int e = threadIdx.x; e < 16 * HC / 4; e += 256) dst[e] = red[e];
}

// Ordered sum of the nb block partials (16 * 512 floats each) into dw in one pass: block =
// 64 float4 outputs x 8 waves, wave w adds partials [w * per, (w + 1) * per) with all its loads
// in flight (per <= 32), then wave 0 adds the 8 wave sums in order onto dw.
constexpr int HW_N = 16 * HC, HW_WAVES = 8, HW_PER = 32;
__global__ __launch_bounds__(64 * HW_WAVES) void head_wgrad_reduce(const float4* __restrict__ part, int nb,
                                                                   float4* __restrict__ dw) {
    __shared__ float4 sums[HW_WAVES][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int i = blockIdx.x * 64 + lane;   // float4 index in [0, HW_N / 4)
    const int per = (nb + HW_WAVES - 1) / HW_WAVES, b0 = wv * per;
    float4 v[HW_PER];
#pragma unroll
    for (int k = 0; k < HW_PER; ++k)
        v[k] = k < per && b0 + k < nb ? part[(long)(b0 + k) * (HW_N / 4) + i] : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 a = v[0];
#pragma unroll
    for (int k = 1; k < HW_PER; ++k) {
        a.x += v[k].x; a.y += v[k].y; a.z += v[k].z; a.w += v[k].w;
    }
    sums[wv][lane] = a;
    __syncthreads();
    if (wv == 0) {
        float4 r = dw[i];
#pragma unroll
        for (int w = 0; w < HW_WAVES; ++w) {
            r.x += sums[w][lane].x; r.y += sums[w][lane].y; r.z += sums[w][lane].z; r.w += sums[w][lane].w;
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
    if (off || C != HC || ldx % 8 || xoff % 8 || N > 65535 || H > 65535 || (long)N * H * W * ldx >= (1L << 31))
        return IRGAN_EUNSUPPORTED;
    const int nstrip = irgan_cdiv(W, HS);
    // rows per wave: the most (<= 8) that still launch >= 1024 waves, then more until the block
    // partials fit the reduce (<= 256)
    auto blocks = [&](int r) { return (long)irgan_cdiv(nstrip, 4) * irgan_cdiv(H, r) * N; };
    int hr = 8;
    while (hr > 1 && 4 * blocks(hr) < 1024) hr >>= 1;
    while (blocks(hr) > HW_WAVES * HW_PER) hr *= 2;
    const dim3 grid(irgan_cdiv(nstrip, 4), irgan_cdiv(H, hr), N);
    const int nb = grid.x * grid.y * grid.z;
    if (!ws || nb > HW_WAVES * HW_PER || (long)nb * HW_N > ws_cap) return IRGAN_EUNSUPPORTED;
    head_wgrad_kernel<<<grid, 256, 0, (hipStream_t)s>>>((const bf16_t*)x, H, W, ldx, xoff, g, ldg, hr, nstrip, ws);
    IRGAN_LAUNCH_CHECK();
    head_wgrad_reduce<<<HW_N / 4 / 64, 64 * HW_WAVES, 0, (hipStream_t)s>>>((const float4*)ws, nb, (float4*)dw);
    IRGAN_LAUNCH_CHECK();
    return 0;
}
