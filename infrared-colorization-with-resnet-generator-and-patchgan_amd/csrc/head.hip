// PatchGAN head: NLayerDiscriminator's last layer, Conv2d(ndf * 8, 1, kernel 4, stride 1, pad 1)
// (ir:625-627), forward and backward-data.  One output channel makes these GEMMs 1 wide: on the
// MFMA kernels they ran as narrow tiles at 8-16 TF/s, latency-bound (30 us for 1 GFLOP at B = 32).
// Here they are VALU kernels bound by their one pass over the 512-channel activation:
//
//  * forward: a wave owns 8 output columns of one output row, a lane 8 channels; the wave
//    walks the 4 input rows once (11 columns each, in registers) and accumulates the 16 taps
//    with v_dot2c_f32_bf16 (two bf16 products per instruction into fp32), then one DPP /
//    readlane sum per output pixel;
//  * backward-data: a wave owns 8 input columns of one input row, a lane 8 channels with the 16
//    taps' weights in fp32 registers; each dx pixel is the sum of the 16 (tap, dy) terms (dy
//    zero outside the output), dy broadcast from one register by v_readlane; packed fp32 FMAs;
//    one 16-byte store per lane.
//
// Deterministic (fixed summation order, no atomics).  C = 512 channels (64 lanes x 8).
#include "common.h"

namespace {

constexpr int HC = 512, HS = 8;  // channels; output (forward) / input (backward) columns per wave

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

IRGAN_HD float dot8(const uint4 a, const uint4 b, float c) {
    c = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a.x), __builtin_bit_cast(bf16x2_t, b.x), c, false);
    c = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a.y), __builtin_bit_cast(bf16x2_t, b.y), c, false);
    c = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a.z), __builtin_bit_cast(bf16x2_t, b.z), c, false);
    c = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a.w), __builtin_bit_cast(bf16x2_t, b.w), c, false);
    return c;
}

// y[n][oy][ox] = bias + sum_{ky, kx, c} w[ky * 4 + kx][c] * x[n][oy + ky - 1][ox + kx - 1][c]
// grid (ceil(nstrip / 4), Ho, N), 4 waves per block, wave = strip of HS output columns
__global__ __launch_bounds__(256) void head_fwd_kernel(const bf16_t* __restrict__ x, int H, int W, int ldx, int xoff,
                                                       const bf16_t* __restrict__ w, const float* __restrict__ bias,
                                                       float* __restrict__ y, int nstrip) {
    const int lane = threadIdx.x & 63;
    const int strip = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (strip >= nstrip) return;  // wave-uniform
    const int oy = blockIdx.y, n = blockIdx.z;
    const int Ho = H - 1, Wo = W - 1, ox0 = strip * HS;
    uint4 wr[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) wr[t] = *(const uint4*)(w + t * HC + lane * 8);
    float acc[HS];
#pragma unroll
    for (int p = 0; p < HS; ++p) acc[p] = 0.f;
    // every column of the 4 input rows in flight at once (zero-padding rows / columns load zeros)
    uint4 col[4][HS + 3];
#pragma unroll
    for (int ky = 0; ky < 4; ++ky) {
        const int iy = oy + ky - 1;
        const bool rok = (unsigned)iy < (unsigned)H;
        const bf16_t* row = x + (long)(n * H + (rok ? iy : 0)) * W * ldx + xoff + lane * 8;
#pragma unroll
        for (int j = 0; j < HS + 3; ++j) {
            const int ix = ox0 - 1 + j;
            col[ky][j] = rok && (unsigned)ix < (unsigned)W ? *(const uint4*)(row + (long)ix * ldx)
                                                            : make_uint4(0u, 0u, 0u, 0u);
        }
    }
#pragma unroll
    for (int ky = 0; ky < 4; ++ky)
#pragma unroll
        for (int p = 0; p < HS; ++p)
#pragma unroll
            for (int kx = 0; kx < 4; ++kx) acc[p] = dot8(col[ky][p + kx], wr[ky * 4 + kx], acc[p]);
    // one sum per output pixel over the 64 lanes: DPP within each 16-lane row, then the four
    // row totals by v_readlane (no LDS round trips), in a fixed order
    const float b = bias ? bias[0] : 0.f;
    float out = 0.f;
#pragma unroll
    for (int p = 0; p < HS; ++p) {
        float v = acc[p];
        v += dpp_xor16<1>(v);
        v += dpp_xor16<2>(v);
        v += dpp_xor16<4>(v);
        v += dpp_xor16<8>(v);
        const float t = (__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0)) +
                         __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16))) +
                        (__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32)) +
                         __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48)));
        if (lane == p) out = t + b;
    }
    if (lane < HS && ox0 + lane < Wo) y[((long)n * Ho + oy) * Wo + ox0 + lane] = out;
}

// dx[n][iy][ix][c] = sum_{ky, kx} w[ky * 4 + kx][c] * g[n][iy + 1 - ky][ix + 1 - kx] (terms inside
// the Ho x Wo output only); g fp32 [N][Ho][Wo] with pixel stride ldg floats.  The 4 x (HS + 3)
// dL/dy values a wave needs are loaded once, one per lane, and broadcast by v_readlane; the
// channel pairs accumulate with packed fp32 FMAs.
// grid (ceil(nstrip / 4), H, N), wave = strip of HS input columns
typedef float f32x2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void head_dgrad_kernel(const float* __restrict__ g, int ldg,
                                                         const bf16_t* __restrict__ w, bf16_t* __restrict__ dx, int H,
                                                         int W, int lddx, int dxoff, int nstrip) {
    constexpr int GC = HS + 3;  // dL/dy columns per window row
    const int lane = threadIdx.x & 63;
    const int strip = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (strip >= nstrip) return;  // wave-uniform
    const int iy = blockIdx.y, n = blockIdx.z;
    const int Ho = H - 1, Wo = W - 1, ix0 = strip * HS;
    // lane r * GC + c holds g[n][iy + 1 - r][ix0 - 2 + c] (0 outside the output), r = ky
    float gl = 0.f;
    if (lane < 4 * GC) {
        const int r = lane / GC, c = lane - r * GC;
        const int oy = iy + 1 - r, ox = ix0 - 2 + c;
        if ((unsigned)oy < (unsigned)Ho && (unsigned)ox < (unsigned)Wo) gl = g[(((long)n * Ho + oy) * Wo + ox) * ldg];
    }
    f32x2 wf[16][4];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
        const uint4 v = *(const uint4*)(w + t * HC + lane * 8);
        const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) wf[t][k] = f32x2{__uint_as_float(u[k] << 16), __uint_as_float(u[k] & 0xffff0000u)};
    }
#pragma unroll
    for (int p = 0; p < HS; ++p) {
        const int ix = ix0 + p;
        if (ix >= W) break;  // wave-uniform
        f32x2 o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = f32x2{0.f, 0.f};
#pragma unroll
        for (int ky = 0; ky < 4; ++ky)
#pragma unroll
            for (int kx = 0; kx < 4; ++kx) {
                // g[iy + 1 - ky][ix + 1 - kx] = window (ky, p + 3 - kx)
                const float gv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(gl), ky * GC + p + 3 - kx));
                const f32x2 g2 = f32x2{gv, gv};
#pragma unroll
                for (int k = 0; k < 4; ++k) o[k] = __builtin_elementwise_fma(wf[ky * 4 + kx][k], g2, o[k]);
            }
        uint4 st;
        st.x = pk_bf16(o[0].x, o[0].y);
        st.y = pk_bf16(o[1].x, o[1].y);
        st.z = pk_bf16(o[2].x, o[2].y);
        st.w = pk_bf16(o[3].x, o[3].y);
        *(uint4*)(dx + ((long)(n * H + iy) * W + ix) * lddx + dxoff + lane * 8) = st;
    }
}

}  // namespace

extern "C" int irgan_patch_head_fwd(const void* x, int32_t N, int32_t H, int32_t W, int32_t C, int32_t ldx,
                                    int32_t xoff, const void* w, const float* bias, float* y, irgan_stream_t s) {
    if (!x || !w || !y) return IRGAN_EINVAL;
    if (N <= 0 || H < 2 || W < 2) return 0;
    if (C != HC || ldx % 8 || xoff % 8 || N > 65535 || H > 65535 || (long)N * H * W * ldx >= (1L << 31))
        return IRGAN_EUNSUPPORTED;
    const int nstrip = irgan_cdiv(W - 1, HS);
    head_fwd_kernel<<<dim3(irgan_cdiv(nstrip, 4), H - 1, N), 256, 0, (hipStream_t)s>>>(
        (const bf16_t*)x, H, W, ldx, xoff, (const bf16_t*)w, bias, y, nstrip);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_patch_head_dgrad(const float* g, int32_t ldg, const void* w, void* dx, int32_t N, int32_t H,
                                      int32_t W, int32_t C, int32_t lddx, int32_t dxoff, irgan_stream_t s) {
    if (!g || !w || !dx || ldg < 1) return IRGAN_EINVAL;
    if (N <= 0 || H < 2 || W < 2) return 0;
    if (C != HC || lddx % 8 || dxoff % 8 || N > 65535 || H > 65535 || (long)N * H * W * lddx >= (1L << 31))
        return IRGAN_EUNSUPPORTED;
    const int nstrip = irgan_cdiv(W, HS);
    head_dgrad_kernel<<<dim3(irgan_cdiv(nstrip, 4), H, N), 256, 0, (hipStream_t)s>>>(
        g, ldg, (const bf16_t*)w, (bf16_t*)dx, H, W, lddx, dxoff, nstrip);
    IRGAN_LAUNCH_CHECK();
    return 0;
}
