// LDS-staged epilogue shared by the bf16 LDS-DMA conv kernels (256-pixel x BN
// block tile, WM x WN waves, 16x16 MFMA fragments: pixel = wm*(256/WM) + i*16 +
// (lane>>4)*4 + r, channel = wn*(BN/WN) + j*16 + (lane&15)).
//
// Writing bf16 straight from the accumulators stores 2 bytes per lane (16-lane
// 32-byte runs), which made output-heavy layers (wide images, short K) store
// bound.  Instead: bias + activation in registers -> fp32 tile in LDS (row
// stride BN+4 floats, conflict-free b32 writes) -> each lane re-reads 8
// consecutive channels of one pixel and applies mask / accumulate with 16-byte
// global loads, then stores 16 bytes (bf16) or 32 bytes (fp32).
#pragma once
#include "common.h"

IRGAN_HD float conv_act(float v, int act) {
    if (act == IRGAN_ACT_RELU) return v > 0.f ? v : 0.f;
    if (act == IRGAN_ACT_LRELU) return v > 0.f ? v : 0.2f * v;
    if (act == IRGAN_ACT_TANH) return tanhf(v);
    return v;
}

IRGAN_HD float mask_mul(float mv, int mask_act) { return mv > 0.f ? 1.f : (mask_act == 2 ? 0.2f : 0.f); }

// Two packed bf16 values times the ReLU mask of two packed bf16 mask values, on the rounded
// bits: a value is kept where its mask is > 0 (bits 0x0001..0x7f80), else it becomes the
// zero of its sign (v * 0.f; Inf / NaN * 0 -> NaN), exactly pk_bf16(v * mask_mul(m, 1)).
IRGAN_HD uint32_t relu_mask_pk(uint32_t v, uint32_t m) {
    uint32_t out = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint32_t vb = (v >> (16 * h)) & 0xffffu, mb = (m >> (16 * h)) & 0xffffu;
        const uint32_t r = (mb - 1u) < 0x7f80u ? vb : ((vb & 0x7f80u) == 0x7f80u ? 0x7fc0u : (vb & 0x8000u));
        out |= r << (16 * h);
    }
    return out;
}

// 8 consecutive output channels co..co+7 of pixel pix: mask, accumulate, store
// (vec: 16-byte aligned full run; else per-channel with the Cout bound)
IRGAN_HD void conv_store8(const irgan_conv_desc& d, float (&v)[8], long pix, int co, bool vec, bool out_f32,
                          void* __restrict__ y, const void* __restrict__ mask) {
    const long off = pix * d.ldy + d.yoff + co;
    if (vec) {
        if (mask) {
            const uint4 u = *(const uint4*)((const bf16_t*)mask + pix * d.ldm + d.moff + co);
            const uint32_t q[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                v[2 * k] *= mask_mul(__uint_as_float(q[k] << 16), d.mask_act);
                v[2 * k + 1] *= mask_mul(__uint_as_float(q[k] & 0xffff0000u), d.mask_act);
            }
        }
        if (out_f32) {
            float4* yp = (float4*)((float*)y + off);
            if (d.accumulate) {
                const float4 y0 = yp[0], y1 = yp[1];
                v[0] += y0.x; v[1] += y0.y; v[2] += y0.z; v[3] += y0.w;
                v[4] += y1.x; v[5] += y1.y; v[6] += y1.z; v[7] += y1.w;
            }
            yp[0] = make_float4(v[0], v[1], v[2], v[3]);
            yp[1] = make_float4(v[4], v[5], v[6], v[7]);
        } else {
            uint4* yp = (uint4*)((bf16_t*)y + off);
            if (d.accumulate) {
                const uint4 u = *yp;
                const uint32_t q[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    v[2 * k] += __uint_as_float(q[k] << 16);
                    v[2 * k + 1] += __uint_as_float(q[k] & 0xffff0000u);
                }
            }
            uint4 o;
            o.x = pk_bf16(v[0], v[1]);
            o.y = pk_bf16(v[2], v[3]);
            o.z = pk_bf16(v[4], v[5]);
            o.w = pk_bf16(v[6], v[7]);
            *yp = o;
        }
    } else {
        for (int k = 0; k < 8 && co + k < d.Cout; ++k) {
            float vk = v[k];
            if (mask) vk *= mask_mul(bf2f(((const bf16_t*)mask)[pix * d.ldm + d.moff + co + k]), d.mask_act);
            if (out_f32) {
                float* yp = (float*)y + off + k;
                *yp = d.accumulate ? *yp + vk : vk;
            } else {
                bf16_t* yp = (bf16_t*)y + off + k;
                *yp = f2bf(d.accumulate ? bf2f(*yp) + vk : vk);
            }
        }
    }
}

// smem must hold (256 / PASSES) * (BN + 4) floats; pix_of(m) -> output pixel
// index or -1.  PASSES > 1 stages the tile in pixel slabs (slab p = the waves
// with wm * PASSES / WM == p) when the whole fp32 tile does not fit in LDS.
template <int BN, int MI, int NJ, int WM, int WN, int NT, int PASSES = 1, typename PixFn>
__device__ __forceinline__ void conv_epilogue(const irgan_conv_desc& d, const f32x4 (&acc)[MI][NJ], char* smem,
                                              int wm, int wn, int n0, const float* __restrict__ bias,
                                              void* __restrict__ y, const void* __restrict__ mask, PixFn pix_of) {
    static_assert(WM % PASSES == 0, "slabs follow the wave rows");
    constexpr int RS = BN + 4, SLAB = 256 / PASSES;
    float* st = (float*)smem;
    const int tid = threadIdx.x, lane = tid & 63;
    constexpr int LPP = BN / 8;    // lanes per pixel (8 channels each)
    constexpr int PPP = NT / LPP;  // pixels per pass
    const int ch = (tid % LPP) * 8, co = n0 + ch;
    const bool out_f32 = d.out_dtype == IRGAN_F32;
    const bool full = co + 8 <= d.Cout;
    const bool vec = full && (out_f32 ? (d.ldy % 4 == 0 && d.yoff % 4 == 0) : (d.ldy % 8 == 0 && d.yoff % 8 == 0)) &&
                     (!mask || (d.ldm % 8 == 0 && d.moff % 8 == 0));
#pragma unroll 1
    for (int pass = 0; pass < PASSES; ++pass) {
        __syncthreads();  // every wave is done reading its operand tiles / the previous slab
        if (wm * PASSES / WM == pass) {
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int cj = wn * (BN / WN) + j * 16 + (lane & 15);
                const int cg = n0 + cj;
                const float b = (bias && cg < d.Cout) ? bias[cg] : 0.f;
#pragma unroll
                for (int i = 0; i < MI; ++i)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int m = wm * (256 / WM) + i * 16 + (lane >> 4) * 4 + r - pass * SLAB;
                        st[m * RS + cj] = conv_act(acc[i][j][r] + b, d.act);
                    }
            }
        }
        __syncthreads();
        if (co >= d.Cout) continue;
        for (int ms = tid / LPP; ms < SLAB; ms += PPP) {
            const int m = ms + pass * SLAB;
            const long pix = pix_of(m);
            if (pix < 0) continue;
            const float4 a0 = *(const float4*)(st + ms * RS + ch), a1 = *(const float4*)(st + ms * RS + ch + 4);
            float v[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
            conv_store8(d, v, pix, co, vec, out_f32, y, mask);
        }
    }
}
