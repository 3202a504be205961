// Shared device helpers for the gfx950 kernels (wave64, NHWC, bf16 as raw u16).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "irgan.h"

typedef uint16_t bf16_t;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4;

#define IRGAN_HD __device__ __forceinline__

IRGAN_HD float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
IRGAN_HD bf16_t f2bf(float f) {
    uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (bf16_t)((u >> 16) | 0x40);  // keep NaN a NaN
    u += 0x7fffu + ((u >> 16) & 1u);                                          // round to nearest even
    return (bf16_t)(u >> 16);
}

// typed scalar load/store through a dtype code (IRGAN_F32 / IRGAN_BF16)
IRGAN_HD float ldv(const void* p, int dt, int64_t i) {
    return dt == IRGAN_BF16 ? bf2f(((const bf16_t*)p)[i]) : ((const float*)p)[i];
}
IRGAN_HD void stv(void* p, int dt, int64_t i, float v) {
    if (dt == IRGAN_BF16) ((bf16_t*)p)[i] = f2bf(v); else ((float*)p)[i] = v;
}

template <typename T> IRGAN_HD float to_f(T v);
template <> IRGAN_HD float to_f<float>(float v) { return v; }
template <> IRGAN_HD float to_f<bf16_t>(bf16_t v) { return bf2f(v); }
template <typename T> IRGAN_HD T from_f(float v);
template <> IRGAN_HD float from_f<float>(float v) { return v; }
template <> IRGAN_HD bf16_t from_f<bf16_t>(float v) { return f2bf(v); }

IRGAN_HD int reflect_idx(int q, int n) {  // nn.ReflectionPad2d index map (|pad| < n)
    q = q < 0 ? -q : q;
    return q >= n ? 2 * n - 2 - q : q;
}

IRGAN_HD float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

#define IRGAN_LAUNCH_CHECK()                      \
    do {                                          \
        hipError_t e__ = hipGetLastError();       \
        if (e__ != hipSuccess) return (int)e__;   \
    } while (0)

static inline int irgan_cdiv(long a, long b) { return (int)((a + b - 1) / b); }
