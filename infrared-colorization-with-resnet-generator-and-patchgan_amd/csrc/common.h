// Shared device helpers for the gfx950 kernels (wave64, NHWC, bf16 as raw u16).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include "irgan.h"

typedef uint16_t bf16_t;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4;

#define IRGAN_HD __device__ __forceinline__


IRGAN_HD float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
// fp32 -> bf16, round to nearest even (NaN stays NaN): gfx950's v_cvt_pk_bf16_f32
IRGAN_HD bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }
// two values -> one packed word (lo in bits 0..15): ONE v_cvt_pk_bf16_f32
IRGAN_HD uint32_t pk_bf16(float lo, float hi) {
    typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
    const bf16x2_t v = {(__bf16)lo, (__bf16)hi};
    return __builtin_bit_cast(uint32_t, v);
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

// dw[i..i+3] += sum over splits s, in order, of slab[s][i..i+3] (the ordered split-K reduce of
// the weight-gradient kernels; deterministic).  The loads of 8 splits are issued together: one
// dependent load per split held the reduce at ~5 TB/s below the copy rate.
IRGAN_HD void slab_sum4(const float* __restrict__ slab, int splits, long n, float* __restrict__ dw, long i) {
    float4 a = ((const float4*)dw)[i];
    for (int s0 = 0; s0 < splits; s0 += 8) {
        float4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k)
            v[k] = s0 + k < splits ? ((const float4*)(slab + (long)(s0 + k) * n))[i] : float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (s0 + k < splits) {
                a.x += v[k].x;
                a.y += v[k].y;
                a.z += v[k].z;
                a.w += v[k].w;
            }
    }
    ((float4*)dw)[i] = a;
}

IRGAN_HD float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// ---- LDS-DMA pipelines ---------------------------------------------------
// global_load_lds_dwordx4: 16 bytes per lane from `src` into lds + 16*lane
// (M0 = the LDS byte offset, wave-uniform).  Issued through inline asm on
// purpose: when the compiler sees the builtin's LDS write it cannot tell the
// ring stage being prefetched from the one being read, and puts
// `s_waitcnt vmcnt(0)` in front of the next ds_read -- which waits for the
// prefetch just issued and serialises the whole pipeline.  The kernels order
// the stages themselves with counted wait_vmcnt<N>() + lds_barrier().
IRGAN_HD void glds16(const void* src, const void* lds) {
    const uint32_t m = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const char*)lds;
    asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "{m0}"(m) : "memory");
}
// Raw buffer resource (gfx9 V#: 64-bit base, num_records bytes, stride 0).
// Wave-uniform: the compiler keeps it in SGPRs.  A lane whose byte offset is
// >= num_records is dropped by the range check and its 16 bytes arrive as zeros.
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
IRGAN_HD i32x4 make_rsrc(const void* base, uint32_t bytes) {
    const uint64_t a = (uint64_t)(uintptr_t)base;
    i32x4 r;
    r.x = (int32_t)(uint32_t)a;
    r.y = (int32_t)(uint32_t)(a >> 32);
    r.z = (int32_t)bytes;
    r.w = 0x00020000;
    return r;
}
constexpr uint32_t IRGAN_OOB = 0x80000000u;  // byte offset that is out of range (num_records < 2^31)
// positions per border line of the line-form reflect ring workspace (conv_ring.hip: dy
// coordinates -2 .. 65 of a <= 64-long line), shared with conv_pp_kernel.h's epilogue fold
constexpr int IRGAN_RING_ROWS = 68;
// buffer_load_dwordx4 ... lds: 16 bytes per lane from rsrc.base + voff into
// lds + 16*lane (same M0 contract as glds16); no 64-bit address math per lane.
IRGAN_HD void blds16(i32x4 rsrc, uint32_t voff, const void* lds) {
    const uint32_t m = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const char*)lds;
    asm volatile("s_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rsrc), "{m0}"(m) : "memory");
}
// same with a wave-uniform byte offset in the instruction's soffset (SGPR)
IRGAN_HD void blds16(i32x4 rsrc, uint32_t voff, uint32_t soff, const void* lds) {
    const uint32_t m = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const char*)lds;
    asm volatile("s_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(voff), "s"(rsrc), "s"(soff), "{m0}"(m)
                 : "memory");
}
template <int N>
IRGAN_HD void wait_vmcnt() {
    static_assert(N >= 0 && N <= 63, "vmcnt");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// v from lane (lane ^ M), M in {1, 2, 4, 8} -- within each 16-lane row, by DPP on the VALU
// (no LDS round trip, unlike __shfl_xor's ds_bpermute): 1, 2 quad_perm; 8 row_ror:8; 4 as
// row_half_mirror (i -> 7 - i) then quad_perm [3,2,1,0] (i -> i ^ 3)
template <int M>
IRGAN_HD float dpp_xor16(float v) {
    int x = __float_as_int(v);
    if constexpr (M == 1) {
        x = __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false);
    } else if constexpr (M == 2) {
        x = __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false);
    } else if constexpr (M == 4) {
        x = __builtin_amdgcn_update_dpp(0, x, 0x141, 0xF, 0xF, false);
        x = __builtin_amdgcn_update_dpp(0, x, 0x1B, 0xF, 0xF, false);
    } else {
        static_assert(M == 8, "dpp_xor16: M in {1, 2, 4, 8}");
        x = __builtin_amdgcn_update_dpp(0, x, 0x128, 0xF, 0xF, false);
    }
    return __int_as_float(x);
}
IRGAN_HD void lds_barrier() { asm volatile("s_barrier" ::: "memory"); }

// XCD-aware tile order.  Workgroups are dealt round-robin to the 8 XCDs
// (b % 8), each with its own L2.  With nb % 8 == 0 the remap hands XCD k the
// contiguous logical range [k*nb/8, (k+1)*nb/8), so tiles that share input rows
// run at the same time on the same L2.  Speed only: any order is correct.
IRGAN_HD int xcd_tile(int b, int nb, int swz) {
    if (!swz || (nb & 7)) return b;
    return (b & 7) * (nb >> 3) + (b >> 3);
}

#define IRGAN_LAUNCH_CHECK()                    \
    do {                                          \
        hipError_t e__ = hipGetLastError();       \
        if (e__ != hipSuccess) return (int)e__;   \
    } while (0)

static inline int irgan_cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// Per-device host caches (a process may drive several GPUs): the CU count and the address
// of a __device__ symbol (a module global has one instance per device).  Lazily filled; two
// threads racing on a slot store the same value.
constexpr int IRGAN_MAX_DEVICES = 64;
static inline int irgan_device() {
    int d = 0;
    return (hipGetDevice(&d) == hipSuccess && d >= 0 && d < IRGAN_MAX_DEVICES) ? d : -1;
}
static inline int irgan_cu_count() {
    static int cache[IRGAN_MAX_DEVICES];
    const int dev = irgan_device();
    if (dev < 0) return 256;
    int c = __atomic_load_n(&cache[dev], __ATOMIC_RELAXED);
    if (!c) {
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c < 1) c = 256;
        __atomic_store_n(&cache[dev], c, __ATOMIC_RELAXED);
    }
    return c;
}
// address of `sym` on the current device; nullptr on failure
static inline void* irgan_symbol(const void* sym, void** cache) {
    const int dev = irgan_device();
    if (dev < 0) return nullptr;
    void* p = __atomic_load_n(&cache[dev], __ATOMIC_ACQUIRE);
    if (!p) {
        if (hipGetSymbolAddress(&p, sym) != hipSuccess) return nullptr;
        __atomic_store_n(&cache[dev], p, __ATOMIC_RELEASE);
    }
    return p;
}
static inline bool irgan_det(const irgan_conv_desc* d) { return (d->flags & IRGAN_CONV_DETERMINISTIC) != 0; }
// XCD-aware tile order (xcd_tile) for every launcher: on unless IRGAN_NO_XCD_SWZ is set (the
// one A/B switch kept for it: the L2 locality it buys is layer-dependent)
static inline int irgan_xcd_swz() {
    static const int v = getenv("IRGAN_NO_XCD_SWZ") ? 0 : 1;
    return v;
}
