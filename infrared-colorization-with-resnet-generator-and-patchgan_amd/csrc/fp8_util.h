// e4m3 packing and the per-block amax record shared by the fp8 quantiser
// (fp8.hip) and the InstanceNorm passes that emit an fp8 copy of their output
// (norm.hip): the conversion is v_cvt_pk_fp8_f32 after a clamp to +-448 (round to
// nearest even = torch's float8_e4m3fn of the clamped value).
#pragma once
#include "common.h"

IRGAN_HD uint32_t pack4_fp8(float a, float b, float c, float d, float q) {
    a = __builtin_amdgcn_fmed3f(a * q, 448.f, -448.f);
    b = __builtin_amdgcn_fmed3f(b * q, 448.f, -448.f);
    c = __builtin_amdgcn_fmed3f(c * q, 448.f, -448.f);
    d = __builtin_amdgcn_fmed3f(d * q, 448.f, -448.f);
    int v = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
    v = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, v, true);
    return (uint32_t)v;
}

// 8 values -> 8 e4m3 bytes (one 8-byte store)
IRGAN_HD uint2 pack8_fp8(const float* v, float q) {
    uint2 o;
    o.x = pack4_fp8(v[0], v[1], v[2], v[3], q);
    o.y = pack4_fp8(v[4], v[5], v[6], v[7], q);
    return o;
}

// block max of m (every thread of a block of <= 1024 threads calls it) raised into
// partial `part % IRGAN_FP8_AMAX_PARTS` of an amax slot
__device__ inline void fp8_block_amax(float m, uint32_t* amax, int part) {
    __shared__ float red_amax[16];
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) red_amax[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < (int)(blockDim.x >> 6); ++k) m = fmaxf(m, red_amax[k]);
        if (m > 0.f) atomicMax(amax + part % IRGAN_FP8_AMAX_PARTS, __float_as_uint(m));
    }
}
