// One-off probe: operand lane maps of the gfx950 fp8 MFMAs and the fp8
// conversion's rounding (DESIGN.md s.fp8).  Built by tools/probe_fp8.py.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

// a, b: [64 lanes][32 bytes]; d: [64][4]
__global__ void k_scaled(const uint8_t* a, const uint8_t* b, float* d) {
    const int l = threadIdx.x;
    v8i va, vb;
    for (int i = 0; i < 8; ++i) {
        va[i] = ((const int*)(a + l * 32))[i];
        vb[i] = ((const int*)(b + l * 32))[i];
    }
    v4f c = {0.f, 0.f, 0.f, 0.f};
    c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(va, vb, c, 0, 0, 0, 127, 0, 127);
    for (int r = 0; r < 4; ++r) d[l * 4 + r] = c[r];
}

// a, b: [64][8 bytes]
__global__ void k_plain(const uint8_t* a, const uint8_t* b, float* d) {
    const int l = threadIdx.x;
    const long va = *(const long*)(a + l * 8), vb = *(const long*)(b + l * 8);
    v4f c = {0.f, 0.f, 0.f, 0.f};
    c = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(va, vb, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) d[l * 4 + r] = c[r];
}

__global__ void k_cvt(const float* x, uint8_t* y, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float v = __builtin_amdgcn_fmed3f(x[i], 448.f, -448.f);
    const int p = __builtin_amdgcn_cvt_pk_fp8_f32(v, v, 0, false);
    y[i] = (uint8_t)(p & 0xff);
}

extern "C" int probe_scaled(const void* a, const void* b, float* d) {
    k_scaled<<<1, 64>>>((const uint8_t*)a, (const uint8_t*)b, d);
    return (int)hipDeviceSynchronize();
}
extern "C" int probe_plain(const void* a, const void* b, float* d) {
    k_plain<<<1, 64>>>((const uint8_t*)a, (const uint8_t*)b, d);
    return (int)hipDeviceSynchronize();
}
extern "C" int probe_cvt(const float* x, void* y, int n) {
    k_cvt<<<(n + 255) / 256, 256>>>(x, (uint8_t*)y, n);
    return (int)hipDeviceSynchronize();
}
