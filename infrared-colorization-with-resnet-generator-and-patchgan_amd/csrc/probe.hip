// MFMA throughput probe: the roofline's MFMA peak measured on the box, beside
// the nominal 2.5 PFLOP/s dense bf16 of MI355X_MICROARCH.md.  Every wave issues back-to-back
// v_mfma_f32_16x16x32_bf16 (16384 FLOP, 16 cycles per SIMD) on operands loaded once from
// `src` -- random data, because the clock the chip holds under MFMA load depends on the
// operand values ('DVFS give-back' in the guide) -- into 8 independent accumulators, and
// writes one reduced float per lane so nothing is dead code.  No LDS, no memory traffic in
// the loop: the rate it reports is what a perfectly fed bf16 MFMA loop reaches on this box.
#include "common.h"

namespace {

constexpr int PROBE_SRC = 4096;  // uint4 entries of random bf16 operands (64 KiB)

__global__ __launch_bounds__(256) void mfma_probe_kernel(const uint4* __restrict__ src, float* __restrict__ out,
                                                         int iters) {
    const int tid = blockIdx.x * 256 + threadIdx.x;
    const uint4 a0 = src[(4 * tid) % PROBE_SRC], a1 = src[(4 * tid + 1) % PROBE_SRC];
    const uint4 b0 = src[(4 * tid + 2) % PROBE_SRC], b1 = src[(4 * tid + 3) % PROBE_SRC];
    const bf16x8_t A0 = __builtin_bit_cast(bf16x8_t, a0), A1 = __builtin_bit_cast(bf16x8_t, a1);
    const bf16x8_t B0 = __builtin_bit_cast(bf16x8_t, b0), B1 = __builtin_bit_cast(bf16x8_t, b1);
    f32x4 acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
            acc[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k & 1 ? A1 : A0, k & 2 ? B1 : B0, acc[k], 0, 0, 0);
    }
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
    out[tid] = s;
}

}  // namespace

extern "C" int irgan_mfma_probe(const void* src, float* out, int32_t blocks, int32_t iters, irgan_stream_t s) {
    if (!src || !out || blocks < 1 || iters < 1) return IRGAN_EINVAL;
    mfma_probe_kernel<<<blocks, 256, 0, (hipStream_t)s>>>((const uint4*)src, out, iters);
    IRGAN_LAUNCH_CHECK();
    return 0;
}
