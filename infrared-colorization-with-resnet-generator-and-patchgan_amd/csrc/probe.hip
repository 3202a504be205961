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
    // inline asm: each accumulator stays in its own registers across iterations (compiled
    // from the builtin, the loop-carried accumulators are rotated through v_accvgpr_mov copies
    // that wait on the MFMAs and halve the rate); a dependent MFMA is 8 issues (128 cycles) away
    f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0, c4 = c0, c5 = c0, c6 = c0, c7 = c0;
    for (int it = 0; it < iters; ++it) {
        asm volatile(
            "v_mfma_f32_16x16x32_bf16 %0, %8, %10, %0\n\t"
            "v_mfma_f32_16x16x32_bf16 %1, %9, %10, %1\n\t"
            "v_mfma_f32_16x16x32_bf16 %2, %8, %11, %2\n\t"
            "v_mfma_f32_16x16x32_bf16 %3, %9, %11, %3\n\t"
            "v_mfma_f32_16x16x32_bf16 %4, %8, %10, %4\n\t"
            "v_mfma_f32_16x16x32_bf16 %5, %9, %10, %5\n\t"
            "v_mfma_f32_16x16x32_bf16 %6, %8, %11, %6\n\t"
            "v_mfma_f32_16x16x32_bf16 %7, %9, %11, %7"
            : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7)
            : "v"(A0), "v"(A1), "v"(B0), "v"(B1));
    }
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");  // MFMA results before the VALU reads them
    const f32x4 t = ((c0 + c1) + (c2 + c3)) + ((c4 + c5) + (c6 + c7));
    const float s = (t[0] + t[1]) + (t[2] + t[3]);
    out[tid] = s;
}

}  // namespace

extern "C" int irgan_mfma_probe(const void* src, float* out, int32_t blocks, int32_t iters, irgan_stream_t s) {
    if (!src || !out || blocks < 1 || iters < 1) return IRGAN_EINVAL;
    mfma_probe_kernel<<<blocks, 256, 0, (hipStream_t)s>>>((const uint4*)src, out, iters);
    IRGAN_LAUNCH_CHECK();
    return 0;
}
