// fp8 (OCP e4m3) operands of the conv path (BASELINE config 5): per-tensor
// power-of-two scales with delayed scaling.
//
//  * fp8_quant_kernel: y = e4m3(clamp(x * q, +-448)) for an NHWC slice (bf16 or
//    fp32 in, dense or strided fp8 out; round to nearest even, the hardware
//    v_cvt_pk_fp8_f32 = torch's float8_e4m3fn conversion), and the max |x| of
//    what it read recorded into the slot's IRGAN_FP8_AMAX_PARTS partial maxima
//    (uint32 bits of a non-negative float, so an integer max orders them; block b
//    updates part b % PARTS, so the atomics do not pile up on one address).  One
//    HBM pass: read 2 B, write 1 B per element.
//  * fp8_amax_kernel: the max only (first use of a tensor, weights).
//  * fp8_scale_kernel: per slot, amax = max of its partials, q =
//    2^floor(log2(448 / amax)) (1 when amax is 0 or not finite), dq = 1 / q;
//    optionally clears the partials for the next step.  A
//    tensor quantised at step t uses the q made from its step t-1 amax (delayed
//    scaling); values beyond 448 / q saturate.
//  * the *_batch kernels run a table of jobs (the per-step weight re-quantisation
//    of every fp8 layer in two launches).
// Byte streams, no LDS beyond the block max, no MFMA.
#include "fp8_util.h"

namespace {

constexpr int TPB = 256;

// 8 channels per thread-item; C % 8 == 0, ld / off % 8 == 0 (bf16) or % 4 (fp32).
template <typename T>
__global__ __launch_bounds__(TPB) void fp8_quant_kernel(const T* __restrict__ x, long P, int C, int ldx, int xoff,
                                                        uint8_t* __restrict__ y, int ldy, int yoff,
                                                        const float* __restrict__ q, uint32_t* __restrict__ amax) {
    const float qs = q ? *q : 1.f;
    const int c8 = C / 8;
    const long items = P * c8;
    float m = 0.f;
    for (long e = blockIdx.x * (long)TPB + threadIdx.x; e < items; e += (long)gridDim.x * TPB) {
        const long p = e / c8;
        const int c = (int)(e - p * c8) * 8;
        float v[8];
        if constexpr (sizeof(T) == 2) {
            const uint4 r = *(const uint4*)(x + p * ldx + xoff + c);
            const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                v[2 * k] = __uint_as_float(w[k] << 16);
                v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
            }
        } else {
            const float4 a = *(const float4*)(x + p * ldx + xoff + c), b = *(const float4*)(x + p * ldx + xoff + c + 4);
            v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) m = fmaxf(m, fabsf(v[k]));
        if (y) {
            *(uint2*)(y + p * ldy + yoff + c) = pack8_fp8(v, qs);
        }
    }
    if (amax) fp8_block_amax(m, amax, blockIdx.x);
}

__global__ void fp8_scale_kernel(uint32_t* __restrict__ amax, int n, float* __restrict__ q, float* __restrict__ dq,
                                 int reset) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t* ap = amax + (long)i * IRGAN_FP8_AMAX_PARTS;
    uint32_t mb = 0;
    for (int k = 0; k < IRGAN_FP8_AMAX_PARTS; ++k) mb = ap[k] > mb ? ap[k] : mb;
    const float a = __uint_as_float(mb);
    float s = 1.f;
    if (a > 0.f && a <= 3.0e38f) s = exp2f(floorf(log2f(448.f / a)));
    s = fminf(fmaxf(s, 0x1p-100f), 0x1p100f);
    q[i] = s;
    dq[i] = 1.f / s;  // exact: s is a power of two
    if (reset)
        for (int k = 0; k < IRGAN_FP8_AMAX_PARTS; ++k) ap[k] = 0u;
}

// job table: {src, dst, n, slot}; src bf16 contiguous, dst fp8 contiguous, n % 8 == 0
struct QJob {
    const bf16_t* src;
    uint8_t* dst;
    int64_t n;
    int32_t slot, pad;
};

__global__ __launch_bounds__(TPB) void fp8_batch_kernel(const QJob* __restrict__ jobs, const float* __restrict__ q,
                                                        uint32_t* __restrict__ amax) {
    const QJob j = jobs[blockIdx.y];
    const long items = j.n / 8;
    const float qs = q ? q[j.slot] : 1.f;
    float m = 0.f;
    for (long e = blockIdx.x * (long)TPB + threadIdx.x; e < items; e += (long)gridDim.x * TPB) {
        const uint4 r = *(const uint4*)(j.src + e * 8);
        const uint32_t w[4] = {r.x, r.y, r.z, r.w};
        float v[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            v[2 * k] = __uint_as_float(w[k] << 16);
            v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
        }
        if (amax) {
#pragma unroll
            for (int k = 0; k < 8; ++k) m = fmaxf(m, fabsf(v[k]));
        } else {
            *(uint2*)(j.dst + e * 8) = pack8_fp8(v, qs);
        }
    }
    if (amax) fp8_block_amax(m, amax + (long)j.slot * IRGAN_FP8_AMAX_PARTS, blockIdx.x);
}

int grid_for(long items) { return (int)std::max<long>(1, std::min<long>(irgan_cdiv(items, TPB), 2048)); }

}  // namespace

extern "C" int irgan_fp8_quant(const void* x, int32_t dt, int64_t P, int32_t C, int32_t ldx, int32_t xoff, void* y,
                               int32_t ldy, int32_t yoff, const float* q, uint32_t* amax, irgan_stream_t s) {
    if (P <= 0 || C <= 0) return 0;
    if (!x || (!y && !amax) || C % 8 || ldx % 8 || xoff % 8 || (y && (ldy % 8 || yoff % 8 || ldy < C + yoff)) ||
        ldx < C + xoff || (dt != IRGAN_BF16 && dt != IRGAN_F32))
        return IRGAN_EINVAL;
    const int g = grid_for(P * (C / 8));
    if (dt == IRGAN_BF16)
        fp8_quant_kernel<bf16_t><<<g, TPB, 0, (hipStream_t)s>>>((const bf16_t*)x, P, C, ldx, xoff, (uint8_t*)y, ldy,
                                                                yoff, q, amax);
    else
        fp8_quant_kernel<float><<<g, TPB, 0, (hipStream_t)s>>>((const float*)x, P, C, ldx, xoff, (uint8_t*)y, ldy,
                                                               yoff, q, amax);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_fp8_scale(uint32_t* amax, int32_t n, float* q, float* dq, int32_t reset, irgan_stream_t s) {
    if (n <= 0) return 0;
    if (!amax || !q || !dq) return IRGAN_EINVAL;
    fp8_scale_kernel<<<irgan_cdiv(n, 64), 64, 0, (hipStream_t)s>>>(amax, n, q, dq, reset);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_fp8_quant_batch(const void* jobs, int32_t njobs, int64_t max_n, const float* q, uint32_t* amax,
                                     irgan_stream_t s) {
    if (njobs <= 0) return 0;
    if (!jobs || njobs > 65535 || max_n <= 0 || (!q && !amax)) return IRGAN_EINVAL;
    dim3 g(grid_for(max_n / 8), njobs);
    fp8_batch_kernel<<<g, TPB, 0, (hipStream_t)s>>>((const QJob*)jobs, amax ? nullptr : q, amax);
    IRGAN_LAUNCH_CHECK();
    return 0;
}
