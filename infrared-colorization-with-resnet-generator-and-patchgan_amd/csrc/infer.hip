// Inference-side conversions and evaluation reductions (SURVEY.md 8(f) rows 1
// and 4): the generator's NHWC fp32 output -> uint8 RGB on the device
// (tensor_to_rgb_image, ir:865-876) and the per-image MAE / MSE sums of
// compute_metrics (ir:1184-1206) over uint8 prediction / ground-truth pairs
// (run_test feeds it pred_u8 / 255 and load_rgb_image(...) = gt_u8 / 255,
// ir:1412-1415).  Both are HBM-bound byte streams: 16 bytes of output per lane
// per iteration, no LDS.
#include "common.h"

namespace {

constexpr int TPB = 256;

// numpy's float32 pipeline of ir:872-874, element by element:
//   x = (x + 1.0) / 2.0 ; x = clip(x, 0, 1) ; (x * 255.0).astype(uint8)
// (NEP 50: the Python scalars stay float32; astype truncates toward zero).
// The division by 2 is exact, so * 0.5f is the same float.  NaN maps to 0
// (np.clip keeps NaN and the cast of NaN is platform-defined; we pin 0).
IRGAN_HD uint32_t to_u8(float x) {
    float v = __fmul_rn(__fadd_rn(x, 1.0f), 0.5f);
    v = v > 0.f ? v : 0.f;  // also NaN -> 0
    v = v < 1.f ? v : 1.f;
    return (uint32_t)(int)__fmul_rn(v, 255.0f);
}

// x: NHWC fp32 slice (pixel p, channel c at x[p*ldx + xoff + c]); out: [P][C] u8.
__global__ __launch_bounds__(TPB) void rgb_u8_kernel(const float* __restrict__ x, int ldx, int xoff, int C, long total,
                                                     uint8_t* __restrict__ out) {
    // each thread writes 16 consecutive output bytes (the total % 16 tail by block 0)
    const long n16 = total / 16;
    for (long i = blockIdx.x * (long)TPB + threadIdx.x; i < n16; i += (long)gridDim.x * TPB) {
        uint32_t w[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            uint32_t acc = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const long e = i * 16 + q * 4 + b;
                const long p = e / C;
                const int c = (int)(e - p * C);
                acc |= to_u8(x[p * ldx + xoff + c]) << (8 * b);
            }
            w[q] = acc;
        }
        *(uint4*)(out + i * 16) = uint4{w[0], w[1], w[2], w[3]};
    }
    if (blockIdx.x == 0) {
        for (long e = n16 * 16 + threadIdx.x; e < total; e += TPB) {
            const long p = e / C;
            const int c = (int)(e - p * C);
            out[e] = (uint8_t)to_u8(x[p * ldx + xoff + c]);
        }
    }
}

// Per-image sums over `per` bytes: d = float(pred)/255 - float(gt)/255 in fp32
// (as numpy forms diff, ir:1197); |d| and d*d accumulated per thread in fp64,
// combined in a fixed order (deterministic).  grid (blocks_per_image, N);
// partials[(n*gridDim.x + b)*2 + {0,1}].
__global__ __launch_bounds__(TPB) void metrics_u8_kernel(const uint8_t* __restrict__ pred,
                                                         const uint8_t* __restrict__ gt, long per,
                                                         double* __restrict__ partials) {
    __shared__ double s0[TPB], s1[TPB];
    const int n = blockIdx.y;
    const uint8_t* a = pred + (long)n * per;
    const uint8_t* b = gt + (long)n * per;
    double ad = 0.0, sq = 0.0;
    const bool vec = (per % 16) == 0 && ((uintptr_t)a % 16) == 0 && ((uintptr_t)b % 16) == 0;
    auto one = [&](uint32_t pa, uint32_t pb) {
        const float d = __fsub_rn(__fdiv_rn((float)pa, 255.0f), __fdiv_rn((float)pb, 255.0f));
        ad += (double)fabsf(d);
        sq += (double)__fmul_rn(d, d);
    };
    if (vec) {
        for (long i = blockIdx.x * (long)TPB + threadIdx.x; i < per / 16; i += (long)gridDim.x * TPB) {
            const uint4 u = *(const uint4*)(a + i * 16), v = *(const uint4*)(b + i * 16);
            const uint32_t ua[4] = {u.x, u.y, u.z, u.w}, vb[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int k = 0; k < 4; ++k) one((ua[q] >> (8 * k)) & 255u, (vb[q] >> (8 * k)) & 255u);
        }
    } else {
        for (long i = blockIdx.x * (long)TPB + threadIdx.x; i < per; i += (long)gridDim.x * TPB) one(a[i], b[i]);
    }
    s0[threadIdx.x] = ad;
    s1[threadIdx.x] = sq;
    __syncthreads();
    for (int w = TPB / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
            s0[threadIdx.x] += s0[threadIdx.x + w];
            s1[threadIdx.x] += s1[threadIdx.x + w];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        partials[((long)n * gridDim.x + blockIdx.x) * 2] = s0[0];
        partials[((long)n * gridDim.x + blockIdx.x) * 2 + 1] = s1[0];
    }
}

__global__ void metrics_finalize_kernel(const double* __restrict__ partials, int nb, int N, double* __restrict__ sums) {
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    double s = 0.0, q = 0.0;
    for (int b = 0; b < nb; ++b) {
        s += partials[((long)n * nb + b) * 2];
        q += partials[((long)n * nb + b) * 2 + 1];
    }
    sums[2 * n] = s;
    sums[2 * n + 1] = q;
}

// skimage.metrics.structural_similarity(gt, pred, data_range=1, channel_axis=2)
// (compute_metrics, ir:1208-1213) on uint8 images that stand for float32(v / 255)
// (run_test, ir:1412-1413; scikit-image then casts to float64): per channel, 7x7
// uniform windows, sample covariance (49/48), C1 = 0.01^2, C2 = 0.03^2, the SSIM
// map averaged over the pixels >= 3 from every border, then over the channels.
// fp64 like scikit-image.  grid (blocks, N): partials[(n*gridDim.x + b)] = sum of
// the block's SSIM map values.
__global__ __launch_bounds__(TPB) void ssim_eval_kernel(const uint8_t* __restrict__ pred,
                                                        const uint8_t* __restrict__ gt, int H, int W, int C,
                                                        double* __restrict__ partials) {
    __shared__ double red[TPB];
    __shared__ double lut[256];  // float32(k / 255) widened, the reference's input values
    lut[threadIdx.x] = (double)((float)threadIdx.x / 255.0f);
    __syncthreads();
    const int n = blockIdx.y;
    const long per = (long)H * W * C;
    const uint8_t* a = gt + n * per;    // im1 = gt (ir:1210)
    const uint8_t* b = pred + n * per;  // im2 = pred
    const int Hv = H - 6, Wv = W - 6;
    const long total = (long)Hv * Wv * C;
    const double inv = 1.0 / 49.0, cov = 49.0 / 48.0;
    const double C1 = 0.01 * 0.01, C2 = 0.03 * 0.03;
    double acc = 0.0;
    for (long e = blockIdx.x * (long)TPB + threadIdx.x; e < total; e += (long)gridDim.x * TPB) {
        const int c = (int)(e % C);
        const long q = e / C;
        const int y = (int)(q / Wv) + 3, x = (int)(q % Wv) + 3;
        double sa = 0, sb = 0, saa = 0, sbb = 0, sab = 0;
        for (int dy = -3; dy <= 3; ++dy) {
            const long row = ((long)(y + dy) * W + x) * C + c;
#pragma unroll
            for (int dx = -3; dx <= 3; ++dx) {
                const double va = lut[a[row + dx * C]], vb = lut[b[row + dx * C]];
                sa += va; sb += vb; saa += va * va; sbb += vb * vb; sab += va * vb;
            }
        }
        const double ux = sa * inv, uy = sb * inv;
        const double vx = cov * (saa * inv - ux * ux), vy = cov * (sbb * inv - uy * uy);
        const double vxy = cov * (sab * inv - ux * uy);
        const double A1 = 2.0 * ux * uy + C1, A2 = 2.0 * vxy + C2;
        const double B1 = ux * ux + uy * uy + C1, B2 = vx + vy + C2;
        acc += (A1 * A2) / (B1 * B2);
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int w = TPB / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) partials[(long)n * gridDim.x + blockIdx.x] = red[0];
}

__global__ void ssim_eval_finalize(const double* __restrict__ partials, int nb, int N, double denom,
                                   double* __restrict__ out) {
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    double s = 0.0;
    for (int b = 0; b < nb; ++b) s += partials[(long)n * nb + b];
    out[n] = s / denom;
}

}  // namespace

extern "C" int irgan_ssim_eval_u8(const void* pred, const void* gt, int32_t N, int32_t H, int32_t W, int32_t C,
                                  double* work, int64_t work_cap, double* ssim, irgan_stream_t s) {
    if (!pred || !gt || !work || !ssim || C < 1) return IRGAN_EINVAL;
    if (N <= 0) return 0;
    if (H < 7 || W < 7) return IRGAN_EINVAL;  // skimage: win_size exceeds image extent
    const long total = (long)(H - 6) * (W - 6) * C;
    int nb = (int)std::min<long>(256, std::max<long>(1, irgan_cdiv(total, TPB)));
    if ((long)nb * N > work_cap) nb = (int)std::max<long>(1, work_cap / N);
    if ((long)nb * N > work_cap || N > 65535) return IRGAN_EINVAL;
    ssim_eval_kernel<<<dim3(nb, N), TPB, 0, (hipStream_t)s>>>((const uint8_t*)pred, (const uint8_t*)gt, H, W, C, work);
    ssim_eval_finalize<<<irgan_cdiv(N, 64), 64, 0, (hipStream_t)s>>>(work, nb, N, (double)total, ssim);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_to_rgb_u8(const float* x, int32_t N, int32_t H, int32_t W, int32_t C, int32_t ldx, int32_t xoff,
                               void* out, irgan_stream_t s) {
    if (!x || !out || C <= 0 || xoff < 0 || ldx < C + xoff) return IRGAN_EINVAL;
    const long total = (long)N * H * W * C;
    if (total <= 0) return 0;
    if ((uintptr_t)out % 16) return IRGAN_EUNSUPPORTED;
    const int blocks = (int)std::max<long>(1, std::min<long>((total / 16 + TPB - 1) / TPB, 4096));
    rgb_u8_kernel<<<blocks, TPB, 0, (hipStream_t)s>>>(x, ldx, xoff, C, total, (uint8_t*)out);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_image_metrics_u8(const void* pred, const void* gt, int32_t N, int64_t per_image, double* work,
                                      int64_t work_cap, double* sums, irgan_stream_t s) {
    if (!pred || !gt || !sums || !work) return IRGAN_EINVAL;
    if (N <= 0 || per_image <= 0) return 0;
    int nb = (int)std::min<long>(64, std::max<long>(1, (per_image / 16 + TPB - 1) / TPB));
    if ((long)nb * N * 2 > work_cap) nb = (int)std::max<long>(1, work_cap / (2L * N));
    if ((long)nb * N * 2 > work_cap) return IRGAN_EINVAL;
    metrics_u8_kernel<<<dim3(nb, N), TPB, 0, (hipStream_t)s>>>((const uint8_t*)pred, (const uint8_t*)gt, per_image,
                                                               work);
    metrics_finalize_kernel<<<irgan_cdiv(N, 64), 64, 0, (hipStream_t)s>>>(work, nb, N, sums);
    IRGAN_LAUNCH_CHECK();
    return 0;
}
