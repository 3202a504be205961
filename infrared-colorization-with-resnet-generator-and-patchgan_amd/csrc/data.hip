// KAIST data pipeline on the device: the per-sample work
// of KAISTPairDataset.__getitem__ (ir:1132-1177) for a whole batch at once.
//
// The reference, per sample and in CPU DataLoader workers: cv2.imread ->
// cv2.resize(..., INTER_AREA) to img_size^2 (uint8 in, uint8 out) -> float32
// / 255 (IR: only when the resized image's max exceeds 1, ir:1142-1146) ->
// random paired horizontal flip (ir:1166-1168) -> x * 2 - 1 (ir:1175-1176).
// Here the host only decodes; the uint8 images of a batch are uploaded once
// and these two launches do resize, flip and normalisation:
//
//  * area_resize_u8_kernel: INTER_AREA as OpenCV's general area path computes
//    it for scale factors >= 1 (resizeArea_: per destination pixel, each
//    source row of the vertical cell reduced horizontally with the x-table
//    weights -- buf = sum alpha * S in table order -- then sum = beta0 * buf0
//    (+ beta1 * buf1 ...), saturate_cast<uchar> = round half to even, clamp).
//    The tables (CSR: per destination index a run of (source index, weight))
//    come from the host (ops.area_table, computeResizeAreaTab's recurrence).
//    Every float op is a separately rounded mul / add (fp contract off: hipcc
//    would fuse them into FMAs), in OpenCV's order.  The flip writes column W-1-x; per-image max of the
//    resized bytes (IR rule) by one atomicMax per block.
//  * unit_kernel: uint8 -> float32 [-1, 1]: v / 255 (correctly rounded float32
//    division, as numpy), then * 2 - 1 (torch float32), the IR max rule applied.
// Byte-sized HBM streams; no LDS, no MFMA.
#include "common.h"

namespace {

constexpr int TPB = 256;

// src: uint8 [N][Hin][Win][C] with image stride img_stride bytes; out: uint8
// [N][C][Hout][Wout] (NCHW, the dataset's tensor layout).  One thread = one
// destination pixel, all C (<= 4) channels.
__global__ __launch_bounds__(TPB) void area_resize_u8_kernel(const uint8_t* __restrict__ src, int Hin, int Win, int C,
                                                             long img_stride, const int* __restrict__ yptr,
                                                             const int* __restrict__ ysrc,
                                                             const float* __restrict__ yw, int Hout,
                                                             const int* __restrict__ xptr,
                                                             const int* __restrict__ xsrc,
                                                             const float* __restrict__ xw, int Wout,
                                                             const uint8_t* __restrict__ flip,
                                                             uint8_t* __restrict__ out, int* __restrict__ img_max) {
#pragma clang fp contract(off)  // OpenCV's separate float mul / add: no FMA contraction (hipcc defaults to fast)
    const int n = blockIdx.y;
    const int e = blockIdx.x * TPB + threadIdx.x;
    __shared__ int bmax;
    if (threadIdx.x == 0) bmax = 0;
    __syncthreads();
    if (e < Hout * Wout) {
        const int y = e / Wout, x = e - y * Wout;
        const uint8_t* S = src + n * img_stride;
        float sum[4] = {0.f, 0.f, 0.f, 0.f};
        const int y0 = yptr[y], y1 = yptr[y + 1], x0 = xptr[x], x1 = xptr[x + 1];
        for (int ty = y0; ty < y1; ++ty) {
            const uint8_t* row = S + (long)ysrc[ty] * Win * C;
            const float beta = yw[ty];
            float buf[4] = {0.f, 0.f, 0.f, 0.f};
            for (int tx = x0; tx < x1; ++tx) {
                const uint8_t* p = row + xsrc[tx] * C;
                const float alpha = xw[tx];
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    if (c < C) buf[c] = buf[c] + (float)p[c] * alpha;
            }
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if (c < C) sum[c] = ty == y0 ? beta * buf[c] : sum[c] + beta * buf[c];
        }
        const int xo = (flip && flip[n]) ? Wout - 1 - x : x;
        int m = 0;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (c >= C) break;
            float r = rintf(sum[c]);                 // cvRound: nearest, ties to even
            r = r < 0.f ? 0.f : (r > 255.f ? 255.f : r);
            const int v = (int)r;
            out[(((long)n * C + c) * Hout + y) * Wout + xo] = (uint8_t)v;
            m = v > m ? v : m;
        }
        if (img_max && m > 1) atomicMax(&bmax, m);
    }
    __syncthreads();
    if (img_max && threadIdx.x == 0 && bmax > 0) atomicMax(img_max + n, bmax);
}

// cv2.resize(INTER_AREA) when an axis UPscales: OpenCV's generic linear resampler with
// area-mode coefficients in 8-bit fixed point (resizeGeneric_, HResizeLinear<uchar, int,
// short, 2048>, VResizeLinear<uchar, int, short, FixedPtCast<..., 22>>): tables from the
// host (data.linear_area_table).  Per destination (y, x) and channel:
//   D(r) = S[r][x0] * a0 + S[r][min(x0 + 1, Win - 1)] * a1   (x >= xlim: S[r][x0] * 2048)
//   v = (((b0 * (D(y0) >> 4)) >> 16) + ((b1 * (D(min(y0 + 1, Hin - 1)) >> 4)) >> 16) + 2) >> 2
// all in int32, stored as uchar (no saturation, as OpenCV).  Flip and the IR max as above.
__global__ __launch_bounds__(TPB) void linear_area_u8_kernel(const uint8_t* __restrict__ src, int Hin, int Win, int C,
                                                             long img_stride, const int* __restrict__ yofs,
                                                             const int* __restrict__ ycoef, int Hout,
                                                             const int* __restrict__ xofs,
                                                             const int* __restrict__ xcoef, int xlim, int Wout,
                                                             const uint8_t* __restrict__ flip,
                                                             uint8_t* __restrict__ out, int* __restrict__ img_max) {
    const int n = blockIdx.y;
    const int e = blockIdx.x * TPB + threadIdx.x;
    __shared__ int bmax;
    if (threadIdx.x == 0) bmax = 0;
    __syncthreads();
    if (e < Hout * Wout) {
        const int y = e / Wout, x = e - y * Wout;
        const uint8_t* S = src + n * img_stride;
        const int y0 = yofs[y], y1 = min(y0 + 1, Hin - 1);
        const int b0 = ycoef[2 * y], b1 = ycoef[2 * y + 1];
        const int x0 = xofs[x], x1 = min(x0 + 1, Win - 1);
        const int a0 = xcoef[2 * x], a1 = xcoef[2 * x + 1];
        const bool one = x >= xlim;
        const int xo = (flip && flip[n]) ? Wout - 1 - x : x;
        int m = 0;
        for (int c = 0; c < C; ++c) {
            const uint8_t* r0 = S + (long)y0 * Win * C + c;
            const uint8_t* r1 = S + (long)y1 * Win * C + c;
            const int d0 = one ? (int)r0[x0 * C] * 2048 : (int)r0[x0 * C] * a0 + (int)r0[x1 * C] * a1;
            const int d1 = one ? (int)r1[x0 * C] * 2048 : (int)r1[x0 * C] * a0 + (int)r1[x1 * C] * a1;
            const int v = ((((b0 * (d0 >> 4)) >> 16) + ((b1 * (d1 >> 4)) >> 16) + 2) >> 2) & 0xFF;
            out[(((long)n * C + c) * Hout + y) * Wout + xo] = (uint8_t)v;
            m = v > m ? v : m;
        }
        if (img_max && m > 1) atomicMax(&bmax, m);
    }
    __syncthreads();
    if (img_max && threadIdx.x == 0 && bmax > 0) atomicMax(img_max + n, bmax);
}

// out[n][i] = f32(in[n][i]) / 255 * 2 - 1; with max_rule (IR) the division is
// skipped for images whose max byte is <= 1 (ir:1142).
__global__ __launch_bounds__(TPB) void unit_kernel(const uint8_t* __restrict__ in, long per_image,
                                                   const int* __restrict__ img_max, int max_rule,
                                                   float* __restrict__ out) {
#pragma clang fp contract(off)
    const int n = blockIdx.y;
    const bool div = !max_rule || img_max[n] > 1;
    for (long i = blockIdx.x * (long)TPB + threadIdx.x; i < per_image; i += (long)gridDim.x * TPB) {
        float v = (float)in[n * per_image + i];
        if (div) v = v / 255.0f;   // IEEE division (hipcc's default correctly rounded fp32 divide)
        v = v < 0.f ? 0.f : (v > 1.f ? 1.f : v);  // np.clip(img, 0, 1)
        out[n * per_image + i] = v * 2.0f - 1.0f;
    }
}

}  // namespace

extern "C" int irgan_area_resize_u8(const void* src, int32_t N, int32_t Hin, int32_t Win, int32_t C, int64_t img_stride,
                                    const int32_t* yptr, const int32_t* ysrc, const float* yw, int32_t Hout,
                                    const int32_t* xptr, const int32_t* xsrc, const float* xw, int32_t Wout,
                                    const void* flip, void* out_u8, int32_t* img_max, irgan_stream_t s) {
    if (N <= 0 || Hout <= 0 || Wout <= 0) return 0;
    if (!src || !yptr || !ysrc || !yw || !xptr || !xsrc || !xw || !out_u8 || C < 1 || C > 4 || Hin < 1 || Win < 1 ||
        img_stride < (long)Hin * Win * C || N > 65535)
        return IRGAN_EINVAL;
    dim3 g(irgan_cdiv((long)Hout * Wout, TPB), N);
    area_resize_u8_kernel<<<g, TPB, 0, (hipStream_t)s>>>((const uint8_t*)src, Hin, Win, C, img_stride, yptr, ysrc, yw,
                                                         Hout, xptr, xsrc, xw, Wout, (const uint8_t*)flip,
                                                         (uint8_t*)out_u8, img_max);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_u8_to_unit(const void* in, int32_t N, int64_t per_image, const int32_t* img_max, int32_t max_rule,
                                float* out, irgan_stream_t s) {
    if (N <= 0 || per_image <= 0) return 0;
    if (!in || !out || (max_rule && !img_max) || N > 65535) return IRGAN_EINVAL;
    const int bx = (int)std::min<long>(irgan_cdiv(per_image, TPB), 1024);
    unit_kernel<<<dim3(bx, N), TPB, 0, (hipStream_t)s>>>((const uint8_t*)in, per_image, img_max, max_rule, out);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_linear_area_resize_u8(const void* src, int32_t N, int32_t Hin, int32_t Win, int32_t C,
                                           int64_t img_stride, const int32_t* yofs, const int32_t* ycoef,
                                           int32_t Hout, const int32_t* xofs, const int32_t* xcoef, int32_t xlim,
                                           int32_t Wout, const void* flip, void* out_u8, int32_t* img_max,
                                           irgan_stream_t s) {
    if (N <= 0 || Hout <= 0 || Wout <= 0) return 0;
    if (!src || !yofs || !ycoef || !xofs || !xcoef || !out_u8 || C < 1 || C > 4 || Hin < 1 || Win < 1 ||
        img_stride < (long)Hin * Win * C || N > 65535)
        return IRGAN_EINVAL;
    dim3 g(irgan_cdiv((long)Hout * Wout, TPB), N);
    linear_area_u8_kernel<<<g, TPB, 0, (hipStream_t)s>>>((const uint8_t*)src, Hin, Win, C, img_stride, yofs, ycoef,
                                                         Hout, xofs, xcoef, xlim, Wout, (const uint8_t*)flip,
                                                         (uint8_t*)out_u8, img_max);
    IRGAN_LAUNCH_CHECK();
    return 0;
}
