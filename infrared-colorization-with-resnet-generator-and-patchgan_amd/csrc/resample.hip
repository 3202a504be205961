// Resampling and layout kernels (NHWC, channel-fastest threads => coalesced).
//   blur-down   : Downsample, reflect pad 1 + binomial [1,2,1]^2/16, stride 2 (ir:269-310)
//   upsample    : UpsampleAA, bilinear x2 align_corners=True + reflect pad 1 + blur (ir:313-355)
//   reflect fold: backward of nn.ReflectionPad2d (ir:381, 402, 459, 528)
//   maxpool 2x2 : VGG-16 features pooling (ir:664)
// Backward passes are written as gathers (each output element sums its
// contributors), so they are deterministic and need no atomics.
#include "common.h"

namespace {

constexpr int TPB = 256;

// blur taps [1,2,1]/4 per dimension (outer product = the reference's 3x3 filt)
IRGAN_HD float tap3(int a) { return a == 1 ? 0.5f : 0.25f; }

// contributors of a padded-domain position set: input coordinate q of an axis of
// length n receives from padded coordinates u with reflect(u - 1) == q.
IRGAN_HD int refl_sources(int q, int n, int* u) {
    int k = 0;
    u[k++] = q + 1;
    if (q == 1) u[k++] = 0;
    if (q == n - 2 && n >= 3) u[k++] = n + 1;
    return k;
}

__global__ __launch_bounds__(TPB) void blur_down_fwd_kernel(const void* __restrict__ x, int dt, int H, int W, int C,
                                                            int ldx, int xoff, void* __restrict__ y, int ldy,
                                                            int yoff, int Ho, int Wo, long total) {
    for (long idx = blockIdx.x * (long)TPB + threadIdx.x; idx < total; idx += (long)gridDim.x * TPB) {
        long t = idx;
        const int c = (int)(t % C); t /= C;
        const int j = (int)(t % Wo); t /= Wo;
        const int i = (int)(t % Ho);
        const int n = (int)(t / Ho);
        float acc = 0.f;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const int qy = reflect_idx(2 * i + a - 1, H);
            float row = 0.f;
#pragma unroll
            for (int b = 0; b < 3; ++b) {
                const int qx = reflect_idx(2 * j + b - 1, W);
                row += tap3(b) * ldv(x, dt, (((long)n * H + qy) * W + qx) * ldx + xoff + c);
            }
            acc += tap3(a) * row;
        }
        stv(y, dt, (((long)n * Ho + i) * Wo + j) * ldy + yoff + c, acc);
    }
}

// dx[q] = sum over padded u with reflect(u-1)=q, taps a with u = 2i + a
__global__ __launch_bounds__(TPB) void blur_down_bwd_kernel(const void* __restrict__ dy, int dt, int H, int W, int C,
                                                            int lddy, int dyoff, void* __restrict__ dx, int dxdt,
                                                            int lddx, int dxoff, int Ho, int Wo, long total) {
    for (long idx = blockIdx.x * (long)TPB + threadIdx.x; idx < total; idx += (long)gridDim.x * TPB) {
        long t = idx;
        const int c = (int)(t % C); t /= C;
        const int qx = (int)(t % W); t /= W;
        const int qy = (int)(t % H);
        const int n = (int)(t / H);
        int uy[3], ux[3];
        const int ny = refl_sources(qy, H, uy), nx = refl_sources(qx, W, ux);
        float acc = 0.f;
        for (int s = 0; s < ny; ++s)
            for (int a = 0; a < 3; ++a) {
                const int vy = uy[s] - a;
                if (vy < 0 || (vy & 1)) continue;
                const int i = vy >> 1;
                if (i >= Ho) continue;
                for (int r = 0; r < nx; ++r)
                    for (int b = 0; b < 3; ++b) {
                        const int vx = ux[r] - b;
                        if (vx < 0 || (vx & 1)) continue;
                        const int j = vx >> 1;
                        if (j >= Wo) continue;
                        acc += tap3(a) * tap3(b) * ldv(dy, dt, (((long)n * Ho + i) * Wo + j) * lddy + dyoff + c);
                    }
            }
        stv(dx, dxdt, (((long)n * H + qy) * W + qx) * lddx + dxoff + c, acc);
    }
}

// bilinear source for output coordinate v of an axis upsampled from n (ATen
// upsample_bilinear2d, align_corners=True: src = v * (n-1)/(2n-1))
struct Bil {
    int i0, i1;
    float l0, l1;
};
IRGAN_HD Bil bil(int v, float scale, int n) {
    Bil b;
    const float r = scale * (float)v;
    b.i0 = (int)r;
    b.i1 = b.i0 + ((b.i0 < n - 1) ? 1 : 0);
    b.l1 = r - (float)b.i0;
    b.l0 = 1.f - b.l1;
    return b;
}

__global__ __launch_bounds__(TPB) void upsample_fwd_kernel(const void* __restrict__ x, int dt, int H, int W, int C,
                                                           int ldx, int xoff, void* __restrict__ y, int ldy, int yoff,
                                                           float sh, float sw, long total) {
    const int H2 = 2 * H, W2 = 2 * W;
    for (long idx = blockIdx.x * (long)TPB + threadIdx.x; idx < total; idx += (long)gridDim.x * TPB) {
        long t = idx;
        const int c = (int)(t % C); t /= C;
        const int ox = (int)(t % W2); t /= W2;
        const int oy = (int)(t % H2);
        const int n = (int)(t / H2);
        const long base = (long)n * H * W;
        float acc = 0.f;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const Bil by = bil(reflect_idx(oy + a - 1, H2), sh, H);
            float row = 0.f;
#pragma unroll
            for (int b = 0; b < 3; ++b) {
                const Bil bx = bil(reflect_idx(ox + b - 1, W2), sw, W);
                auto X = [&](int yy, int xx) { return ldv(x, dt, (base + (long)yy * W + xx) * ldx + xoff + c); };
                const float v = by.l0 * (bx.l0 * X(by.i0, bx.i0) + bx.l1 * X(by.i0, bx.i1)) +
                                by.l1 * (bx.l0 * X(by.i1, bx.i0) + bx.l1 * X(by.i1, bx.i1));
                row += tap3(b) * v;
            }
            acc += tap3(a) * row;
        }
        stv(y, dt, (((long)n * H2 + oy) * W2 + ox) * ldy + yoff + c, acc);
    }
}

// backward part 1: transpose of (reflect pad 1 + blur, stride 1) on the 2H x 2W grid -> fp32 work
__global__ __launch_bounds__(TPB) void upsample_bwd_blur_kernel(const void* __restrict__ dy, int dt, int H2, int W2,
                                                                int C, int lddy, int dyoff, float* __restrict__ work,
                                                                long total) {
    for (long idx = blockIdx.x * (long)TPB + threadIdx.x; idx < total; idx += (long)gridDim.x * TPB) {
        long t = idx;
        const int c = (int)(t % C); t /= C;
        const int qx = (int)(t % W2); t /= W2;
        const int qy = (int)(t % H2);
        const int n = (int)(t / H2);
        int uy[3], ux[3];
        const int ny = refl_sources(qy, H2, uy), nx = refl_sources(qx, W2, ux);
        float acc = 0.f;
        for (int s = 0; s < ny; ++s)
            for (int a = 0; a < 3; ++a) {
                const int oy = uy[s] - a;
                if (oy < 0 || oy >= H2) continue;
                for (int r = 0; r < nx; ++r)
                    for (int b = 0; b < 3; ++b) {
                        const int ox = ux[r] - b;
                        if (ox < 0 || ox >= W2) continue;
                        acc += tap3(a) * tap3(b) * ldv(dy, dt, (((long)n * H2 + oy) * W2 + ox) * lddy + dyoff + c);
                    }
            }
        work[idx] = acc;
    }
}

// backward part 2: transpose of the bilinear map (gather over the ~5 output
// rows/cols whose stencil touches each input row/col)
__global__ __launch_bounds__(TPB) void upsample_bwd_bil_kernel(const float* __restrict__ work, int H, int W, int C,
                                                               float sh, float sw, void* __restrict__ dx, int dxdt,
                                                               int lddx, int dxoff, int accumulate, long total) {
    const int H2 = 2 * H, W2 = 2 * W;
    for (long idx = blockIdx.x * (long)TPB + threadIdx.x; idx < total; idx += (long)gridDim.x * TPB) {
        long t = idx;
        const int c = (int)(t % C); t /= C;
        const int w = (int)(t % W); t /= W;
        const int h = (int)(t % H);
        const int n = (int)(t / H);
        // output rows v with bil(v).i0 or .i1 == h: v*sh in [h-1, h+1)
        const int vy0 = max(0, (int)floorf((h - 1) / fmaxf(sh, 1e-30f)) - 1);
        const int vy1 = min(H2 - 1, sh > 0.f ? (int)ceilf((h + 1) / sh) + 1 : H2 - 1);
        const int vx0 = max(0, (int)floorf((w - 1) / fmaxf(sw, 1e-30f)) - 1);
        const int vx1 = min(W2 - 1, sw > 0.f ? (int)ceilf((w + 1) / sw) + 1 : W2 - 1);
        float acc = 0.f;
        for (int vy = vy0; vy <= vy1; ++vy) {
            const Bil by = bil(vy, sh, H);
            float wy = (by.i0 == h ? by.l0 : 0.f) + (by.i1 == h ? by.l1 : 0.f);
            if (wy == 0.f) continue;
            for (int vx = vx0; vx <= vx1; ++vx) {
                const Bil bx = bil(vx, sw, W);
                float wx = (bx.i0 == w ? bx.l0 : 0.f) + (bx.i1 == w ? bx.l1 : 0.f);
                if (wx == 0.f) continue;
                acc += wy * wx * work[(((long)n * H2 + vy) * W2 + vx) * C + c];
            }
        }
        const long o = (((long)n * H + h) * W + w) * lddx + dxoff + c;
        if (accumulate) acc += ldv(dx, dxdt, o);
        stv(dx, dxdt, o, acc);
    }
}

__global__ __launch_bounds__(TPB) void reflect_fold_kernel(const float* __restrict__ dxp, int H, int W, int C, int p,
                                                           void* __restrict__ dx, int dxdt, int lddx, int dxoff,
                                                           int accumulate, long total) {
    const int Hp = H + 2 * p, Wp = W + 2 * p;
    for (long idx = blockIdx.x * (long)TPB + threadIdx.x; idx < total; idx += (long)gridDim.x * TPB) {
        long t = idx;
        const int c = (int)(t % C); t /= C;
        const int qx = (int)(t % W); t /= W;
        const int qy = (int)(t % H);
        const int n = (int)(t / H);
        int uy[3], ux[3], ny = 0, nx = 0;
        uy[ny++] = qy + p;
        if (qy >= 1 && qy <= p) uy[ny++] = p - qy;
        if (qy <= H - 2 && qy >= H - 1 - p) uy[ny++] = p + 2 * (H - 1) - qy;
        ux[nx++] = qx + p;
        if (qx >= 1 && qx <= p) ux[nx++] = p - qx;
        if (qx <= W - 2 && qx >= W - 1 - p) ux[nx++] = p + 2 * (W - 1) - qx;
        float acc = 0.f;
        for (int a = 0; a < ny; ++a)
            for (int b = 0; b < nx; ++b) acc += dxp[(((long)n * Hp + uy[a]) * Wp + ux[b]) * C + c];
        const long o = (((long)n * H + qy) * W + qx) * lddx + dxoff + c;
        if (accumulate) acc += ldv(dx, dxdt, o);
        stv(dx, dxdt, o, acc);
    }
}

__global__ __launch_bounds__(TPB) void maxpool_fwd_kernel(const void* __restrict__ x, int dt, int H, int W, int C,
                                                          void* __restrict__ y, long total) {
    const int Ho = H / 2, Wo = W / 2;
    for (long idx = blockIdx.x * (long)TPB + threadIdx.x; idx < total; idx += (long)gridDim.x * TPB) {
        long t = idx;
        const int c = (int)(t % C); t /= C;
        const int j = (int)(t % Wo); t /= Wo;
        const int i = (int)(t % Ho);
        const int n = (int)(t / Ho);
        float m = -INFINITY;
        for (int a = 0; a < 2; ++a)
            for (int b = 0; b < 2; ++b) {
                float v = ldv(x, dt, (((long)n * H + 2 * i + a) * W + 2 * j + b) * C + c);
                if (v > m || isnan(v)) m = v;
            }
        stv(y, dt, idx, m);
    }
}

__global__ __launch_bounds__(TPB) void maxpool_bwd_kernel(const void* __restrict__ x, const void* __restrict__ dy,
                                                          int dt, int H, int W, int C, void* __restrict__ dx,
                                                          int relu_mask, long total) {
    const int Ho = H / 2, Wo = W / 2;
    for (long idx = blockIdx.x * (long)TPB + threadIdx.x; idx < total; idx += (long)gridDim.x * TPB) {
        long t = idx;
        const int c = (int)(t % C); t /= C;
        const int j = (int)(t % Wo); t /= Wo;
        const int i = (int)(t % Ho);
        const int n = (int)(t / Ho);
        float m = -INFINITY;
        int am = 0;
        for (int k = 0; k < 4; ++k) {
            float v = ldv(x, dt, (((long)n * H + 2 * i + (k >> 1)) * W + 2 * j + (k & 1)) * C + c);
            if (v > m || isnan(v)) { m = v; am = k; }
        }
        float g = ldv(dy, dt, idx);
        if (relu_mask && !(m > 0.f)) g = 0.f;  // pool input is a ReLU output: fold relu' in
        for (int k = 0; k < 4; ++k)
            stv(dx, dt, (((long)n * H + 2 * i + (k >> 1)) * W + 2 * j + (k & 1)) * C + c, k == am ? g : 0.f);
    }
}

__global__ __launch_bounds__(TPB) void nchw_to_nhwc_kernel(const float* __restrict__ x, int C, int HW,
                                                           void* __restrict__ y, int dt, int ldy, int yoff,
                                                           const float* __restrict__ scale,
                                                           const float* __restrict__ shift, long total) {
    for (long idx = blockIdx.x * (long)TPB + threadIdx.x; idx < total; idx += (long)gridDim.x * TPB) {
        long t = idx;
        const int c = (int)(t % C); t /= C;
        const long p = t;  // n*HW + hw
        const long n = p / HW, hw = p - n * HW;
        float v = x[(n * C + c) * HW + hw];
        if (scale) v = v * scale[c] + shift[c];
        stv(y, dt, p * ldy + yoff + c, v);
    }
}

__global__ __launch_bounds__(TPB) void nhwc_to_nchw_kernel(const void* __restrict__ x, int dt, int ldx, int xoff,
                                                           int C, int HW, float* __restrict__ y, float scale,
                                                           int accumulate, long total) {
    for (long idx = blockIdx.x * (long)TPB + threadIdx.x; idx < total; idx += (long)gridDim.x * TPB) {
        long t = idx;
        const int hw = (int)(t % HW); t /= HW;
        const int c = (int)(t % C);
        const long n = t / C;
        float v = scale * ldv(x, dt, (n * HW + hw) * ldx + xoff + c);
        y[idx] = accumulate ? y[idx] + v : v;
    }
}

__global__ __launch_bounds__(TPB) void axpby_kernel(const void* __restrict__ x, int xdt, int ldx, int xoff, float a,
                                                    void* __restrict__ y, int ydt, int ldy, int yoff, float b, int C,
                                                    long total) {
    for (long idx = blockIdx.x * (long)TPB + threadIdx.x; idx < total; idx += (long)gridDim.x * TPB) {
        const long p = idx / C;
        const int c = (int)(idx - p * C);
        float v = a * ldv(x, xdt, p * ldx + xoff + c);
        const long o = p * ldy + yoff + c;
        if (b != 0.f) v += b * ldv(y, ydt, o);
        stv(y, ydt, o, v);
    }
}

__global__ __launch_bounds__(TPB) void affine_kernel(const void* __restrict__ x, int xdt, int ldx, int xoff,
                                                     const float* __restrict__ scale, const float* __restrict__ shift,
                                                     void* __restrict__ y, int ydt, int ldy, int yoff, int accumulate,
                                                     int C, long total) {
    for (long idx = blockIdx.x * (long)TPB + threadIdx.x; idx < total; idx += (long)gridDim.x * TPB) {
        const long p = idx / C;
        const int c = (int)(idx - p * C);
        float v = ldv(x, xdt, p * ldx + xoff + c) * scale[c];
        if (shift) v += shift[c];
        const long o = p * ldy + yoff + c;
        if (accumulate) v += ldv(y, ydt, o);
        stv(y, ydt, o, v);
    }
}

__global__ __launch_bounds__(TPB) void act_bwd_kernel(const void* __restrict__ dy, int dydt, int lddy, int dyoff,
                                                      const void* __restrict__ a, int adt, int lda, int aoff, int act,
                                                      void* __restrict__ dx, int dxdt, int lddx, int dxoff, int C,
                                                      long total) {
    for (long idx = blockIdx.x * (long)TPB + threadIdx.x; idx < total; idx += (long)gridDim.x * TPB) {
        const long p = idx / C;
        const int c = (int)(idx - p * C);
        const float g = ldv(dy, dydt, p * lddy + dyoff + c);
        const float av = ldv(a, adt, p * lda + aoff + c);
        float f;
        if (act == IRGAN_ACT_RELU) f = av > 0.f ? 1.f : 0.f;
        else if (act == IRGAN_ACT_LRELU) f = av > 0.f ? 1.f : 0.2f;
        else if (act == IRGAN_ACT_TANH) f = 1.f - av * av;
        else f = 1.f;
        stv(dx, dxdt, p * lddx + dxoff + c, g * f);
    }
}

int nblocks(long total) { return (int)std::max<long>(1, std::min<long>((total + TPB - 1) / TPB, 16384)); }

}  // namespace

#define RS_CHECK(total) \
    if ((total) <= 0) return 0

extern "C" int irgan_blur_down_fwd(const void* x, int32_t dt, int32_t N, int32_t H, int32_t W, int32_t C, int32_t ldx,
                                   int32_t xoff, void* y, int32_t ldy, int32_t yoff, irgan_stream_t s) {
    const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
    long total = (long)N * Ho * Wo * C;
    RS_CHECK(total);
    blur_down_fwd_kernel<<<nblocks(total), TPB, 0, (hipStream_t)s>>>(x, dt, H, W, C, ldx, xoff, y, ldy, yoff, Ho, Wo,
                                                                     total);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_blur_down_bwd(const void* dy, int32_t dt, int32_t N, int32_t H, int32_t W, int32_t C,
                                   int32_t lddy, int32_t dyoff, void* dx, int32_t dxdt, int32_t lddx, int32_t dxoff,
                                   irgan_stream_t s) {
    const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
    long total = (long)N * H * W * C;
    RS_CHECK(total);
    blur_down_bwd_kernel<<<nblocks(total), TPB, 0, (hipStream_t)s>>>(dy, dt, H, W, C, lddy, dyoff, dx, dxdt, lddx,
                                                                     dxoff, Ho, Wo, total);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

static float up_scale(int n) { return n > 1 ? (float)(n - 1) / (float)(2 * n - 1) : 0.f; }

extern "C" int irgan_upsample_fwd(const void* x, int32_t dt, int32_t N, int32_t H, int32_t W, int32_t C, int32_t ldx,
                                  int32_t xoff, void* y, int32_t ldy, int32_t yoff, irgan_stream_t s) {
    long total = (long)N * 4 * H * W * C;
    RS_CHECK(total);
    upsample_fwd_kernel<<<nblocks(total), TPB, 0, (hipStream_t)s>>>(x, dt, H, W, C, ldx, xoff, y, ldy, yoff,
                                                                    up_scale(H), up_scale(W), total);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_upsample_bwd(const void* dy, int32_t dt, int32_t N, int32_t H, int32_t W, int32_t C,
                                  int32_t lddy, int32_t dyoff, float* work, void* dx, int32_t dxdt, int32_t lddx,
                                  int32_t dxoff, int32_t accumulate, irgan_stream_t s) {
    long t1 = (long)N * 4 * H * W * C, t2 = (long)N * H * W * C;
    RS_CHECK(t2);
    upsample_bwd_blur_kernel<<<nblocks(t1), TPB, 0, (hipStream_t)s>>>(dy, dt, 2 * H, 2 * W, C, lddy, dyoff, work, t1);
    upsample_bwd_bil_kernel<<<nblocks(t2), TPB, 0, (hipStream_t)s>>>(work, H, W, C, up_scale(H), up_scale(W), dx, dxdt,
                                                                     lddx, dxoff, accumulate, t2);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_reflect_fold(const float* dxpad, int32_t N, int32_t H, int32_t W, int32_t C, int32_t p, void* dx,
                                  int32_t dxdt, int32_t lddx, int32_t dxoff, int32_t accumulate, irgan_stream_t s) {
    long total = (long)N * H * W * C;
    RS_CHECK(total);
    reflect_fold_kernel<<<nblocks(total), TPB, 0, (hipStream_t)s>>>(dxpad, H, W, C, p, dx, dxdt, lddx, dxoff,
                                                                    accumulate, total);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_maxpool_fwd(const void* x, int32_t dt, int32_t N, int32_t H, int32_t W, int32_t C, void* y,
                                 irgan_stream_t s) {
    long total = (long)N * (H / 2) * (W / 2) * C;
    RS_CHECK(total);
    maxpool_fwd_kernel<<<nblocks(total), TPB, 0, (hipStream_t)s>>>(x, dt, H, W, C, y, total);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_maxpool_bwd(const void* x, const void* dy, int32_t dt, int32_t N, int32_t H, int32_t W, int32_t C,
                                 void* dx, int32_t relu_mask, irgan_stream_t s) {
    long total = (long)N * (H / 2) * (W / 2) * C;
    RS_CHECK(total);
    maxpool_bwd_kernel<<<nblocks(total), TPB, 0, (hipStream_t)s>>>(x, dy, dt, H, W, C, dx, relu_mask, total);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_nchw_to_nhwc(const float* x, int32_t N, int32_t C, int32_t H, int32_t W, void* y, int32_t dt,
                                  int32_t ldy, int32_t yoff, const float* scale, const float* shift, irgan_stream_t s) {
    long total = (long)N * C * H * W;
    RS_CHECK(total);
    nchw_to_nhwc_kernel<<<nblocks(total), TPB, 0, (hipStream_t)s>>>(x, C, H * W, y, dt, ldy, yoff, scale, shift,
                                                                    total);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_nhwc_to_nchw(const void* x, int32_t dt, int32_t ldx, int32_t xoff, int32_t N, int32_t C,
                                  int32_t H, int32_t W, float* y, float scale, int32_t accumulate, irgan_stream_t s) {
    long total = (long)N * C * H * W;
    RS_CHECK(total);
    nhwc_to_nchw_kernel<<<nblocks(total), TPB, 0, (hipStream_t)s>>>(x, dt, ldx, xoff, C, H * W, y, scale, accumulate,
                                                                    total);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_axpby(const void* x, int32_t xdt, int32_t ldx, int32_t xoff, float a, void* y, int32_t ydt,
                           int32_t ldy, int32_t yoff, float b, int32_t P, int32_t C, irgan_stream_t s) {
    long total = (long)P * C;
    RS_CHECK(total);
    axpby_kernel<<<nblocks(total), TPB, 0, (hipStream_t)s>>>(x, xdt, ldx, xoff, a, y, ydt, ldy, yoff, b, C, total);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_act_bwd(const void* dy, int32_t dydt, int32_t lddy, int32_t dyoff, const void* a, int32_t adt,
                             int32_t lda, int32_t aoff, int32_t act, void* dx, int32_t dxdt, int32_t lddx,
                             int32_t dxoff, int32_t P, int32_t C, irgan_stream_t s) {
    long total = (long)P * C;
    RS_CHECK(total);
    act_bwd_kernel<<<nblocks(total), TPB, 0, (hipStream_t)s>>>(dy, dydt, lddy, dyoff, a, adt, lda, aoff, act, dx, dxdt,
                                                               lddx, dxoff, C, total);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_affine(const void* x, int32_t xdt, int32_t ldx, int32_t xoff, const float* scale,
                            const float* shift, void* y, int32_t ydt, int32_t ldy, int32_t yoff, int32_t accumulate,
                            int32_t P, int32_t C, irgan_stream_t s) {
    long total = (long)P * C;
    RS_CHECK(total);
    affine_kernel<<<nblocks(total), TPB, 0, (hipStream_t)s>>>(x, xdt, ldx, xoff, scale, shift, y, ydt, ldy, yoff,
                                                              accumulate, C, total);
    IRGAN_LAUNCH_CHECK();
    return 0;
}
