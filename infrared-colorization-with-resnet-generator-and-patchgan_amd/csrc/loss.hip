// Loss kernels of the G/D objectives (ir:1647-1679) and the fused Adam update
// (ir:1601-1604, 1651, 1681).  Images are NHWC fp32 (B, H, W, 3).  Every loss
// is reduced per block in fp32 and across blocks with one fp64 atomic, and
// writes its gradient in the same pass (no autograd tape).
#include "common.h"

namespace {

constexpr int TPB = 256;

IRGAN_HD void block_add(double* dst, float v) {
    __shared__ float red[TPB / 64];
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) red[wid] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        float t = 0.f;
        for (int i = 0; i < TPB / 64; ++i) t += red[i];
        atomicAdd(dst, (double)t);
    }
}

IRGAN_HD float sgn(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }

int nblocks(long total) { return (int)std::max<long>(1, std::min<long>((total + TPB - 1) / TPB, 8192)); }
// kernels that finish with block_add: every block adds into the SAME fp64 word,
// and same-address atomics serialise at the memory side (~10 ns each), so keep
// the grid small and let threads loop
int nblocks_red(long total) { return (int)std::max<long>(1, std::min<long>((total + TPB - 1) / TPB, 512)); }

// mode 0: pred = [real (n) ; fake (n)] -> 0.5*(mean relu(1-r) + mean relu(1+f))   (ir:1647-1649)
// mode 1: pred = fake (n) -> -mean(p) * scale                                    (ir:1662, x lambda_gan)
__global__ __launch_bounds__(TPB) void hinge_kernel(const float* __restrict__ pred, int n, int mode, float scale,
                                                    float* __restrict__ grad, double* __restrict__ loss) {
    const long total = mode == 0 ? 2L * n : n;
    float acc = 0.f;
    const float inv = 1.f / (float)n;
    for (long i = blockIdx.x * (long)TPB + threadIdx.x; i < total; i += (long)gridDim.x * TPB) {
        const float p = pred[i];
        if (mode == 0) {  // [real; fake]
            if (i < n) {
                const float t = 1.f - p;
                acc += t > 0.f ? t : 0.f;
                grad[i] = t > 0.f ? -0.5f * inv * scale : 0.f;
            } else {
                const float t = 1.f + p;
                acc += t > 0.f ? t : 0.f;
                grad[i] = t > 0.f ? 0.5f * inv * scale : 0.f;
            }
        } else {
            acc += p;
            grad[i] = -scale * inv;
        }
    }
    block_add(loss, mode == 0 ? 0.5f * acc * inv * scale : -acc * inv * scale);
}

template <typename T>
IRGAN_HD void ld8t(const T* p, long i, float* o) {
    if constexpr (sizeof(T) == 2) {
        const uint4 u = *(const uint4*)(p + i);
        const uint32_t q[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            o[2 * k] = __uint_as_float(q[k] << 16);
            o[2 * k + 1] = __uint_as_float(q[k] & 0xffff0000u);
        }
    } else {
        const float4 x0 = *(const float4*)(p + i), x1 = *(const float4*)(p + i + 4);
        o[0] = x0.x; o[1] = x0.y; o[2] = x0.z; o[3] = x0.w; o[4] = x1.x; o[5] = x1.y; o[6] = x1.z; o[7] = x1.w;
    }
}
template <typename T>
IRGAN_HD void st8t(T* p, long i, const float* v) {
    if constexpr (sizeof(T) == 2) {
        uint4 u;
        u.x = pk_bf16(v[0], v[1]);
        u.y = pk_bf16(v[2], v[3]);
        u.z = pk_bf16(v[4], v[5]);
        u.w = pk_bf16(v[6], v[7]);
        *(uint4*)(p + i) = u;
    } else {
        *(float4*)(p + i) = make_float4(v[0], v[1], v[2], v[3]);
        *(float4*)(p + i + 4) = make_float4(v[4], v[5], v[6], v[7]);
    }
}

// VEC: 8 elements per thread-iteration (16/32-byte accesses; count % 8 == 0)
template <typename T, typename G, bool VEC>
__global__ __launch_bounds__(TPB) void l1_kernel(const T* __restrict__ a, const T* __restrict__ b, long count, float w,
                                                 G* __restrict__ ga, int accumulate, double* __restrict__ loss) {
    float acc = 0.f;
    const float inv = w / (float)count;
    if constexpr (VEC) {
        for (long i = (blockIdx.x * (long)TPB + threadIdx.x) * 8; i < count; i += (long)gridDim.x * TPB * 8) {
            float av[8], bv[8], gv[8];
            ld8t<T>(a, i, av);
            ld8t<T>(b, i, bv);
            if (ga && accumulate) ld8t<G>(ga, i, gv);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const float d = av[k] - bv[k];
                acc += fabsf(d);
                gv[k] = (ga && accumulate ? gv[k] : 0.f) + sgn(d) * inv;
            }
            if (ga) st8t<G>(ga, i, gv);
        }
    } else {
        for (long i = blockIdx.x * (long)TPB + threadIdx.x; i < count; i += (long)gridDim.x * TPB) {
            const float d = to_f<T>(a[i]) - to_f<T>(b[i]);
            acc += fabsf(d);
            if (ga) {
                float gv = sgn(d) * inv;
                if (accumulate) gv += to_f<G>(ga[i]);
                ga[i] = from_f<G>(gv);
            }
        }
    }
    block_add(loss, acc * inv);
}

// TV (ir:686-694): mean|x[h+1]-x[h]| + mean|x[w+1]-x[w]| over N*C*(H-1)*W and N*C*H*(W-1).
// Grid-stride over image rows (n*H + y), threads over pixels x, channel loop.
__global__ __launch_bounds__(TPB) void tv_kernel(const float* __restrict__ x, int N, int H, int W, int C, float w,
                                                 float* __restrict__ g, double* __restrict__ loss, float inv_v,
                                                 float inv_h) {
    float acc = 0.f;
    const int WC = W * C;
    for (int row = blockIdx.x; row < N * H; row += gridDim.x) {
        const int yh = row % H;
        const float* xr = x + (long)row * WC;
        float* gr = g + (long)row * WC;
        for (int xw = threadIdx.x; xw < W; xw += TPB) {
            for (int c = 0; c < C; ++c) {
                const int e = xw * C + c;
                const float v = xr[e];
                float gv = 0.f;
                if (yh + 1 < H) {
                    const float d = xr[e + WC] - v;
                    acc += fabsf(d) * inv_v;
                    gv -= sgn(d) * inv_v;
                }
                if (yh > 0) gv += sgn(v - xr[e - WC]) * inv_v;
                if (xw + 1 < W) {
                    const float d = xr[e + C] - v;
                    acc += fabsf(d) * inv_h;
                    gv -= sgn(d) * inv_h;
                }
                if (xw > 0) gv += sgn(v - xr[e - C]) * inv_h;
                gr[e] += w * gv;
            }
        }
    }
    block_add(loss, w * acc);
}

// the separable Gaussian window of ssim_loss_torch (ir:699-712): K taps, K odd
template <int K>
struct WinK {
    float g[K];
};

// SSIM (ir:714-750) on a' = (a+1)/2, b' = (b+1)/2 with the separable 11-tap
// Gaussian (sigma 1.5) and zero padding 5.  Planar fp32 work maps of size S.
template <int K>
__global__ __launch_bounds__(TPB) void ssim_h5_kernel(const float* __restrict__ a, const float* __restrict__ b, int W,
                                                      int C, WinK<K> win, float* __restrict__ out, long S) {
    constexpr int HK = K / 2;
    const int xw = blockIdx.x * TPB + threadIdx.x;
    if (xw >= W) return;
    const long rowb = (long)blockIdx.y * W * C;
    for (int c = 0; c < C; ++c) {
        const long idx = rowb + (long)xw * C + c;
        float m1 = 0.f, m2 = 0.f, e11 = 0.f, e22 = 0.f, e12 = 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int xx = xw + k - HK;
            if (xx < 0 || xx >= W) continue;
            const long j = idx + (long)(k - HK) * C;
            const float p = (a[j] + 1.f) * 0.5f, q = (b[j] + 1.f) * 0.5f, gk = win.g[k];
            m1 += gk * p;
            m2 += gk * q;
            e11 += gk * p * p;
            e22 += gk * q * q;
            e12 += gk * p * q;
        }
        out[idx] = m1;
        out[S + idx] = m2;
        out[2 * S + idx] = e11;
        out[3 * S + idx] = e22;
        out[4 * S + idx] = e12;
    }
}

// Horizontal 11-tap pass, one image row per block: the row's NI input maps are
// staged in LDS with coalesced loads (FIRST: a' = (a+1)/2 and b' = (b+1)/2, five
// outputs mu1, mu2, E[a'^2], E[b'^2], E[a'b']; else NI = NO planar maps), then every
// output element reads its 11 taps from LDS.  Same tap order as ssim_h5_kernel /
// ssim_h_kernel (bit-identical results) without their stride-C global re-reads.
template <int K, int NI, int NO, bool FIRST>
__global__ __launch_bounds__(TPB) void ssim_hrow_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                        const float* __restrict__ in, int W, int C, WinK<K> win,
                                                        float* __restrict__ out, long S) {
    constexpr int HK = K / 2;
    extern __shared__ float rowm[];  // NI x W*C
    const int WC = W * C;
    const long rb = (long)blockIdx.x * WC;
    for (int e = threadIdx.x; e < WC; e += TPB) {
        if (FIRST) {
            rowm[e] = (a[rb + e] + 1.f) * 0.5f;
            rowm[WC + e] = (b[rb + e] + 1.f) * 0.5f;
        } else {
#pragma unroll
            for (int m = 0; m < NI; ++m) rowm[m * WC + e] = in[m * S + rb + e];
        }
    }
    __syncthreads();
    for (int e = threadIdx.x; e < WC; e += TPB) {
        const int xw = e / C;
        float acc[NO];
#pragma unroll
        for (int m = 0; m < NO; ++m) acc[m] = 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int xx = xw + k - HK;
            if (xx < 0 || xx >= W) continue;
            const int j = e + (k - HK) * C;
            const float gk = win.g[k];
            if (FIRST) {
                const float p = rowm[j], q = rowm[WC + j];
                acc[0] += gk * p;
                acc[1] += gk * q;
                acc[2] += gk * p * p;
                acc[3] += gk * q * q;
                acc[4] += gk * p * q;
            } else {
#pragma unroll
                for (int m = 0; m < NO; ++m) acc[m] += gk * rowm[m * WC + j];
            }
        }
#pragma unroll
        for (int m = 0; m < NO; ++m) out[m * S + rb + e] = acc[m];
    }
}

// Round 6: the vertical pass fused with its elementwise consumer -- the five moment maps'
// vertical sums feed the SSIM map and dL/d{mu1, e11, e12} (ssim_map_kernel's arithmetic) in
// registers, and the three adjoint maps' sums feed the input gradient (ssim_grad_kernel's),
// so neither the 5 nor the 3 vertically filtered maps are written and re-read (5 + 3 fp32
// maps of N*H*W*C).  Per element the operations and their order are those of the unfused
// pair: d3 and g bit-identical; the loss is the same sum in another block grouping.
template <int K, int R, bool MAP>
__global__ __launch_bounds__(TPB) void ssim_vfused_kernel(const float* __restrict__ in, int H, int W, int C,
                                                          WinK<K> win, float w, float* __restrict__ d3,
                                                          double* __restrict__ loss, const float* __restrict__ a,
                                                          const float* __restrict__ b, float* __restrict__ g,
                                                          long S) {
    constexpr int HK = K / 2, NM = MAP ? 5 : 3;
    const int e = blockIdx.x * TPB + threadIdx.x;  // element within the row (x*C + c)
    float lacc = 0.f;
    if (e < W * C) {
        const int hb = (H + R - 1) / R;
        const int n = blockIdx.y / hb, y0 = (blockIdx.y - n * hb) * R;
        const long WC = (long)W * C;
        const long base = (long)n * H * WC + e;
        float v[NM][R + K - 1];
#pragma unroll
        for (int r = 0; r < R + K - 1; ++r) {
            const int yy = y0 + r - HK;
            const bool ok = yy >= 0 && yy < H;
#pragma unroll
            for (int m = 0; m < NM; ++m) v[m][r] = ok ? in[m * S + base + yy * WC] : 0.f;
        }
        const float C1 = 0.01f * 0.01f, C2 = 0.03f * 0.03f;
        const float dLdS = -w / (float)S;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (y0 + r >= H) break;
            float mom[NM];
#pragma unroll
            for (int m = 0; m < NM; ++m) {
                float acc = 0.f;
#pragma unroll
                for (int k = 0; k < K; ++k) acc += win.g[k] * v[m][r + k];
                mom[m] = acc;
            }
            const long idx = base + (y0 + r) * WC;
            if constexpr (MAP) {
                const float mu1 = mom[0], mu2 = mom[1], e11 = mom[2], e22 = mom[3], e12 = mom[4];
                const float m11 = mu1 * mu1, m22 = mu2 * mu2, m12 = mu1 * mu2;
                const float s11 = e11 - m11, s22 = e22 - m22, s12 = e12 - m12;
                const float A1 = 2.f * m12 + C1, A2 = 2.f * s12 + C2;
                const float B1 = m11 + m22 + C1, B2 = s11 + s22 + C2;
                const float den = B1 * B2;
                const float Sv = (A1 * A2) / den;
                lacc += 1.f - Sv;
                const float dmu1 = (2.f * mu2 * (A2 - A1)) / den - Sv * 2.f * mu1 / B1 + Sv * 2.f * mu1 / B2;
                const float de11 = -Sv / B2;
                const float de12 = 2.f * A1 / den;
                d3[idx] = dLdS * dmu1;
                d3[S + idx] = dLdS * de11;
                d3[2 * S + idx] = dLdS * de12;
            } else {
                const float p = (a[idx] + 1.f) * 0.5f, q = (b[idx] + 1.f) * 0.5f;
                const float gp = mom[0] + 2.f * p * mom[1] + q * mom[2];
                g[idx] += 0.5f * gp;  // d a'/d a = 1/2
            }
        }
    }
    if constexpr (MAP) block_add(loss, w * lacc / (float)S);
}

// horizontal 11-tap pass over NM planar maps
template <int K, int NM>
__global__ __launch_bounds__(TPB) void ssim_h_kernel(const float* __restrict__ in, int W, int C, WinK<K> win,
                                                     float* __restrict__ out, long S) {
    constexpr int HK = K / 2;
    const int xw = blockIdx.x * TPB + threadIdx.x;
    if (xw >= W) return;
    const long rowb = (long)blockIdx.y * W * C;
    for (int c = 0; c < C; ++c) {
        const long idx = rowb + (long)xw * C + c;
        float acc[NM];
#pragma unroll
        for (int m = 0; m < NM; ++m) acc[m] = 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int xx = xw + k - HK;
            if (xx < 0 || xx >= W) continue;
            const long j = idx + (long)(k - HK) * C;
#pragma unroll
            for (int m = 0; m < NM; ++m) acc[m] += win.g[k] * in[m * S + j];
        }
#pragma unroll
        for (int m = 0; m < NM; ++m) out[m * S + idx] = acc[m];
    }
}

// prm (device, nullable): {step_size, bc2s} written by adam_prep_kernel in the same stream
// (graph replay: the step count lives on the device, so a captured step stays valid)
__global__ __launch_bounds__(TPB) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, long n,
                                                   float step_size, float b1, float b2, float bc2s, float eps,
                                                   const float* __restrict__ prm = nullptr) {
    if (prm) {
        step_size = prm[0];
        bc2s = prm[1];
    }
    const float w1 = 1.f - b1, w2 = 1.f - b2;
    for (long i = blockIdx.x * (long)TPB + threadIdx.x; i < n; i += (long)gridDim.x * TPB) {
        const float gi = g[i];
        float mi = m[i];
        // torch lerp: weight < 0.5 ? m + w*(g-m) : g - (g-m)*(1-w)
        mi = (w1 < 0.5f) ? mi + w1 * (gi - mi) : gi - (gi - mi) * (1.f - w1);
        float vi = v[i] * b2 + w2 * gi * gi;
        const float denom = sqrtf(vi) / bc2s + eps;
        p[i] = p[i] + (-step_size) * (mi / denom);
        m[i] = mi;
        v[i] = vi;
    }
}

template <int K>
WinK<K> gauss_win() {
    // ir:699-703 in fp32: coords = arange(K) - (K-1)/2, exp(-c^2 / (2*1.5^2)), normalised
    WinK<K> w;
    float s = 0.f;
    for (int k = 0; k < K; ++k) {
        float c = (float)k - (float)(K - 1) / 2.0f;
        w.g[k] = expf(-(c * c) / (2.f * 1.5f * 1.5f));
        s += w.g[k];
    }
    for (int k = 0; k < K; ++k) w.g[k] /= s;
    return w;
}

// the forward + gradient launches for one window size (S = N*H*W*C, maps in work)
template <int K>
int ssim_launch(const float* a, const float* b, int N, int H, int W, int C, float w, float* g, double* loss,
                float* work, hipStream_t st) {
    const long S = (long)N * H * W * C;
    const WinK<K> win = gauss_win<K>();
    float* w0 = work;          // 5 maps
    float* w1 = work + 5 * S;  // 5 maps
    constexpr int VR = 8;  // rows per thread in the vertical passes
    const dim3 gx(irgan_cdiv(W, TPB), N * H), ge(irgan_cdiv((long)W * C, TPB), N * irgan_cdiv(H, VR));
    const size_t row5 = (size_t)W * C * 2 * sizeof(float), row3 = (size_t)W * C * 3 * sizeof(float);
    if (row3 <= 64 * 1024) {  // row-staged horizontal passes (W*C <= 5461)
        ssim_hrow_kernel<K, 2, 5, true><<<N * H, TPB, row5, st>>>(a, b, nullptr, W, C, win, w0, S);
    } else {
        ssim_h5_kernel<K><<<gx, TPB, 0, st>>>(a, b, W, C, win, w0, S);
    }
    // vertical pass + SSIM map + its gradient maps (into w1's first 3 maps)
    ssim_vfused_kernel<K, VR, true><<<ge, TPB, 0, st>>>(w0, H, W, C, win, w, w1, loss, nullptr, nullptr, nullptr, S);
    if (row3 <= 64 * 1024) {
        ssim_hrow_kernel<K, 3, 3, false><<<N * H, TPB, row3, st>>>(nullptr, nullptr, w1, W, C, win, w0, S);
    } else {
        ssim_h_kernel<K, 3><<<gx, TPB, 0, st>>>(w1, W, C, win, w0, S);
    }
    // vertical pass of the adjoint + the input gradient
    ssim_vfused_kernel<K, VR, false><<<ge, TPB, 0, st>>>(w0, H, W, C, win, w, nullptr, nullptr, a, b, g, S);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

}  // namespace

extern "C" int irgan_hinge(const float* pred, int32_t n_half, int32_t mode, float scale, float* grad, double* loss,
                           irgan_stream_t s) {
    if (mode != 0 && mode != 1) return IRGAN_EINVAL;
    long total = mode == 0 ? 2L * n_half : n_half;
    hinge_kernel<<<nblocks_red(total), TPB, 0, (hipStream_t)s>>>(pred, n_half, mode, scale, grad, loss);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_l1(const void* a, const void* b, int32_t dtype, int64_t count, float w, void* ga,
                        int32_t ga_dtype, int32_t accumulate, double* loss, irgan_stream_t s) {
    hipStream_t st = (hipStream_t)s;
    if (count <= 0) return 0;
    const bool vec = count % 8 == 0 && ((uintptr_t)a % 16 == 0) && ((uintptr_t)b % 16 == 0) &&
                     (!ga || (uintptr_t)ga % 16 == 0);
    const int nb = nblocks_red(vec ? count / 8 : count);
#define L1_LAUNCH(T, G)                                                                                       \
    do {                                                                                                      \
        if (vec)                                                                                              \
            l1_kernel<T, G, true><<<nb, TPB, 0, st>>>((const T*)a, (const T*)b, count, w, (G*)ga, accumulate, \
                                                      loss);                                                  \
        else                                                                                                  \
            l1_kernel<T, G, false><<<nb, TPB, 0, st>>>((const T*)a, (const T*)b, count, w, (G*)ga, accumulate, \
                                                       loss);                                                 \
    } while (0)
    if (dtype == IRGAN_F32) {
        if (ga_dtype == IRGAN_BF16) L1_LAUNCH(float, bf16_t);
        else L1_LAUNCH(float, float);
    } else {
        if (ga_dtype == IRGAN_BF16) L1_LAUNCH(bf16_t, bf16_t);
        else L1_LAUNCH(bf16_t, float);
    }
#undef L1_LAUNCH
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_tv(const float* x, int32_t N, int32_t H, int32_t W, int32_t C, float w, float* g, double* loss,
                        irgan_stream_t s) {
    if ((long)N * H * W * C <= 0) return 0;
    float inv_v = H > 1 ? 1.f / (float)((long)N * C * (H - 1) * W) : 0.f;
    float inv_h = W > 1 ? 1.f / (float)((long)N * C * H * (W - 1)) : 0.f;
    tv_kernel<<<std::min(N * H, 512), TPB, 0, (hipStream_t)s>>>(x, N, H, W, C, w, g, loss, inv_v, inv_h);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_ssim_ws(const float* a, const float* b, int32_t N, int32_t H, int32_t W, int32_t C, float w,
                             float* g, double* loss, float* work, int32_t window, irgan_stream_t s) {
    hipStream_t st = (hipStream_t)s;
    if ((long)N * H * W * C <= 0) return 0;
    if ((long)N * H > 65535) return IRGAN_EUNSUPPORTED;
    switch (window) {
        case 1: return ssim_launch<1>(a, b, N, H, W, C, w, g, loss, work, st);
        case 3: return ssim_launch<3>(a, b, N, H, W, C, w, g, loss, work, st);
        case 5: return ssim_launch<5>(a, b, N, H, W, C, w, g, loss, work, st);
        case 7: return ssim_launch<7>(a, b, N, H, W, C, w, g, loss, work, st);
        case 9: return ssim_launch<9>(a, b, N, H, W, C, w, g, loss, work, st);
        case 11: return ssim_launch<11>(a, b, N, H, W, C, w, g, loss, work, st);
        case 13: return ssim_launch<13>(a, b, N, H, W, C, w, g, loss, work, st);
        case 15: return ssim_launch<15>(a, b, N, H, W, C, w, g, loss, work, st);
        default: return IRGAN_EUNSUPPORTED;
    }
}

extern "C" int irgan_ssim(const float* a, const float* b, int32_t N, int32_t H, int32_t W, int32_t C, float w,
                          float* g, double* loss, float* work, irgan_stream_t s) {
    return irgan_ssim_ws(a, b, N, H, W, C, w, g, loss, work, 11, s);
}

// t = ++*count; prm = {lr / (1 - b1^t), sqrt(1 - b2^t)}: the host formula of irgan_adam's
// arguments (ops.adam), in fp64 and then rounded to fp32, evaluated on the device
static __global__ void adam_prep_kernel(int32_t* count, double lr, double b1, double b2, float* prm) {
    if (threadIdx.x != 0) return;
    const int t = *count + 1;
    *count = t;
    const double bc1 = 1.0 - pow(b1, (double)t), bc2 = 1.0 - pow(b2, (double)t);
    prm[0] = (float)(lr / bc1);
    prm[1] = (float)sqrt(bc2);
}

extern "C" int irgan_adam_prep(int32_t* count, double lr, double beta1, double beta2, float* prm, irgan_stream_t s) {
    if (!count || !prm) return IRGAN_EINVAL;
    adam_prep_kernel<<<1, 64, 0, (hipStream_t)s>>>(count, lr, beta1, beta2, prm);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_adam_dev(float* p, const float* g, float* m, float* v, int64_t n, const float* prm, float beta1,
                              float beta2, float eps, irgan_stream_t s) {
    if (!prm) return IRGAN_EINVAL;
    if (n <= 0) return 0;
    adam_kernel<<<nblocks(n), TPB, 0, (hipStream_t)s>>>(p, g, m, v, n, 0.f, beta1, beta2, 1.f, eps, prm);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_adam(float* p, const float* g, float* m, float* v, int64_t n, float step_size, float beta1,
                          float beta2, float bc2_sqrt, float eps, irgan_stream_t s) {
    if (n <= 0) return 0;
    adam_kernel<<<nblocks(n), TPB, 0, (hipStream_t)s>>>(p, g, m, v, n, step_size, beta1, beta2, bc2_sqrt, eps);
    IRGAN_LAUNCH_CHECK();
    return 0;
}
