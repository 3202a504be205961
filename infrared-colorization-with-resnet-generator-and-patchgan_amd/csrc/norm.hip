// InstanceNorm forward / backward and channel reductions (NHWC, per (n, c)
// over H*W).  Replaces nn.InstanceNorm2d (ir:154-165: eps 1e-5, no affine, no
// running stats) + the fused ReLU / LeakyReLU(0.2) / residual add of ir:392,
// 417-418, 601-624 and their autograd backward.
//
// Statistics are accumulated per block in fp32 and across blocks in fp64
// atomics (one add per (n, c) per block), then finalised to fp32 (mean, rstd)
// or (mean g, mean g*xhat) by a second tiny launch.
#include "common.h"

namespace {

constexpr int TPB = 256;

// thread -> (channel, row lane) layout for a C-wide NHWC row block
struct RowLayout {
    int cpt, rpar;  // channels covered per pass, rows processed in parallel
    __device__ RowLayout(int C) {
        cpt = C < TPB ? C : TPB;
        rpar = TPB / cpt;
    }
};

// derivative of the activation that followed the norm, at xhat
IRGAN_HD float act_grad(float xh, int act) {
    if (act == IRGAN_ACT_RELU) return xh > 0.f ? 1.f : 0.f;
    if (act == IRGAN_ACT_LRELU) return xh > 0.f ? 1.f : 0.2f;
    return 1.f;
}

// generic per-(n,c) two-moment reduction; MODE 0: (x, x^2); MODE 1: (g, g*xhat)
template <int MODE>
__global__ __launch_bounds__(TPB) void reduce2_kernel(const void* __restrict__ x, int xdt, int ldx, int xoff,
                                                      const void* __restrict__ dy2, int d2dt, int ld2, int off2,
                                                      const void* __restrict__ a, int adt, int lda, int aoff,
                                                      int act, const float* __restrict__ mr, int HW, int C,
                                                      int rows_per_block, double* __restrict__ work) {
    __shared__ float s0[TPB], s1[TPB];
    const int n = blockIdx.y;
    const int r0 = blockIdx.x * rows_per_block;
    const int r1 = min(HW, r0 + rows_per_block);
    RowLayout L(C);
    const int tid = threadIdx.x;
    const int cl = tid % L.cpt, rl = tid / L.cpt;
    const bool active = rl < L.rpar;
    for (int cbase = 0; cbase < C; cbase += L.cpt) {
        const int c = cbase + cl;
        float acc0 = 0.f, acc1 = 0.f;
        if (active && c < C) {
            float2 st = make_float2(0.f, 0.f);
            if (MODE == 1) st = ((const float2*)mr)[(long)n * C + c];
            for (int r = r0 + rl; r < r1; r += L.rpar) {
                const long p = (long)n * HW + r;
                float v = ldv(x, xdt, p * ldx + xoff + c);
                if (MODE == 0) {
                    acc0 += v;
                    acc1 += v * v;
                } else {
                    if (dy2) v += ldv(dy2, d2dt, p * ld2 + off2 + c);
                    const float xh = (ldv(a, adt, p * lda + aoff + c) - st.x) * st.y;
                    const float g = v * act_grad(xh, act);
                    acc0 += g;
                    acc1 += g * xh;
                }
            }
        }
        s0[tid] = acc0;
        s1[tid] = acc1;
        __syncthreads();
        if (active && rl == 0 && c < C) {
            float t0 = 0.f, t1 = 0.f;
            for (int k = 0; k < L.rpar; ++k) {
                t0 += s0[cl + k * L.cpt];
                t1 += s1[cl + k * L.cpt];
            }
            atomicAdd(work + ((long)n * C + c) * 2 + 0, (double)t0);
            atomicAdd(work + ((long)n * C + c) * 2 + 1, (double)t1);
        }
        __syncthreads();
    }
}

__global__ void finalize_stats_kernel(const double* __restrict__ work, float* __restrict__ mr, int NC, int HW,
                                      int mode) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= NC) return;
    double s = work[2 * i], q = work[2 * i + 1];
    double mean = s / HW;
    if (mode == 0) {
        double var = q / HW - mean * mean;
        if (var < 0) var = 0;
        mr[2 * i] = (float)mean;
        mr[2 * i + 1] = (float)(1.0 / sqrt(var + 1e-5));
    } else {
        mr[2 * i] = (float)mean;
        mr[2 * i + 1] = (float)(q / HW);
    }
}

__global__ __launch_bounds__(TPB) void in_apply_kernel(const void* __restrict__ x, int dt, int HW, int C, int ldx,
                                                       int xoff, const float* __restrict__ mr, int act,
                                                       const void* __restrict__ res, int ldr, int roff,
                                                       void* __restrict__ y, int ldy, int yoff,
                                                       void* __restrict__ xhat, long total) {
    for (long idx = blockIdx.x * (long)TPB + threadIdx.x; idx < total; idx += (long)gridDim.x * TPB) {
        const long p = idx / C;
        const int c = (int)(idx - p * C);
        const int n = (int)(p / HW);
        const float2 st = ((const float2*)mr)[(long)n * C + c];
        float v = (ldv(x, dt, p * ldx + xoff + c) - st.x) * st.y;
        if (xhat) stv(xhat, dt, p * C + c, v);
        if (act == IRGAN_ACT_RELU) v = v > 0.f ? v : 0.f;
        else if (act == IRGAN_ACT_LRELU) v = v > 0.f ? v : 0.2f * v;
        if (res) v += ldv(res, dt, p * ldr + roff + c);
        stv(y, dt, p * ldy + yoff + c, v);
    }
}

__global__ __launch_bounds__(TPB) void in_bwd_apply_kernel(
    const void* __restrict__ dy, int dydt, int lddy, int dyoff, const void* __restrict__ dy2, int d2dt, int ld2,
    int off2, const void* __restrict__ a, int adt, int lda, int aoff, int act, int HW, int C,
    const float* __restrict__ mr, const float* __restrict__ red, void* __restrict__ dx, int dxdt, int lddx,
    int dxoff, float* __restrict__ db, int rows_per_block) {
    __shared__ float sdb[TPB];
    const int n = blockIdx.y;
    const int r0 = blockIdx.x * rows_per_block;
    const int r1 = min(HW, r0 + rows_per_block);
    RowLayout L(C);
    const int tid = threadIdx.x;
    const int cl = tid % L.cpt, rl = tid / L.cpt;
    const bool active = rl < L.rpar;
    for (int cbase = 0; cbase < C; cbase += L.cpt) {
        const int c = cbase + cl;
        float accd = 0.f;
        if (active && c < C) {
            const float2 st = ((const float2*)mr)[(long)n * C + c];
            const float2 rd = ((const float2*)red)[(long)n * C + c];
            for (int r = r0 + rl; r < r1; r += L.rpar) {
                const long p = (long)n * HW + r;
                float v = ldv(dy, dydt, p * lddy + dyoff + c);
                if (dy2) v += ldv(dy2, d2dt, p * ld2 + off2 + c);
                const float xh = (ldv(a, adt, p * lda + aoff + c) - st.x) * st.y;
                const float g = v * act_grad(xh, act);
                const float o = st.y * (g - rd.x - xh * rd.y);
                stv(dx, dxdt, p * lddx + dxoff + c, o);
                accd += o;
            }
        }
        if (db) {
            sdb[tid] = accd;
            __syncthreads();
            if (active && rl == 0 && c < C) {
                float t = 0.f;
                for (int k = 0; k < L.rpar; ++k) t += sdb[cl + k * L.cpt];
                atomicAdd(db + c, t);
            }
            __syncthreads();
        }
    }
}

__global__ __launch_bounds__(TPB) void channel_sum_kernel(const void* __restrict__ g, int dt, long P, int C, int ld,
                                                          int off, float* __restrict__ db, int rows_per_block) {
    __shared__ float s[TPB];
    const long r0 = (long)blockIdx.x * rows_per_block;
    const long r1 = min(P, r0 + rows_per_block);
    RowLayout L(C);
    const int tid = threadIdx.x, cl = tid % L.cpt, rl = tid / L.cpt;
    const bool active = rl < L.rpar;
    for (int cbase = 0; cbase < C; cbase += L.cpt) {
        const int c = cbase + cl;
        float acc = 0.f;
        if (active && c < C)
            for (long r = r0 + rl; r < r1; r += L.rpar) acc += ldv(g, dt, r * ld + off + c);
        s[tid] = acc;
        __syncthreads();
        if (active && rl == 0 && c < C) {
            float t = 0.f;
            for (int k = 0; k < L.rpar; ++k) t += s[cl + k * L.cpt];
            atomicAdd(db + c, t);
        }
        __syncthreads();
    }
}

int rows_for(long HW, int N) {
    // ~1-4k rows per block, enough blocks to cover 256 CUs
    long want_blocks = 1024 / (N > 0 ? N : 1);
    if (want_blocks < 1) want_blocks = 1;
    long r = (HW + want_blocks - 1) / want_blocks;
    if (r < 256) r = 256;
    return (int)r;
}

}  // namespace

extern "C" int irgan_in_stats(const void* x, int32_t dtype, int32_t N, int32_t HW, int32_t C, int32_t ld,
                              int32_t off, double* work, float* mr, irgan_stream_t s) {
    hipStream_t st = (hipStream_t)s;
    hipMemsetAsync(work, 0, sizeof(double) * 2 * (size_t)N * C, st);
    int rows = rows_for(HW, N);
    dim3 g(irgan_cdiv(HW, rows), N);
    reduce2_kernel<0><<<g, TPB, 0, st>>>(x, dtype, ld, off, nullptr, 0, 0, 0, nullptr, 0, 0, 0, 0, nullptr, HW, C,
                                         rows, work);
    finalize_stats_kernel<<<irgan_cdiv((long)N * C, 256), 256, 0, st>>>(work, mr, N * C, HW, 0);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_in_apply(const void* x, int32_t dtype, int32_t N, int32_t HW, int32_t C, int32_t ldx,
                              int32_t xoff, const float* mr, int32_t act, const void* res, int32_t ldr, int32_t roff,
                              void* y, int32_t ldy, int32_t yoff, void* xhat, irgan_stream_t s) {
    long total = (long)N * HW * C;
    if (total <= 0) return 0;
    int blocks = (int)std::min<long>((total + TPB - 1) / TPB, 8192);
    in_apply_kernel<<<blocks, TPB, 0, (hipStream_t)s>>>(x, dtype, HW, C, ldx, xoff, mr, act, res, ldr, roff, y, ldy,
                                                        yoff, xhat, total);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_in_bwd_reduce(const void* dy, int32_t dy_dtype, int32_t lddy, int32_t dyoff, const void* dy2,
                                   int32_t dy2_dtype, int32_t lddy2, int32_t dy2off, const void* x, int32_t x_dtype,
                                   int32_t ldx, int32_t xoff, int32_t act, int32_t N, int32_t HW, int32_t C,
                                   const float* mr, double* work, float* red, irgan_stream_t s) {
    hipStream_t st = (hipStream_t)s;
    hipMemsetAsync(work, 0, sizeof(double) * 2 * (size_t)N * C, st);
    int rows = rows_for(HW, N);
    dim3 g(irgan_cdiv(HW, rows), N);
    reduce2_kernel<1><<<g, TPB, 0, st>>>(dy, dy_dtype, lddy, dyoff, dy2, dy2_dtype, lddy2, dy2off, x, x_dtype, ldx,
                                         xoff, act, mr, HW, C, rows, work);
    finalize_stats_kernel<<<irgan_cdiv((long)N * C, 256), 256, 0, st>>>(work, red, N * C, HW, 1);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_in_bwd_apply(const void* dy, int32_t dy_dtype, int32_t lddy, int32_t dyoff, const void* dy2,
                                  int32_t dy2_dtype, int32_t lddy2, int32_t dy2off, const void* x, int32_t x_dtype,
                                  int32_t ldx, int32_t xoff, int32_t act, int32_t N, int32_t HW, int32_t C,
                                  const float* mr, const float* red, void* dx, int32_t dx_dtype, int32_t lddx,
                                  int32_t dxoff, float* db, irgan_stream_t s) {
    int rows = rows_for(HW, N);
    dim3 g(irgan_cdiv(HW, rows), N);
    in_bwd_apply_kernel<<<g, TPB, 0, (hipStream_t)s>>>(dy, dy_dtype, lddy, dyoff, dy2, dy2_dtype, lddy2, dy2off, x,
                                                       x_dtype, ldx, xoff, act, HW, C, mr, red, dx, dx_dtype, lddx,
                                                       dxoff, db, rows);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_channel_sum(const void* g, int32_t dtype, int32_t P, int32_t C, int32_t ld, int32_t off,
                                 float* db, irgan_stream_t s) {
    if (P <= 0) return 0;
    int rows = rows_for(P, 1);
    channel_sum_kernel<<<irgan_cdiv(P, rows), TPB, 0, (hipStream_t)s>>>(g, dtype, P, C, ld, off, db, rows);
    IRGAN_LAUNCH_CHECK();
    return 0;
}
