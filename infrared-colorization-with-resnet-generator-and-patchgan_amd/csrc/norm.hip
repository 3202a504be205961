// InstanceNorm forward / backward and channel reductions (NHWC, per (n, c)
// over H*W).  Replaces nn.InstanceNorm2d (ir:154-165: eps 1e-5, no affine, no
// running stats) + the fused ReLU / LeakyReLU(0.2) / residual add of ir:392,
// 417-418, 601-624 and their autograd backward.
//
// HBM-bound: every thread owns 8 consecutive channels (one 16-byte bf16 load /
// two 16-byte fp32 loads per pixel) and walks >= 8 rows; a block covers a run of
// rows of one image and reduces its partial sums through LDS.  Reductions are
// two-level and atomic-free: each block stores one float2 partial per channel
// (<= IN_PARTS blocks per image), and the finalize launch sums the partials of
// each (n, c) in fp64, in a fixed order (deterministic), into fp32 (mean, rstd)
// or (mean g, mean g*xhat).
#include "fp8_util.h"

namespace {

// optional fp8 copy of a pass's bf16 output (the fp8 path's conv operands,
// GeneratorEngine(fp8=True)): y8 = e4m3(clamp(bf16(y) * q[0])), max |bf16(y)|
// into the amax slot -- the same bytes irgan_fp8_quant makes from the stored y
struct Q8 {
    uint8_t* p;
    int ld, off;
    const float* q;
    uint32_t* amax;
};

constexpr int TPB = 256;
constexpr int V = 8;          // channels per thread
constexpr int IN_PARTS = 128; // max rows-kernel blocks (partials) per image (<= IRGAN_IN_PARTS, the work size)

IRGAN_HD void ld8(const void* p, int dt, long i, float* o) {
    if (dt == IRGAN_BF16) {
        const uint4 u = *(const uint4*)((const bf16_t*)p + i);
        const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            o[2 * k] = __uint_as_float(w[k] << 16);
            o[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
        }
    } else {
        const float4 a = *(const float4*)((const float*)p + i), b = *(const float4*)((const float*)p + i + 4);
        o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
    }
}
IRGAN_HD void st8(void* p, int dt, long i, const float* v) {
    if (dt == IRGAN_BF16) {
        uint4 u;
        u.x = pk_bf16(v[0], v[1]);
        u.y = pk_bf16(v[2], v[3]);
        u.z = pk_bf16(v[4], v[5]);
        u.w = pk_bf16(v[6], v[7]);
        *(uint4*)((bf16_t*)p + i) = u;
    } else {
        *(float4*)((float*)p + i) = make_float4(v[0], v[1], v[2], v[3]);
        *(float4*)((float*)p + i + 4) = make_float4(v[4], v[5], v[6], v[7]);
    }
}
template <int VW>
IRGAN_HD void ldv_(const void* p, int dt, long i, float* o) {
    if constexpr (VW == 8) ld8(p, dt, i, o);
    else o[0] = ldv(p, dt, i);
}
template <int VW>
IRGAN_HD void stv_(void* p, int dt, long i, const float* v) {
    if constexpr (VW == 8) st8(p, dt, i, v);
    else stv(p, dt, i, v[0]);
}

// derivative of the activation that followed the norm, at xhat
IRGAN_HD float act_grad(float xh, int act) {
    if (act == IRGAN_ACT_RELU) return xh > 0.f ? 1.f : 0.f;
    if (act == IRGAN_ACT_LRELU) return xh > 0.f ? 1.f : 0.2f;
    return 1.f;
}

struct Slice {
    const void* p;
    int dt, ld, off;
};

// block layout: CL lanes per row (VW channels each), RP rows in parallel
struct Lay {
    int CL, RP, cl, rl;
    __device__ Lay(int C, int VW) {
        CL = (C + VW - 1) / VW;
        if (CL > TPB) CL = TPB;
        RP = TPB / CL;
        cl = threadIdx.x % CL;
        rl = threadIdx.x / CL;
    }
};

// MODE 0: (sum x, sum x^2); MODE 1: (sum g, sum g*xhat), g = (dy+dy2)*act'(xhat),
// xhat = (x-mean)*rstd;  MODE 2: MODE-1 pass that also writes dx and sums dx (db);
// MODE 3: plain channel sum of x into db (bias gradients)
template <int MODE, int VW>
__global__ __launch_bounds__(TPB) void rows_kernel(Slice X, Slice DY, Slice DY2, int act, const float* __restrict__ mr,
                                                   const float* __restrict__ red, void* __restrict__ dx, int dxdt,
                                                   int lddx, int dxoff, int HW, int C, int rows_per_block,
                                                   float2* __restrict__ part, float* __restrict__ db) {
    __shared__ float s0[TPB * VW], s1[TPB * VW];
    const int n = blockIdx.y;
    const int r0 = blockIdx.x * rows_per_block;
    const int r1 = min(HW, r0 + rows_per_block);
    Lay L(C, VW);
    const bool active = L.rl < L.RP;
    for (int cb = 0; cb < C; cb += L.CL * VW) {
        const int c = cb + L.cl * VW;
        const bool on = active && c < C;
        float a0[VW], a1[VW], mean[VW], rstd[VW], mg[VW], mgx[VW];
#pragma unroll
        for (int k = 0; k < VW; ++k) { a0[k] = 0.f; a1[k] = 0.f; }
        if (on && MODE >= 1) {
#pragma unroll
            for (int k = 0; k < VW; ++k) {
                const float2 st = ((const float2*)mr)[(long)n * C + c + k];
                mean[k] = st.x; rstd[k] = st.y;
                if (MODE == 2) {
                    const float2 rd = ((const float2*)red)[(long)n * C + c + k];
                    mg[k] = rd.x; mgx[k] = rd.y;
                }
            }
        }
        if (on) {
#pragma unroll 8
            for (int r = r0 + L.rl; r < r1; r += L.RP) {
                const long p = (long)n * HW + r;
                float xv[VW];
                ldv_<VW>(X.p, X.dt, p * X.ld + X.off + c, xv);
                if (MODE == 0 || MODE == 3) {
#pragma unroll
                    for (int k = 0; k < VW; ++k) { a0[k] += xv[k]; a1[k] += xv[k] * xv[k]; }
                } else {
                    float gv[VW], g2[VW];
                    ldv_<VW>(DY.p, DY.dt, p * DY.ld + DY.off + c, gv);
                    if (DY2.p) {
                        ldv_<VW>(DY2.p, DY2.dt, p * DY2.ld + DY2.off + c, g2);
#pragma unroll
                        for (int k = 0; k < VW; ++k) gv[k] += g2[k];
                    }
                    float o[VW];
#pragma unroll
                    for (int k = 0; k < VW; ++k) {
                        const float xh = (xv[k] - mean[k]) * rstd[k];
                        const float g = gv[k] * act_grad(xh, act);
                        if (MODE == 1) { a0[k] += g; a1[k] += g * xh; }
                        else { o[k] = rstd[k] * (g - mg[k] - xh * mgx[k]); a0[k] += o[k]; }
                    }
                    if (MODE == 2) stv_<VW>(dx, dxdt, p * lddx + dxoff + c, o);
                }
            }
        }
        if ((MODE == 2 || MODE == 3) && !db) continue;  // uniform across the block
        if (L.CL <= 64 && (64 % L.CL) == 0) {
            // rows of one wave share a lane's channels every CL lanes: butterfly
            // over them, then one LDS slot per (wave, channel lane)
            for (int o = L.CL; o < 64; o <<= 1) {
#pragma unroll
                for (int k = 0; k < VW; ++k) {
                    a0[k] += __shfl_xor(a0[k], o, 64);
                    a1[k] += __shfl_xor(a1[k], o, 64);
                }
            }
            const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
            if (lane < L.CL) {
#pragma unroll
                for (int k = 0; k < VW; ++k) {
                    s0[(wv * L.CL + lane) * VW + k] = a0[k];
                    s1[(wv * L.CL + lane) * VW + k] = a1[k];
                }
            }
            __syncthreads();
            if (threadIdx.x < L.CL && cb + threadIdx.x * VW < C) {
                const int cc = cb + threadIdx.x * VW;
#pragma unroll
                for (int k = 0; k < VW; ++k) {
                    float t0 = 0.f, t1 = 0.f;
                    for (int j = 0; j < TPB / 64; ++j) {
                        t0 += s0[(j * L.CL + threadIdx.x) * VW + k];
                        t1 += s1[(j * L.CL + threadIdx.x) * VW + k];
                    }
                    if (MODE == 2 || MODE == 3) atomicAdd(db + cc + k, t0);
                    else part[((long)n * gridDim.x + blockIdx.x) * C + cc + k] = make_float2(t0, t1);
                }
            }
            __syncthreads();
            continue;
        }
#pragma unroll
        for (int k = 0; k < VW; ++k) {
            s0[threadIdx.x * VW + k] = a0[k];
            s1[threadIdx.x * VW + k] = a1[k];
        }
        __syncthreads();
        // first RP-row of lanes reduces over the RP rows
        if (on && L.rl == 0) {
#pragma unroll
            for (int k = 0; k < VW; ++k) {
                float t0 = 0.f, t1 = 0.f;
                for (int j = 0; j < L.RP; ++j) {
                    t0 += s0[(j * L.CL + L.cl) * VW + k];
                    t1 += s1[(j * L.CL + L.cl) * VW + k];
                }
                if (MODE == 2 || MODE == 3) {
                    atomicAdd(db + c + k, t0);
                } else {  // partial of block b of image n: part[(n*nb + b)*C + c]
                    part[((long)n * gridDim.x + blockIdx.x) * C + c + k] = make_float2(t0, t1);
                }
            }
        }
        __syncthreads();
    }
}

IRGAN_HD void bf8f(const uint4 u, float* o) {
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        o[2 * k] = __uint_as_float(w[k] << 16);
        o[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
    }
}

// Block-wide per-channel sums of (a0, a1) (8 channels per thread) ->
// part[(n*gridDim.x + blockIdx.x)*C + c]; the same order as rows_kernel's.
IRGAN_HD void block_partials8(float* a0, float* a1, const Lay& L, bool on, int cb, int c, int C, int n, float* s0,
                              float* s1, float2* __restrict__ part) {
    if (L.CL <= 64 && (64 % L.CL) == 0) {
        for (int o = L.CL; o < 64; o <<= 1) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                a0[k] += __shfl_xor(a0[k], o, 64);
                a1[k] += __shfl_xor(a1[k], o, 64);
            }
        }
        const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
        if (lane < L.CL) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                s0[(wv * L.CL + lane) * 8 + k] = a0[k];
                s1[(wv * L.CL + lane) * 8 + k] = a1[k];
            }
        }
        __syncthreads();
        if (threadIdx.x < L.CL && cb + threadIdx.x * 8 < C) {
            const int cc = cb + threadIdx.x * 8;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                float t0 = 0.f, t1 = 0.f;
                for (int j = 0; j < TPB / 64; ++j) {
                    t0 += s0[(j * L.CL + threadIdx.x) * 8 + k];
                    t1 += s1[(j * L.CL + threadIdx.x) * 8 + k];
                }
                part[((long)n * gridDim.x + blockIdx.x) * C + cc + k] = make_float2(t0, t1);
            }
        }
        __syncthreads();
        return;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        s0[threadIdx.x * 8 + k] = a0[k];
        s1[threadIdx.x * 8 + k] = a1[k];
    }
    __syncthreads();
    if (on && L.rl == 0) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            float t0 = 0.f, t1 = 0.f;
            for (int j = 0; j < L.RP; ++j) {
                t0 += s0[(j * L.CL + L.cl) * 8 + k];
                t1 += s1[(j * L.CL + L.cl) * 8 + k];
            }
            part[((long)n * gridDim.x + blockIdx.x) * C + c + k] = make_float2(t0, t1);
        }
    }
    __syncthreads();
}

// All-bf16 fast path of rows_kernel<MODE, 8> for MODE 0 (stats), 1 (backward
// reduce) and 2 (backward apply without db), and MODE 4: the forward apply
// y = act((x - mean) * rstd) [+ res] (res in the dy slot, nullable) -- apply_kernel's job
// without its per-element index divisions and per-element {mean, rstd} reloads: a
// thread's 8 channels and image are fixed, so their table entries are loaded once.  rows_kernel issues one row's
// loads at a time at ~150 VGPRs (3 waves per SIMD), so only ~24 KB of loads are
// in flight per CU and the backward reduce streams at ~2 TB/s.  Here each
// thread walks its rows in batches of U and issues every 16-byte load of a
// batch, unconverted, before using any; tail rows of the last batch re-load a
// valid row and are masked.  dx may alias dy (no __restrict__ on either): a
// thread stores only rows it has already loaded.
// ROWS8_DB = 1: two register batches in flight (U rows each, the next batch's loads issued
// before the current one is used); 0 (default): one batch at a time with twice the rows.
// Measured same box: no faster standalone (tools/norm_bench.py) and -0.5 % on the step
// (profiles/r05_s5_nab.txt), so the round-4 schedule stays
#ifndef ROWS8_DB
#define ROWS8_DB 0
#endif
template <int MODE, int U, bool F8 = false>
__global__ __launch_bounds__(TPB) void rows8_kernel(const bf16_t* x, int ldx, int xoff, const bf16_t* dy, int lddy,
                                                    int dyoff, const bf16_t* dy2, int lddy2, int dy2off, int act,
                                                    const float* __restrict__ mr, const float* __restrict__ red,
                                                    bf16_t* dx, int lddx, int dxoff, int HW, int C, int rows_per_block,
                                                    float2* __restrict__ part, Q8 q8 = Q8{}) {
    __shared__ float s0[TPB * 8], s1[TPB * 8];
    const float qs = F8 ? *q8.q : 1.f;
    float amx = 0.f;
    const int n = blockIdx.y;
    const int r0 = blockIdx.x * rows_per_block;
    const int r1 = min(HW, r0 + rows_per_block);
    Lay L(C, 8);
    const bool active = L.rl < L.RP;
    const long pb = (long)n * HW;
    for (int cb = 0; cb < C; cb += L.CL * 8) {
        const int c = cb + L.cl * 8;
        const bool on = active && c < C;
        float a0[8], a1[8], mean[8], rstd[8], mg[8], mgx[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) { a0[k] = 0.f; a1[k] = 0.f; }
        if (on && MODE >= 1) {   // (MODE 4 as well)
            const float4* m4 = (const float4*)(mr + 2 * ((long)n * C + c));
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float4 t = m4[k];
                mean[2 * k] = t.x; rstd[2 * k] = t.y; mean[2 * k + 1] = t.z; rstd[2 * k + 1] = t.w;
            }
            if (MODE == 2) {
                const float4* r4 = (const float4*)(red + 2 * ((long)n * C + c));
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const float4 t = r4[k];
                    mg[2 * k] = t.x; mgx[2 * k] = t.y; mg[2 * k + 1] = t.z; mgx[2 * k + 1] = t.w;
                }
            }
        }
        if (on) {
            // two register batches: batch b + 1's loads are issued before batch b is used, so a
            // wave keeps a batch in flight while it computes (one batch at a time held the
            // passes at 2.9-4.8 TB/s, the waves idle between their batches)
            uint4 xr[2][U], gr[2][U], hr[2][U];
            auto load = [&](int b, int r) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const long p = pb + min(r + u * L.RP, r1 - 1);
                    xr[b][u] = *(const uint4*)(x + p * ldx + xoff + c);
                    if (MODE != 0 && (MODE != 4 || dy)) gr[b][u] = *(const uint4*)(dy + p * lddy + dyoff + c);
                }
                if (MODE != 0 && dy2) {
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const long p = pb + min(r + u * L.RP, r1 - 1);
                        hr[b][u] = *(const uint4*)(dy2 + p * lddy2 + dy2off + c);
                    }
                }
            };
            auto process = [&](int b, int r) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    if (r + u * L.RP >= r1) break;
                    float xv[8];
                    bf8f(xr[b][u], xv);
                    if (MODE == 0) {
#pragma unroll
                        for (int k = 0; k < 8; ++k) { a0[k] += xv[k]; a1[k] += xv[k] * xv[k]; }
                        continue;
                    }
                    float gv[8];
                    if (MODE != 4 || dy) bf8f(gr[b][u], gv);
                    if (dy2) {
                        float hv[8];
                        bf8f(hr[b][u], hv);
#pragma unroll
                        for (int k = 0; k < 8; ++k) gv[k] += hv[k];
                    }
                    float o[8];
                    if (MODE == 4) {   // forward apply (as apply_kernel, same float ops)
#pragma unroll
                        for (int k = 0; k < 8; ++k) {
                            float h = (xv[k] - mean[k]) * rstd[k];
                            if (act == IRGAN_ACT_RELU) h = h > 0.f ? h : 0.f;
                            else if (act == IRGAN_ACT_LRELU) h = h > 0.f ? h : 0.2f * h;
                            o[k] = dy ? h + gv[k] : h;
                        }
                    } else {
#pragma unroll
                        for (int k = 0; k < 8; ++k) {
                            const float xh = (xv[k] - mean[k]) * rstd[k];
                            const float g = gv[k] * act_grad(xh, act);
                            if (MODE == 1) { a0[k] += g; a1[k] += g * xh; }
                            else o[k] = rstd[k] * (g - mg[k] - xh * mgx[k]);
                        }
                    }
                    if (MODE == 2 || MODE == 4) {
                        uint4 w;
                        w.x = pk_bf16(o[0], o[1]);
                        w.y = pk_bf16(o[2], o[3]);
                        w.z = pk_bf16(o[4], o[5]);
                        w.w = pk_bf16(o[6], o[7]);
                        *(uint4*)(dx + (pb + r + u * L.RP) * lddx + dxoff + c) = w;
                        if constexpr (F8) {
                            float vb[8];
                            bf8f(w, vb);
#pragma unroll
                            for (int k = 0; k < 8; ++k) amx = fmaxf(amx, fabsf(vb[k]));
                            *(uint2*)(q8.p + (pb + r + u * L.RP) * q8.ld + q8.off + c) = pack8_fp8(vb, qs);
                        }
                    }
                }
            };
            const int step = U * L.RP;
            int r = r0 + L.rl;
#if ROWS8_DB
            if (r < r1) load(0, r);
#pragma unroll 1
            for (; r < r1; r += 2 * step) {
                if (r + step < r1) load(1, r + step);
                process(0, r);
                if (r + step >= r1) break;
                if (r + 2 * step < r1) load(0, r + 2 * step);
                process(1, r + step);
            }
#else
#pragma unroll 1
            for (; r < r1; r += step) {
                load(0, r);
                process(0, r);
            }
#endif
        }
        if (MODE == 2 || MODE == 4) continue;  // uniform across the block
        block_partials8(a0, a1, L, on, cb, c, C, n, s0, s1, part);
    }
    if constexpr (F8) fp8_block_amax(amx, q8.amax, blockIdx.y * gridDim.x + blockIdx.x);
}

// Rows per thread and rows per load batch (U) of each pass, by key: 0 stats, 1 backward
// reduce, 2 backward apply, 4 forward apply, 5 forward apply + residual / with the fp8 copy.
// Measured at the resblock shape, B = 16 (profiles/r05_nsw_norm_sweep.txt, tools/norm_sweep.sh
// with IRGAN_IN_RPT_M<key> / IRGAN_IN_U_M<key>): forward apply 16.2 -> 14.4 us and backward
// apply 17.9 -> 17.5 at 4 rows per thread in one batch; the reduce stays at 16 rows in batches
// of 4 (one batch of 4: 20.7 us, 4x the partials), apply + residual at 8 rows in batches of 4
constexpr int PASS_RPT[6] = {16, 16, 4, 0, 4, 8}, PASS_U[6] = {16, 4, 4, 0, 4, 4};  // U: the batch cap (larger maps: several batches)
int pass_env(const char* what, int key, int dflt) {
    char k[32];
    snprintf(k, sizeof(k), "IRGAN_IN_%s_M%d", what, key);
    const char* v = getenv(k);
    return v && atoi(v) > 0 ? atoi(v) : dflt;
}
int pass_rpt(int key, int dflt) {
    static int cache[6] = {0, 0, 0, 0, 0, 0};
    if (!cache[key]) cache[key] = pass_env("RPT", key, dflt);
    return cache[key];
}
int pass_u(int key) {
    static int cache[6] = {0, 0, 0, 0, 0, 0};
    if (!cache[key]) cache[key] = pass_env("U", key, PASS_U[key]);
    return cache[key];
}

// rows8_kernel with U = min(the thread's rows, the pass's batch), from the instances 2 / 4 / 8 / 16
template <int MODE, bool F8 = false, typename... A>
void rows8_go(int key, int rows_per_thread, dim3 g, hipStream_t st, A... args) {
    const int u = std::min(pass_u(key), rows_per_thread);
    if (u <= 2) rows8_kernel<MODE, 2, F8><<<g, TPB, 0, st>>>(args...);
    else if (u <= 4) rows8_kernel<MODE, 4, F8><<<g, TPB, 0, st>>>(args...);
    else if (u <= 8) rows8_kernel<MODE, 8, F8><<<g, TPB, 0, st>>>(args...);
    else rows8_kernel<MODE, 16, F8><<<g, TPB, 0, st>>>(args...);
}

// fp64 sum of the nb block partials of each (n, c).  Block (FC channels x FS
// partial lanes) per (image, channel group): a lane adds partials sub, sub + FS,
// ... (at most nb / FS dependent loads: the launch is latency-bound, so the
// partial lanes are many and the channel groups narrow), then the FS lanes of a
// channel combine through LDS in a fixed order (deterministic).
constexpr int FC = 8, FS = 32;
__global__ __launch_bounds__(256) void finalize_kernel(const float2* __restrict__ part, float* __restrict__ mr, int N,
                                                       int C, int nb, int HW, int mode) {
    __shared__ double s0[FS][FC], s1[FS][FC];
    const int n = blockIdx.y, cl = threadIdx.x % FC, sub = threadIdx.x / FC;
    const int c = blockIdx.x * FC + cl;
    double s = 0.0, q = 0.0;
    if (c < C) {
        for (int b = sub; b < nb; b += FS) {
            const float2 v = part[((long)n * nb + b) * C + c];
            s += v.x;
            q += v.y;
        }
    }
    s0[sub][cl] = s;
    s1[sub][cl] = q;
    __syncthreads();
    if (sub != 0 || c >= C) return;
    s = 0.0;
    q = 0.0;
    for (int k = 0; k < FS; ++k) {
        s += s0[k][cl];
        q += s1[k][cl];
    }
    const long i = (long)n * C + c;
    const double mean = s / HW;
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

template <int VW, bool F8 = false>
__global__ __launch_bounds__(TPB) void apply_kernel(Slice X, int HW, int C, const float* __restrict__ mr, int act,
                                                    Slice R, void* __restrict__ y, int ldy, int yoff,
                                                    void* __restrict__ xhat, long total, Q8 q8 = Q8{}) {
    const int CV = C / VW;
    const float qs = F8 ? *q8.q : 1.f;
    float amx = 0.f;
    for (long idx = blockIdx.x * (long)TPB + threadIdx.x; idx < total; idx += (long)gridDim.x * TPB) {
        const long p = idx / CV;
        const int c = (int)(idx - p * CV) * VW;
        const int n = (int)(p / HW);
        float v[VW];
        ldv_<VW>(X.p, X.dt, p * X.ld + X.off + c, v);
        const float4* m4 = (const float4*)(mr + 2 * ((long)n * C + c));
#pragma unroll
        for (int k = 0; k < VW; k += 2) {
            float4 st;
            if constexpr (VW == 8) st = m4[k / 2];
            else { st = make_float4(mr[2 * ((long)n * C + c)], mr[2 * ((long)n * C + c) + 1], 0.f, 0.f); }
            v[k] = (v[k] - st.x) * st.y;
            if (VW > 1) v[k + 1] = (v[k + 1] - st.z) * st.w;
        }
        if (xhat) stv_<VW>(xhat, X.dt, p * C + c, v);
#pragma unroll
        for (int k = 0; k < VW; ++k) {
            if (act == IRGAN_ACT_RELU) v[k] = v[k] > 0.f ? v[k] : 0.f;
            else if (act == IRGAN_ACT_LRELU) v[k] = v[k] > 0.f ? v[k] : 0.2f * v[k];
        }
        if (R.p) {
            float rv[VW];
            ldv_<VW>(R.p, R.dt, p * R.ld + R.off + c, rv);
#pragma unroll
            for (int k = 0; k < VW; ++k) v[k] += rv[k];
        }
        stv_<VW>(y, X.dt, p * ldy + yoff + c, v);
        if constexpr (F8) {  // bf16 output, VW == 8
            float vb[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                vb[k] = bf2f(f2bf(v[k]));
                amx = fmaxf(amx, fabsf(vb[k]));
            }
            *(uint2*)(q8.p + p * q8.ld + q8.off + c) = pack8_fp8(vb, qs);
        }
    }
    if constexpr (F8) fp8_block_amax(amx, q8.amax, blockIdx.x);
}


bool vec_ok(int C, std::initializer_list<int> lds) {
    if (C % V) return false;
    for (int l : lds)
        if (l % V) return false;
    return true;
}

int rp_of(int C, int VW) {
    int cl = (C + VW - 1) / VW;
    if (cl > TPB) cl = TPB;
    return TPB / cl;
}

// blocks per image: ~4096 blocks over the grid, >= rpt rows per thread, <= IN_PARTS.
// rpt 16 for the reductions (stats, backward reduce: half the partials for the finalize)
// and the plain forward apply, 8 for the three-stream passes (backward apply, apply +
// residual) -- measured per pass at the resblock shape (tools/norm_sweep.sh, r03_e:
// backward reduce + finalize 20.6 -> 17.2 us, apply + ReLU 17.4 -> 16.5, apply + residual
// 18.1 -> 18.8, backward apply 18.4 -> 18.6; U = 2 / a 128-VGPR cap on the reduce: no gain)
int blocks_per_image(long HW, int N, int RP, long rpt = 8) {
    long nb = (4096 + N - 1) / (N > 0 ? N : 1);
    const long maxnb = (HW + rpt * RP - 1) / (rpt * RP);
    if (nb > maxnb) nb = maxnb;
    if (nb > IN_PARTS) nb = IN_PARTS;
    if (nb < 1) nb = 1;
    return (int)nb;
}

template <int MODE>
int launch_rows(Slice X, Slice DY, Slice DY2, int act, const float* mr, const float* red, void* dx, int dxdt, int lddx,
                int dxoff, int N, int HW, int C, float2* part, float* db, bool vec, hipStream_t st, int* nb_out,
                const Q8* q8 = nullptr) {
    const int VW = vec ? V : 1;
    const int rpt = pass_rpt(MODE, PASS_RPT[MODE]);
    const int RP = rp_of(C, VW);
    int nb = blocks_per_image(HW, N, RP, rpt);
    const int rows = irgan_cdiv(HW, nb);
    nb = irgan_cdiv(HW, rows);
    const int rpth = irgan_cdiv(rows, RP);
    dim3 g(nb, N);
    static const bool fast = !getenv("IRGAN_NO_ROWS8");
    const bool bf = X.dt == IRGAN_BF16 && (MODE == 0 || (DY.dt == IRGAN_BF16 && (!DY2.p || DY2.dt == IRGAN_BF16))) &&
                    (MODE != 2 || (dxdt == IRGAN_BF16 && !db));
    if (q8 && !(vec && bf && MODE == 2)) return IRGAN_EUNSUPPORTED;
    if ((fast || q8) && vec && bf && MODE <= 2) {
        const bf16_t *xp = (const bf16_t*)X.p, *gp = (const bf16_t*)DY.p, *hp = (const bf16_t*)DY2.p;
        if (MODE == 2 && q8)
            rows8_go<2, true>(2, rpth, g, st, xp, X.ld, X.off, gp, DY.ld, DY.off, hp, DY2.ld, DY2.off, act, mr, red,
                              (bf16_t*)dx, lddx, dxoff, HW, C, rows, part, *q8);
        else if (MODE == 0)
            rows8_go<0>(0, rpth, g, st, xp, X.ld, X.off, (const bf16_t*)nullptr, 0, 0, (const bf16_t*)nullptr, 0, 0, act, mr,
                        red, (bf16_t*)nullptr, 0, 0, HW, C, rows, part, Q8{});
        else
            rows8_go<MODE>(MODE, rpth, g, st, xp, X.ld, X.off, gp, DY.ld, DY.off, hp, DY2.ld, DY2.off, act, mr, red,
                           (bf16_t*)dx, lddx, dxoff, HW, C, rows, part, Q8{});
        if (nb_out) *nb_out = nb;
        return 0;
    }
    if (vec)
        rows_kernel<MODE, V><<<g, TPB, 0, st>>>(X, DY, DY2, act, mr, red, dx, dxdt, lddx, dxoff, HW, C, rows, part, db);
    else
        rows_kernel<MODE, 1><<<g, TPB, 0, st>>>(X, DY, DY2, act, mr, red, dx, dxdt, lddx, dxoff, HW, C, rows, part, db);
    if (nb_out) *nb_out = nb;
    return 0;
}

}  // namespace

extern "C" int irgan_in_stats(const void* x, int32_t dtype, int32_t N, int32_t HW, int32_t C, int32_t ld,
                              int32_t off, double* work, float* mr, irgan_stream_t s) {
    hipStream_t st = (hipStream_t)s;
    if ((long)N * HW * C <= 0) return 0;
    Slice X{x, dtype, ld, off}, Z{nullptr, 0, 0, 0};
    int nb = 1;
    launch_rows<0>(X, Z, Z, 0, nullptr, nullptr, nullptr, 0, 0, 0, N, HW, C, (float2*)work, nullptr,
                   vec_ok(C, {ld, off}), st, &nb);
    finalize_kernel<<<dim3(irgan_cdiv(C, FC), N), 256, 0, st>>>((const float2*)work, mr, N, C, nb, HW, 0);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_in_finalize(const void* part, int32_t N, int32_t HW, int32_t C, int32_t nb, float* mr,
                                 irgan_stream_t s) {
    if ((long)N * HW * C <= 0) return 0;
    if (!part || !mr || nb < 1 || nb > IRGAN_IN_PARTS) return IRGAN_EINVAL;
    finalize_kernel<<<dim3(irgan_cdiv(C, FC), N), 256, 0, (hipStream_t)s>>>((const float2*)part, mr, N, C, nb, HW, 0);
    IRGAN_LAUNCH_CHECK();
    return 0;
}



// the forward apply as rows8_kernel<4> (bf16, 8-channel vectors, no xhat), grid as the
// other row passes; q8: also the fp8 copy of y (irgan_in_apply_fp8)
bool apply_rows(const void* x, int ldx, int xoff, int N, int HW, int C, const float* mr, int act, const void* res,
                int ldr, int roff, void* y, int ldy, int yoff, hipStream_t st, const Q8* q8 = nullptr) {
    static const bool off = getenv("IRGAN_NO_APPLY_ROWS") != nullptr;
    if (off) return false;
    const int key = res || q8 ? 5 : 4;  // 5: apply + residual, or with the fp8 copy
    const int rpt = pass_rpt(key, PASS_RPT[key]);
    const int RP = rp_of(C, 8);
    int nb = blocks_per_image(HW, N, RP, rpt);
    const int rows = irgan_cdiv(HW, nb);
    nb = irgan_cdiv(HW, rows);
    const int rpth = irgan_cdiv(rows, RP);
    dim3 g(nb, N);
    const bf16_t *xp = (const bf16_t*)x, *rp = (const bf16_t*)res;
    if (q8)
        rows8_go<4, true>(key, rpth, g, st, xp, ldx, xoff, rp, ldr, roff, (const bf16_t*)nullptr, 0, 0, act, mr,
                          (const float*)nullptr, (bf16_t*)y, ldy, yoff, HW, C, rows, (float2*)nullptr, *q8);
    else
        rows8_go<4>(key, rpth, g, st, xp, ldx, xoff, rp, ldr, roff, (const bf16_t*)nullptr, 0, 0, act, mr,
                    (const float*)nullptr, (bf16_t*)y, ldy, yoff, HW, C, rows, (float2*)nullptr, Q8{});
    return true;
}

extern "C" int irgan_in_apply(const void* x, int32_t dtype, int32_t N, int32_t HW, int32_t C, int32_t ldx,
                              int32_t xoff, const float* mr, int32_t act, const void* res, int32_t ldr, int32_t roff,
                              void* y, int32_t ldy, int32_t yoff, void* xhat, irgan_stream_t s) {
    const bool vec = vec_ok(C, {ldx, xoff, ldy, yoff}) && (!res || vec_ok(C, {ldr, roff}));
    if (vec && dtype == IRGAN_BF16 && !xhat && (long)N * HW * C > 0 &&
        apply_rows(x, ldx, xoff, N, HW, C, mr, act, res, ldr, roff, y, ldy, yoff, (hipStream_t)s)) {
        IRGAN_LAUNCH_CHECK();
        return 0;
    }
    const int VW = vec ? V : 1;
    long total = (long)N * HW * (C / VW);
    if (total <= 0) return 0;
    int blocks = (int)std::min<long>((total + TPB - 1) / TPB, 16384);
    Slice X{x, dtype, ldx, xoff}, R{res, dtype, ldr, roff};
    if (vec)
        apply_kernel<V><<<blocks, TPB, 0, (hipStream_t)s>>>(X, HW, C, mr, act, R, y, ldy, yoff, xhat, total);
    else
        apply_kernel<1><<<blocks, TPB, 0, (hipStream_t)s>>>(X, HW, C, mr, act, R, y, ldy, yoff, xhat, total);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_in_bwd_reduce(const void* dy, int32_t dy_dtype, int32_t lddy, int32_t dyoff, const void* dy2,
                                   int32_t dy2_dtype, int32_t lddy2, int32_t dy2off, const void* x, int32_t x_dtype,
                                   int32_t ldx, int32_t xoff, int32_t act, int32_t N, int32_t HW, int32_t C,
                                   const float* mr, double* work, float* red, irgan_stream_t s) {
    hipStream_t st = (hipStream_t)s;
    if ((long)N * HW * C <= 0) return 0;
    const bool vec = vec_ok(C, {lddy, dyoff, ldx, xoff}) && (!dy2 || vec_ok(C, {lddy2, dy2off}));
    Slice X{x, x_dtype, ldx, xoff}, DY{dy, dy_dtype, lddy, dyoff}, DY2{dy2, dy2_dtype, lddy2, dy2off};
    int nb = 1;
    launch_rows<1>(X, DY, DY2, act, mr, nullptr, nullptr, 0, 0, 0, N, HW, C, (float2*)work, nullptr, vec, st, &nb);
    finalize_kernel<<<dim3(irgan_cdiv(C, FC), N), 256, 0, st>>>((const float2*)work, red, N, C, nb, HW, 1);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_in_bwd_apply(const void* dy, int32_t dy_dtype, int32_t lddy, int32_t dyoff, const void* dy2,
                                  int32_t dy2_dtype, int32_t lddy2, int32_t dy2off, const void* x, int32_t x_dtype,
                                  int32_t ldx, int32_t xoff, int32_t act, int32_t N, int32_t HW, int32_t C,
                                  const float* mr, const float* red, void* dx, int32_t dx_dtype, int32_t lddx,
                                  int32_t dxoff, float* db, irgan_stream_t s) {
    const bool vec = vec_ok(C, {lddy, dyoff, ldx, xoff, lddx, dxoff}) && (!dy2 || vec_ok(C, {lddy2, dy2off}));
    Slice X{x, x_dtype, ldx, xoff}, DY{dy, dy_dtype, lddy, dyoff}, DY2{dy2, dy2_dtype, lddy2, dy2off};
    launch_rows<2>(X, DY, DY2, act, mr, red, dx, dx_dtype, lddx, dxoff, N, HW, C, nullptr, db, vec, (hipStream_t)s,
                   nullptr);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

// db[c] += sum of the nb partials' .x: FC channels x FS partial lanes per block (lane k adds
// partials k, k + FS, ...), then the FS lanes of a channel in order (deterministic)
static __global__ __launch_bounds__(256) void colsum_finalize_kernel(const float2* __restrict__ part, float* __restrict__ db,
                                                              int nb, int C) {
    __shared__ double sp[FS][FC];
    const int cl = threadIdx.x % FC, sub = threadIdx.x / FC, c = blockIdx.x * FC + cl;
    double t = 0.0;
    if (c < C)
        for (int b = sub; b < nb; b += FS) t += part[(long)b * C + c].x;
    sp[sub][cl] = t;
    __syncthreads();
    if (sub != 0 || c >= C) return;
    t = 0.0;
    for (int k = 0; k < FS; ++k) t += sp[k][cl];
    db[c] += (float)t;
}

// Bias gradient (sum over the P rows of each channel).  The rows are split into S <= 16
// equal segments run as S "images" of launch_rows (S x <= IN_PARTS block partials: with one
// image a single row of <= IN_PARTS blocks streamed the D input layer's 67 MB gradient at
// ~1.6 TB/s), then summed in a fixed order (no atomics).  work: 16 * IN_PARTS * C doubles.
extern "C" int irgan_channel_sum(const void* g, int32_t dtype, int32_t P, int32_t C, int32_t ld, int32_t off,
                                 float* db, double* work, irgan_stream_t s) {
    if (P <= 0) return 0;
    hipStream_t st = (hipStream_t)s;
    Slice X{g, dtype, ld, off}, Z{nullptr, 0, 0, 0};
    int S = 16;
    while (S > 1 && (P % S || P / S < 4096)) S >>= 1;
    int nb = 1;
    launch_rows<0>(X, Z, Z, 0, nullptr, nullptr, nullptr, 0, 0, 0, S, P / S, C, (float2*)work, nullptr,
                   vec_ok(C, {ld, off}), st, &nb);
    colsum_finalize_kernel<<<irgan_cdiv(C, FC), 256, 0, st>>>((const float2*)work, db, S * nb, C);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

// irgan_in_apply / irgan_in_bwd_apply that also write the fp8 copy of their bf16
// output (Q8 above): the producers of the fp8 path's ResnetBlock conv operands.
extern "C" int irgan_in_apply_fp8(const void* x, int32_t N, int32_t HW, int32_t C, int32_t ldx, int32_t xoff,
                                  const float* mr, int32_t act, const void* res, int32_t ldr, int32_t roff, void* y,
                                  int32_t ldy, int32_t yoff, void* y8, int32_t ld8, int32_t off8, const float* q,
                                  uint32_t* amax, irgan_stream_t s) {
    if (!x || !mr || !y || !y8 || !q || !amax) return IRGAN_EINVAL;
    if (!vec_ok(C, {ldx, xoff, ldy, yoff, ld8, off8}) || (res && !vec_ok(C, {ldr, roff}))) return IRGAN_EUNSUPPORTED;
    const long total = (long)N * HW * (C / V);
    if (total <= 0) return 0;
    const Q8 q8v{(uint8_t*)y8, ld8, off8, q, amax};
    if (apply_rows(x, ldx, xoff, N, HW, C, mr, act, res, ldr, roff, y, ldy, yoff, (hipStream_t)s, &q8v)) {
        IRGAN_LAUNCH_CHECK();
        return 0;
    }
    const int blocks = (int)std::min<long>((total + TPB - 1) / TPB, 16384);
    Slice X{x, IRGAN_BF16, ldx, xoff}, R{res, IRGAN_BF16, ldr, roff};
    apply_kernel<V, true><<<blocks, TPB, 0, (hipStream_t)s>>>(X, HW, C, mr, act, R, y, ldy, yoff, nullptr, total,
                                                               q8v);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_in_bwd_apply_fp8(const void* dy, int32_t lddy, int32_t dyoff, const void* dy2, int32_t lddy2,
                                      int32_t dy2off, const void* x, int32_t ldx, int32_t xoff, int32_t act, int32_t N,
                                      int32_t HW, int32_t C, const float* mr, const float* red, void* dx, int32_t lddx,
                                      int32_t dxoff, void* y8, int32_t ld8, int32_t off8, const float* q,
                                      uint32_t* amax, irgan_stream_t s) {
    if (!dy || !x || !mr || !red || !dx || !y8 || !q || !amax) return IRGAN_EINVAL;
    if ((long)N * HW * C <= 0) return 0;
    const bool vec = vec_ok(C, {lddy, dyoff, ldx, xoff, lddx, dxoff, ld8, off8}) && (!dy2 || vec_ok(C, {lddy2, dy2off}));
    if (!vec) return IRGAN_EUNSUPPORTED;
    Slice X{x, IRGAN_BF16, ldx, xoff}, DY{dy, IRGAN_BF16, lddy, dyoff}, DY2{dy2, IRGAN_BF16, lddy2, dy2off};
    const Q8 q8{(uint8_t*)y8, ld8, off8, q, amax};
    const int rc = launch_rows<2>(X, DY, DY2, act, mr, red, dx, IRGAN_BF16, lddx, dxoff, N, HW, C, nullptr, nullptr,
                                  true, (hipStream_t)s, nullptr, &q8);
    if (rc) return rc;
    IRGAN_LAUNCH_CHECK();
    return 0;
}
