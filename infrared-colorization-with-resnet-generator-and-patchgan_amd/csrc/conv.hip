// Implicit-GEMM convolutions for gfx950 (CDNA4): forward / backward-data (one
// kernel, re-packed weights) and backward-weight (split-K over pixels).
//
// Replaces the ATen convolution / convolution_backward / reflection_pad2d /
// cat work of the reference hot path (ir:390-411, 458-531, 595-630, vgg 664).
//
// Tiling: 256 threads = 4 waves (2x2).  A K-tile row is 128 bytes (64 bf16 or
// 32 fp32) stored in LDS with a 16-byte-chunk XOR swizzle (chunk ^ (row & 7)),
// which makes the ds_read_b128 fragment reads conflict-free.  Each lane reads
// one 16 B chunk per 64 B half-row: for bf16 that is exactly the
// v_mfma_f32_16x16x32_bf16 operand (k = 8*(lane>>4) + j); for fp32 the four
// words feed four v_mfma_f32_16x16x4_f32 with k = 4*(lane>>4) + s, the same
// permutation on both operands, so the K sum is complete (exact fp32 FMA chain).
#include "common.h"
#include <stdlib.h>

extern "C" int irgan_conv_fwd_glds(const irgan_conv_desc* d, const void* x, const void* w, const float* bias, void* y,
                                   const void* mask, hipStream_t st);
extern "C" int irgan_conv_fwd_glds_split(const irgan_conv_desc* d, const void* x, const void* w, const float* bias,
                                         void* y, const void* mask, int ksplit, long sstride, hipStream_t st);
extern "C" int irgan_conv_fwd_pp(const irgan_conv_desc* d, const void* x, const void* w, const float* bias, void* y,
                                 const void* mask, hipStream_t st);
extern "C" int irgan_conv_fwd_halo(const irgan_conv_desc* d, const void* x, const void* w, const float* bias, void* y,
                                   const void* mask, hipStream_t st);
extern "C" int irgan_conv_fwd_c8(const irgan_conv_desc* d, const void* x, const void* w, const float* bias, void* y,
                                 const void* mask, hipStream_t st);
extern "C" int irgan_conv_wgrad_halo(const irgan_conv_desc* d, const void* x, const void* dy, float* dw, int splitk,
                                     float* ws, long ws_cap, hipStream_t st);
extern "C" int irgan_conv_wgrad_rowspan(const irgan_conv_desc* d, const void* x, const void* dy, float* dw, float* ws,
                                        long ws_cap, hipStream_t st);
extern "C" int irgan_conv_wgrad_pc(const irgan_conv_desc* d, const void* x, const void* dy, float* dw, int splitk,
                                   float* ws, long ws_cap, hipStream_t st);
extern "C" int irgan_conv_wgrad_narrow(const irgan_conv_desc* d, const void* x, const void* dy, float* dw, float* ws,
                                       long ws_cap, hipStream_t st);
extern "C" int irgan_conv_wgrad_glds(const irgan_conv_desc* d, const void* x, const void* dy, float* dw, int splitk,
                                     hipStream_t st, float* ws, long ws_cap);

namespace {

constexpr int ROWB = 128;  // bytes per LDS tile row (one K-tile)

template <typename T> struct TT;
template <> struct TT<float>  { static constexpr int EPC = 4; };
template <> struct TT<bf16_t> { static constexpr int EPC = 8; };

IRGAN_HD int lds_off(int row, int chunk) { return row * ROWB + ((chunk ^ (row & 7)) << 4); }

IRGAN_HD void mma16(f32x4& acc, const uint4& a, const uint4& b, const float*) {
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), __uint_as_float(b.x), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), __uint_as_float(b.y), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), __uint_as_float(b.z), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), __uint_as_float(b.w), acc, 0, 0, 0);
}
IRGAN_HD void mma16(f32x4& acc, const uint4& a, const uint4& b, const bf16_t*) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                  __builtin_bit_cast(bf16x8_t, b), acc, 0, 0, 0);
}

IRGAN_HD float apply_act(float v, int act) {
    if (act == IRGAN_ACT_RELU) return v > 0.f ? v : 0.f;
    if (act == IRGAN_ACT_LRELU) return v > 0.f ? v : 0.2f * v;
    if (act == IRGAN_ACT_TANH) return tanhf(v);
    return v;
}

// map an input coordinate; returns false when it falls in the zero padding
IRGAN_HD bool map_q(int& qy, int& qx, int H, int W, int mode) {
    if (mode == IRGAN_PAD_REFLECT) {
        qy = reflect_idx(qy, H);
        qx = reflect_idx(qx, W);
        return true;
    }
    return qy >= 0 && qy < H && qx >= 0 && qx < W;
}

// ---------------------------------------------------------------------------
// forward / backward-data:  Y[m][co] = sum_k A[m][k] * W[co][k]
//   m = (n, i, j) launch position, k = (ty, tx, ci)
// ---------------------------------------------------------------------------
template <typename T, int BN, bool FAST>
__global__ __launch_bounds__(256) void conv_fwd_kernel(const irgan_conv_desc d, const T* __restrict__ x,
                                                       const T* __restrict__ w, const float* __restrict__ bias,
                                                       void* __restrict__ y, const void* __restrict__ mask) {
    constexpr int BM = 128, EPC = TT<T>::EPC, BKE = ROWB / (int)sizeof(T);
    constexpr int MI = 4, NJ = BN / 32, BR = BN / 32;
    __shared__ __attribute__((aligned(16))) char smem[2 * (BM + BN) * ROWB];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    const int HoWo = d.Ho * d.Wo;
    const long M = (long)d.N * HoWo;
    const int K = d.KH * d.KW * d.Cin;
    const long m0 = (long)blockIdx.x * BM;
    const int n0 = blockIdx.y * BN;
    const int lc = tid & 7, lr = tid >> 3;

    int a_nb[4], a_iy[4], a_ix[4];
    bool a_ok[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        long m = m0 + lr + 32 * u;
        a_ok[u] = m < M;
        int mm = a_ok[u] ? (int)m : 0;
        int n = mm / HoWo, r = mm - n * HoWo, i = r / d.Wo, j = r - i * d.Wo;
        a_nb[u] = n * d.H;
        a_iy[u] = i * d.sy + d.c0y;
        a_ix[u] = j * d.sx + d.c0x;
    }

    uint4 ra[4], rb[BR];
    const uint4 z4 = make_uint4(0, 0, 0, 0);

    auto load_tile = [&](int kt) {
        const int k0 = kt * BKE;
        if constexpr (FAST) {
            const int tap = k0 / d.Cin, cin0 = k0 - tap * d.Cin;
            const int ty = tap / d.KW, tx = tap - ty * d.KW;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                int qy = a_iy[u] + ty, qx = a_ix[u] + tx;
                bool v = map_q(qy, qx, d.H, d.W, d.pad_mode) && a_ok[u];
                ra[u] = v ? *(const uint4*)(x + ((long)(a_nb[u] + qy) * d.W + qx) * d.ldx + d.xoff + cin0 + lc * EPC)
                          : z4;
            }
#pragma unroll
            for (int u = 0; u < BR; ++u) {
                int co = n0 + lr + 32 * u;
                rb[u] = co < d.Cout ? *(const uint4*)(w + (long)co * K + k0 + lc * EPC) : z4;
            }
        } else {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                T tmp[EPC];
#pragma unroll
                for (int e = 0; e < EPC; ++e) {
                    int k = k0 + lc * EPC + e;
                    T val = from_f<T>(0.f);
                    if (a_ok[u] && k < K) {
                        int tap = k / d.Cin, ci = k - tap * d.Cin;
                        int ty = tap / d.KW, tx = tap - ty * d.KW;
                        int qy = a_iy[u] + ty, qx = a_ix[u] + tx;
                        if (map_q(qy, qx, d.H, d.W, d.pad_mode))
                            val = x[((long)(a_nb[u] + qy) * d.W + qx) * d.ldx + d.xoff + ci];
                    }
                    tmp[e] = val;
                }
                __builtin_memcpy(&ra[u], tmp, 16);
            }
#pragma unroll
            for (int u = 0; u < BR; ++u) {
                int co = n0 + lr + 32 * u;
                T tmp[EPC];
#pragma unroll
                for (int e = 0; e < EPC; ++e) {
                    int k = k0 + lc * EPC + e;
                    tmp[e] = (co < d.Cout && k < K) ? w[(long)co * K + k] : from_f<T>(0.f);
                }
                __builtin_memcpy(&rb[u], tmp, 16);
            }
        }
    };
    auto store_tile = [&](int buf) {
        char* A = smem + buf * (BM + BN) * ROWB;
        char* B = A + BM * ROWB;
#pragma unroll
        for (int u = 0; u < 4; ++u) *(uint4*)(A + lds_off(lr + 32 * u, lc)) = ra[u];
#pragma unroll
        for (int u = 0; u < BR; ++u) *(uint4*)(B + lds_off(lr + 32 * u, lc)) = rb[u];
    };

    f32x4 acc[MI][NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = (K + BKE - 1) / BKE;
    load_tile(0);
    store_tile(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nk) load_tile(kt + 1);
        const char* A = smem + cur * (BM + BN) * ROWB;
        const char* B = A + BM * ROWB;
        // fp32 parity mode: blocked summation (one fresh partial per K-tile) keeps the
        // fp32 error at O(32 + K/32) ulps instead of a K-long FMA chain
        f32x4 part[MI][NJ];
        constexpr bool BLOCKED = sizeof(T) == 4;
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) part[i][j] = BLOCKED ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[i][j];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            uint4 af[MI], bfr[NJ];
            const int ch = h * 4 + (lane >> 4);
#pragma unroll
            for (int i = 0; i < MI; ++i) af[i] = *(const uint4*)(A + lds_off(wm * 64 + i * 16 + (lane & 15), ch));
#pragma unroll
            for (int j = 0; j < NJ; ++j) bfr[j] = *(const uint4*)(B + lds_off(wn * (BN / 2) + j * 16 + (lane & 15), ch));
#pragma unroll
            for (int i = 0; i < MI; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j) mma16(part[i][j], af[i], bfr[j], (const T*)nullptr);
        }
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) acc[i][j] = BLOCKED ? acc[i][j] + part[i][j] : part[i][j];
        if (kt + 1 < nk) store_tile(cur ^ 1);
        __syncthreads();
    }

    // epilogue: C[row = (lane>>4)*4 + r][col = lane & 15] of each 16x16 fragment
#pragma unroll
    for (int i = 0; i < MI; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const long m = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
            if (m >= M) continue;
            const int mm = (int)m;
            const int n = mm / HoWo, rr = mm - n * HoWo, ii = rr / d.Wo, jj = rr - ii * d.Wo;
            const long pix = ((long)n * d.OH + ii * d.omy + d.ooy) * d.OW + jj * d.omx + d.oox;
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int co = n0 + wn * (BN / 2) + j * 16 + (lane & 15);
                if (co >= d.Cout) continue;
                float v = acc[i][j][r] + (bias ? bias[co] : 0.f);
                v = apply_act(v, d.act);
                if (mask) {
                    float mv = ldv(mask, d.dtype, pix * d.ldm + d.moff + co);
                    v *= mv > 0.f ? 1.f : (d.mask_act == 2 ? 0.2f : 0.f);
                }
                const long off = pix * d.ldy + d.yoff + co;
                if (d.out_dtype == IRGAN_F32) {
                    float* yp = (float*)y;
                    yp[off] = d.accumulate ? yp[off] + v : v;
                } else {
                    bf16_t* yp = (bf16_t*)y;
                    yp[off] = f2bf(d.accumulate ? bf2f(yp[off]) + v : v);
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// backward-weight:  dW[co][col] += sum_p dY[p][co] * im2col(X)[p][col]
//   rows = co (BM), cols = (ty, tx, ci) (BN = 64), K = pixels (split over z)
// Both operands arrive pixel-major from HBM; they are transposed into the
// k-contiguous LDS image on the store (pixel pairs packed per LDS write).
// ---------------------------------------------------------------------------
template <typename T, int BM, bool FASTA, bool FASTB>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(const irgan_conv_desc d, const T* __restrict__ x,
                                                         const T* __restrict__ dy, float* __restrict__ dw,
                                                         int kchunk) {
    constexpr int BN = 64, EPC = TT<T>::EPC, BKP = ROWB / (int)sizeof(T);
    constexpr int MI = BM / 32, NJ = 2;
    constexpr int ACH = BM / EPC, BCH = BN / EPC, NPP = BKP / 2;  // chunks per pixel, pixel pairs
    constexpr int IA = ACH * NPP / 256, IB = BCH * NPP / 256;
    static_assert(IA >= 1 && IB >= 1, "tile too small");
    __shared__ __attribute__((aligned(16))) char smem[2 * (BM + BN) * ROWB];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    const int HoWo = d.Ho * d.Wo;
    const long P = (long)d.N * HoWo;
    const int K = d.KH * d.KW * d.Cin;
    const int co0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
    const long pb = (long)blockIdx.z * kchunk;
    const long pe = min(P, pb + kchunk);
    if (pb >= pe) return;

    // FASTB: whole tile inside one tap
    const int tapB = n0 / d.Cin, cinB = n0 - tapB * d.Cin;
    const int tyB = tapB / d.KW, txB = tapB - tyB * d.KW;

    // packed pixel pairs: bf16 -> one u32 (lo = p, hi = p+1); fp32 -> u64
    typedef typename std::conditional<sizeof(T) == 2, uint32_t, uint2>::type pair_t;
    pair_t pa[IA][EPC], pbv[IB][EPC];
    // generic B path: each thread covers 8 (col, pair) items; generic A: BM*NPP/256 items
    constexpr int GB = BN * NPP / 256;
    constexpr int GA = BM * NPP / 256;
    pair_t ga[FASTA ? 1 : GA], gb[FASTB ? 1 : GB];

    auto pix_in = [&](long p, int ty, int tx, long& off) -> bool {
        if (p >= pe) return false;
        int pp = (int)p;
        int n = pp / HoWo, r = pp - n * HoWo, i = r / d.Wo, j = r - i * d.Wo;
        int qy = i * d.sy + ty + d.c0y, qx = j * d.sx + tx + d.c0x;
        if (!map_q(qy, qx, d.H, d.W, d.pad_mode)) return false;
        off = ((long)n * d.H + qy) * d.W + qx;
        return true;
    };
    auto mkpair = [&](T lo, T hi) -> pair_t {
        if constexpr (sizeof(T) == 2) return (uint32_t)lo | ((uint32_t)hi << 16);
        else return make_uint2(__float_as_uint(lo), __float_as_uint(hi));
    };

    auto load_tile = [&](long p0) {
        if constexpr (FASTA) {
#pragma unroll
            for (int u = 0; u < IA; ++u) {
                int it = tid + 256 * u, cc = it % ACH, pp = it / ACH;
                long p = p0 + 2 * pp;
                int co = co0 + cc * EPC;
                uint4 c0 = make_uint4(0, 0, 0, 0), c1 = c0;
                if (co < d.Cout) {
                    if (p < pe) c0 = *(const uint4*)(dy + p * d.ldy + d.yoff + co);
                    if (p + 1 < pe) c1 = *(const uint4*)(dy + (p + 1) * d.ldy + d.yoff + co);
                }
                T e0[EPC], e1[EPC];
                __builtin_memcpy(e0, &c0, 16);
                __builtin_memcpy(e1, &c1, 16);
#pragma unroll
                for (int e = 0; e < EPC; ++e) pa[u][e] = mkpair(e0[e], e1[e]);
            }
        } else {
#pragma unroll
            for (int u = 0; u < GA; ++u) {
                int it = tid + 256 * u, row = it % BM, pp = it / BM;
                long p = p0 + 2 * pp;
                int co = co0 + row;
                T lo = from_f<T>(0.f), hi = from_f<T>(0.f);
                if (co < d.Cout) {
                    if (p < pe) lo = dy[p * d.ldy + d.yoff + co];
                    if (p + 1 < pe) hi = dy[(p + 1) * d.ldy + d.yoff + co];
                }
                ga[u] = mkpair(lo, hi);
            }
        }
        if constexpr (FASTB) {
#pragma unroll
            for (int u = 0; u < IB; ++u) {
                int it = tid + 256 * u, cc = it % BCH, pp = it / BCH;
                long p = p0 + 2 * pp, o0, o1;
                uint4 c0 = make_uint4(0, 0, 0, 0), c1 = c0;
                const long coff = d.xoff + cinB + cc * EPC;
                if (pix_in(p, tyB, txB, o0)) c0 = *(const uint4*)(x + o0 * d.ldx + coff);
                if (pix_in(p + 1, tyB, txB, o1)) c1 = *(const uint4*)(x + o1 * d.ldx + coff);
                T e0[EPC], e1[EPC];
                __builtin_memcpy(e0, &c0, 16);
                __builtin_memcpy(e1, &c1, 16);
#pragma unroll
                for (int e = 0; e < EPC; ++e) pbv[u][e] = mkpair(e0[e], e1[e]);
            }
        } else {
#pragma unroll
            for (int u = 0; u < GB; ++u) {
                int it = tid + 256 * u, col = it % BN, pp = it / BN;
                int kc = n0 + col;
                long p = p0 + 2 * pp, o;
                T lo = from_f<T>(0.f), hi = from_f<T>(0.f);
                if (kc < K) {
                    int tap = kc / d.Cin, ci = kc - tap * d.Cin, ty = tap / d.KW, tx = tap - ty * d.KW;
                    if (pix_in(p, ty, tx, o)) lo = x[o * d.ldx + d.xoff + ci];
                    if (pix_in(p + 1, ty, tx, o)) hi = x[o * d.ldx + d.xoff + ci];
                }
                gb[u] = mkpair(lo, hi);
            }
        }
    };
    // LDS image: row = co (A) / col (B), k = pixel within the tile, 128 B rows
    auto put = [&](char* base, int row, int pp, pair_t v) {
        const int byte = pp * (int)sizeof(pair_t);
        *(pair_t*)(base + lds_off(row, byte >> 4) + (byte & 15)) = v;
    };
    auto store_tile = [&](int buf) {
        char* A = smem + buf * (BM + BN) * ROWB;
        char* B = A + BM * ROWB;
        if constexpr (FASTA) {
#pragma unroll
            for (int u = 0; u < IA; ++u) {
                int it = tid + 256 * u, cc = it % ACH, pp = it / ACH;
#pragma unroll
                for (int e = 0; e < EPC; ++e) put(A, cc * EPC + e, pp, pa[u][e]);
            }
        } else {
#pragma unroll
            for (int u = 0; u < GA; ++u) {
                int it = tid + 256 * u;
                put(A, it % BM, it / BM, ga[u]);
            }
        }
        if constexpr (FASTB) {
#pragma unroll
            for (int u = 0; u < IB; ++u) {
                int it = tid + 256 * u, cc = it % BCH, pp = it / BCH;
#pragma unroll
                for (int e = 0; e < EPC; ++e) put(B, cc * EPC + e, pp, pbv[u][e]);
            }
        } else {
#pragma unroll
            for (int u = 0; u < GB; ++u) {
                int it = tid + 256 * u;
                put(B, it % BN, it / BN, gb[u]);
            }
        }
    };

    f32x4 acc[MI][NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = (int)((pe - pb + BKP - 1) / BKP);
    load_tile(pb);
    store_tile(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nk) load_tile(pb + (long)(kt + 1) * BKP);
        const char* A = smem + cur * (BM + BN) * ROWB;
        const char* B = A + BM * ROWB;
        f32x4 part[MI][NJ];
        constexpr bool BLOCKED = sizeof(T) == 4;  // see conv_fwd_kernel
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) part[i][j] = BLOCKED ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[i][j];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            uint4 af[MI], bfr[NJ];
            const int ch = h * 4 + (lane >> 4);
#pragma unroll
            for (int i = 0; i < MI; ++i) af[i] = *(const uint4*)(A + lds_off(wm * (BM / 2) + i * 16 + (lane & 15), ch));
#pragma unroll
            for (int j = 0; j < NJ; ++j) bfr[j] = *(const uint4*)(B + lds_off(wn * 32 + j * 16 + (lane & 15), ch));
#pragma unroll
            for (int i = 0; i < MI; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j) mma16(part[i][j], af[i], bfr[j], (const T*)nullptr);
        }
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) acc[i][j] = BLOCKED ? acc[i][j] + part[i][j] : part[i][j];
        if (kt + 1 < nk) store_tile(cur ^ 1);
        __syncthreads();
    }

#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int co = co0 + wm * (BM / 2) + i * 16 + (lane >> 4) * 4 + r;
            if (co >= d.Cout) continue;
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int kc = n0 + wn * 32 + j * 16 + (lane & 15);
                if (kc < K) atomicAdd(dw + (long)co * K + kc, acc[i][j][r]);
            }
        }
}

// dst rows: [R][Kp] with Kp = roundup(taps*Cp, kalign) (taps and channels zero-padded)
//   transpose=0: R = Cout, taps = KH*KW, channel = ci (Cp >= Cin)
//   transpose=1: R = Cin,  taps = Ay*Ax, channel = co (Cp >= Cout), flipped / phase-selected
template <typename T>
__global__ void weight_pack_kernel(const float* __restrict__ src, T* __restrict__ dst, int Cout, int KH, int KW,
                                   int Cin, int transpose, int s, int tyr, int Ay, int txr, int Ax, int Cp, int Kp) {
    const int R = transpose ? Cin : Cout;
    const int taps = transpose ? Ay * Ax : KH * KW;
    const int Cr = transpose ? Cout : Cin;
    long total = (long)R * Kp;
    for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
        const int row = (int)(idx / Kp), k = (int)(idx - (long)row * Kp);
        const int tap = k / Cp, c = k - tap * Cp;
        float v = 0.f;
        if (tap < taps && c < Cr) {
            if (!transpose) {
                v = src[((long)row * KH * KW + tap) * Cin + c];
            } else {
                const int a = tap / Ax, b = tap - a * Ax;
                const int ky = tyr + s * (Ay - 1 - a), kx = txr + s * (Ax - 1 - b);
                v = src[(((long)c * KH + ky) * KW + kx) * Cin + row];
            }
        }
        dst[idx] = from_f<T>(v);
    }
}

// irgan_weight_pack_batch: block row y serves descs[y] (grid-stride over its R x Kp)
__global__ __launch_bounds__(256) void weight_pack_batch_kernel(const irgan_pack_desc* __restrict__ descs) {
    const irgan_pack_desc q = descs[blockIdx.y];
    const int R = q.transpose ? q.Cin : q.Cout;
    const int taps = q.transpose ? q.Ay * q.Ax : q.KH * q.KW;
    const int Cr = q.transpose ? q.Cout : q.Cin;
    const int Cp = q.cpad > Cr ? q.cpad : Cr;
    const int ka = q.kalign > 0 ? q.kalign : 1;
    const int Kp = (taps * Cp + ka - 1) / ka * ka;
    const long total = (long)R * Kp;
    if (q.transpose) {
        // backward-data pack dst[ci][tap*Cp + co] = src[co][ky][kx][ci]: per tap a 2-D
        // transpose, staged through a 64x64 LDS tile so both the fp32 reads (along ci)
        // and the stores (along co) are coalesced
        __shared__ float tile[64][65];
        const int ntc = (Cp + 63) / 64, ntr = (R + 63) / 64;
        const long ntiles = (long)taps * ntc * ntr;
        for (long t = blockIdx.x; t < ntiles; t += gridDim.x) {
            const int rt = (int)(t % ntr);
            const long t2 = t / ntr;
            const int ct = (int)(t2 % ntc), tap = (int)(t2 / ntc);
            const int a = tap / q.Ax, b = tap - a * q.Ax;
            const int ky = q.tyr + q.s * (q.Ay - 1 - a), kx = q.txr + q.s * (q.Ax - 1 - b);
            for (int e = threadIdx.x; e < 4096; e += 256) {
                const int cc = e >> 6, rr = e & 63, c = ct * 64 + cc, row = rt * 64 + rr;
                tile[cc][rr] = (c < Cr && row < R) ? q.src[(((long)c * q.KH + ky) * q.KW + kx) * q.Cin + row] : 0.f;
            }
            __syncthreads();
            for (int e = threadIdx.x; e < 4096; e += 256) {
                const int rr = e >> 6, cc = e & 63, c = ct * 64 + cc, row = rt * 64 + rr;
                if (row < R && c < Cp) {
                    const long o = (long)row * Kp + tap * Cp + c;
                    if (q.dtype == IRGAN_BF16) ((bf16_t*)q.dst)[o] = f2bf(tile[cc][rr]);
                    else ((float*)q.dst)[o] = tile[cc][rr];
                }
            }
            __syncthreads();
        }
        const int tail = Kp - taps * Cp;  // K padding up to kalign: zeros
        for (long idx = blockIdx.x * 256L + threadIdx.x; idx < (long)R * tail; idx += (long)gridDim.x * 256) {
            const long o = (idx / tail) * Kp + taps * Cp + idx % tail;
            if (q.dtype == IRGAN_BF16) ((bf16_t*)q.dst)[o] = 0;
            else ((float*)q.dst)[o] = 0.f;
        }
        return;
    }
    if (q.dtype == IRGAN_BF16 && Cp == Cr && Kp == taps * Cp && total % 8 == 0 && (uintptr_t)q.src % 16 == 0 &&
        (uintptr_t)q.dst % 16 == 0) {
        // unpadded forward pack: dst row = src row (taps x Cin contiguous) in bf16, 8 per thread
        const float4* s4 = (const float4*)q.src;
        uint4* d4 = (uint4*)q.dst;
        for (long i = blockIdx.x * 256L + threadIdx.x; i < total / 8; i += (long)gridDim.x * 256) {
            const float4 a = s4[2 * i], b = s4[2 * i + 1];
            d4[i] = make_uint4(pk_bf16(a.x, a.y), pk_bf16(a.z, a.w), pk_bf16(b.x, b.y), pk_bf16(b.z, b.w));
        }
        return;
    }
    for (long idx = blockIdx.x * 256L + threadIdx.x; idx < total; idx += (long)gridDim.x * 256) {
        const int row = (int)(idx / Kp), k = (int)(idx - (long)row * Kp);
        const int tap = k / Cp, c = k - tap * Cp;
        float v = 0.f;
        if (tap < taps && c < Cr) {
            if (!q.transpose) {
                v = q.src[((long)row * q.KH * q.KW + tap) * q.Cin + c];
            } else {
                const int a = tap / q.Ax, b = tap - a * q.Ax;
                const int ky = q.tyr + q.s * (q.Ay - 1 - a), kx = q.txr + q.s * (q.Ax - 1 - b);
                v = q.src[(((long)c * q.KH + ky) * q.KW + kx) * q.Cin + row];
            }
        }
        if (q.dtype == IRGAN_BF16) ((bf16_t*)q.dst)[idx] = f2bf(v);
        else ((float*)q.dst)[idx] = v;
    }
}

template <typename T>
int launch_fwd(const irgan_conv_desc* d, const void* x, const void* w, const float* bias, void* y,
               const void* mask, hipStream_t st) {
    constexpr int EPC = TT<T>::EPC, BKE = ROWB / (int)sizeof(T);
    const long M = (long)d->N * d->Ho * d->Wo;
    if (M <= 0 || d->Cout <= 0) return 0;
    const bool fast = (d->Cin % BKE == 0) && (d->ldx % EPC == 0) && (d->xoff % EPC == 0);
    if constexpr (sizeof(T) == 2) {
        static const bool use_glds = !getenv("IRGAN_NO_GLDS");
        const bool narrow = (d->Cin == 8 || d->Cin == 16 || d->Cin == 32) && d->ldx % 8 == 0 && d->xoff % 8 == 0;
        static const bool use_halo = !getenv("IRGAN_NO_HALO");
        const int taps = d->KH * d->KW;
        static const bool use_pp = !getenv("IRGAN_NO_PP");
        if (fast && use_pp && ((d->sy == 1 && d->sx == 1) || (d->sy == 2 && d->sx == 2 && d->KH == 4 && d->KW == 4)) &&
            taps >= 2 && d->Cout % 64 == 0) {
            const int rc = irgan_conv_fwd_pp(d, x, w, bias, y, mask, st);
            if (rc != IRGAN_EUNSUPPORTED) return rc;
        }
        if (fast && use_halo && d->sy == 1 && d->sx == 1 && taps >= 2) {
            const int rc = irgan_conv_fwd_halo(d, x, w, bias, y, mask, st);
            if (rc != IRGAN_EUNSUPPORTED) return rc;
        }
        // 8-channel inputs: (tap, channel) flattened into the MFMA K axis (conv_c8.hip)
        static const bool use_c8 = !getenv("IRGAN_NO_C8");
        if (narrow && use_c8 && d->Cin == 8) {
            const int rc = irgan_conv_fwd_c8(d, x, w, bias, y, mask, st);
            if (rc != IRGAN_EUNSUPPORTED) return rc;
        }
        if ((fast || narrow) && use_glds) return irgan_conv_fwd_glds(d, x, w, bias, y, mask, st);
    }
    const bool wide = d->Cout > 64;
    dim3 grid(irgan_cdiv(M, 128), irgan_cdiv(d->Cout, wide ? 128 : 64));
    const T* xp = (const T*)x;
    const T* wp = (const T*)w;
    if (wide) {
        if (fast) conv_fwd_kernel<T, 128, true><<<grid, 256, 0, st>>>(*d, xp, wp, bias, y, mask);
        else conv_fwd_kernel<T, 128, false><<<grid, 256, 0, st>>>(*d, xp, wp, bias, y, mask);
    } else {
        if (fast) conv_fwd_kernel<T, 64, true><<<grid, 256, 0, st>>>(*d, xp, wp, bias, y, mask);
        else conv_fwd_kernel<T, 64, false><<<grid, 256, 0, st>>>(*d, xp, wp, bias, y, mask);
    }
    IRGAN_LAUNCH_CHECK();
    return 0;
}

template <typename T, int BM, bool FA, bool FB>
void wg_launch(dim3 g, hipStream_t st, const irgan_conv_desc* d, const void* x, const void* dy, float* dw, int kc) {
    conv_wgrad_kernel<T, BM, FA, FB><<<g, 256, 0, st>>>(*d, (const T*)x, (const T*)dy, dw, kc);
}

template <typename T>
int launch_wgrad(const irgan_conv_desc* d, const void* x, const void* dy, float* dw, int splitk, hipStream_t st,
                 float* ws = nullptr, long ws_cap = 0) {
    constexpr int EPC = TT<T>::EPC, BKP = ROWB / (int)sizeof(T);
    const long P = (long)d->N * d->Ho * d->Wo;
    const int K = d->KH * d->KW * d->Cin;
    if (P <= 0) return 0;
    const bool fa = (d->Cout % EPC == 0) && (d->ldy % EPC == 0) && (d->yoff % EPC == 0);
    const bool fb = (d->Cin % 64 == 0) && (d->ldx % EPC == 0) && (d->xoff % EPC == 0);
    if constexpr (sizeof(T) == 2) {
        {   // 8-channel inputs (G inc, D model.0): conv_wgrad_narrow.hip
            const int rc = irgan_conv_wgrad_narrow(d, x, dy, dw, ws, ws_cap, st);
            if (rc != IRGAN_EUNSUPPORTED) return rc;
        }
        {   // Cout <= 8, 7x7, one 64-channel input chunk (G outc): row-span GEMM (conv_rowspan.hip)
            const int rc = irgan_conv_wgrad_rowspan(d, x, dy, dw, ws, ws_cap, st);
            if (rc != IRGAN_EUNSUPPORTED) return rc;
        }
        {   // 3x3 stride-1, Cout % 128: producer/consumer row-segment kernel (conv_wgrad_pc.hip)
            const int rc = irgan_conv_wgrad_pc(d, x, dy, dw, splitk, ws, ws_cap, st);
            if (rc != IRGAN_EUNSUPPORTED) return rc;
        }
        static const bool use_wgh = !getenv("IRGAN_NO_WGRAD_HALO");
        if (use_wgh) {
            const int rc = irgan_conv_wgrad_halo(d, x, dy, dw, splitk, ws, ws_cap, st);
            if (rc != IRGAN_EUNSUPPORTED) return rc;
        }
        static const bool use_glds = !getenv("IRGAN_NO_GLDS");
        if (use_glds && fb && (d->Cout % 64 == 0 || d->Cout < 64) && d->ldy % 8 == 0 && d->yoff % 8 == 0)
            return irgan_conv_wgrad_glds(d, x, dy, dw, splitk, st, ws, ws_cap);
    }
    const int BM = d->Cout > 64 ? 128 : 64;
    const int tiles = irgan_cdiv(d->Cout, BM) * irgan_cdiv(K, 64);
    if (irgan_det(d)) splitk = 1;  // deterministic: one block per output element (its single atomic add)
    if (splitk <= 0) {  // aim at ~4 workgroups per CU over 256 CUs
        splitk = irgan_cdiv(1024, tiles);
        long maxs = (P + 4 * BKP - 1) / (4 * BKP);  // keep >= 4 K-tiles per split
        if (splitk > maxs) splitk = (int)maxs;
        if (splitk < 1) splitk = 1;
    }
    long kc = (P + splitk - 1) / splitk;
    kc = (kc + BKP - 1) / BKP * BKP;
    splitk = (int)((P + kc - 1) / kc);
    dim3 g(irgan_cdiv(d->Cout, BM), irgan_cdiv(K, 64), splitk);
#define WG(BMV, A, B) wg_launch<T, BMV, A, B>(g, st, d, x, dy, dw, (int)kc)
    if (BM == 128) {
        if (fa && fb) WG(128, true, true); else if (fa) WG(128, true, false);
        else if (fb) WG(128, false, true); else WG(128, false, false);
    } else {
        if (fa && fb) WG(64, true, true); else if (fa) WG(64, true, false);
        else if (fb) WG(64, false, true); else WG(64, false, false);
    }
#undef WG
    IRGAN_LAUNCH_CHECK();
    return 0;
}

}  // namespace

extern "C" int irgan_conv_fwd(const irgan_conv_desc* d, const void* x, const void* w, const float* bias,
                              void* y, const void* mask, irgan_stream_t s) {
    if (!d || !x || !w || !y) return IRGAN_EINVAL;
    if (d->accumulate && d->out_dtype != IRGAN_F32 && d->out_dtype != IRGAN_BF16) return IRGAN_EINVAL;
    hipStream_t st = (hipStream_t)s;
    if (d->dtype == IRGAN_BF16) return launch_fwd<bf16_t>(d, x, w, bias, y, mask, st);
    if (d->dtype == IRGAN_F32) return launch_fwd<float>(d, x, w, bias, y, mask, st);
    return IRGAN_EUNSUPPORTED;
}

extern "C" int irgan_conv_wgrad(const irgan_conv_desc* d, const void* x, const void* dy, float* dw,
                                int32_t splitk, irgan_stream_t s) {
    if (!d || !x || !dy || !dw) return IRGAN_EINVAL;
    hipStream_t st = (hipStream_t)s;
    if (d->dtype == IRGAN_BF16) return launch_wgrad<bf16_t>(d, x, dy, dw, splitk, st);
    if (d->dtype == IRGAN_F32) return launch_wgrad<float>(d, x, dy, dw, splitk, st);
    return IRGAN_EUNSUPPORTED;
}

extern "C" int irgan_conv_wgrad_ws(const irgan_conv_desc* d, const void* x, const void* dy, float* dw,
                                   int32_t splitk, float* ws, int64_t ws_floats, irgan_stream_t s) {
    if (!d || !x || !dy || !dw) return IRGAN_EINVAL;
    hipStream_t st = (hipStream_t)s;
    if (d->dtype == IRGAN_BF16)
        return launch_wgrad<bf16_t>(d, x, dy, dw, splitk, st, ws, ws_floats);
    if (d->dtype == IRGAN_F32) return launch_wgrad<float>(d, x, dy, dw, splitk, st);
    return IRGAN_EUNSUPPORTED;
}

extern "C" int irgan_weight_pack(const float* src, void* dst, int32_t dtype, int32_t Cout, int32_t KH, int32_t KW,
                                 int32_t Cin, int32_t transpose, int32_t s, int32_t tyr, int32_t Ay, int32_t txr,
                                 int32_t Ax, int32_t cpad, int32_t kalign, irgan_stream_t st) {
    const int R = transpose ? Cin : Cout, taps = transpose ? Ay * Ax : KH * KW;
    const int Cr = transpose ? Cout : Cin;
    const int Cp = cpad > Cr ? cpad : Cr;
    const int ka = kalign > 0 ? kalign : 1;
    const int Kp = (taps * Cp + ka - 1) / ka * ka;
    long total = (long)R * Kp;
    int blocks = (int)std::min<long>((total + 255) / 256, 4096);
    if (blocks <= 0) return 0;
    if (dtype == IRGAN_BF16)
        weight_pack_kernel<bf16_t><<<blocks, 256, 0, (hipStream_t)st>>>(src, (bf16_t*)dst, Cout, KH, KW, Cin,
                                                                          transpose, s, tyr, Ay, txr, Ax, Cp, Kp);
    else
        weight_pack_kernel<float><<<blocks, 256, 0, (hipStream_t)st>>>(src, (float*)dst, Cout, KH, KW, Cin,
                                                                         transpose, s, tyr, Ay, txr, Ax, Cp, Kp);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_weight_pack_batch(const irgan_pack_desc* descs, int32_t n, irgan_stream_t st) {
    if (n <= 0) return 0;
    if (!descs || n > 65535) return IRGAN_EINVAL;
    // 256 blocks per job: the largest (a 256 x 256 x 3 x 3 backward-data pack, 144 64 x 64 tiles;
    // D model.8's, 512) in one or two rounds; a small job's spare blocks exit at once
    weight_pack_batch_kernel<<<dim3(256, n), 256, 0, (hipStream_t)st>>>(descs);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_version(void) { return 1; }


// Split-K partial sums (no bias / activation / mask): partial ks of the
// fp32 output lands at y + ks*split_stride.  Used for thin output domains
// (the reflect-pad ring) whose full-K blocks would run a long serial K loop.
extern "C" int irgan_conv_fwd_splitk(const irgan_conv_desc* d, const void* x, const void* w, float* y,
                                     int32_t ksplit, int64_t split_stride, irgan_stream_t s) {
    if (d->out_dtype != IRGAN_F32 || d->act != IRGAN_ACT_NONE || d->accumulate || ksplit < 1) return IRGAN_EINVAL;
    const bool fast = (d->Cin % 64 == 0) && (d->ldx % 8 == 0) && (d->xoff % 8 == 0);
    const bool narrow = (d->Cin == 8 || d->Cin == 16 || d->Cin == 32) && d->ldx % 8 == 0 && d->xoff % 8 == 0;
    if (d->dtype == IRGAN_BF16 && (fast || narrow))
        return irgan_conv_fwd_glds_split(d, x, w, nullptr, y, nullptr, ksplit, (long)split_stride, (hipStream_t)s);
    if (ksplit != 1) return IRGAN_EUNSUPPORTED;
    return irgan_conv_fwd(d, x, w, nullptr, y, nullptr, s);
}
