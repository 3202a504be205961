// Resampling and layout kernels (NHWC, channel-fastest threads => coalesced).
//   separable resample: Downsample (ir:269-310), UpsampleAA (ir:313-355), the
//                       nn.ReflectionPad2d fold (ir:381, 402, 459, 528) and their
//                       adjoints, all as per-axis (index, weight) tables
//   maxpool 2x2       : VGG-16 features pooling (ir:664)
// Backward passes are gathers (each output element sums its contributors), so
// they are deterministic and need no atomics.
#include "common.h"
#include "fp8_util.h"

namespace {

constexpr int TPB = 256;

// ---------------------------------------------------------------------------
// separable resampling: out[n][oy][ox][c] = sum_i sum_j wy[oy][i] wx[ox][j] in[n][iy][ix][c]
// One kernel serves Downsample (blur s2), UpsampleAA (bilinear x2 + blur), the
// reflection-pad fold and all their adjoints: each is separable per axis, so a
// per-axis (index, weight) table of at most T taps describes it exactly.
// Threads own 8 channels (16-byte loads) when the slices allow.
// ---------------------------------------------------------------------------
template <int VW>
IRGAN_HD void ldvec(const void* p, int dt, long i, float* o) {
    if constexpr (VW == 8) {
        if (dt == IRGAN_BF16) {
            const uint4 u = *(const uint4*)((const bf16_t*)p + i);
            const uint32_t q[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                o[2 * k] = __uint_as_float(q[k] << 16);
                o[2 * k + 1] = __uint_as_float(q[k] & 0xffff0000u);
            }
        } else {
            const float4 a = *(const float4*)((const float*)p + i), b = *(const float4*)((const float*)p + i + 4);
            o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
        }
    } else {
        o[0] = ldv(p, dt, i);
    }
}
template <int VW>
IRGAN_HD void stvec(void* p, int dt, long i, const float* v) {
    if constexpr (VW == 8) {
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
    } else {
        stv(p, dt, i, v[0]);
    }
}

// One block row per output image row (blockIdx.y = n*Hout + oy): the vertical
// taps are block-uniform (scalar loads), threads run over (ox, channel group)
// with 32-bit index math and 16-byte loads/stores.
template <int VW>
__global__ __launch_bounds__(TPB) void sep_kernel(const void* __restrict__ in, int idt, int Hin, int Win, int C,
                                                  int ldi, int offi, void* __restrict__ out, int odt, int Hout,
                                                  int Wout, int ldo, int offo, const int* __restrict__ ty,
                                                  const float* __restrict__ wy, int Ty, const int* __restrict__ tx,
                                                  const float* __restrict__ wx, int Tx, int accumulate) {
    const int CV = C / VW;
    const int row = blockIdx.y;
    const int n = row / Hout, oy = row - n * Hout;
    const int idx = blockIdx.x * TPB + threadIdx.x;
    if (idx >= Wout * CV) return;
    const int ox = idx / CV, c = (idx - ox * CV) * VW;
    float acc[VW];
#pragma unroll
    for (int k = 0; k < VW; ++k) acc[k] = 0.f;
    for (int i = 0; i < Ty; ++i) {
        const float w1 = wy[oy * Ty + i];
        if (w1 == 0.f) continue;
        const long rowb = ((long)n * Hin + ty[oy * Ty + i]) * Win;
        for (int j = 0; j < Tx; ++j) {
            const float w2 = wx[ox * Tx + j];
            if (w2 == 0.f) continue;
            const float w = w1 * w2;
            float v[VW];
            ldvec<VW>(in, idt, (rowb + tx[ox * Tx + j]) * ldi + offi + c, v);
#pragma unroll
            for (int k = 0; k < VW; ++k) acc[k] += w * v[k];
        }
    }
    const long o = (((long)n * Hout + oy) * Wout + ox) * ldo + offo + c;
    if (accumulate) {
        float v[VW];
        ldvec<VW>(out, odt, o, v);
#pragma unroll
        for (int k = 0; k < VW; ++k) acc[k] += v[k];
    }
    stvec<VW>(out, odt, o, acc);
}

// Two-stage form of the same map through LDS.  Block = one output row (n, oy)
// x a group of CB channels, 1024 threads.  Stage 1 applies the row's vertical
// taps to every input column (16-byte coalesced loads of the <= TM input rows;
// the taps are block-uniform, so they come from scalar loads) and keeps the
// fp32 result [Win][CB] in LDS; stage 2 applies the horizontal taps from LDS and
// writes the output row with 16-byte stores.  The tap loops run to the
// compile-time bound TM (tables are compacted to their widest row on the host),
// so a thread's loads are issued back to back.  Global loads per output drop
// from Ty*Tx (sep_kernel) to about Ty*Win/Wout.
//
// NORM (irgan_sep_resample_in): the input is a pre-InstanceNorm tensor z and every
// loaded value becomes act((z - mean[n][c]) * rstd[n][c]) before the vertical taps --
// the InstanceNorm apply + ReLU of down1 / down2 / up1_conv (ir:469-482, 557) fused into
// the Downsample / UpsampleAA that consumes it, so the normalised tensor is never stored.
// LTPB % G == 0, so a thread's channel group (and its 8 (mean, rstd) pairs) is fixed.
//
// Q8 (irgan_sep_resample_fp8): the stored bf16 output also as e4m3 bytes (o8: an NHWC slice,
// e4m3(clamp(bf16(out) * q8[0], +-448))) with max |bf16(out)| raised into the amax slot --
// the fp8 path's producers of the down2 / up1_conv operands (x1 from down1's Downsample, the
// up-sampled bottleneck from UpsampleAA: the two halves of up1_conv's concat), so no separate
// quantise pass reads them back.
struct ResQ8 {
    uint8_t* p;
    int ld, off;
    const float* q;
    uint32_t* amax;
};
constexpr int LTPB = 1024;
template <int TM, bool NORM = false, int NT = LTPB, bool Q8 = false>
__global__ __launch_bounds__(NT) void sep_lds_kernel(const void* __restrict__ in, int idt, int Hin, int Win,
                                                       int ldi, int offi, void* __restrict__ out, int odt, int Hout,
                                                       int Wout, int ldo, int offo, const int* __restrict__ ty,
                                                       const float* __restrict__ wy, int Ty,
                                                       const int* __restrict__ tx, const float* __restrict__ wx,
                                                       int Tx, int accumulate, int CB,
                                                       const float* __restrict__ mr = nullptr, int C = 0,
                                                       int act = 0, int swz = 0, ResQ8 q8 = ResQ8{}) {
    extern __shared__ float4 sm4[];
    float* const sm = (float*)sm4;
    // XCD-aware row order: consecutive output rows (which share input rows through the
    // vertical taps) run on the same XCD, so the shared rows hit that XCD's L2
    const int row = xcd_tile(blockIdx.x, gridDim.x, swz);
    const int n = row / Hout, oy = row - n * Hout;
    const int c0 = blockIdx.y * CB;
    const int G = CB >> 3;  // 8-channel groups
    float nm[NORM ? 8 : 1], nr[NORM ? 8 : 1];
    if constexpr (NORM) {
        const float4* m4 = (const float4*)(mr + 2 * ((long)n * C + c0 + (threadIdx.x % G) * 8));
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float4 t = m4[k];
            nm[2 * k] = -t.x * t.y; nr[2 * k] = t.y; nm[2 * k + 1] = -t.z * t.w; nr[2 * k + 1] = t.w;
        }  // nm = -mean * rstd: (z - mean) * rstd as one FMA per loaded element
    }
    float wyv[TM];
    long rb[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        wyv[i] = i < Ty ? wy[oy * Ty + i] : 0.f;
        rb[i] = i < Ty ? (long)(n * Hin + ty[oy * Ty + i]) * Win : 0;
    }
    for (int v = threadIdx.x; v < Win * G; v += NT) {
        const int col = v / G, g = v - col * G;
        float acc[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            if (wyv[i] == 0.f) continue;
            float xv[8];
            ldvec<8>(in, idt, (rb[i] + col) * ldi + offi + c0 + g * 8, xv);
            if constexpr (NORM) {
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const float h = fmaf(xv[k], nr[k], nm[k]);
                    xv[k] = act == IRGAN_ACT_RELU ? fmaxf(h, 0.f) : (act == IRGAN_ACT_LRELU && h < 0.f ? 0.2f * h : h);
                }
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[k] += wyv[i] * xv[k];
        }
        float4* d = (float4*)(sm + (col * CB + g * 8));
        d[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
        d[1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
    }
    __syncthreads();
    const float qs = Q8 ? *q8.q : 1.f;
    float amx = 0.f;
    for (int v = threadIdx.x; v < Wout * G; v += NT) {
        const int ox = v / G, g = v - ox * G;
        float wxv[TM];
        int ix[TM];
#pragma unroll
        for (int j = 0; j < TM; ++j) {
            wxv[j] = j < Tx ? wx[ox * Tx + j] : 0.f;
            ix[j] = j < Tx ? tx[ox * Tx + j] : 0;
        }
        float acc[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] = 0.f;
#pragma unroll
        for (int j = 0; j < TM; ++j) {
            const float w = wxv[j];
            if (w == 0.f) continue;  // padding slot (keeps inf/nan in a skipped column out)
            const float4* sp = (const float4*)(sm + (ix[j] * CB + g * 8));
            const float4 a = sp[0], b = sp[1];
            acc[0] += w * a.x; acc[1] += w * a.y; acc[2] += w * a.z; acc[3] += w * a.w;
            acc[4] += w * b.x; acc[5] += w * b.y; acc[6] += w * b.z; acc[7] += w * b.w;
        }
        const long o = (((long)n * Hout + oy) * Wout + ox) * ldo + offo + c0 + g * 8;
        if (accumulate) {
            float pv[8];
            ldvec<8>(out, odt, o, pv);
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[k] += pv[k];
        }
        if constexpr (Q8) {  // bf16 out (host-checked): quantise the stored values
            uint4 u;
            u.x = pk_bf16(acc[0], acc[1]);
            u.y = pk_bf16(acc[2], acc[3]);
            u.z = pk_bf16(acc[4], acc[5]);
            u.w = pk_bf16(acc[6], acc[7]);
            *(uint4*)((bf16_t*)out + o) = u;
            const uint32_t wd[4] = {u.x, u.y, u.z, u.w};
            float vb[8];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                vb[2 * k] = __uint_as_float(wd[k] << 16);
                vb[2 * k + 1] = __uint_as_float(wd[k] & 0xffff0000u);
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) amx = fmaxf(amx, fabsf(vb[k]));
            const long o8 = (((long)n * Hout + oy) * Wout + ox) * q8.ld + q8.off + c0 + g * 8;
            *(uint2*)(q8.p + o8) = pack8_fp8(vb, qs);
        } else {
            stvec<8>(out, odt, o, acc);
        }
    }
    if constexpr (Q8) fp8_block_amax(amx, q8.amax, blockIdx.y * gridDim.x + blockIdx.x);
}

// Round 6: sep_lds_kernel's map with R output rows per block and the next row's vertical
// taps in flight under the current row's horizontal pass.  sep_lds_kernel runs one output row
// per block: load its <= TM input rows, barrier, horizontal taps, store, exit -- every block
// exposes its loads' latency and the resamplers ran at 1.4-3.9 TB/s.  Here a block walks rows
// oy0 .. oy0 + R - 1 of one image and channel group with two [Win][CB] fp32 row buffers:
//   * the vertical-tap loads of row r + 1 are issued (raw 16-byte buffer loads, invalid
//     items and zero-weight taps at the out-of-range offset) right after row r's vertical
//     sums are written to LDS, and consumed at the top of the next row;
//   * the horizontal tables live in LDS (loaded once per block), the output goes through raw
//     buffer stores (an item past the row at the out-of-range offset), so a row issues a
//     fixed number of VMEM ops and the wait for the prefetched taps is a counted vmcnt that
//     leaves the previous row's stores in flight;
//   * one barrier per row (a buffer is rewritten two rows later, after every thread passed
//     the next row's barrier).
// Same per-element arithmetic and tap order as sep_lds_kernel (bf16 in, bf16 out, no
// accumulate; NORM / Q8 as there).  IPT / OPT: input / output items per thread (host-sized).
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
int sep_swz();

template <int TM, bool NORM, bool Q8, int IPT, int OPT>
__global__ __launch_bounds__(512) void sep_pipe_kernel(const bf16_t* __restrict__ in, int Hin, int Win, int ldi,
                                                       int offi, bf16_t* __restrict__ out, int Hout, int Wout,
                                                       int ldo, int offo, const int* __restrict__ ty,
                                                       const float* __restrict__ wy, int Ty,
                                                       const int* __restrict__ tx, const float* __restrict__ wx,
                                                       int Tx, int CB, int CBP, int R, const float* __restrict__ mr,
                                                       int C, int act, int swz, ResQ8 q8) {
    constexpr int NT = 512;
    extern __shared__ float4 sm4[];
    float* const sm = (float*)sm4;                       // [2][Win][CBP] fp32 rows (CBP >= CB: bank spread)
    const int G = CB >> 3;
    const int WG = Win * G, OG = Wout * G;
    float* const tw = sm + 2 * Win * CBP;                // [Wout][TM] horizontal weights
    int* const ti = (int*)(tw + Wout * TM);              // [Wout][TM] horizontal taps (input column)
    // block -> (row block, channel group), groups fastest: the C / CB blocks that read the
    // same input pixels (each a CB-channel slice of every pixel row) are consecutive logical
    // tiles, i.e. (XCD-aware order) dispatched together on one XCD, so a 64 / 128-byte slice
    // read pulls the whole pixel row into that L2 once for all of them
    const int nrb = (Hout + R - 1) / R, ng = C / CB;
    const int t = xcd_tile(blockIdx.x, gridDim.x, swz);
    const int rbk = t / ng;
    const int n = rbk / nrb, oy0 = (rbk - n * nrb) * R;
    const int oy1 = min(Hout, oy0 + R);
    const int c0 = (t - rbk * ng) * CB;
    const int tid = threadIdx.x;
    for (int e = tid; e < Wout * TM; e += NT) {
        const int ox = e / TM, j = e - ox * TM;
        tw[e] = j < Tx ? wx[ox * Tx + j] : 0.f;
        ti[e] = j < Tx ? tx[ox * Tx + j] : 0;
    }
    float nm[NORM ? 8 : 1], nr[NORM ? 8 : 1];
    if constexpr (NORM) {
        const float4* m4 = (const float4*)(mr + 2 * ((long)n * C + c0 + (tid % G) * 8));
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float4 t = m4[k];
            nm[2 * k] = -t.x * t.y; nr[2 * k] = t.y; nm[2 * k + 1] = -t.z * t.w; nr[2 * k + 1] = t.w;
        }
    }
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)in, (short)0, (int)((long)(n + 1) * Hin * Win * ldi * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(
        out, (short)0, (int)((long)(n + 1) * Hout * Wout * ldo * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t qr = __builtin_amdgcn_make_buffer_rsrc(
        Q8 ? (void*)q8.p : (void*)out, (short)0, Q8 ? (int)((long)(n + 1) * Hout * Wout * q8.ld) : 0, 0x00020000);
    // this thread's input items (col, group) and their offsets within an input row
    int icol[IPT], ig[IPT];
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
        const int v = tid + k * NT;
        icol[k] = v < WG ? v / G : -1;
        ig[k] = v - (v / G) * G;
    }
    uint4 pre[IPT][TM];   // raw bf16x8 of the next row's vertical taps
    float wnext[TM];
    auto issue = [&](int oy) {
        int trow[TM];   // the row's taps (block-uniform: scalar loads, all issued before any use)
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            wnext[i] = i < Ty ? wy[oy * Ty + i] : 0.f;
            trow[i] = i < Ty ? ty[oy * Ty + i] : 0;
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const long rb = (long)(n * Hin + trow[i]) * Win;
#pragma unroll
            for (int k = 0; k < IPT; ++k) {
                const bool ok = icol[k] >= 0 && wnext[i] != 0.f;
                const uint32_t off = ok ? (uint32_t)(((rb + icol[k]) * ldi + offi + c0 + ig[k] * 8) * 2) : IRGAN_OOB;
                pre[k][i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
            }
        }
    };
    issue(oy0);
    __syncthreads();  // the horizontal tables
    const float qs = Q8 ? *q8.q : 1.f;
    float amx = 0.f;
    int buf = 0;
#pragma unroll 1
    for (int oy = oy0; oy < oy1; ++oy, buf ^= 1) {
        float wcur[TM];
#pragma unroll
        for (int i = 0; i < TM; ++i) wcur[i] = wnext[i];
        // vertical taps of row oy (its loads were issued one row ago)
        float* const row = sm + buf * Win * CBP;
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
            if (icol[k] < 0) continue;
            float acc[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) acc[q] = 0.f;
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                if (wcur[i] == 0.f) continue;
                const uint32_t wd[4] = {pre[k][i].x, pre[k][i].y, pre[k][i].z, pre[k][i].w};
                float xv[8];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    xv[2 * q] = __uint_as_float(wd[q] << 16);
                    xv[2 * q + 1] = __uint_as_float(wd[q] & 0xffff0000u);
                }
                if constexpr (NORM) {
#pragma unroll
                    for (int q = 0; q < 8; ++q) {
                        const float h = fmaf(xv[q], nr[q], nm[q]);
                        xv[q] = act == IRGAN_ACT_RELU ? fmaxf(h, 0.f) : (act == IRGAN_ACT_LRELU && h < 0.f ? 0.2f * h : h);
                    }
                }
#pragma unroll
                for (int q = 0; q < 8; ++q) acc[q] += wcur[i] * xv[q];
            }
            float4* d = (float4*)(row + (icol[k] * CBP + ig[k] * 8));
            d[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
            d[1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
        }
        if (oy + 1 < oy1) issue(oy + 1);
        __syncthreads();  // row oy's vertical sums complete
        // horizontal taps of row oy
#pragma unroll
        for (int k = 0; k < OPT; ++k) {
            const int v = tid + k * NT;
            const bool okv = v < OG;
            const int ox = okv ? v / G : 0, g = v - (v / G) * G;
            float acc[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) acc[q] = 0.f;
#pragma unroll
            for (int j = 0; j < TM; ++j) {
                const float w = tw[ox * TM + j];
                if (w == 0.f) continue;
                const float4* sp = (const float4*)(row + (ti[ox * TM + j] * CBP + g * 8));
                const float4 a = sp[0], b = sp[1];
                acc[0] += w * a.x; acc[1] += w * a.y; acc[2] += w * a.z; acc[3] += w * a.w;
                acc[4] += w * b.x; acc[5] += w * b.y; acc[6] += w * b.z; acc[7] += w * b.w;
            }
            u32x4_t u;
            u.x = pk_bf16(acc[0], acc[1]);
            u.y = pk_bf16(acc[2], acc[3]);
            u.z = pk_bf16(acc[4], acc[5]);
            u.w = pk_bf16(acc[6], acc[7]);
            const long o = (((long)n * Hout + oy) * Wout + ox) * ldo + offo + c0 + g * 8;
            __builtin_amdgcn_raw_buffer_store_b128(u, yr, okv ? (int)(o * 2) : (int)IRGAN_OOB, 0, 0);
            if constexpr (Q8) {
                const uint32_t wd[4] = {u.x, u.y, u.z, u.w};
                float vb[8];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    vb[2 * q] = __uint_as_float(wd[q] << 16);
                    vb[2 * q + 1] = __uint_as_float(wd[q] & 0xffff0000u);
                }
                if (okv) {
#pragma unroll
                    for (int q = 0; q < 8; ++q) amx = fmaxf(amx, fabsf(vb[q]));
                }
                const uint2 p8 = pack8_fp8(vb, qs);
                const long o8 = (((long)n * Hout + oy) * Wout + ox) * q8.ld + q8.off + c0 + g * 8;
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, p8), qr, okv ? (int)o8 : (int)IRGAN_OOB,
                                                      0, 0);
            }
        }
    }
    if constexpr (Q8) fp8_block_amax(amx, q8.amax, blockIdx.x);
}

// the pipelined form for a (bf16 -> bf16, no accumulate) resample, or false (nothing launched)
bool sep_pipe_launch(const void* in, int in_dtype, int N, int Hin, int Win, int C, int ldi, int offi, void* out,
                     int out_dtype, int Hout, int Wout, int ldo, int offo, const int* ty, const float* wy, int Ty,
                     const int* tx, const float* wx, int Tx, const float* mr, int act, const ResQ8* q8,
                     hipStream_t st) {
    static const bool off = getenv("IRGAN_SEP_ROWS1") != nullptr;   // A/B: sep_lds_kernel
    if (off || in_dtype != IRGAN_BF16 || out_dtype != IRGAN_BF16) return false;
    const int TM = Ty > Tx ? Ty : Tx;
    if (TM > 8 || C % 8 || ldi % 8 || offi % 8 || ldo % 8 || offo % 8) return false;
    if (q8 && (q8->ld % 8 || q8->off % 8)) return false;
    int CB = 0;
    for (int cb = 128; cb >= 8 && !CB; cb >>= 1)
        if (C % cb == 0 && (long)Win * cb <= 8192) CB = cb;
    if (!CB) return false;
    const int G = CB / 8;
    const long WG = (long)Win * G, OG = (long)Wout * G;
    const int ipt = WG <= 512 ? 1 : (WG <= 1024 ? 2 : 0);
    const int opt = OG <= 512 ? 1 : (OG <= 1024 ? 2 : (OG <= 2048 ? 4 : 0));
    if (!ipt || !opt || 512 % G) return false;
    if ((long)N * Hin * Win * ldi * 2 >= (1L << 31) || (long)N * Hout * Wout * ldo * 2 >= (1L << 31)) return false;
    const int R = Hout >= 64 ? 8 : (Hout >= 16 ? 4 : 1);
    const int TMt = TM <= 2 ? 2 : (TM <= 4 ? 4 : (TM <= 6 ? 6 : 8));
    // rows padded by 4 floats where two blocks per CU still fit: a stride-2 horizontal read
    // (Downsample, the UpsampleAA adjoint) otherwise lands every 64-float step on one bank
    int CBP = CB + 4;
    size_t sh = (size_t)2 * Win * CBP * 4 + (size_t)Wout * TMt * 8;
    if (sh > 80 * 1024) {
        CBP = CB;
        sh = (size_t)2 * Win * CBP * 4 + (size_t)Wout * TMt * 8;
    }
    if (sh > 80 * 1024) return false;
    const dim3 g(N * irgan_cdiv(Hout, R) * (C / CB));
    const ResQ8 qq = q8 ? *q8 : ResQ8{};
    const int swz = sep_swz();
#define SPK(TMV, NORMV, Q8V, IP, OP)                                                                               \
    sep_pipe_kernel<TMV, NORMV, Q8V, IP, OP><<<g, 512, sh, st>>>((const bf16_t*)in, Hin, Win, ldi, offi,          \
                                                                 (bf16_t*)out, Hout, Wout, ldo, offo, ty, wy, Ty, \
                                                                 tx, wx, Tx, CB, CBP, R, mr, C, act, swz, qq)
#define SPO(TMV, NORMV, Q8V, IP)                              \
    if (opt == 1) SPK(TMV, NORMV, Q8V, IP, 1);                \
    else if (opt == 2) SPK(TMV, NORMV, Q8V, IP, 2);           \
    else SPK(TMV, NORMV, Q8V, IP, 4);
#define SPI(TMV, NORMV, Q8V)                                  \
    if (ipt == 1) { SPO(TMV, NORMV, Q8V, 1) } else { SPO(TMV, NORMV, Q8V, 2) }
#define SPT(NORMV, Q8V)                                       \
    if (TM <= 2) { SPI(2, NORMV, Q8V) }                       \
    else if (TM <= 4) { SPI(4, NORMV, Q8V) }                  \
    else if (TM <= 6) { SPI(6, NORMV, Q8V) }                  \
    else { SPI(8, NORMV, Q8V) }
    if (mr && q8) { SPT(true, true) }
    else if (mr) { SPT(true, false) }
    else if (q8) { SPT(false, true) }
    else { SPT(false, false) }
#undef SPT
#undef SPI
#undef SPO
#undef SPK
    return true;
}

// Threads per block of sep_lds_kernel and the LDS row cap (floats) that sizes its channel
// group: 512 threads with CB <= 8192 / Win.  Half-size groups (against 1024 threads) double
// the blocks and let two resident blocks per CU overlap one's load with the other's taps: the
// six resample launches of a step sum 659 -> 576 us standalone and the step goes 1191 -> 1204
// img/s (same box, 3 reps each; profiles/r03_resample_nt_sweep.txt).
constexpr int sep_nt() { return 512; }

// XCD-aware row order for sep_lds_kernel: each XCD takes a contiguous range of output rows,
// so the input rows their vertical taps share stay in that XCD's L2 (IRGAN_NO_XCD_SWZ)
int sep_swz() { return irgan_xcd_swz(); }

// Reflect-pad backward, border part.  The backward-data result g over the
// padded domain (H+2p) x (W+2p) has its interior in dx already; its RING comes
// as nsplit split-K partials in compact buffers rows[ks][N][2p][Wp][C] and
// cols[ks][N][H][2p][C].  Along one axis dx index i receives padded u = i+p
// (interior) and at most one mirror: u = p-i (1 <= i <= p) or u = 2H-2-i+p
// (H-1-p <= i <= H-2).  Each band element of dx gathers every (uy, ux) pair
// except the interior-interior one (deterministic, no atomics).
// blockIdx.y = n*H + iy, threads over (ix, channel group).
IRGAN_HD int mirrors(int i, int n, int p, int* u) {  // padded coords != i+p mapping to i
    int k = 0;
    if (i >= 1 && i <= p) u[k++] = p - i;
    if (i >= n - 1 - p && i <= n - 2) u[k++] = 2 * n - 2 - i + p;
    return k;
}

template <int VW>
__global__ __launch_bounds__(TPB) void ring_fold_kernel(const float* __restrict__ rows, const float* __restrict__ cols,
                                                        int nsplit, int N, int H, int W, int C, int p,
                                                        void* __restrict__ dx, int dt, int lddx, int dxoff) {
    const int CV = C / VW;
    const int e = blockIdx.x * TPB + threadIdx.x;
    if (e >= W * CV) return;
    const int ix = e / CV, c = (e - ix * CV) * VW;
    const int n = blockIdx.y / H, iy = blockIdx.y - n * H;
    int uy[3], ux[3];
    uy[0] = iy + p;
    ux[0] = ix + p;
    const int ky = 1 + mirrors(iy, H, p, uy + 1), kx = 1 + mirrors(ix, W, p, ux + 1);
    if (ky == 1 && kx == 1) return;  // not in the band
    const int Wp = W + 2 * p;
    const long rstride = (long)N * 2 * p * Wp * C, cstride = (long)N * H * 2 * p * C;
    float acc[VW];
#pragma unroll
    for (int k = 0; k < VW; ++k) acc[k] = 0.f;
    for (int a = 0; a < ky; ++a)
        for (int b = 0; b < kx; ++b) {
            if (a == 0 && b == 0) continue;
            const int y = uy[a], x = ux[b];
            const float* src;
            long stride;
            if (y < p || y >= H + p) {
                const int r = y < p ? y : p + (y - H - p);
                src = rows + (((long)n * 2 * p + r) * Wp + x) * C + c;
                stride = rstride;
            } else {
                const int cc = x < p ? x : p + (x - W - p);
                src = cols + (((long)n * H + (y - p)) * 2 * p + cc) * C + c;
                stride = cstride;
            }
            for (int ks = 0; ks < nsplit; ++ks) {
                float v[VW];
                ldvec<VW>(src, IRGAN_F32, ks * stride, v);
#pragma unroll
                for (int k = 0; k < VW; ++k) acc[k] += v[k];
            }
        }
    const long o = (((long)n * H + iy) * W + ix) * lddx + dxoff + c;
    float d[VW];
    ldvec<VW>(dx, dt, o, d);
#pragma unroll
    for (int k = 0; k < VW; ++k) d[k] += acc[k];
    stvec<VW>(dx, dt, o, d);
}

// 2x2/2 max pooling; blockIdx.y = n*Ho + i, threads over (j, channel group of VW)
template <int VW>
__global__ __launch_bounds__(TPB) void maxpool_fwd_kernel(const void* __restrict__ x, int dt, int H, int W, int C,
                                                          void* __restrict__ y) {
    const int Ho = H / 2, Wo = W / 2, CV = C / VW;
    const int e = blockIdx.x * TPB + threadIdx.x;
    if (e >= Wo * CV) return;
    const int j = e / CV, c = (e - j * CV) * VW;
    const int n = blockIdx.y / Ho, i = blockIdx.y - n * Ho;
    float m[VW];
#pragma unroll
    for (int k = 0; k < VW; ++k) m[k] = -INFINITY;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            float v[VW];
            ldvec<VW>(x, dt, (((long)n * H + 2 * i + a) * W + 2 * j + b) * C + c, v);
#pragma unroll
            for (int k = 0; k < VW; ++k)
                if (v[k] > m[k] || isnan(v[k])) m[k] = v[k];
        }
    stvec<VW>(y, dt, (((long)n * Ho + i) * Wo + j) * C + c, m);
}

// gradient routed to the (first) argmax; relu_mask folds the ReLU' of the pool input
template <int VW>
__global__ __launch_bounds__(TPB) void maxpool_bwd_kernel(const void* __restrict__ x, const void* __restrict__ dy,
                                                          int dt, int H, int W, int C, void* __restrict__ dx,
                                                          int relu_mask) {
    const int Ho = H / 2, Wo = W / 2, CV = C / VW;
    const int e = blockIdx.x * TPB + threadIdx.x;
    if (e >= Wo * CV) return;
    const int j = e / CV, c = (e - j * CV) * VW;
    const int n = blockIdx.y / Ho, i = blockIdx.y - n * Ho;
    float xv[4][VW], m[VW];
    int am[VW];
#pragma unroll
    for (int k = 0; k < VW; ++k) { m[k] = -INFINITY; am[k] = 0; }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        ldvec<VW>(x, dt, (((long)n * H + 2 * i + (q >> 1)) * W + 2 * j + (q & 1)) * C + c, xv[q]);
#pragma unroll
        for (int k = 0; k < VW; ++k)
            if (xv[q][k] > m[k] || isnan(xv[q][k])) { m[k] = xv[q][k]; am[k] = q; }
    }
    float g[VW];
    ldvec<VW>(dy, dt, (((long)n * Ho + i) * Wo + j) * C + c, g);
#pragma unroll
    for (int k = 0; k < VW; ++k)
        if (relu_mask && !(m[k] > 0.f)) g[k] = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        float o[VW];
#pragma unroll
        for (int k = 0; k < VW; ++k) o[k] = am[k] == q ? g[k] : 0.f;
        stvec<VW>(dx, dt, (((long)n * H + 2 * i + (q >> 1)) * W + 2 * j + (q & 1)) * C + c, o);
    }
}

// The bf16 form for C = 8 CL channels (CL = 8, 16, 32: the VGG pools, C = 64 / 128 / 256), laid
// out for whole-row memory transactions: 2 CL lanes per pooled pixel, lane (b, chunk) reading
// input column 2j + b of both rows as 16-byte pieces, so one wave instruction covers
// 64 / (2 CL) pooled pixels' 2 C contiguous channels (maxpool_bwd_kernel's thread per pooled
// pixel read every other 128-256 B segment).  The partner column's values come by lane
// exchange; the argmax is taken in maxpool_bwd_kernel's order over the four window positions
// (first maximum, NaN wins), so dx is bit-identical.
template <int CL>
IRGAN_HD uint32_t xchg(uint32_t v) {   // value of lane ^ CL
    if constexpr (CL < 16) return (uint32_t)__float_as_int(dpp_xor16<CL>(__int_as_float((int)v)));
    else return (uint32_t)__shfl_xor((int)v, CL, 64);
}
template <int CL>
__global__ __launch_bounds__(TPB) void maxpool_bwd_rows_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
                                                               int H, int W, bf16_t* __restrict__ dx, int relu_mask) {
    constexpr int C = CL * 8, PPW = 64 / (2 * CL);  // pooled pixels per wave
    const int Ho = H / 2, Wo = W / 2;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int n = blockIdx.y / Ho, i = blockIdx.y - n * Ho;
    const int b = (lane / CL) & 1, ch = lane % CL;
    const int j = (blockIdx.x * (TPB / 64) + wv) * PPW + lane / (2 * CL);
    const bool on = j < Wo;   // whole pixel groups: the partner lane has the same j
    const long r0 = ((long)n * H + 2 * i) * W + 2 * j + b, r1 = r0 + W;
    uint4 x0 = make_uint4(0u, 0u, 0u, 0u), x1 = x0, g4 = x0;
    if (on) {
        x0 = *(const uint4*)(x + r0 * C + ch * 8);
        x1 = *(const uint4*)(x + r1 * C + ch * 8);
        g4 = *(const uint4*)(dy + (((long)n * Ho + i) * Wo + j) * C + ch * 8);
    }
    const uint32_t own0[4] = {x0.x, x0.y, x0.z, x0.w}, own1[4] = {x1.x, x1.y, x1.z, x1.w};
    uint32_t oth0[4], oth1[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        oth0[k] = xchg<CL>(own0[k]);
        oth1[k] = xchg<CL>(own1[k]);
    }
    if (!on) return;
    const uint32_t gw[4] = {g4.x, g4.y, g4.z, g4.w};
    uint32_t o0[4], o1[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        // window order q = 2a + b': (0,0), (0,1), (1,0), (1,1)
        const uint32_t q[4] = {b ? oth0[k] : own0[k], b ? own0[k] : oth0[k], b ? oth1[k] : own1[k],
                               b ? own1[k] : oth1[k]};
        float r[2][2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            float m = -INFINITY;
            int am = 0;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const float v = __uint_as_float(h ? q[t] & 0xffff0000u : q[t] << 16);
                if (v > m || isnan(v)) { m = v; am = t; }
            }
            float gv = __uint_as_float(h ? gw[k] & 0xffff0000u : gw[k] << 16);
            if (relu_mask && !(m > 0.f)) gv = 0.f;
            r[0][h] = am == b ? gv : 0.f;        // row 2i, this lane's column
            r[1][h] = am == 2 + b ? gv : 0.f;    // row 2i + 1
        }
        o0[k] = pk_bf16(r[0][0], r[0][1]);
        o1[k] = pk_bf16(r[1][0], r[1][1]);
    }
    *(uint4*)(dx + r0 * C + ch * 8) = make_uint4(o0[0], o0[1], o0[2], o0[3]);
    *(uint4*)(dx + r1 * C + ch * 8) = make_uint4(o1[0], o1[1], o1[2], o1[3]);
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

// nn.Dropout(p), training mode (ResnetBlock use_dropout, ir:394-395): keep element e with
// probability 1 - p from a counter-based hash of (seed, e), e = pixel * C + channel, and
// scale kept values by 1 / (1 - p).  The backward is the same launch on the gradient
// (same seed: same mask, same scale), so no mask is stored.
IRGAN_HD uint64_t mix64(uint64_t z) {  // splitmix64 finaliser
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
__global__ __launch_bounds__(TPB) void dropout_kernel(const void* x, int xdt, int ldx, int xoff,
                                                      void* y, int ydt, int ldy, int yoff, int C,
                                                      long total, uint64_t seed, uint32_t thresh, float scale) {
    for (long idx = blockIdx.x * (long)TPB + threadIdx.x; idx < total; idx += (long)gridDim.x * TPB) {
        const long p = idx / C;
        const int c = (int)(idx - p * C);
        const uint32_t u = (uint32_t)(mix64(seed + 0x9e3779b97f4a7c15ull * (uint64_t)(idx + 1)) >> 40);  // 24 bits
        const float v = ldv(x, xdt, p * ldx + xoff + c);
        stv(y, ydt, p * ldy + yoff + c, u >= thresh ? v * scale : 0.f);
    }
}

int nblocks(long total) { return (int)std::max<long>(1, std::min<long>((total + TPB - 1) / TPB, 16384)); }

}  // namespace

#define RS_CHECK(total) \
    if ((total) <= 0) return 0

// ---- per-axis tables (host only) -------------------------------------------
namespace {
int refl_host(int q, int n) {
    q = q < 0 ? -q : q;
    return q >= n ? 2 * n - 2 - q : q;
}
struct Tab {
    int n_out, T;
    int32_t* idx;
    float* w;
    int add(int row, int i, float wt) {  // merge duplicate indices
        for (int k = 0; k < T; ++k) {
            if (w[row * T + k] != 0.f && idx[row * T + k] == i) { w[row * T + k] += wt; return 0; }
        }
        for (int k = 0; k < T; ++k) {
            if (w[row * T + k] == 0.f) { idx[row * T + k] = i; w[row * T + k] = wt; return 0; }
        }
        return -1;  // table too narrow
    }
};
// forward map of `kind` on an axis of length n_in: calls add(out_row, in_index, weight)
template <typename F>
int axis_map(int kind, int n_in, int p, F&& add) {
    const float f3[3] = {0.25f, 0.5f, 0.25f};
    if (kind == 0) {  // Downsample: reflect pad 1, [1,2,1]/4, stride 2 (ir:269-310)
        const int n_out = (n_in - 1) / 2 + 1;
        for (int o = 0; o < n_out; ++o)
            for (int a = 0; a < 3; ++a)
                if (add(o, refl_host(2 * o + a - 1, n_in), f3[a])) return -1;
        return n_out;
    }
    if (kind == 1) {  // UpsampleAA: bilinear x2 align_corners=True, reflect pad 1, blur (ir:313-355)
        const int n2 = 2 * n_in;
        const float scale = n_in > 1 ? (float)(n_in - 1) / (float)(n2 - 1) : 0.f;
        for (int o = 0; o < n2; ++o)
            for (int a = 0; a < 3; ++a) {
                const int v = refl_host(o + a - 1, n2);
                const float r = scale * (float)v;
                const int i0 = (int)r, i1 = i0 + (i0 < n_in - 1 ? 1 : 0);
                const float l1 = r - (float)i0, l0 = 1.f - l1;
                if (add(o, i0, f3[a] * l0)) return -1;
                if (l1 != 0.f && add(o, i1, f3[a] * l1)) return -1;
            }
        return n2;
    }
    if (kind == 2) {  // nn.ReflectionPad2d(p): padded coordinate u reads refl(u - p)
        const int n_out = n_in + 2 * p;
        for (int u = 0; u < n_out; ++u)
            if (add(u, refl_host(u - p, n_in), 1.f)) return -1;
        return n_out;
    }
    return -1;
}
}  // namespace

extern "C" int irgan_resample_table(int32_t kind, int32_t n_in, int32_t p, int32_t transpose, int32_t* idx,
                                    float* w, int32_t tmax, int32_t rows_cap) {
    // forward: rows = output coordinates; transpose: rows = input coordinates (adjoint map)
    int n_out_fwd = axis_map(kind, n_in, p, [](int, int, float) { return 0; });
    if (n_out_fwd < 0) return -IRGAN_EINVAL;
    const int rows = transpose ? n_in : n_out_fwd;
    if (rows > rows_cap) return -IRGAN_EINVAL;
    for (long i = 0; i < (long)rows * tmax; ++i) { idx[i] = 0; w[i] = 0.f; }
    Tab t{rows, tmax, idx, w};
    int rc = axis_map(kind, n_in, p, [&](int o, int i, float wt) {
        return transpose ? t.add(i, o, wt) : t.add(o, i, wt);
    });
    return rc < 0 ? -IRGAN_EUNSUPPORTED : rows;
}

extern "C" int irgan_sep_resample(const void* in, int32_t in_dtype, int32_t N, int32_t Hin, int32_t Win, int32_t C,
                                  int32_t ldi, int32_t offi, void* out, int32_t out_dtype, int32_t Hout, int32_t Wout,
                                  int32_t ldo, int32_t offo, const int32_t* ty, const float* wy, int32_t Ty,
                                  const int32_t* tx, const float* wx, int32_t Tx, int32_t accumulate,
                                  irgan_stream_t s) {
    const bool vec = (C % 8 == 0) && (ldi % 8 == 0) && (offi % 8 == 0) && (ldo % 8 == 0) && (offo % 8 == 0);
    const int VW = vec ? 8 : 1;
    if ((long)N * Hout * Wout * C <= 0) return 0;
    if (Ty < 1 || Tx < 1) return IRGAN_EINVAL;
    static const bool use_lds = !getenv("IRGAN_NO_SEP_LDS");
    const int TM = Ty > Tx ? Ty : Tx;
    if (use_lds && !accumulate &&
        sep_pipe_launch(in, in_dtype, N, Hin, Win, C, ldi, offi, out, out_dtype, Hout, Wout, ldo, offo, ty, wy, Ty, tx,
                        wx, Tx, nullptr, 0, nullptr, (hipStream_t)s)) {
        IRGAN_LAUNCH_CHECK();
        return 0;
    }
    if (vec && use_lds && TM <= 8) {
        // channel group: the widest of 128..8 dividing C whose fp32 row [Win][CB] fits the cap
        const int nt = sep_nt();
        int CB = 0;
        for (int cb = 128; cb >= 8 && !CB; cb >>= 1)
            if (C % cb == 0 && (long)Win * cb <= 16384 * nt / 1024) CB = cb;
        if (CB) {
            dim3 g(N * Hout, C / CB);
            const size_t sh = (size_t)Win * CB * 4;
            hipStream_t st = (hipStream_t)s;
#define SEPL(T, NTV)                                                                                                 \
    sep_lds_kernel<T, false, NTV><<<g, NTV, sh, st>>>(in, in_dtype, Hin, Win, ldi, offi, out, out_dtype, Hout, Wout,   \
                                                      ldo, offo, ty, wy, Ty, tx, wx, Tx, accumulate, CB, nullptr, 0,   \
                                                      0, sep_swz())
#define SEPT(NTV)                          \
    if (TM <= 2) SEPL(2, NTV);             \
    else if (TM <= 4) SEPL(4, NTV);        \
    else if (TM <= 6) SEPL(6, NTV);        \
    else SEPL(8, NTV);
            if (nt == 256) { SEPT(256) } else if (nt == 512) { SEPT(512) } else { SEPT(1024) }
#undef SEPT
#undef SEPL
            IRGAN_LAUNCH_CHECK();
            return 0;
        }
    }
    if ((long)N * Hout > 65535) return IRGAN_EUNSUPPORTED;
    dim3 g(irgan_cdiv((long)Wout * (C / VW), TPB), N * Hout);
    if (vec)
        sep_kernel<8><<<g, TPB, 0, (hipStream_t)s>>>(in, in_dtype, Hin, Win, C, ldi, offi, out, out_dtype, Hout, Wout,
                                                     ldo, offo, ty, wy, Ty, tx, wx, Tx, accumulate);
    else
        sep_kernel<1><<<g, TPB, 0, (hipStream_t)s>>>(in, in_dtype, Hin, Win, C, ldi, offi, out, out_dtype, Hout, Wout,
                                                     ldo, offo, ty, wy, Ty, tx, wx, Tx, accumulate);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

// out = (Wy (x) Wx) act(IN(in)) with IN's per-(n, c) {mean, rstd} table mr (the
// InstanceNorm apply fused into the resample that consumes it); the LDS form only
// (IRGAN_EUNSUPPORTED otherwise: the caller applies the norm itself, then resamples).
extern "C" int irgan_sep_resample_in(const void* in, int32_t in_dtype, int32_t N, int32_t Hin, int32_t Win,
                                     int32_t C, int32_t ldi, int32_t offi, const float* mr, int32_t act, void* out,
                                     int32_t out_dtype, int32_t Hout, int32_t Wout, int32_t ldo, int32_t offo,
                                     const int32_t* ty, const float* wy, int32_t Ty, const int32_t* tx,
                                     const float* wx, int32_t Tx, irgan_stream_t s) {
    if (!mr) return IRGAN_EINVAL;
    const bool vec = (C % 8 == 0) && (ldi % 8 == 0) && (offi % 8 == 0) && (ldo % 8 == 0) && (offo % 8 == 0);
    if ((long)N * Hout * Wout * C <= 0) return 0;
    if (Ty < 1 || Tx < 1) return IRGAN_EINVAL;
    const int TM = Ty > Tx ? Ty : Tx;
    if (!vec || TM > 8 || getenv("IRGAN_NO_SEP_LDS") || getenv("IRGAN_NO_IN_RESAMPLE")) return IRGAN_EUNSUPPORTED;
    if (sep_pipe_launch(in, in_dtype, N, Hin, Win, C, ldi, offi, out, out_dtype, Hout, Wout, ldo, offo, ty, wy, Ty, tx,
                        wx, Tx, mr, act, nullptr, (hipStream_t)s)) {
        IRGAN_LAUNCH_CHECK();
        return 0;
    }
    const int nt = sep_nt();
    int CB = 0;
    for (int cb = 128; cb >= 8 && !CB; cb >>= 1)
        if (C % cb == 0 && (long)Win * cb <= 16384 * nt / 1024) CB = cb;
    if (!CB) return IRGAN_EUNSUPPORTED;
    dim3 g(N * Hout, C / CB);
    const size_t sh = (size_t)Win * CB * 4;
    hipStream_t st = (hipStream_t)s;
#define SEPN(T, NTV)                                                                                               \
    sep_lds_kernel<T, true, NTV><<<g, NTV, sh, st>>>(in, in_dtype, Hin, Win, ldi, offi, out, out_dtype, Hout, Wout, \
                                                     ldo, offo, ty, wy, Ty, tx, wx, Tx, 0, CB, mr, C, act, sep_swz())
#define SEPT(NTV)                          \
    if (TM <= 2) SEPN(2, NTV);             \
    else if (TM <= 4) SEPN(4, NTV);        \
    else if (TM <= 6) SEPN(6, NTV);        \
    else SEPN(8, NTV);
    if (nt == 256) { SEPT(256) } else if (nt == 512) { SEPT(512) } else { SEPT(1024) }
#undef SEPT
#undef SEPN
    IRGAN_LAUNCH_CHECK();
    return 0;
}

// irgan_sep_resample (mr == NULL) / irgan_sep_resample_in (mr: act(IN(in)) on load) into a
// bf16 out, no accumulate, that also writes out's e4m3 copy y8 (ld8 / off8: an NHWC slice) with
// the quantisation factor q[0] and raises max |bf16(out)| into the amax slot (the LDS form only:
// IRGAN_EUNSUPPORTED otherwise, nothing launched)
extern "C" int irgan_sep_resample_fp8(const void* in, int32_t in_dtype, int32_t N, int32_t Hin, int32_t Win,
                                      int32_t C, int32_t ldi, int32_t offi, const float* mr, int32_t act, void* out,
                                      int32_t out_dtype, int32_t Hout, int32_t Wout, int32_t ldo, int32_t offo,
                                      const int32_t* ty, const float* wy, int32_t Ty, const int32_t* tx,
                                      const float* wx, int32_t Tx, void* y8, int32_t ld8, int32_t off8,
                                      const float* q, uint32_t* amax, irgan_stream_t s) {
    if (!in || !out || !y8 || !q || !amax) return IRGAN_EINVAL;
    const bool vec = (C % 8 == 0) && (ldi % 8 == 0) && (offi % 8 == 0) && (ldo % 8 == 0) && (offo % 8 == 0) &&
                     ld8 % 8 == 0 && off8 % 8 == 0;
    if ((long)N * Hout * Wout * C <= 0) return 0;
    if (Ty < 1 || Tx < 1) return IRGAN_EINVAL;
    const int TM = Ty > Tx ? Ty : Tx;
    if (!vec || TM > 8 || out_dtype != IRGAN_BF16) return IRGAN_EUNSUPPORTED;
    const ResQ8 q8{(uint8_t*)y8, ld8, off8, q, amax};
    if (sep_pipe_launch(in, in_dtype, N, Hin, Win, C, ldi, offi, out, out_dtype, Hout, Wout, ldo, offo, ty, wy, Ty, tx,
                        wx, Tx, mr, act, &q8, (hipStream_t)s)) {
        IRGAN_LAUNCH_CHECK();
        return 0;
    }
    const int nt = sep_nt();
    int CB = 0;
    for (int cb = 128; cb >= 8 && !CB; cb >>= 1)
        if (C % cb == 0 && (long)Win * cb <= 16384 * nt / 1024) CB = cb;
    if (!CB) return IRGAN_EUNSUPPORTED;
    dim3 g(N * Hout, C / CB);
    const size_t sh = (size_t)Win * CB * 4;
    hipStream_t st = (hipStream_t)s;
#define SEPQ(T, NORMV)                                                                                            \
    sep_lds_kernel<T, NORMV, 512, true><<<g, 512, sh, st>>>(in, in_dtype, Hin, Win, ldi, offi, out, out_dtype, Hout, \
                                                            Wout, ldo, offo, ty, wy, Ty, tx, wx, Tx, 0, CB, mr, C,    \
                                                            act, sep_swz(), q8)
#define SEPT(NORMV)                  \
    if (TM <= 2) SEPQ(2, NORMV);     \
    else if (TM <= 4) SEPQ(4, NORMV); \
    else if (TM <= 6) SEPQ(6, NORMV); \
    else SEPQ(8, NORMV);
    if (mr) { SEPT(true) } else { SEPT(false) }
#undef SEPT
#undef SEPQ
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_reflect_ring_fold(const float* rows, const float* cols, int32_t nsplit, int32_t N, int32_t H,
                                      int32_t W, int32_t C, int32_t p, void* dx, int32_t dx_dtype, int32_t lddx,
                                      int32_t dxoff, irgan_stream_t s) {
    if ((long)N * H * W * C <= 0 || p <= 0) return 0;
    if ((long)N * H > 65535 || p >= H || p >= W || nsplit < 1) return IRGAN_EUNSUPPORTED;
    const bool vec = C % 8 == 0 && lddx % 8 == 0 && dxoff % 8 == 0;
    if (vec) {
        dim3 gr(irgan_cdiv((long)W * (C / 8), TPB), N * H);
        ring_fold_kernel<8><<<gr, TPB, 0, (hipStream_t)s>>>(rows, cols, nsplit, N, H, W, C, p, dx, dx_dtype, lddx,
                                                            dxoff);
    } else {
        dim3 gr(irgan_cdiv((long)W * C, TPB), N * H);
        ring_fold_kernel<1><<<gr, TPB, 0, (hipStream_t)s>>>(rows, cols, nsplit, N, H, W, C, p, dx, dx_dtype, lddx,
                                                            dxoff);
    }
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_maxpool_fwd(const void* x, int32_t dt, int32_t N, int32_t H, int32_t W, int32_t C, void* y,
                                 irgan_stream_t s) {
    long total = (long)N * (H / 2) * (W / 2) * C;
    RS_CHECK(total);
    if ((long)N * (H / 2) > 65535) return IRGAN_EUNSUPPORTED;
    if (C % 8 == 0) {
        dim3 g(irgan_cdiv((long)(W / 2) * (C / 8), TPB), N * (H / 2));
        maxpool_fwd_kernel<8><<<g, TPB, 0, (hipStream_t)s>>>(x, dt, H, W, C, y);
    } else {
        dim3 g(irgan_cdiv((long)(W / 2) * C, TPB), N * (H / 2));
        maxpool_fwd_kernel<1><<<g, TPB, 0, (hipStream_t)s>>>(x, dt, H, W, C, y);
    }
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_maxpool_bwd(const void* x, const void* dy, int32_t dt, int32_t N, int32_t H, int32_t W, int32_t C,
                                 void* dx, int32_t relu_mask, irgan_stream_t s) {
    long total = (long)N * (H / 2) * (W / 2) * C;
    RS_CHECK(total);
    if ((long)N * (H / 2) > 65535) return IRGAN_EUNSUPPORTED;
    static const bool rows = !getenv("IRGAN_NO_POOL_ROWS");
    if (rows && dt == IRGAN_BF16 && (C == 64 || C == 128 || C == 256)) {
        const int ppb = (TPB / 64) * (64 / (2 * (C / 8)));   // pooled pixels per block
        dim3 g(irgan_cdiv(W / 2, ppb), N * (H / 2));
        const bf16_t *xp = (const bf16_t*)x, *gp = (const bf16_t*)dy;
        if (C == 64) maxpool_bwd_rows_kernel<8><<<g, TPB, 0, (hipStream_t)s>>>(xp, gp, H, W, (bf16_t*)dx, relu_mask);
        else if (C == 128) maxpool_bwd_rows_kernel<16><<<g, TPB, 0, (hipStream_t)s>>>(xp, gp, H, W, (bf16_t*)dx, relu_mask);
        else maxpool_bwd_rows_kernel<32><<<g, TPB, 0, (hipStream_t)s>>>(xp, gp, H, W, (bf16_t*)dx, relu_mask);
    } else if (C % 8 == 0) {
        dim3 g(irgan_cdiv((long)(W / 2) * (C / 8), TPB), N * (H / 2));
        maxpool_bwd_kernel<8><<<g, TPB, 0, (hipStream_t)s>>>(x, dy, dt, H, W, C, dx, relu_mask);
    } else {
        dim3 g(irgan_cdiv((long)(W / 2) * C, TPB), N * (H / 2));
        maxpool_bwd_kernel<1><<<g, TPB, 0, (hipStream_t)s>>>(x, dy, dt, H, W, C, dx, relu_mask);
    }
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

extern "C" int irgan_dropout(const void* x, int32_t xdt, int32_t P, int32_t C, int32_t ldx, int32_t xoff, void* y,
                             int32_t ydt, int32_t ldy, int32_t yoff, uint64_t seed, float p, irgan_stream_t s) {
    const long total = (long)P * C;
    RS_CHECK(total);
    if (!x || !y || !(p >= 0.f && p < 1.f)) return IRGAN_EINVAL;
    const uint32_t thresh = (uint32_t)(p * 16777216.f);  // keep iff u24 >= p * 2^24
    dropout_kernel<<<nblocks(total), TPB, 0, (hipStream_t)s>>>(x, xdt, ldx, xoff, y, ydt, ldy, yoff, C, total, seed,
                                                                thresh, 1.f / (1.f - p));
    IRGAN_LAUNCH_CHECK();
    return 0;
}
