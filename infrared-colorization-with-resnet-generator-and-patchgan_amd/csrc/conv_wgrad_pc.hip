// bf16 backward-weight convolution, producer/consumer form (3x3, stride 1,
// Cout % 64 == 0, Cin % 64 == 0, Wo % 64 == 0): the ResnetBlock weight
// gradients (ir:390, 411) and the encoder / decoder 3x3 convs that qualify
// (down1, down2, up1_conv, up2_conv: ir:470, 478, 504, 520).  co tiles of 128 (BMC 128,
// Cout % 128 == 0) or 64 (BMC 64: up2_conv's 64 output channels; its dY rows are 128 B
// and use the X span's swizzle).
//
//   dW[co][ty][tx][ci] += sum_p dY[p][co] * X[iy(p, ty)][ix(p, tx)][ci]
//
// Same work decomposition as conv_wgrad_halo.hip: a block owns (BMC-channel co
// tile, 64-channel ci chunk, kernel row ty, all three tx taps) and walks 64-pixel
// row segments of dY (split-K over segments); per segment the dY tile
// [64 px][BMC co] and ONE input row span [66][64 ci] sit in LDS and the three tx
// taps are row shifts of the span.  What is different is who does what
// (measured on the halo kernel: 5 VALU per MFMA, fragment reads and DMA issue
// serialised with the MFMAs):
//
//  * 8 waves: waves 0-3 only compute (one per SIMD), waves 4-7 only load (one
//    per SIMD).  A loader wave issues its ~6 LDS-DMA pieces per segment with
//    precomputed per-lane offsets (dY: a lane-invariant offset + the segment's
//    scalar soffset; X span: a few VALU per piece for the reflect / zero edge),
//    so the compute waves issue no VMEM and almost no VALU;
//  * 4-stage LDS ring (4 x 25 KiB at BMC 128, 4 x 17 KiB at 64), one s_barrier per segment, the DMA two
//    segments ahead of its consumer: the loaders retire segment k+1 with a
//    counted vmcnt before barrier k, then issue segment k+3 into the stage that
//    segment k-1 (fully consumed before barrier k) used;
//  * compute waves keep two fragment register sets: the reads of the next half
//    segment (32 pixels) are issued before the MFMAs of the current one, and
//    every fragment address is a precomputed per-lane offset plus the stage base
//    (the read for pixel rows +4 / +32 is an immediate offset: the XOR swizzles
//    below do not change over those steps).
//
// LDS images (conflict-free ds_read_b64_tr_b16, as conv_wgrad_halo.hip):
//   dY, 256-B rows (BMC 128): 16-B chunk XOR 2*((r&3)|((r>>3&1)<<2));
//   X span and dY at BMC 64, 128-B rows: chunk XOR 2*((r>>1&1)|((r>>3&1)<<1)).
// Split-K partials go to a caller slab (plain stores, ordered reduce) or, with
// no slab, fp32 atomics into dW.
#include "common.h"

#ifndef PC_EXP
#define PC_EXP 0  // A/B timing experiments only (tools/build_variant.sh); 0 = the real kernel
#endif
// bits: 1 loaders skip the in-loop vmcnt wait, 2 no DMA in the loop, 4 no fragment reads, 8 no barriers,
// 16 compiler-scheduled reads (no sched_group_barrier), 32 s_setprio 1 on the compute waves
#define PCX(b) ((PC_EXP & (b)) != 0)

namespace {

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s4;

IRGAN_HD int pc_t128(int r) { return ((r >> 1) & 1) | (((r >> 3) & 1) << 1); }
IRGAN_HD int pc_t256(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }

constexpr int XPIECES = 9;               // 72 X span positions, 8 per piece
#ifndef WGPC_LW
#define WGPC_LW 4   // loader waves per block (8: twice the DMA issue slots, 1024 threads, <= 128 VGPRs)
#endif
#ifndef WGPC_STAGES
#define WGPC_STAGES 4
#endif
// LDS ring depth: segment k + STAGES - 1 is issued after barrier k, so STAGES - 2
// segments are in flight while segment k + 1 is read (4: 100 KiB at BMC 128; 6: 150 KiB)
// (BMC 64 keeps 4 stages: two of its blocks share a CU)
template <int BMC>
constexpr int stages_of() { return BMC == 128 ? WGPC_STAGES : 4; }
static_assert(WGPC_STAGES >= 4, "the schedule needs segment k-1's stage free after barrier k");

// wait until at most c segments of this loader's pieces (np per segment: PPL or PPL - 1)
// are outstanding, c wave-uniform in [0, C]
template <int PPL, int C>
IRGAN_HD void wait_segs(int c, bool full) {
    if constexpr (C == 0) {
        wait_vmcnt<0>();
    } else {
        if (c >= C) {
            if (full) wait_vmcnt<C * PPL>(); else wait_vmcnt<C * (PPL - 1)>();
        } else {
            wait_segs<PPL, C - 1>(c, full);
        }
    }
}
// BMC: co tile (128 or 64).  CW compute waves: 4 -> BMC co x 48 n per wave (1 per SIMD);
// 8 -> BMC/2 co x 48 n (2 per SIMD)
template <int BMC, int CW>
struct PC {
    static constexpr int DYR = BMC * 2;             // dY tile row bytes
    static constexpr int APIECES = 64 * DYR / 1024; // dY tile pieces (16 of 4 rows / 8 of 8 rows)
    static constexpr int TP = APIECES + XPIECES;    // pieces per segment (25 / 17)
    static constexpr int STAGE = TP * 1024;
    static constexpr int LW = WGPC_LW;              // loader waves
    static constexpr int PPL = (TP + LW - 1) / LW;  // max pieces per loader wave (LW 4: 7 / 5)
    static constexpr int MI = BMC / 16 / (CW / 4);  // co fragments per compute wave
    static constexpr int NT = (CW + LW) * 64;       // threads: CW compute + LW loader waves
    static_assert(TP % LW == 1, "loader 0 takes PPL pieces, the others PPL - 1");
};
template <int BMC>
IRGAN_HD int pc_dsw(int r) { return BMC == 128 ? pc_t256(r) : pc_t128(r); }  // dY row swizzle

IRGAN_HD uint4 ld_tr_pair(const char* lo, const char* hi) {
    const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)lo);
    const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)hi);
    uint4 out;
    __builtin_memcpy(&out, &a, 8);
    __builtin_memcpy((char*)&out + 8, &b, 8);
    return out;
}

template <int MI, int NJ>
struct Frag {
    uint4 a[MI], b[NJ];
};

// KW: 3 or 4 taps per kernel row (NJ = KW (tx, 16-ci) fragments per compute wave).
// PAIR (Wo <= 32: D model.8, 31 wide): a 64-pixel segment is TWO output rows of 32 (pixel
// 32 h + c of row oy0 + h), and the X span holds both input rows: positions [36 h, 36 h +
// 35) are row h's, so k-step h reads position 36 h + k + tx.
template <int BMC, int CW, int KW = 3, bool PAIR = false>
__global__ __launch_bounds__((PC<BMC, CW>::NT), 1) void wgrad_pc_kernel(const irgan_conv_desc d, const bf16_t* __restrict__ x,
                                                          const bf16_t* __restrict__ dy, float* __restrict__ dw,
                                                          int segs_per_block, int nseg, int ntco, int nci, int swz,
                                                          float* __restrict__ slab) {
    using Q = PC<BMC, CW>;
    constexpr int STAGES = stages_of<BMC>();
    constexpr int APIECES = Q::APIECES, TP = Q::TP, STAGE = Q::STAGE, PPL = Q::PPL, DYR = Q::DYR;
    constexpr int DROWS = 1024 / DYR;  // dY rows per piece
    constexpr int NJ = KW, XPOS = 63 + KW;
    static_assert(KW == 3 || KW == 4, "taps per row");
    __shared__ __attribute__((aligned(1024))) char smem[STAGES * STAGE];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    constexpr int MI = Q::MI;
    const bool loader = wid >= CW;
    const int tiles = ntco * nci * d.KH;
    const int t = xcd_tile(blockIdx.x, gridDim.x, swz);
    const int split = t / tiles;
    int r = t - split * tiles;
    const int ty = r % d.KH;
    r /= d.KH;
    const int cic = r % nci, cot = r / nci;
    const int co0 = cot * BMC, ci0 = cic * 64;
    const int s_beg = split * segs_per_block;
    const int s_end = min(nseg, s_beg + segs_per_block);
    if (s_beg >= s_end) return;  // block-uniform
    const int nk = s_end - s_beg;
    const int segs_row = d.Wo / 64;

    if (loader) {
        // ------------------------------------------------------------------
        // loader wave l issues pieces j = l, l+4, ... (< TP) of every segment
        constexpr int LW = Q::LW;
        const int l = wid - CW;
        const int np = (TP - l + LW - 1) / LW;  // PPL for l = 0, else PPL - 1
        const bool reflect = d.pad_mode == IRGAN_PAD_REFLECT;
        // dY: buffer base at dy + yoff + co0; lane offset fixed per piece, the
        // segment's first pixel enters as the scalar soffset
        const i32x4 rs_dy = make_rsrc(dy + d.yoff + co0,
                                      (uint32_t)(((long)d.N * d.Ho * d.Wo * d.ldy - d.yoff - co0) * 2));
        const i32x4 rs_x = make_rsrc(x + d.xoff + ci0, (uint32_t)(((long)d.N * d.H * d.W * d.ldx - d.xoff - ci0) * 2));
        const int cout8 = (d.Cout + 7) / 8 * 8;
        uint32_t voff[PPL];
        int xpos[PPL], xc16[PPL];
        uint32_t second = 0;  // PAIR: bit u set when piece u's lane row is in the segment's 2nd output row
#pragma unroll
        for (int u = 0; u < PPL; ++u) {
            const int j = l + LW * u;
            voff[u] = IRGAN_OOB;
            xpos[u] = 0;
            xc16[u] = 0;
            if (j < APIECES) {
                const int pos = j * DROWS + lane / (64 / DROWS), slot = lane % (64 / DROWS);
                const int c16 = slot ^ (2 * pc_dsw<BMC>(pos));
                // PAIR: tile row pos = pixel (pos & 31) of output row pos >> 5 (masked past Wo)
                const int mpix = PAIR ? (pos >> 5) * d.Wo + (pos & 31) : pos;
                const bool pix_ok = !PAIR || (pos & 31) < d.Wo;
                if (PAIR && pos >= 32) second |= 1u << u;
                if (co0 + c16 * 8 < cout8 && pix_ok) voff[u] = (uint32_t)((mpix * d.ldy + c16 * 8) * 2);
            } else if (j < TP) {
                const int pos = (j - APIECES) * 8 + (lane >> 3), slot = lane & 7;
                xpos[u] = pos;
                xc16[u] = (slot ^ (2 * pc_t128(pos))) * 16;  // byte offset of the lane's 16-B chunk
            }
        }
        const int hpair = (d.Ho + 1) >> 1;  // PAIR: row pairs per image
        auto issue = [&](int s, int stage) {
            int n, oy, x0;
            if (PAIR) {
                n = s / hpair;
                oy = (s - n * hpair) * 2;
                x0 = 0;
            } else {
                const int rowi = s / segs_row;
                x0 = (s - rowi * segs_row) * 64;
                n = rowi / d.Ho;
                oy = rowi - n * d.Ho;
            }
            const bool second_ok = !PAIR || oy + 1 < d.Ho;
            int iy0 = oy * d.sy + ty + d.c0y, iy1 = (oy + 1) * d.sy + ty + d.c0y;
            if (reflect) {
                iy0 = reflect_idx(iy0, d.H);
                iy1 = reflect_idx(iy1, d.H);
            }
            const bool row0_ok = (unsigned)iy0 < (unsigned)d.H, row1_ok = second_ok && (unsigned)iy1 < (unsigned)d.H;
            const uint32_t dy_soff = (uint32_t)((((long)n * d.Ho + oy) * d.Wo + x0) * d.ldy * 2);
            const long xrow0 = ((long)n * d.H + iy0) * d.W, xrow1 = ((long)n * d.H + iy1) * d.W;
            char* base = smem + stage * STAGE;
#pragma unroll
            for (int u = 0; u < PPL; ++u) {
                if (u >= np) break;
                const int j = l + LW * u;
                if (j < APIECES) {
                    const uint32_t vo = (PAIR && !second_ok && ((second >> u) & 1)) ? IRGAN_OOB : voff[u];
                    blds16(rs_dy, vo, dy_soff, base + j * 1024);
                } else {
                    const bool hi = PAIR && xpos[u] >= 36;
                    const int xp = hi ? xpos[u] - 36 : xpos[u];
                    int ix = x0 + d.c0x + xp;
                    if (reflect) ix = reflect_idx(ix, d.W);
                    const bool ok = (hi ? row1_ok : row0_ok) & (xp < (PAIR ? 32 + KW - 1 : XPOS)) &
                                    ((unsigned)ix < (unsigned)d.W);
                    const uint32_t off = ok ? (uint32_t)(((hi ? xrow1 : xrow0) + ix) * d.ldx * 2) + xc16[u] : IRGAN_OOB;
                    blds16(rs_x, off, base + j * 1024);
                }
            }
        };
        // prologue: segments 0..STAGES-2 in flight, retire segment 0
        for (int k = 0; k < STAGES - 1; ++k)
            if (k < nk) issue(s_beg + k, k);
        wait_segs<PPL, STAGES - 2>(min(nk - 1, STAGES - 2), np == PPL);
        lds_barrier();
        for (int kt = 0; kt < nk; ++kt) {
            // retire segment kt+1 (segments kt+2 .. kt+STAGES-2 may stay in flight), then barrier kt
            if (kt + 1 < nk && !PCX(1)) wait_segs<PPL, STAGES - 3>(min(nk - kt - 2, STAGES - 3), np == PPL);
#if !PCX(8)
            lds_barrier();
#endif
            if (kt + STAGES - 1 < nk && !PCX(2)) issue(s_beg + kt + STAGES - 1, (kt + STAGES - 1) % STAGES);
        }
        return;
    }

    // ----------------------------------------------------------------------
    // compute wave wn: co 128 x n 48 (fragments jj = 3 wn + j: tx = jj >> 2,
    // 16-ci group jj & 3), two 32-pixel k-steps per segment
    const int wn = wid & 3, wm = wid >> 2;  // n group, co group (CW = 8)
    const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
    const int k_lo = 8 * g + q;  // pixel row of the lane's low 4-row half (k-step 0)
    // per-lane byte offsets inside a stage (k-step 0, low half); +4 / +32 rows for the
    // high half / k-step 1 (the row swizzles do not change over those steps)
    int aoff[MI];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
        const int col = (wm * MI + i) * 16 + 4 * p, c16 = col >> 3, within = (col & 7) * 2;
        aoff[i] = k_lo * DYR + ((c16 ^ (2 * pc_dsw<BMC>(k_lo))) << 4) + within;
    }
    // [j][high half][k-step]: k-step 1 is the +32-row image of k-step 0 (the swizzle repeats)
    // except in PAIR mode, where it starts at position 36 (its own swizzle phase)
    constexpr int NH = PAIR ? 2 : 1;
    int boff[NJ][2][NH];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int jj = wn * NJ + j, tx = jj >> 2, col = (jj & 3) * 16 + 4 * p;
        const int c16 = col >> 3, within = (col & 7) * 2;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh)
#pragma unroll
            for (int h = 0; h < NH; ++h) {
                const int pos = 36 * h + k_lo + 4 * hh + tx;
                boff[j][hh][h] = APIECES * 1024 + pos * 128 + ((c16 ^ (2 * pc_t128(pos))) << 4) + within;
            }
    }
    f32x4 acc[MI][NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // MFMAs on `cur` with the 11 fragment-pair reads of `nxt` (stage, half h)
    // interleaved one pair per MFMA: the first MFMA retires cur's reads with no
    // newer read in flight, every later one needs no wait (lgkmcnt counts 15).
    auto step = [&](const Frag<MI, NJ>& cur, Frag<MI, NJ>& nxt, int stage, int h) {
        const char* S = smem + stage * STAGE + h * 32 * DYR;
        const char* X = smem + stage * STAGE + (PAIR ? 0 : h * 4096);
        const int hb = PAIR ? h : 0;
#pragma unroll
        for (int idx = 0; idx < MI * NJ; ++idx) {
            const int i = idx / NJ, j = idx % NJ;
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, cur.a[i]),
                                                                __builtin_bit_cast(bf16x8_t, cur.b[j]), acc[i][j], 0,
                                                                0, 0);
#if !PCX(4)
            if (idx < MI) nxt.a[idx] = ld_tr_pair(S + aoff[idx], S + aoff[idx] + 4 * DYR);
            else if (idx < MI + NJ)
                nxt.b[idx - MI] = ld_tr_pair(X + boff[idx - MI][0][hb], X + boff[idx - MI][1][hb]);
#else
            if (idx < MI) nxt.a[idx] = cur.a[idx] ^ make_uint4(idx, 1, 2, 3);
            else if (idx < MI + NJ) nxt.b[idx - MI] = cur.b[idx - MI] ^ make_uint4(idx, 1, 2, 3);
#endif
        }
#if !PCX(16)
#pragma unroll
        for (int k = 0; k < MI + NJ; ++k) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // 2 DS reads
        }
        __builtin_amdgcn_sched_group_barrier(0x008, MI * NJ - MI - NJ, 0);
#endif
    };
    auto barrier = [] {
        __builtin_amdgcn_sched_barrier(0);
#if !PCX(8)
        lds_barrier();
#endif
        __builtin_amdgcn_sched_barrier(0);
    };
    Frag<MI, NJ> f0, f1;
#if PCX(32)
    __builtin_amdgcn_s_setprio(1);  // compute waves win issue arbitration over the loaders
#endif
    barrier();  // prologue barrier: segment 0 landed
    {
        const char* S = smem;
#pragma unroll
        for (int i = 0; i < MI; ++i) f0.a[i] = ld_tr_pair(S + aoff[i], S + aoff[i] + 4 * DYR);
#pragma unroll
        for (int j = 0; j < NJ; ++j) f0.b[j] = ld_tr_pair(S + boff[j][0][0], S + boff[j][1][0]);
    }
    for (int kt = 0; kt < nk; ++kt) {
        step(f0, f1, kt % STAGES, 1);        // segment kt, pixels 0-31 | read pixels 32-63
        barrier();                           // barrier kt: segment kt+1 landed; segment kt-1 fully read
        step(f1, f0, (kt + 1) % STAGES, 0);  // segment kt, pixels 32-63 | read segment kt+1, pixels 0-31
    }                                        // (the last iteration's reads are unused)

    // C[row = co][col = n]: co = co0 + i*16 + 4g + rr, n = jj*16 + (lane & 15)
    const int K = d.KH * KW * d.Cin;
    float* const dst = slab ? slab + (long)split * d.Cout * K : nullptr;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            const int co = co0 + (wm * MI + i) * 16 + g * 4 + rr;
            if (co >= d.Cout) continue;
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int jj = wn * NJ + j, tx = jj >> 2;
                const int ci = ci0 + (jj & 3) * 16 + (lane & 15);
                const long o = (long)co * K + (ty * KW + tx) * d.Cin + ci;
                if (dst) dst[o] = acc[i][j][rr];
                else atomicAdd(dw + o, acc[i][j][rr]);
            }
        }
}

// ---- Wide-n variant for Cin % 128 == 0 (the ResnetBlock convs, ir:386-411): block = (128 co,
// 128 ci as TWO 64-channel planes of the X span, kernel row ty, the 3 tx taps), n = 384.  Per
// 64-pixel segment a block does twice the MFMAs of wgrad_pc_kernel<128, 8> for 34 DMA pieces
// instead of 25 and one barrier: fewer DMA issues, fragment reads (0.42 instead of 0.58 per
// MFMA) and barriers per MFMA.  A compute wave holds 4 co x 6 n fragments (96 accumulator
// VGPRs) and ONE operand set that it re-reads right after each fragment's last MFMA of the
// k-step (b[j] after its 4 MFMAs, a[i] in the last column), so the 12-wave block stays within
// 168 VGPRs; the other compute wave of the SIMD covers the reads' latency.  12 tiles x 21
// splits = 252 blocks (wgrad_pc_kernel: 24 x 10 = 240).  Resblock shape incl. the reduce:
// 93.8 -> 84.8 us (profiles/r04_w2_wgrad_ab.txt); the default wherever Cin % 128 == 0.
constexpr int W2_AP = 16;                    // dY tile: 64 px x 128 co x 2 B
constexpr int W2_XP = 2 * XPIECES;           // X span: 2 planes x 72 positions x 128 B
constexpr int W2_TP = W2_AP + W2_XP;         // 34 pieces per segment
constexpr int W2_STAGE = W2_TP * 1024;
constexpr int W2_LW = 4, W2_CW = 8, W2_NT = (W2_CW + W2_LW) * 64;
constexpr int W2_PPL = (W2_TP + W2_LW - 1) / W2_LW;  // 9 (loaders 0, 1) / 8 (loaders 2, 3)
constexpr int W2_STAGES = 4;                 // 136 KiB
// ablations for variant builds (tools/build_variant.sh -DW2_EXP=...): 1 no epilogue stores,
// 2 no DMA after the prologue (the MFMAs run on stale stages), 4 no MFMAs (operand reads kept),
// 8 fp32 atomics into dW instead of the split slabs + reduce
#ifndef W2_EXP
#define W2_EXP 0
#endif

// XCD-aware order for any grid size: XCD x (blocks b % 8 == x) takes a contiguous range of
// logical tiles (xcd_tile needs nb % 8 == 0)
IRGAN_HD int xcd_tile_any(int b, int nb) {
    const int x = b & 7, k = b >> 3, per = nb >> 3, rem = nb & 7;
    return x * per + (x < rem ? x : rem) + k;
}

__global__ __launch_bounds__(W2_NT, 1) void wgrad_w2_kernel(const irgan_conv_desc d, const bf16_t* __restrict__ x,
                                                            const bf16_t* __restrict__ dy, float* __restrict__ dw,
                                                            int segs_per_block, int nseg, int ntco, int nci2, int swz,
                                                            float* __restrict__ slab) {
    constexpr int DYR = 256, MI = 4, NJ = 6;
    __shared__ __attribute__((aligned(1024))) char smem[W2_STAGES * W2_STAGE];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int tiles = ntco * nci2 * d.KH;
    const int t = swz ? xcd_tile_any(blockIdx.x, gridDim.x) : blockIdx.x;
    const int split = t / tiles;
    int r = t - split * tiles;
    const int ty = r % d.KH;
    r /= d.KH;
    const int cic = r % nci2, cot = r / nci2;
    const int co0 = cot * 128, ci0 = cic * 128;
    const int s_beg = split * segs_per_block;
    const int s_end = min(nseg, s_beg + segs_per_block);
    if (s_beg >= s_end) return;  // block-uniform
    const int nk = s_end - s_beg;
    const int segs_row = (d.Wo + 63) / 64;  // the last segment of a row may be partial (Wo % 64)

    if (wid >= W2_CW) {
        // ------------------------------------------------------------------ loaders
        const int l = wid - W2_CW;
        const int np = (W2_TP - l + W2_LW - 1) / W2_LW;  // PPL (loaders 0, 1) or PPL - 1
        const bool reflect = d.pad_mode == IRGAN_PAD_REFLECT;
        const i32x4 rs_dy = make_rsrc(dy + d.yoff + co0,
                                      (uint32_t)(((long)d.N * d.Ho * d.Wo * d.ldy - d.yoff - co0) * 2));
        const i32x4 rs_x = make_rsrc(x + d.xoff + ci0, (uint32_t)(((long)d.N * d.H * d.W * d.ldx - d.xoff - ci0) * 2));
        uint32_t voff[W2_PPL];
        int xpos[W2_PPL], xc16[W2_PPL];
#pragma unroll
        for (int u = 0; u < W2_PPL; ++u) {
            const int j = l + W2_LW * u;
            voff[u] = IRGAN_OOB;
            xpos[u] = 0;
            xc16[u] = 0;
            if (j < W2_AP) {
                const int pos = j * 4 + lane / 16, slot = lane % 16;
                const int c16 = slot ^ (2 * pc_t256(pos));
                voff[u] = (uint32_t)((pos * d.ldy + c16 * 8) * 2);
                xpos[u] = pos;   // the dY pixel within the segment (a partial segment zero-fills past Wo)
            } else if (j < W2_TP) {
                const int jx = j - W2_AP, plane = jx / XPIECES;
                const int pos = (jx - plane * XPIECES) * 8 + (lane >> 3), slot = lane & 7;
                xpos[u] = pos;
                xc16[u] = ((slot ^ (2 * pc_t128(pos))) * 8 + plane * 64) * 2;  // byte offset: chunk + plane
            }
        }
        auto issue = [&](int s, int stage) {
            const int rowi = s / segs_row;
            const int x0 = (s - rowi * segs_row) * 64;
            const int n = rowi / d.Ho, oy = rowi - n * d.Ho;
            int iy = oy + ty + d.c0y;
            if (reflect) iy = reflect_idx(iy, d.H);
            const bool row_ok = (unsigned)iy < (unsigned)d.H;
            const uint32_t dy_soff = (uint32_t)((((long)n * d.Ho + oy) * d.Wo + x0) * d.ldy * 2);
            const long xrow = ((long)n * d.H + iy) * d.W;
            char* base = smem + stage * W2_STAGE;
#pragma unroll
            for (int u = 0; u < W2_PPL; ++u) {
                if (u >= np) break;
                const int j = l + W2_LW * u;
                if (j < W2_AP) {
                    blds16(rs_dy, x0 + xpos[u] < d.Wo ? voff[u] : IRGAN_OOB, dy_soff, base + j * 1024);
                } else {
                    int ix = x0 + d.c0x + xpos[u];
                    if (reflect) ix = reflect_idx(ix, d.W);
                    const bool ok = row_ok & (xpos[u] < 66) & ((unsigned)ix < (unsigned)d.W);
                    const uint32_t off = ok ? (uint32_t)((xrow + ix) * d.ldx * 2) + xc16[u] : IRGAN_OOB;
                    blds16(rs_x, off, base + j * 1024);
                }
            }
        };
        for (int k = 0; k < W2_STAGES - 1; ++k)
            if (k < nk) issue(s_beg + k, k);
        wait_segs<W2_PPL, W2_STAGES - 2>(min(nk - 1, W2_STAGES - 2), np == W2_PPL);
        lds_barrier();
        for (int kt = 0; kt < nk; ++kt) {
            if (kt + 1 < nk) wait_segs<W2_PPL, W2_STAGES - 3>(min(nk - kt - 2, W2_STAGES - 3), np == W2_PPL);
            lds_barrier();
            if (!(W2_EXP & 2) && kt + W2_STAGES - 1 < nk)
                issue(s_beg + kt + W2_STAGES - 1, (kt + W2_STAGES - 1) % W2_STAGES);
        }
        return;
    }

    // ---------------------------------------------------------------------- compute
    // wave (wm, wn): co fragments wm*4 + i, n fragments jj = 6 wn + j: tap jj >> 3, 16-channel
    // ci group cg = jj & 7 (plane cg >> 2), two 32-pixel k-steps per segment
    const int wn = wid & 3, wm = wid >> 2;
    const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
    const int k_lo = 8 * g + q;
    // fragment addresses as one per-lane base XOR a wave-uniform chunk term: the 16-B chunk
    // index c16 = 2 * (16-channel group) + (p >> 1) enters the swizzle by XOR only, so the
    // group's part is (32 * group) XORed into the base (bits 5..7, above `within`, below the row)
    const int a_base = k_lo * DYR + (((p >> 1) ^ (2 * pc_t256(k_lo))) << 4) + (p & 1) * 8;
    int xb[3][2];  // X span rows pos = k_lo + tx (+ 4 for the high half): plane 0, group 0
#pragma unroll
    for (int tx = 0; tx < 3; ++tx)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            const int pos = k_lo + 4 * hh + tx;
            xb[tx][hh] = W2_AP * 1024 + pos * 128 + (((p >> 1) ^ (2 * pc_t128(pos))) << 4) + (p & 1) * 8;
        }
    auto aoff = [&](int i) { return a_base ^ (32 * (wm * MI + i)); };
    auto boff = [&](int j, int hh) {
        const int jj = wn * NJ + j, tx = jj >> 3, cg = jj & 7;
        return (xb[tx][hh] ^ (32 * (cg & 3))) + (cg >> 2) * XPIECES * 1024;
    };
    f32x4 acc[MI][NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    uint4 a[MI], b[NJ];
    // the MFMAs of the current k-step, each operand re-read from (stage, half h) after its last use
    auto step = [&](int stage, int h) {
        const char* S = smem + stage * W2_STAGE + h * 32 * DYR;
        const char* X = smem + stage * W2_STAGE + h * 4096;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
#pragma unroll
            for (int i = 0; i < MI; ++i) {
                if constexpr (W2_EXP & 4) {   // operands consumed by a cheap dependency only
                    acc[i][j][0] += __uint_as_float(a[i].x ^ b[j].y);
                } else {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a[i]),
                                                                        __builtin_bit_cast(bf16x8_t, b[j]), acc[i][j],
                                                                        0, 0, 0);
                }
                if (j == NJ - 1) a[i] = ld_tr_pair(S + aoff(i), S + aoff(i) + 4 * DYR);
            }
            b[j] = ld_tr_pair(X + boff(j, 0), X + boff(j, 1));
        }
    };
    auto barrier = [] {
        __builtin_amdgcn_sched_barrier(0);
        lds_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    barrier();  // prologue barrier: segment 0 landed
#pragma unroll
    for (int i = 0; i < MI; ++i) a[i] = ld_tr_pair(smem + aoff(i), smem + aoff(i) + 4 * DYR);
#pragma unroll
    for (int j = 0; j < NJ; ++j) b[j] = ld_tr_pair(smem + boff(j, 0), smem + boff(j, 1));
    for (int kt = 0; kt < nk; ++kt) {
        step(kt % W2_STAGES, 1);        // segment kt, pixels 0-31 | read pixels 32-63
        barrier();                      // barrier kt: segment kt+1 landed; segment kt-1 fully read
        step((kt + 1) % W2_STAGES, 0);  // segment kt, pixels 32-63 | read segment kt+1, pixels 0-31
    }                                   // (the last iteration's reads are unused)

    // C[row = co][col = n]: co = co0 + (wm*4 + i)*16 + 4g + rr, n = jj*16 + (lane & 15)
    const int K = d.KH * 3 * d.Cin;
    float* const dst = slab ? slab + (long)split * d.Cout * K : nullptr;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            const int co = co0 + (wm * MI + i) * 16 + g * 4 + rr;
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int jj = wn * NJ + j, tx = jj >> 3;
                const int ci = ci0 + (jj & 7) * 16 + (lane & 15);
                const long o = (long)co * K + (ty * 3 + tx) * d.Cin + ci;
                if ((W2_EXP & 1) && acc[i][j][rr] != 1234.5f) continue;
                if (dst) dst[o] = acc[i][j][rr];
                else atomicAdd(dw + o, acc[i][j][rr]);
            }
        }
}

__global__ __launch_bounds__(256) void wgrad_pc_reduce(const float* __restrict__ slab, int splits, long n,
                                                        float* __restrict__ dw) {
    const long n4 = n / 4;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
        slab_sum4(slab, splits, n, dw, i);
    }
}

}  // namespace

// Preconditions (else IRGAN_EUNSUPPORTED, nothing launched): bf16 operands, stride 1,
// Cin % 64 == 0, ldx, xoff, ldy, yoff % 8 == 0, byte extents < 2^31, and either KH x 3 taps,
// Cout % 64 == 0, Wo % 64 == 0 (64-pixel row segments) or 4 x 4 taps, Cout % 128 == 0,
// Wo <= 32 (paired-row segments: D model.8).
extern "C" int irgan_conv_wgrad_pc(const irgan_conv_desc* d, const void* x, const void* dy, float* dw, int splitk,
                                   float* ws, long ws_cap, hipStream_t st) {
    if ((long)d->N * d->Ho * d->Wo <= 0) return 0;
    const int BMC = d->Cout % 128 == 0 ? 128 : 64;
    const bool pair = d->KW == 4 && d->KH == 4 && d->Wo <= 32 && BMC == 128;
    // the wide-n kernel takes any Wo: a row's last 64-pixel segment may be partial (its dY
    // pieces past Wo zero-filled), e.g. the 128 x 160 ResnetBlock maps of 512 x 640 (config 4)
    const bool w2 = !pair && BMC == 128 && d->KW == 3 && d->Cin % 128 == 0 && splitk <= 0;
    if (d->dtype != IRGAN_BF16 || (d->KW != 3 && !pair) || d->sx != 1 || d->sy != 1 ||
        d->Cout % BMC || d->Cin % 64 || (d->Wo % 64 && !pair && !w2) || d->ldx % 8 || d->xoff % 8 ||
        d->ldy % 8 || d->yoff % 8 || (long)d->N * d->H * d->W * d->ldx * 2 >= (1L << 31) ||
        (long)d->N * d->Ho * d->Wo * d->ldy * 2 >= (1L << 31))
        return IRGAN_EUNSUPPORTED;
    const int cus = irgan_cu_count();
    const int swz = irgan_xcd_swz();
    if (w2) {
        const int ntco = d->Cout / 128, nci2 = d->Cin / 128;
        const int tiles = ntco * nci2 * d->KH;
        const int nseg = d->N * d->Ho * irgan_cdiv(d->Wo, 64);
        int sk = cus / tiles;
        if (sk < 1) sk = 1;
        const int maxs = irgan_cdiv(nseg, 4);
        if (sk > maxs) sk = maxs;
        const long n = (long)d->Cout * d->KH * 3 * d->Cin;
        if (irgan_det(d)) {
            const long fit = ws ? ws_cap / n : 1;
            if (sk > fit) sk = (int)(fit > 1 ? fit : 1);
        }
        const int spb = irgan_cdiv(nseg, sk);
        sk = irgan_cdiv(nseg, spb);
        float* slab = (!(W2_EXP & 8) && ws && sk > 1 && (long)sk * n <= ws_cap) ? ws : nullptr;
        wgrad_w2_kernel<<<tiles * sk, W2_NT, 0, st>>>(*d, (const bf16_t*)x, (const bf16_t*)dy, dw, spb, nseg, ntco,
                                                      nci2, swz, slab);
        if (slab) {
            const int blocks = (int)std::min<long>(irgan_cdiv(n / 4, 256), 2048);
            wgrad_pc_reduce<<<blocks, 256, 0, st>>>(slab, sk, n, dw);
        }
        IRGAN_LAUNCH_CHECK();
        return 0;
    }
    const int ntco = d->Cout / BMC, nci = d->Cin / 64;
    const int tiles = ntco * nci * d->KH;
    const int nseg = pair ? d->N * ((d->Ho + 1) / 2) : d->N * d->Ho * (d->Wo / 64);
    if (splitk <= 0) {  // one block per CU (BMC 64: two fit): the largest split count whose grid fits one round
        splitk = (BMC == 64 ? 2 : 1) * cus / tiles;
        if (splitk < 1) splitk = 1;
        const int maxs = irgan_cdiv(nseg, 4);  // >= 4 segments per split
        if (splitk > maxs) splitk = maxs;
        if (swz && (tiles * splitk) % 8) {
            for (int s2 = splitk - 1; s2 >= 1 && s2 >= splitk - 8; --s2)
                if ((tiles * s2) % 8 == 0) { splitk = s2; break; }
        }
    }
    if (irgan_det(d)) {  // deterministic: no atomics -- at most the splits the workspace holds
        const long fit = ws ? ws_cap / ((long)d->Cout * d->KH * d->KW * d->Cin) : 1;
        if (splitk > fit) splitk = (int)(fit > 1 ? fit : 1);
    }
    const int spb = irgan_cdiv(nseg, splitk);
    splitk = irgan_cdiv(nseg, spb);
    const long n = (long)d->Cout * d->KH * d->KW * d->Cin;
    float* slab = (ws && splitk > 1 && n % 4 == 0 && (long)splitk * n <= ws_cap) ? ws : nullptr;
#define WPC(B, C, ...)                                                                                          \
    wgrad_pc_kernel<B, C, ##__VA_ARGS__><<<tiles * splitk, PC<B, C>::NT, 0, st>>>(                             \
        *d, (const bf16_t*)x, (const bf16_t*)dy, dw, spb, nseg, ntco, nci, swz, slab)
    if (pair) WPC(128, 8, 4, true);
    else if (BMC == 64) WPC(64, 4);   // 4 co fragments x 3 per compute wave (8 waves would hold 2 x 3)
    else WPC(128, 8);
#undef WPC
    if (slab) {
        const int blocks = (int)std::min<long>(irgan_cdiv(n / 4, 256), 2048);
        wgrad_pc_reduce<<<blocks, 256, 0, st>>>(slab, splitk, n, dw);
    } else if (splitk == 1) {
        // (atomics with one split: still correct, dw accumulates)
    }
    IRGAN_LAUNCH_CHECK();
    return 0;
}
