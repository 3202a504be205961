// bf16 / fp8 stride-1 convolution kernel template (conv_pp_kernel), launched by conv_pp.hip
// (forward, backward-data, fused statistics, the fp8 ResnetBlock path).  Design notes:
//
// bf16 stride-1 convolution, resident input halo, ping-pong wave groups.
//
// Same operand staging as conv_halo.hip (a block owns a 16x16 output patch of
// one image; per 64-channel chunk the (16+KH-1)x(16+KW-1) input halo is DMA'd
// into LDS once and every tap is an LDS row shift of it; the weight tile of a
// K-step = one tap x 64 channels streams through a 2-stage ring), but the
// schedule is built for MFMA occupancy at one block per CU:
//
//  * block tile 256 pixels x 256 output channels, 8 waves = 2 groups x 4 waves;
//    group g owns patch rows [8g, 8g+8), wave wn owns channels [64wn, 64wn+64):
//    a 128 x 64 wave tile (8 x 4 fragments of mfma_f32_16x16x32_bf16), so a
//    32-deep sub-step is 12 ds_read_b128 per 32 MFMAs (narrower channel tiles
//    split the group's rows instead, see PP<BN>);
//  * each sub-step (one tap, 32 channels) is two phases per wave: READ (issue
//    the 12 fragment reads and this wave's share of the next K-step's DMA) and
//    MFMA (32 MFMAs), each closed by a block barrier.  Group 1 starts one
//    barrier late, so in every barrier window one group multiplies while the
//    other reads: each SIMD holds one wave of each group;
//  * taps are compile-time (KH, KW template); the K-step loop keeps its
//    chunk / tap counters in scalars, so a phase costs a few SALU ops plus
//    4 VALU per swizzled fragment address;
//  * the MFMA computes C^T (weights are the A operand): a lane's 4 accumulator
//    rows are 4 consecutive output channels of one pixel, so the epilogue
//    stages bf16 [pixel][channel] rows with 8-byte LDS writes in one pass and
//    stores 16-byte runs.
//
// DMA ordering: K-step k's weights sit in stage k&1 and are read in windows
// 4k..4k+3 (group 0: 4k, 4k+2; group 1: 4k+1, 4k+3).  W(k+1) is issued in each
// wave's first READ of step k (that stage was last read in window 4k-1) and is
// retired by every wave with a counted vmcnt before the barrier closing window
// 4k+3.  The halo of chunk c+1 is issued after W(k+1) at the first tap of chunk
// c (its buffer last served chunk c-1).  Reads need no lgkmcnt wait before
// their barrier except group 1's last READ of a K-step (window 4k+3): the next
// window may overwrite that stage; every other READ is consumed by the same
// wave's MFMA phase before any DMA can target its buffer.
//
// fp8 (F8, irgan_conv_fwd_fp8): the same kernel on OCP e4m3 operands.  A K-step
// is one tap x 128 channels (a 128-byte halo / weight row, so every DMA, LDS
// image and barrier window is byte-for-byte the bf16 schedule); its MFMA is
// mfma_scale_f32_32x32x64_f8f6f4 (unit block scales: 2x the bf16 rate).  The
// wave tile is the bf16 one (MIW patch rows x NJ*16 channels) as 32 x 32
// fragments: a weight fragment is 32 channels, a pixel fragment two patch rows
// (lane bit 4 picks the row), each lane's 32 operand bytes are chunks
// 4h + (lane >> 5) and + 2 of the 128-byte row in sub-step h (the same K bytes
// for both operands).  So a sub-step is (MIW / 2) x (NJ / 2) MFMAs of 64 cycles
// on 48 operand VGPRs -- the bf16 kernel's 512-cycle windows, 12 fragment reads
// and registers at twice the FLOPs (the 16x16x128 form needed 4 sub-steps of
// 256 cycles per K-step to stay in registers: twice the barriers per FLOP).
// Accumulator (p, q) register 4*i4 + r is channel 32q + 8*i4 + 4*(lane >> 5) + r
// of pixel 32p + (lane & 31); the epilogue sees it as the bf16 fragment
// (i, j) = (2p + (i4 >> 1), 2q + (i4 & 1)) through m_of / cl_of.  The per-tensor
// scales are undone in the epilogue: y = acc * (dqx[0] * dqw[0]) + bias.
//
// Preconditions (checked by irgan_conv_fwd_pp): bf16, sy = sx = 1, Cin % 64 == 0,
// (KH, KW) in {(3,3), (4,4)}, ldx, xoff % 8 == 0, Cout % 256 == 0 (channel
// tiles of 256), no tanh epilogue, input slice and weights < 2^30 elements (byte offsets
// below the buffer-resource out-of-range marker 2^31).

#pragma once
#include <type_traits>

#include "conv_epilogue.h"

#ifndef PP_EXP
#define PP_EXP 0  // A/B timing experiments only (tools/build_variant.sh); 0 = the real kernel
#endif
// bits: 1 no MFMA, 2 no weight DMA in the loop, 4 no fragment reads, 8 no barriers in the loop, 16 no epilogue
#define PPX(b) ((PP_EXP & (b)) != 0)

namespace {

IRGAN_HD int lds_off(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }

IRGAN_HD void sched_fence() { __builtin_amdgcn_sched_barrier(0); }
// block barrier that the scheduler cannot move instructions across
IRGAN_HD void phase_barrier() {
    sched_fence();
#if !PPX(8)
    lds_barrier();
#endif
    sched_fence();
}
IRGAN_HD void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

constexpr int PH = 16, PW = 16;   // output patch
constexpr int HPMAX = 46;         // halo pieces (8 rows of 128 B) for taps up to 4x4: 19*19 = 361 rows
constexpr int HBYTES = HPMAX * 1024;
// per output-channel tile BN (256: resblock / D / VGG conv3; 192: up2 dgrad; 128: down1,
// up1, VGG conv2; 64: up2, down1 dgrad, VGG conv1_2).  A group's 128 pixels (8 patch rows)
// x BN channels are split over its 4 waves as RW row bands x CW channel bands; the wave
// tile is MIW pixel fragments x NJ channel fragments.  Narrow BN splits rows rather than
// channels, so every wave keeps 4 channel fragments: LDS fragment reads per MFMA are
// (MIW + NJ) / (MIW * NJ) = 0.375 (BN 256), 0.5 (128), 0.75 (64) instead of
// 0.625 / 1.125 with 128-pixel wave tiles.
template <int BN>
struct PP {
    static constexpr int BBYTES = BN * 128;
    static constexpr int LDS = 2 * HBYTES + 2 * BBYTES;
    static constexpr int MIW = BN >= 192 ? 8 : (BN == 128 ? 4 : 2);  // pixel fragments (patch rows) per wave
    static constexpr int RW = 8 / MIW, CW = 4 / RW;
    static constexpr int NJ = BN / 16 / CW;            // 16-channel fragments per wave
    static constexpr int WU = BBYTES / 1024 / 8;       // weight pieces per wave per K-step
    static constexpr int RSB = BN * 2 + 16;            // bf16 staging row (pixel) stride, bytes
    static constexpr int LPP = BN / 8;                 // epilogue lanes per pixel row (8 channels each)
    static constexpr int PPASS = 512 / LPP;            // pixel rows stored per pass (BN = 192: 21, lanes 504+ idle)
    static_assert(256 * RSB <= LDS && BN % 64 == 0 && WU * 8 * 1024 == BBYTES && NJ * 16 * CW == BN, "tile");
};

typedef int v8i_t __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
IRGAN_HD v8i_t cat8(i32x4 a, i32x4 b) { return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7); }

// rg (irgan_conv_dgrad_reflect_line): the line-form reflect ring of a ResnetBlock backward-data
// (conv_ring.hip: g[n][line][pos][c], lines top / bottom / left / right) folded onto the staged
// bf16 dx before the store pass -- ring_line_fold_kernel's terms, order and roundings, so dx is
// bit-identical to the interior launch + fold launch
// v = the ring terms of dx pixel (y, x) (a border-band pixel: row 1 / H-2 or column 1 / W-2),
// channels c .. c+7, summed in ring_line_fold_kernel's order
IRGAN_HD void ring_line_sum(const irgan_conv_desc& d, const float* __restrict__ g, int n, int y, int x, int c,
                            float (&v)[8]) {
    const int H = d.Ho, W = d.Wo;
    const bool row = y == 1 || y == H - 2;
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = 0.f;
    auto add = [&](int line, int pos) {
        const float4* q = (const float4*)(g + (((long)n * 4 + line) * IRGAN_RING_ROWS + pos) * d.Cout + c);
        const float4 a = q[0], b = q[1];
        v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
        v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
    };
    if (row) {
        const int line = y == 1 ? 0 : 1;
        add(line, x + 1);
        if (x == 1) { add(line, 0); add(2, y + 1); }
        if (x == W - 2) { add(line, W + 1); add(3, y + 1); }
    } else {
        add(x == 1 ? 2 : 3, y + 1);
    }
}
// o (8 bf16 of dx, the interior's rounded values) += its ring terms, one more rounding
IRGAN_HD void ring_line_apply(const float (&v)[8], uint4& o) {
    const uint32_t wd[4] = {o.x, o.y, o.z, o.w};
    uint32_t o4[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        o4[k] = pk_bf16(__uint_as_float(wd[k] << 16) + v[2 * k], __uint_as_float(wd[k] & 0xffff0000u) + v[2 * k + 1]);
    o = make_uint4(o4[0], o4[1], o4[2], o4[3]);
}

// ONE: a single halo buffer, so at BN = 64 the block fits twice per CU (LDS 62 KiB,
// <= 128 VGPRs) and one block's halo loads / epilogue overlap the other's MFMA loop
// (BN = 128 would need 159 VGPRs: at 128 it spills 30 and runs slower than two BN-64
// tiles, profiles/r02_s5_pp_one_ab.txt).  With more than one channel chunk the next chunk's halo cannot be
// prefetched: after the last window that reads chunk c (4k+3 of its last tap) every
// wave issues its pieces of chunk c+1, retires them and meets at one extra barrier.
// S2D: a 4x4 stride-2 convolution (the PatchGAN's model.2 / model.5, ir:607-615) run as the
// 2x2 stride-1 convolution it is over the space-to-depth input x''[u][v][(p, q, c)] =
// x[2u + p + c0y][2v + q + c0x][c]: KH = KW = 2 here, the descriptor keeps the layer's own
// 4x4 / stride-2 geometry.  x'' is never stored: a chunk of x'' (64 channels of one phase
// (p, q)) is a halo DMA that gathers every other pixel of x, and the weight tile of K-step
// (tap (a, b), chunk) is read from the layer's plain 4x4 pack at tap (2a + p, 2b + q) -- the
// halo reuse of the stride-1 kernel (each input pixel loaded once per output patch instead of
// once per tap) for the layers the generic implicit GEMM ran at 0.2 of peak.
//
// PH4: the four output phases of a stride-2 backward-data (4x4 stride 2: each phase a 2x2
// stride-1 conv of dY onto every other dx pixel) in ONE launch: block = (channel tile, phase,
// patch); the phase picks its taps' origin (c0y, c0x), its output pixel phase (ooy, oox) and
// its packed weight image from `tab`; d carries the rest (omy = omx = 2, the per-phase Ho / Wo).
struct PhaseTab {
    const bf16_t* w[4];
    int c0y[4], c0x[4], ooy[4], oox[4];
};
IRGAN_HD int pick4(const int (&a)[4], int i) { return i == 0 ? a[0] : (i == 1 ? a[1] : (i == 2 ? a[2] : a[3])); }

template <int KH, int KW, int BN, bool ACC, bool STATS = false, bool F8 = false, bool ONE = false, bool S2D = false,
          bool PH4 = false>
__global__ __launch_bounds__(512, ONE ? 2 : 1) void conv_pp_kernel(const irgan_conv_desc d, const bf16_t* __restrict__ x,
                                                         const bf16_t* __restrict__ w, const float* __restrict__ bias,
                                                         void* __restrict__ y, const void* __restrict__ mask,
                                                         int ntn, int tpx, int tpy, int swz,
                                                         float2* __restrict__ part = nullptr,
                                                         const float* __restrict__ dqx = nullptr,
                                                         const float* __restrict__ dqw = nullptr,
                                                         const float* __restrict__ rg = nullptr,
                                                         const PhaseTab tab = PhaseTab{}) {
    constexpr int ESZ = F8 ? 1 : 2, CHN = 128 / ESZ;  // operand bytes, channels per 128-byte chunk
    const char* const xb = (const char*)x;
    const char* wb = (const char*)w;
    constexpr int TAPS = KH * KW, HWd = PW + KW - 1, HROWS = (PH + KH - 1) * HWd, HP = (HROWS + 7) / 8;
    constexpr int BBYTES = PP<BN>::BBYTES, NJ = PP<BN>::NJ, WU = PP<BN>::WU, RSB = PP<BN>::RSB;
    constexpr int LDS = ONE ? HBYTES + 2 * BBYTES : PP<BN>::LDS;
    static_assert(!ONE || (BN == 64 && 256 * RSB <= LDS && !F8), "single-halo variant: staging must fit");
    constexpr int MI = PP<BN>::MIW, RW = PP<BN>::RW;
    // sub-steps per K-step: 2 (bf16: 32 channels each; fp8: 64)
    constexpr int HS = 2;
    constexpr int NP = F8 ? MI / 2 : 1, NQ = F8 ? NJ / 2 : 1;  // fp8 32 x 32 fragments per wave
    static_assert(!F8 || (MI % 2 == 0 && NJ % 2 == 0), "fp8: 32 x 32 fragments");
    static_assert(HP <= HPMAX && HP > 32 && TAPS >= 2, "halo pieces per wave are 4 to 6");
    static_assert(!S2D || (KH == 2 && KW == 2 && !F8), "space-to-depth: the 2x2 form of a 4x4 stride-2 conv");
    static_assert(!PH4 || (!S2D && !F8 && !STATS), "four-phase backward-data: plain bf16");
    __shared__ __attribute__((aligned(1024))) char smem[LDS];
    char* const sH = smem;
    char* const sB = smem + (ONE ? 1 : 2) * HBYTES;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wid >> 2, wn = wid & 3;
    const int prow = grp * 8 + (wn % RW) * MI;  // first patch row of this wave's pixel fragments
    const int cb = (wn / RW) * NJ * 16;         // first block-local channel of this wave
    int t = xcd_tile(blockIdx.x, gridDim.x, swz);
    const int nt = t % ntn;
    t /= ntn;
    int c0y = d.c0y, c0x = d.c0x, ooy = d.ooy, oox = d.oox;
    if constexpr (PH4) {  // the phases of one patch are adjacent blocks: their dY halos share L2
        const int ph = t & 3;
        t >>= 2;
        c0y = pick4(tab.c0y, ph);
        c0x = pick4(tab.c0x, ph);
        ooy = pick4(tab.ooy, ph);
        oox = pick4(tab.oox, ph);
        wb = (const char*)(ph == 0 ? tab.w[0] : (ph == 1 ? tab.w[1] : (ph == 2 ? tab.w[2] : tab.w[3])));
    }
    const int pxi = t % tpx;
    t /= tpx;
    const int pyi = t % tpy;
    const int img = t / tpy;
    const int py0 = pyi * PH, px0 = pxi * PW, n0 = nt * BN;
    const int nh = (HP - wid + 7) >> 3;  // halo pieces this wave loads: wid, wid+8, ... (4 to 6)
    const int Kw = (S2D ? 16 : TAPS) * d.Cin;      // weight row stride (S2D: the 4x4 pack)
    const int cpp = d.Cin / CHN;                   // S2D: chunks per phase
    const int nchunk = (S2D ? 4 : 1) * d.Cin / CHN;
    const int sub = lane >> 3;
    const int chunk = (lane & 7) ^ sub;  // source chunk for this lane's LDS slot (row & 7 == sub)
    const bool reflect = d.pad_mode == IRGAN_PAD_REFLECT;

    // DMA sources as byte offsets into buffer resources (out-of-range offsets
    // arrive as zeros: padding and Cout tails cost no address math in the loop)
    const uint32_t xbytes = (uint32_t)((long)d.N * d.H * d.W * d.ldx * ESZ);
    // byte offset of this lane's row of halo piece (u*8 + wid) (computed at issue
    // time, once per chunk: keeping six offsets live costs registers the MFMA
    // tile needs)
    auto halo_off = [&](int u, int lsub, int ph) -> uint32_t {
        const int h = (u * 8 + wid) * 8 + lsub;
        const int hy = h / HWd, hx = h - hy * HWd;
        int iy = py0 + hy + c0y, ix = px0 + hx + c0x;
        if constexpr (S2D) {  // x''[py0 + hy][px0 + hx] of phase (p, q) = ph
            iy = 2 * (py0 + hy) + (ph >> 1) + c0y;
            ix = 2 * (px0 + hx) + (ph & 1) + c0x;
        }
        if (reflect) {
            iy = reflect_idx(iy, d.H);
            ix = reflect_idx(ix, d.W);
        }
        const bool ok = (h < HROWS) & ((unsigned)iy < (unsigned)d.H) & ((unsigned)ix < (unsigned)d.W);
        return ok ? (uint32_t)((((img * d.H + iy) * d.W + ix) * d.ldx + d.xoff) * ESZ + ((lane & 7) ^ lsub) * 16)
                  : IRGAN_OOB;
    };
    // weight rows co >= Cout lie beyond num_records: they arrive as zeros
    const uint32_t wbytes = (uint32_t)((long)d.Cout * Kw * ESZ);
    const uint32_t b_off = (uint32_t)((n0 + wid * WU * 8 + sub) * Kw * ESZ + chunk * 16);  // piece u (8 rows): + u*8*Kw*ESZ
    auto issue_halo = [&](int c) {
        char* dst = sH + (ONE ? 0 : (c & 1) * HBYTES);
        const int cc = S2D ? c % cpp : c, ph = S2D ? c / cpp : 0;
        const i32x4 rs = make_rsrc(xb + cc * 128, xbytes - cc * 128);
        int lsub = sub;
        asm volatile("" : "+v"(lsub));  // recompute the offsets here instead of hoisting them out of the loop
#pragma unroll
        for (int u = 0; u < 6; ++u)
            if (u < nh) blds16(rs, halo_off(u, lsub, ph), dst + (u * 8 + wid) * 1024);
    };
    auto issue_w = [&](int c, int tp, int stage) {
        int kcol = tp * d.Cin + c * CHN;
        if constexpr (S2D) {  // tap (a, b) of phase (p, q): the 4x4 tap (2a + p, 2b + q)
            const int ph = c / cpp;
            kcol = ((2 * (tp >> 1) + (ph >> 1)) * 4 + 2 * (tp & 1) + (ph & 1)) * d.Cin + (c % cpp) * CHN;
        }
        const i32x4 rs = make_rsrc(wb + kcol * ESZ, wbytes - kcol * ESZ);
        char* dst = sB + stage * BBYTES + wid * WU * 1024;
#pragma unroll
        for (int u = 0; u < WU; ++u) blds16(rs, b_off, (uint32_t)(u * 8 * Kw * ESZ), dst + u * 1024);
    };
    // ONE: chunk c's halo after the barrier closing its last reading window (the same
    // barrier instance for both groups), landed before anyone reads it
    auto reload_halo = [&](int c) {
        issue_halo(c);
        wait_vmcnt<0>();
        phase_barrier();
    };
    // W(k+1) landed; the halo issued at step k (after W(k+1)) may stay in flight
    auto retire = [&](bool halo_now) {
        if (!halo_now) wait_vmcnt<0>();
        else if (nh == 6) wait_vmcnt<6>();
        else if (nh == 5) wait_vmcnt<5>();
        else wait_vmcnt<4>();
    };

    f32x4 acc[F8 ? 1 : MI][F8 ? 1 : NJ];
    f32x16 acc32[NP][NQ];
    if constexpr (F8) {
#pragma unroll
        for (int p = 0; p < NP; ++p)
#pragma unroll
            for (int q = 0; q < NQ; ++q)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc32[p][q][r] = 0.f;
    } else {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    uint4 af[F8 ? 1 : MI], bfr[F8 ? 1 : NJ];
    v8i_t pf8[NP], wf8[NQ];  // fp8: 32-byte fragments (chunks 4h + (lane >> 5), + 2)
    // prologue: W(0), halo(0), W(1); retire the first two
    issue_w(0, 0, 0);
    issue_halo(0);
    issue_w(0, 1, 1);
    wait_vmcnt<WU>();
    phase_barrier();
    if (grp == 1) phase_barrier();  // group 1 runs one window behind

    // LDS addressing.  Fragment rows of a tap are constant shifts K of the
    // lane's row arow0 and lds_off's XOR term depends only on (arow0 + K) & 7,
    // so with the tap loop unrolled an A address is tsw[K & 7] + hb plus the
    // ds_read immediate K * 128: one VALU add per fragment read.
    // halo row of fragment 0 at tap (0,0) (fp8: lane bit 4 = the second patch row of a fragment)
    const int arow0 = (prow + (F8 ? (lane >> 4) & 1 : 0)) * HWd + (lane & 15);
    const int brow0 = cb + (lane & (F8 ? 31 : 15));  // weight row of fragment 0 (rows +16j / +32q share the XOR)
    // bf16: sub-step h reads chunk (lane >> 4) + 4h; fp8: chunks 4h + (lane >> 5) and + 2 (the
    // same byte <-> channel map for both operands)
    const int g0 = F8 ? lane >> 5 : lane >> 4;
    const int bb0 = lds_off(brow0, g0), bb1 = lds_off(brow0, 4 + g0);
    int tsw[8];  // h = 1 flips chunk bit 2 (tsw ^ 64), the second fp8 chunk bit 1 (^ 32)
#pragma unroll
    for (int k8 = 0; k8 < 8; ++k8) tsw[k8] = (g0 ^ ((arow0 + k8) & 7)) << 4;
#pragma unroll 1
    for (int c = 0; c < nchunk; ++c) {
        const int hb = arow0 * 128 + (ONE ? 0 : (c & 1) * HBYTES);
        const bool more = c + 1 < nchunk;
#pragma unroll
        for (int tp = 0; tp < TAPS; ++tp) {
            const int ty = tp / KW, tx = tp % KW;
            const int k = c * TAPS + tp;  // K-step
            const char* B = sB + (k & 1) * BBYTES;
            const bool last_k = !more && tp == TAPS - 1;
            const bool halo_now = tp == 0 && more && !ONE;
            const bool reload = ONE && more && tp == TAPS - 1;  // single buffer: chunk c+1 after window 4k+3
#pragma unroll
            for (int h = 0; h < HS; ++h) {
                // ---- READ phase (group 0: even windows, group 1: odd)
                const int bb = h ? bb1 : bb0;
                int hbp = hb;
                asm volatile("" : "+v"(hbp));  // per-phase base: the address adds stay here, not hoisted
                if constexpr (F8) {
#pragma unroll
                    for (int q = 0; q < NQ; ++q)
                        wf8[q] = cat8(*(const i32x4*)(B + bb + q * 4096), *(const i32x4*)(B + (bb ^ 32) + q * 4096));
#pragma unroll
                    for (int p = 0; p < NP; ++p) {
                        const int K = (2 * p + ty) * HWd + tx;
                        const int sw = tsw[K & 7] ^ (h * 64);
                        pf8[p] = cat8(*(const i32x4*)(sH + (hbp + sw) + K * 128),
                                      *(const i32x4*)(sH + (hbp + (sw ^ 32)) + K * 128));
                    }
                } else {
#if !PPX(4)
#pragma unroll
                for (int j = 0; j < NJ; ++j) bfr[j] = *(const uint4*)(B + bb + j * 2048);
#pragma unroll
                for (int i = 0; i < MI; ++i) {
                    const int K = (i + ty) * HWd + tx;
                    af[i] = *(const uint4*)(sH + (hbp + (tsw[K & 7] ^ (h * 64))) + K * 128);
                }
#else
                if (k == 0 && h == 0) {
#pragma unroll
                    for (int j = 0; j < NJ; ++j) bfr[j] = *(const uint4*)(B + bb + j * 2048);
#pragma unroll
                    for (int i = 0; i < MI; ++i) af[i] = *(const uint4*)(sH + hbp + i * 128);
                }
#endif
                }
                if (h == 0 && !PPX(2)) {
                    // W(k+1) (W(1) came with the prologue), then the next chunk's halo
                    if (k >= 1 && !last_k) {
                        if (tp + 1 < TAPS) issue_w(c, tp + 1, (k + 1) & 1);
                        else issue_w(c + 1, 0, (k + 1) & 1);
                    }
                    if (halo_now) issue_halo(c + 1);
                }
                if (h == HS - 1 && grp == 1) {  // last window of step k (4k+3 in bf16): last reads, then retire
                    wait_lgkm0();
                    if (!last_k) retire(halo_now);
                }
                phase_barrier();
                if (reload && h == HS - 1 && grp == 1) reload_halo(c + 1);
                // ---- MFMA phase: C^T fragment (weights as A, pixels as B)
                if constexpr (F8) {
#pragma unroll
                    for (int p = 0; p < NP; ++p)
#pragma unroll
                        for (int q = 0; q < NQ; ++q)
                            acc32[p][q] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
                                wf8[q], pf8[p], acc32[p][q], 0, 0, 0, 127, 0, 127);
                    // pin the scaled MFMAs inside this phase: hipcc otherwise sinks them past the
                    // barriers to the end of the chunk, keeping every tap's fragments live (spills)
#pragma unroll
                    for (int p = 0; p < NP; ++p)
#pragma unroll
                        for (int q = 0; q < NQ; ++q) asm volatile("" : "+v"(acc32[p][q]));
                } else {
#pragma unroll
                    for (int i = 0; i < MI * !PPX(1); ++i)
#pragma unroll
                        for (int j = 0; j < NJ; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                                __builtin_bit_cast(bf16x8_t, bfr[j]), __builtin_bit_cast(bf16x8_t, af[i]), acc[i][j],
                                0, 0, 0);
                }
                if (h == HS - 1 && grp == 0 && !last_k) retire(halo_now);  // last window of step k
                phase_barrier();
                if (reload && h == HS - 1 && grp == 0) reload_halo(c + 1);
            }
        }
    }
    if (grp == 0) phase_barrier();  // match group 1's extra barrier
    __syncthreads();                // all operand reads done: LDS becomes the staging buffer
    // bf16 accumulate (a dgrad into a tensor that holds another branch's gradient): the old
    // tile is DMA'd straight into the staging layout (16-byte slots of RSB-byte pixel rows; the
    // row's padding slot and pixels / channels outside the output are out-of-range loads) in
    // one batch of ~17 loads per wave, so its latency is paid once per launch; the emit then
    // adds each lane's 4 old channels from LDS and writes the sum back to the same slot.
    // (Loaded in registers per fragment row the latency was exposed MI times.)
    const bool out_f32 = d.out_dtype == IRGAN_F32;
    const bool acc_lds = ACC && !out_f32 && d.ldy % 8 == 0 && d.yoff % 8 == 0 &&
                         (long)d.N * d.OH * d.OW * d.ldy * 2 < (1L << 31);
    if constexpr (ACC) {
        if (acc_lds) {
            constexpr int SPR = RSB / 16, SLOTS = 256 * SPR;  // slots per staged pixel row / tile
            const i32x4 rs = make_rsrc(y, (uint32_t)((long)d.N * d.OH * d.OW * d.ldy * 2));
            for (int k = wid; k * 64 < SLOTS; k += 8) {  // wave-uniform
                const int e = k * 64 + lane, m = e / SPR, sl = e - m * SPR;
                const int oy = py0 + (m >> 4), ox = px0 + (m & 15), co = n0 + sl * 8;
                const bool ok = e < SLOTS && sl < BN / 8 && oy < d.Ho && ox < d.Wo && co + 8 <= d.Cout;
                const long pix = ((long)img * d.OH + oy * d.omy + ooy) * d.OW + ox * d.omx + oox;
                blds16(rs, ok ? (uint32_t)((pix * d.ldy + d.yoff + co) * 2) : IRGAN_OOB, smem + k * 1024);
            }
        }
    }
#if PPX(16)
    {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) s += F8 ? acc32[i >> 1][j >> 1][0] : acc[i][j][0] + acc[i][j][3];
        if (s == 123.f) *(float*)y = s;
        return;
    }
#endif

    // ---- epilogue.  Fragment (i, j): pixel m = m_of(i), block-local channels cl_of(i, j) + r,
    // r = 0..3 (bf16: m = (prow + i)*16 + (lane & 15), cl = cb + j*16 + 4*(lane >> 4); fp8: the
    // 32 x 32 accumulator's quarter i4 = 2 (i & 1) + (j & 1) of fragment (i >> 1, j >> 1))
    auto m_of = [&](int i) {
        return F8 ? (prow + 2 * (i >> 1) + ((lane >> 4) & 1)) * 16 + (lane & 15) : (prow + i) * 16 + (lane & 15);
    };
    auto cl_of = [&](int i, int j) {
        return F8 ? cb + 32 * (j >> 1) + 8 * (2 * (i & 1) + (j & 1)) + 4 * (lane >> 5) : cb + 4 * (lane >> 4) + j * 16;
    };
    auto accv = [&](int i, int j) -> f32x4 {
        if constexpr (F8) {
            const int o = 4 * (2 * (i & 1) + (j & 1));
            const f32x16& t = acc32[i >> 1][j >> 1];
            return f32x4{t[o], t[o + 1], t[o + 2], t[o + 3]};
        } else {
            return acc[i][j];
        }
    };
    const float osc = F8 ? *dqx * *dqw : 1.f;  // fp8: 1 / (x scale * w scale), powers of two
    constexpr int NB = F8 ? 2 : 1;  // bias quads per channel fragment (fp8: by i & 1)
    float4 b4[NB][NJ];
#pragma unroll
    for (int ib = 0; ib < NB; ++ib)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int co = n0 + cl_of(ib, j);
        b4[ib][j] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (bias) {
            if (co + 3 < d.Cout) {
                b4[ib][j] = *(const float4*)(bias + co);
            } else {
                if (co < d.Cout) b4[ib][j].x = bias[co];
                if (co + 1 < d.Cout) b4[ib][j].y = bias[co + 1];
                if (co + 2 < d.Cout) b4[ib][j].z = bias[co + 2];
            }
        }
    }
    auto pix_of = [&](int m) -> long {
        const int oy = py0 + (m >> 4), ox = px0 + (m & 15);
        if (oy >= d.Ho || ox >= d.Wo) return -1;
        return ((long)img * d.OH + oy * d.omy + ooy) * d.OW + ox * d.omx + oox;
    };
    // Each lane owns (pixel, 4 consecutive channels) per fragment: mask and
    // accumulate are applied right here on those 4 channels.
    // bf16 output: stage bf16 [256 px][256 ch] in LDS, then 16-byte row stores;
    // fp32 output: 16-byte stores straight from the registers.
    // ReLU backward mask on a plain bf16 store (the VGG backward-data chain): applied in the
    // store pass on the rounded values with 16-byte coalesced mask loads issued together
    // (x * {0, 1} commutes with the bf16 rounding: bit-identical to masking before it);
    // otherwise (LReLU 0.2, accumulate, fp32 out) in registers, one 8-byte load per fragment
    // row issued for all NJ fragments before any is used
    const bool late_mask = mask && d.mask_act == 1 && !ACC && !out_f32 && !STATS && !rg && d.ldm % 8 == 0 &&
                           d.moff % 8 == 0 && d.ldy % 8 == 0 && d.yoff % 8 == 0;
    const bool mask_vec = mask && d.ldm % 4 == 0 && d.moff % 4 == 0;
    auto emit = [&](auto actc) {
        constexpr int A = decltype(actc)::value;
#pragma unroll
        for (int i = 0; i < MI; ++i) {
            const int m = m_of(i);
            const long pix = pix_of(m);
            uint2 mk[NJ];
            if (mask_vec && !late_mask && pix >= 0) {
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    const int co = n0 + cl_of(i, j);
                    mk[j] = co + 4 <= d.Cout ? *(const uint2*)((const bf16_t*)mask + pix * d.ldm + d.moff + co)
                                             : make_uint2(0u, 0u);
                }
            }
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int cl = cl_of(i, j), co = n0 + cl;
                const float4 b = b4[F8 ? i & 1 : 0][j];
                const f32x4 a = accv(i, j);
                float v[4] = {a[0] + b.x, a[1] + b.y, a[2] + b.z, a[3] + b.w};
                if constexpr (F8) {
                    v[0] = a[0] * osc + b.x;
                    v[1] = a[1] * osc + b.y;
                    v[2] = a[2] * osc + b.z;
                    v[3] = a[3] * osc + b.w;
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = conv_act(v[r], A);
                const bool full = co + 4 <= d.Cout;
                if (pix >= 0 && mask && !late_mask) {
                    if (mask_vec && full) {
                        v[0] *= mask_mul(__uint_as_float(mk[j].x << 16), d.mask_act);
                        v[1] *= mask_mul(__uint_as_float(mk[j].x & 0xffff0000u), d.mask_act);
                        v[2] *= mask_mul(__uint_as_float(mk[j].y << 16), d.mask_act);
                        v[3] *= mask_mul(__uint_as_float(mk[j].y & 0xffff0000u), d.mask_act);
                    } else {
                        const bf16_t* mp = (const bf16_t*)mask + pix * d.ldm + d.moff + co;
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            if (full || co + r < d.Cout) v[r] *= mask_mul(bf2f(mp[r]), d.mask_act);
                    }
                }
                if (out_f32) {
                    if (pix < 0) continue;
                    float* yp = (float*)y + pix * d.ldy + d.yoff + co;
                    if (full && ((pix * d.ldy + d.yoff + co) & 3) == 0) {
                        float4 o = make_float4(v[0], v[1], v[2], v[3]);
                        if (ACC) {
                            const float4 p = *(const float4*)yp;
                            o.x += p.x; o.y += p.y; o.z += p.z; o.w += p.w;
                        }
                        *(float4*)yp = o;
                    } else {
                        for (int r = 0; r < 4 && co + r < d.Cout; ++r) yp[r] = ACC ? yp[r] + v[r] : v[r];
                    }
                } else {
                    if (acc_lds && pix >= 0 && full) {
                        const uint2 old = *(const uint2*)(smem + m * RSB + cl * 2);
                        v[0] += bf2f((bf16_t)(old.x & 0xffffu));
                        v[1] += bf2f((bf16_t)(old.x >> 16));
                        v[2] += bf2f((bf16_t)(old.y & 0xffffu));
                        v[3] += bf2f((bf16_t)(old.y >> 16));
                    } else if (ACC && pix >= 0) {
                        const bf16_t* yp = (const bf16_t*)y + pix * d.ldy + d.yoff + co;
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            if (full || co + r < d.Cout) v[r] += bf2f(yp[r]);
                    }
                    uint2 pk;
                    pk.x = pk_bf16(v[0], v[1]);
                    pk.y = pk_bf16(v[2], v[3]);
                    *(uint2*)(smem + m * RSB + cl * 2) = pk;
                }
            }
        }
    };
    // rg: the patch's border-band pixels (rows 1 / H-2, columns 1 / W-2 of the image: at most
    // two rows and two columns of the patch, 4 lines x 16 positions x LPP 8-channel slots) get
    // their ring terms in a pass over the staged tile between the staging and the store pass.
    // Every slot's line loads are issued here, before the staging, so their latency hides
    // under it -- added in the store pass they stalled a border pixel's wave once per pixel row.
    constexpr int RSL = 4 * 16 * PP<BN>::LPP / 512;  // ring slots per thread
    float rv[RSL][8];
    int rm[RSL];
    if (rg) {
        constexpr int LPPr = PP<BN>::LPP;
        const int H = d.Ho, W = d.Wo;
        const int rr1 = 1 - py0, rr2 = H - 2 - py0, cc1 = 1 - px0, cc2 = W - 2 - px0;
        auto in16 = [](int a) { return (unsigned)a < 16u; };
        const bool r1 = in16(rr1), r2 = in16(rr2), c1 = in16(cc1), c2 = in16(cc2);
#pragma unroll
        for (int k = 0; k < RSL; ++k) {
            const int sl = tid + 512 * k;
            const int line = sl / (16 * LPPr), pos = (sl / LPPr) % 16, ch = sl % LPPr;
            int pr = -1, pc = -1;
            if (line == 0 && r1) { pr = rr1; pc = pos; }
            else if (line == 1 && r2) { pr = rr2; pc = pos; }
            else if (line == 2 && c1 && !(r1 && pos == rr1) && !(r2 && pos == rr2)) { pr = pos; pc = cc1; }
            else if (line == 3 && c2 && !(r1 && pos == rr1) && !(r2 && pos == rr2)) { pr = pos; pc = cc2; }
            const int y = py0 + pr, x = px0 + pc;
            rm[k] = (pr >= 0 && y < H && x < W && n0 + ch * 8 < d.Cout) ? pr * 16 + pc : -1;
            if (rm[k] >= 0) ring_line_sum(d, rg, img, y, x, n0 + ch * 8, rv[k]);
        }
    }
    if (acc_lds) {  // the old tile landed (every wave's DMA) before any lane reads a slot
        wait_vmcnt<0>();
        __syncthreads();
    }
    switch (d.act) {
        case IRGAN_ACT_RELU: emit(std::integral_constant<int, IRGAN_ACT_RELU>()); break;
        case IRGAN_ACT_LRELU: emit(std::integral_constant<int, IRGAN_ACT_LRELU>()); break;
        default: emit(std::integral_constant<int, IRGAN_ACT_NONE>()); break;
    }
    if (out_f32) return;
    __syncthreads();
    if (rg) {  // the ring terms onto the staged pixels (each (pixel, slot) owned by one thread)
#pragma unroll
        for (int k = 0; k < RSL; ++k) {
            if (rm[k] < 0) continue;
            const int ch = (tid + 512 * k) % PP<BN>::LPP;
            uint4* sp = (uint4*)(smem + rm[k] * RSB + ch * 16);
            uint4 o = *sp;
            ring_line_apply(rv[k], o);
            *sp = o;
        }
        __syncthreads();
    }
    constexpr int LPP = PP<BN>::LPP;
    constexpr int PPASS = PP<BN>::PPASS;
    if constexpr (STATS) {
        // InstanceNorm statistics of the stored (bf16) outputs fused into the store
        // pass: per-channel (sum, sum of squares) over this block's valid pixels, one
        // float2 partial per (image, patch, channel) in the layout finalize_kernel
        // (norm.hip) reduces.  Host guarantees Cout % BN == 0, LPP * PPASS == 512.
        static_assert(!STATS || PP<BN>::LPP * PP<BN>::PPASS == 512, "all threads store");
        const int c8 = (tid % LPP) * 8, co8 = n0 + c8;
        float s1[8], s2[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) s1[k] = s2[k] = 0.f;
        for (int m = tid / LPP; m < 256; m += PPASS) {
            const long pix = pix_of(m);
            if (pix < 0) continue;
            const uint4 v = *(const uint4*)(smem + m * RSB + c8 * 2);
            *(uint4*)((bf16_t*)y + pix * d.ldy + d.yoff + co8) = v;
            const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float lo = __uint_as_float(wv[k] << 16), hi = __uint_as_float(wv[k] & 0xffff0000u);
                s1[2 * k] += lo; s2[2 * k] += lo * lo;
                s1[2 * k + 1] += hi; s2[2 * k + 1] += hi * hi;
            }
        }
        __syncthreads();  // staging reads done: reuse LDS for the cross-row reduction
        float2* red = (float2*)smem;  // [PPASS][BN]
#pragma unroll
        for (int k = 0; k < 8; ++k) red[(tid / LPP) * BN + c8 + k] = make_float2(s1[k], s2[k]);
        __syncthreads();
        // two-level fixed-order sum over the PPASS row groups: NR = 512 / BN threads per
        // channel each add PPASS / NR rows, then one thread per channel adds the NR
        constexpr int NR = 512 / BN, RPT = PPASS / NR;
        static_assert(RPT * NR == PPASS, "row split");
        float a = 0.f, b = 0.f;
        {
            const int c = tid % BN, r0 = tid / BN;
#pragma unroll
            for (int r = 0; r < RPT; ++r) {
                const float2 e = red[(r0 * RPT + r) * BN + c];
                a += e.x;
                b += e.y;
            }
        }
        __syncthreads();
        red[tid] = make_float2(a, b);  // [NR][BN]
        __syncthreads();
        if (tid < BN) {
            a = 0.f;
            b = 0.f;
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const float2 e = red[r * BN + tid];
                a += e.x;
                b += e.y;
            }
            const long patch = (long)img * (tpx * tpy) + pyi * tpx + pxi;
            part[patch * d.Cout + n0 + tid] = make_float2(a, b);
        }
        return;
    }
    if (tid >= PPASS * LPP) return;
    const int c8 = (tid % LPP) * 8, co8 = n0 + c8;
    if (co8 >= d.Cout) return;
    const bool vec = co8 + 8 <= d.Cout && d.ldy % 8 == 0 && d.yoff % 8 == 0;
    if (late_mask && vec) {
        constexpr int NIT = (256 + PPASS - 1) / PPASS;  // pixel rows per thread
        uint4 mk[NIT];
#pragma unroll
        for (int q = 0; q < NIT; ++q) {  // every mask load in flight before the first store
            const int m = tid / LPP + q * PPASS;
            const long pix = m < 256 ? pix_of(m) : -1;
            mk[q] = pix >= 0 ? *(const uint4*)((const bf16_t*)mask + pix * d.ldm + d.moff + co8)
                             : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int q = 0; q < NIT; ++q) {
            const int m = tid / LPP + q * PPASS;
            const long pix = m < 256 ? pix_of(m) : -1;
            if (pix < 0) continue;
            const uint4 o = *(const uint4*)(smem + m * RSB + c8 * 2);
            *(uint4*)((bf16_t*)y + pix * d.ldy + d.yoff + co8) = make_uint4(
                relu_mask_pk(o.x, mk[q].x), relu_mask_pk(o.y, mk[q].y), relu_mask_pk(o.z, mk[q].z),
                relu_mask_pk(o.w, mk[q].w));
        }
        return;
    }
    for (int m = tid / LPP; m < 256; m += PPASS) {
        const long pix = pix_of(m);
        if (pix < 0) continue;
        bf16_t* yp = (bf16_t*)y + pix * d.ldy + d.yoff + co8;
        const char* sp = smem + m * RSB + c8 * 2;
        if (vec) {
            *(uint4*)yp = *(const uint4*)sp;
        } else {
            for (int q = 0; q < 8 && co8 + q < d.Cout; ++q) yp[q] = ((const bf16_t*)sp)[q];
        }
    }
}

}  // namespace
