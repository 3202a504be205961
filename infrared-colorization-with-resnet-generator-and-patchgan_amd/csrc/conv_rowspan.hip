// Narrow-output stride-1 convolution as a row-span GEMM plus a shift-add: G outc
// (64 -> 3, 7x7 reflect, ir:529-531) and the backward-data of VGG conv1_1 (64 -> 3,
// 3x3: the input gradient of the perceptual term, ir:664).
//
// With Cout <= 8 the tile-per-tap kernel (conv_halo.hip conv_narrow_kernel) spends a
// 16-column MFMA on 3 output channels and a fragment read per MFMA and a half.  Here
// the N axis carries (tx, co) -- KW * Cout <= 32 columns, 21 of 32 used for outc --
// and the M axis carries INPUT positions q of an output row segment:
//
//   Z[q][tx * Cout + co] = sum_ty sum_ci  x[oy + ty + c0y][x0 + q + c0x][ci] * W[co][ty][tx][ci]
//   y[oy][x0 + j][co]    = act(bias[co] + sum_tx Z[j + tx][tx * Cout + co])
//
// Z accumulates over ty in the MFMA accumulators (the tx shift is the same for every
// ty), so a 32-pixel segment costs KH x 2 K-steps x 3 M fragments (40 input positions)
// x 2 N fragments of mfma_f32_16x16x32_bf16 -- 84 MFMAs for 7x7 where the tap-per-step
// kernel needed 196 per 16 pixels -- and the shift-add is KW fp32 adds per output value
// out of LDS.
//
// Block = one image, a 32-column strip, 64 output rows.  8 waves, one output row each
// per iteration (8 rows per iteration).  The input rows live in an LDS ring of
// 8 + KH - 1 rows x 40 positions x 128 B (one 64-channel chunk): after an iteration's
// MFMAs the 8 oldest rows are dead and the next 8 rows are DMA'd (buffer_load ... lds,
// reflect / zero padding by address, out-of-range arrives as zeros) into their slots
// while the waves run the shift-add and store.  All KH x 32 weight rows of the B
// operand ([ty][n = tx*Cout + co][ci]) stay in LDS.  Every LDS image uses the
// lds_off row swizzle (conflict-free 16-byte fragment reads).
#include "conv_epilogue.h"

#ifndef RS_EXP
#define RS_EXP 0  // A/B timing experiments only (tools/build_variant.sh); 0 = the real kernels
#endif
// wgrad bits: 1 no MFMA phase, 2 no A build, 4 no loads in the loop
#define RSX(b) ((RS_EXP & (b)) != 0)

namespace {

constexpr int RS_SEG = 32;     // output pixels per row segment
constexpr int RS_QP = 40;      // input positions per ring row (>= SEG + KW - 1, multiple of 8)
constexpr int RS_QF = 3;       // M fragments (48 positions; 40..47 read the next row: unused)
constexpr int RS_NR = 8;       // output rows per iteration (one per wave)
constexpr int RS_RB = 64;      // output rows per block
constexpr int RS_ZS = 33;      // Z row stride (floats): conflict-free column reads

IRGAN_HD int rs_lds_off(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }

template <int KH, int KW>
struct RSL {
    static constexpr int RR = RS_NR + KH - 1;                    // ring rows
    static constexpr int RING = (RR * RS_QP + 8) * 128;          // + 8 rows of slack for the q >= 40 reads
    static constexpr int WB = KH * 32 * 128;                      // B operand
    static constexpr int ZB = RS_NR * RS_QF * 16 * RS_ZS * 4;     // per-wave Z tiles
    static constexpr int LDS = RING + WB + ZB;
    static_assert(LDS <= 160 * 1024, "lds");
};

template <int KH, int KW>
__global__ __launch_bounds__(512, 1) void conv_rowspan_kernel(const irgan_conv_desc d, const bf16_t* __restrict__ x,
                                                              const bf16_t* __restrict__ w,
                                                              const float* __restrict__ bias, void* __restrict__ y,
                                                              int nsx, int nrb) {
    using L = RSL<KH, KW>;
    constexpr int RR = L::RR;
    __shared__ __attribute__((aligned(1024))) char smem[L::LDS];
    char* const sR = smem;
    char* const sW = smem + L::RING;
    float* const sZ = (float*)(smem + L::RING + L::WB);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    int t = blockIdx.x;
    const int sx = t % nsx;
    t /= nsx;
    const int rb = t % nrb;
    const int img = t / nrb;
    const int x0 = sx * RS_SEG, R0 = rb * RS_RB;
    const int R1 = min(d.Ho, R0 + RS_RB);
    const int Cout = d.Cout;
    const bool reflect = d.pad_mode == IRGAN_PAD_REFLECT;

    // ---- B operand: row (ty*32 + n), n = tx*Cout + co < KW*Cout, 64 input channels
    {
        const int Kw = KH * KW * d.Cin;
        for (int e = tid; e < KH * 32 * 8; e += 512) {
            const int row = e >> 3, c = e & 7, ty = row >> 5, n = row & 31;
            uint4 v = make_uint4(0u, 0u, 0u, 0u);
            if (n < KW * Cout) {
                const int tx = n / Cout, co = n - tx * Cout;
                v = *(const uint4*)(w + (long)co * Kw + (ty * KW + tx) * d.Cin + c * 8);
            }
            *(uint4*)(sW + rs_lds_off(row, c)) = v;
        }
    }
    // ---- ring rows: input row R0 + c0y + rel lives in slot rel % RR.  One wave-instruction
    // = 8 positions x 128 B of one row (5 per row)
    const i32x4 rs = make_rsrc(x, (uint32_t)((long)d.N * d.H * d.W * d.ldx * 2));
    const int sub = lane >> 3, cl = lane & 7;
    auto load_row = [&](int rel, int part) {  // part 0..4 of row rel
        const int slot = rel % RR;
        const int lrow = slot * RS_QP + part * 8 + sub;  // LDS row this lane writes
        const int q = part * 8 + sub;
        int iy = R0 + d.c0y + rel, ix = x0 + q + d.c0x;
        if (reflect) {
            iy = reflect_idx(iy, d.H);
            ix = reflect_idx(ix, d.W);
        }
        const bool ok = q < RS_SEG + KW - 1 && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W;
        const int chunk = cl ^ (lrow & 7);
        const uint32_t off =
            ok ? (uint32_t)((((img * d.H + iy) * d.W + ix) * d.ldx + d.xoff) * 2 + chunk * 16) : IRGAN_OOB;
        blds16(rs, off, sR + (slot * RS_QP + part * 8) * 128);
    };
    // prologue: rows rel 0 .. RR-1 (5 * RR instructions over the 8 waves)
    for (int e = wid; e < RR * 5; e += 8) load_row(e / 5, e % 5);
    wait_vmcnt<0>();
    __syncthreads();

    float bv[8];
#pragma unroll
    for (int co = 0; co < 8; ++co) bv[co] = (bias && co < Cout) ? bias[co] : 0.f;
    float* const Zw = sZ + wid * RS_QF * 16 * RS_ZS;
    const int g = lane >> 4, c16 = lane & 15;

#pragma unroll 1
    for (int it = 0; R0 + it * RS_NR < R1; ++it) {
        const int oy = R0 + it * RS_NR + wid;
        f32x4 acc[RS_QF][2];
#pragma unroll
        for (int m = 0; m < RS_QF; ++m) acc[m][0] = acc[m][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ty = 0; ty < KH; ++ty) {
            const int slot = (it * RS_NR + wid + ty) % RR;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                uint4 a[RS_QF], b[2];
#pragma unroll
                for (int nf = 0; nf < 2; ++nf) b[nf] = *(const uint4*)(sW + rs_lds_off(ty * 32 + nf * 16 + c16, 4 * h + g));
#pragma unroll
                for (int m = 0; m < RS_QF; ++m)
                    a[m] = *(const uint4*)(sR + rs_lds_off(slot * RS_QP + m * 16 + c16, 4 * h + g));
#pragma unroll
                for (int m = 0; m < RS_QF; ++m)
#pragma unroll
                    for (int nf = 0; nf < 2; ++nf)
                        acc[m][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a[m]),
                                                                             __builtin_bit_cast(bf16x8_t, b[nf]),
                                                                             acc[m][nf], 0, 0, 0);
            }
        }
        __syncthreads();  // every wave is done with the 8 oldest ring rows
        const bool more = R0 + (it + 1) * RS_NR < R1;
        if (more)  // the next iteration's 8 new rows: rel (it+1)*8 + KH-1 ..
            for (int e = wid; e < RS_NR * 5; e += 8) load_row((it + 1) * RS_NR + KH - 1 + e / 5, e % 5);
        // Z[q][n] (lane: q = 16m + 4g + r, n = 16nf + c16) -> this wave's LDS tile
#pragma unroll
        for (int m = 0; m < RS_QF; ++m)
#pragma unroll
            for (int nf = 0; nf < 2; ++nf)
#pragma unroll
                for (int r = 0; r < 4; ++r) Zw[(m * 16 + 4 * g + r) * RS_ZS + nf * 16 + c16] = acc[m][nf][r];
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's Z writes landed (LDS ops are in order)
        if (lane < RS_SEG && oy < R1 && x0 + lane < d.Wo) {
            const long pix = ((long)img * d.OH + oy * d.omy + d.ooy) * d.OW + (x0 + lane) * d.omx + d.oox;
            for (int co = 0; co < Cout; ++co) {
                float v = bv[co];
#pragma unroll
                for (int tx = 0; tx < KW; ++tx) v += Zw[(lane + tx) * RS_ZS + tx * Cout + co];
                v = conv_act(v, d.act);
                if (d.out_dtype == IRGAN_F32) {
                    float* yp = (float*)y + pix * d.ldy + d.yoff + co;
                    *yp = d.accumulate ? *yp + v : v;
                } else {
                    bf16_t* yp = (bf16_t*)y + pix * d.ldy + d.yoff + co;
                    *yp = f2bf(d.accumulate ? bf2f(*yp) + v : v);
                }
            }
        }
        wait_vmcnt<0>();  // the new rows landed (and this wave's stores retired)
        __syncthreads();
    }
}

template <int KH, int KW>
void launch_rowspan(const irgan_conv_desc* d, const void* x, const void* w, const float* bias, void* y, hipStream_t st) {
    const int nsx = irgan_cdiv(d->Wo, RS_SEG), nrb = irgan_cdiv(d->Ho, RS_RB);
    conv_rowspan_kernel<KH, KW><<<d->N * nsx * nrb, 512, 0, st>>>(*d, (const bf16_t*)x, (const bf16_t*)w, bias, y,
                                                                 nsx, nrb);
}

// ---- weight gradient of the same layers (G outc, 7x7): the same row-span trick with the
// shift moved onto dY.  For output row oy, segment x0 and kernel row ty:
//
//   dW[ty][n = tx*Cout + co][ci] += sum_q A[q][n] * X[oy + ty + c0y][x0 + q + c0x][ci],
//   A[q][n] = dY[oy][x0 + q - tx][co]   (0 <= q - tx < 32, else 0)
//
// an MFMA GEMM with M = n (32 rows, 21 used), N = ci (64), K = q (64: 38 used; the rest
// multiplies zeros of A).  Wave ty (< KH) owns the 2 x 4 accumulator tiles of kernel row
// ty for the whole block (one A fragment feeds 4 MFMAs, one X fragment 2); both operands
// are K-major in LDS ([q][n] and the [q][ci] ring) and are read with ds_read_b64_tr_b16
// pairs (conv_wgrad_pc.hip's operand reads).  Per batch of 8 output rows every wave
// builds its share of the 8 A tiles (64 q x 32 n bf16; rows r and r + 4 share one 128-B
// row image, n in its columns 32 (r >> 2) ..) from dY.  The ring holds two batches of
// input rows: batch it + 1's 8 new rows and its dY rows are DMA'd when batch it's MFMAs
// start (into the slots batch it - 1 released), so the HBM latency hides under them.
// Block partials -> slab (ordered reduce) or fp32 atomics.
typedef __attribute__((ext_vector_type(4))) short rs_s16x4;
typedef __attribute__((address_space(3))) rs_s16x4 rs_lds_s4;
IRGAN_HD uint4 rs_tr_pair(const char* lo, const char* hi) {
    const rs_s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((rs_lds_s4*)lo);
    const rs_s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((rs_lds_s4*)hi);
    uint4 out;
    __builtin_memcpy(&out, &a, 8);
    __builtin_memcpy((char*)&out + 8, &b, 8);
    return out;
}

// K-major operand images for the transposed reads, 128-B rows, 16-B chunk XOR 2*t(r)
// (conv_wgrad_pc.hip's X-span swizzle: conflict-free ds_read_b64_tr_b16 pairs)
IRGAN_HD int rs_t128(int r) { return ((r >> 1) & 1) | (((r >> 3) & 1) << 1); }
IRGAN_HD int rs_tr_off(int row, int col) { return row * 128 + (((col >> 3) ^ (2 * rs_t128(row))) << 4) + (col & 7) * 2; }

template <int KH, int KW>
struct RSW {
    // output pixels per row segment: 7x7 takes 26 so that its 32 input positions are ONE K-step
    // (a 32-pixel segment needs 38: two K-steps, the second with 6 of 32 positions used)
    static constexpr int SEG = KW == 7 ? 32 - (KW - 1) : RS_SEG;
    static constexpr int HS = (SEG + KW - 1 + 31) / 32;           // K-steps per row
    static constexpr int RR = RS_NR + KH - 1;                     // input rows one batch reads
    static constexpr int RQ = RR + RS_NR;                         // ring slots: + the next batch's rows
    static constexpr int RING = (RQ * RS_QP + 32) * 128;          // + 32 rows: K-step 1 of the last slot
    static constexpr int AB = RS_NR / 2 * 64 * 128;               // 8 A tiles [64 q][32 n], two per row image
    static constexpr int DBH = RS_NR * RS_SEG * 16;               // one batch's dY rows (8 channels)
    static constexpr int DB = 2 * DBH;
    static constexpr int LDS = RING + AB + DB;
    static_assert(LDS <= 160 * 1024 && KH <= 8, "lds / one kernel row per wave");
};

template <int KH, int KW>
__global__ __launch_bounds__(512, 1) void wgrad_rowspan_kernel(const irgan_conv_desc d, const bf16_t* __restrict__ x,
                                                               const bf16_t* __restrict__ dy, float* __restrict__ dw,
                                                               float* __restrict__ slab, int nsx, int nrb,
                                                               int nchunk) {
    using L = RSW<KH, KW>;
    constexpr int RR = L::RR, RQ = L::RQ;
    __shared__ __attribute__((aligned(1024))) char smem[L::LDS];
    char* const sR = smem;
    char* const sA = smem + L::RING;
    char* const sD = sA + L::AB;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    // block = (64-channel input chunk, image, strip, row block); a group (image, strip, row
    // block) of nchunk blocks writes one slab partial, each block its chunk's columns
    const int chunk = blockIdx.x % nchunk, grp = blockIdx.x / nchunk;
    int t = grp;
    const int sx = t % nsx;
    t /= nsx;
    const int rb = t % nrb;
    const int img = t / nrb;
    const int x0 = sx * L::SEG, R0 = rb * RS_RB;
    const int R1 = min(d.Ho, R0 + RS_RB);
    const int Cout = d.Cout;
    const bool reflect = d.pad_mode == IRGAN_PAD_REFLECT;

    // K-step 1 of a slot reads the first rows of the next slot (the slack rows after the last
    // one), times zeros of A: they must hold finite values, also while a prefetch is landing
    // in them -- the slots the prologue does not load start as zeros
    for (int e = tid; e < ((RQ - RR) * RS_QP + 32) * 8; e += 512)
        *(uint4*)(sR + (RR * RS_QP) * 128 + e * 16) = make_uint4(0u, 0u, 0u, 0u);
    const i32x4 rs = make_rsrc(x, (uint32_t)((long)d.N * d.H * d.W * d.ldx * 2));
    const int sub = lane >> 3, cl = lane & 7;
    auto load_row = [&](int rel, int part) {
        const int slot = rel % RQ;
        const int lrow = slot * RS_QP + part * 8 + sub;
        const int q = part * 8 + sub;
        int iy = R0 + d.c0y + rel, ix = x0 + q + d.c0x;
        if (reflect) {
            iy = reflect_idx(iy, d.H);
            ix = reflect_idx(ix, d.W);
        }
        const bool ok = q < L::SEG + KW - 1 && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W;
        const int ck = cl ^ (2 * rs_t128(lrow));
        const uint32_t off =
            ok ? (uint32_t)((((img * d.H + iy) * d.W + ix) * d.ldx + d.xoff) * 2 + chunk * 128 + ck * 16)
               : IRGAN_OOB;
        blds16(rs, off, sR + (slot * RS_QP + part * 8) * 128);
    };
    // batch it's dY rows -> sD[it & 1] [8 rows][32 px][8 channels] (4 wave-instructions; out
    // of range -> zeros)
    const i32x4 rsd = make_rsrc(dy, (uint32_t)((long)d.N * d.Ho * d.Wo * d.ldy * 2));
    auto load_dy = [&](int it) {
        if (wid < 4) {
            const int r = wid * 2 + (lane >> 5), j = lane & 31, oy = R0 + it * RS_NR + r, ox = x0 + j;
            const bool ok = oy < R1 && ox < d.Wo;
            const uint32_t off = ok ? (uint32_t)((((long)img * d.Ho + oy) * d.Wo + ox) * d.ldy + d.yoff) * 2 : IRGAN_OOB;
            blds16(rsd, off, sD + (it & 1) * L::DBH + wid * 1024);
        }
    };
    // A tiles of batch `it` (from sD): row r, q, 8 consecutive n -> one 16-byte LDS write
    auto build_a = [&](int it) {
        const char* const sDi = sD + (it & 1) * L::DBH;
        constexpr int QB = 32 * L::HS;  // the A rows the K-steps read
        for (int e = tid; e < RS_NR * QB * 4; e += 512) {
            const int r = e / (QB * 4), q = (e >> 2) % QB, n8 = (e & 3) * 8;
            float v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int n = n8 + k, tx = n / Cout, co = n - tx * Cout, j = q - tx;
                const bool ok = n < KW * Cout && j >= 0 && j < L::SEG;
                v[k] = ok ? bf2f(*(const bf16_t*)(sDi + (r * RS_SEG + j) * 16 + co * 2)) : 0.f;
            }
            uint4 u;
            u.x = pk_bf16(v[0], v[1]);
            u.y = pk_bf16(v[2], v[3]);
            u.z = pk_bf16(v[4], v[5]);
            u.w = pk_bf16(v[6], v[7]);
            *(uint4*)(sA + (r & 3) * 8192 + rs_tr_off(q, n8 + (r >> 2) * 32)) = u;
        }
    };
    for (int e = wid; e < RR * 5; e += 8) load_row(e / 5, e % 5);
    load_dy(0);
    wait_vmcnt<0>();
    __syncthreads();
    build_a(0);
    __syncthreads();

    // lane roles of the transposed operand reads (conv_wgrad_pc.hip): k row k_lo (+4 for the
    // high half, +32 for K-step 1), 4 consecutive columns from 4p
    const int g = lane >> 4, qq = (lane & 15) >> 2, p = lane & 3;
    const int k_lo = 8 * g + qq;
    // Wave roles: wave w owns the kernel-row PAIR (2 pr, 2 pr + 1), pr = w % NPR, over the
    // batch's rows [rh * RPW, rh * RPW + RPW), rh = w / NPR.  Output row r of kernel row ty
    // reads input row r + ty, so the pair's second row at r is its first row at r + 1: the
    // X fragments slide through registers and each step reads one A tile and ONE new X row
    // for 16 MFMAs (one kernel row per wave read an A tile and an X row for 8).  The NRS
    // waves of a pair sum their partials through LDS in a fixed order after the loop.
    // (4x4, two K-steps per row: the window's registers would spill -- one kernel row per
    // wave, the batch's rows split over two waves)
    constexpr bool PAIRS = KH == 7;
    constexpr int NPR = PAIRS ? (KH + 1) / 2 : KH, NRS = 8 / NPR, RPW = RS_NR / NRS, HS = L::HS;
    static_assert(NPR * NRS == 8 && RS_NR % NRS == 0, "wave roles");
    const int pr = wid % NPR, rh = wid / NPR, ty0 = PAIRS ? 2 * pr : pr;
    const bool two = PAIRS && ty0 + 1 < KH;  // wave-uniform
    f32x4 acc[2][2][4];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[u][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    int xo[4];  // X column byte terms of ci fragment j (swizzle applied per row below)
#pragma unroll
    for (int j = 0; j < 4; ++j) xo[j] = (16 * j + 4 * p);
    // the ci fragments of input row `rel` (relative to the block's first row), both K-steps
    auto read_x = [&](int rel, uint4 (&b)[HS][4]) {
        const int slot = rel % RQ;
#pragma unroll
        for (int h = 0; h < HS; ++h)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int row = slot * RS_QP + 32 * h + k_lo;
                b[h][j] = rs_tr_pair(sR + rs_tr_off(row, xo[j]), sR + rs_tr_off(row + 4, xo[j]));
            }
    };

#pragma unroll 1
    for (int it = 0; R0 + it * RS_NR < R1; ++it) {
        const bool nxt = R0 + (it + 1) * RS_NR < R1;
        if (nxt && !RSX(4)) {  // batch it + 1: its 8 new input rows and its dY rows
            for (int e = wid; e < RS_NR * 5; e += 8) load_row((it + 1) * RS_NR + KH - 1 + e / 5, e % 5);
            load_dy(it + 1);
        }
        if (!RSX(1)) {
            uint4 xc[HS][4], xn[PAIRS ? HS : 1][4];
#pragma unroll
            for (int k = 0; k < RPW; ++k) {
                const int r = rh * RPW + k;
                if (k == 0 || !two) read_x(it * RS_NR + r + ty0, xc);
                if constexpr (PAIRS)
                    if (two) read_x(it * RS_NR + r + ty0 + 1, xn);
                const char* Ar = sA + (r & 3) * 8192;
                const int ac = (r >> 2) * 32;
#pragma unroll
                for (int h = 0; h < HS; ++h) {
                    uint4 a[2];
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        const int q0 = 32 * h + k_lo, col = ac + 16 * i + 4 * p;
                        a[i] = rs_tr_pair(Ar + rs_tr_off(q0, col), Ar + rs_tr_off(q0 + 4, col));
                    }
#pragma unroll
                    for (int i = 0; i < 2; ++i)
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            acc[0][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                                __builtin_bit_cast(bf16x8_t, a[i]), __builtin_bit_cast(bf16x8_t, xc[h][j]), acc[0][i][j], 0,
                                0, 0);
                            if constexpr (PAIRS)
                                if (two)
                                    acc[1][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                                        __builtin_bit_cast(bf16x8_t, a[i]), __builtin_bit_cast(bf16x8_t, xn[h][j]),
                                        acc[1][i][j], 0, 0, 0);
                        }
                }
                if constexpr (PAIRS)
                    if (two) {
#pragma unroll
                        for (int h = 0; h < HS; ++h)
#pragma unroll
                            for (int j = 0; j < 4; ++j) xc[h][j] = xn[h][j];
                    }
            }
        }
        if (nxt) wait_vmcnt<0>();
        __syncthreads();  // this batch's A tiles consumed, the next batch's rows landed
        if (nxt) {
            if (!RSX(2)) build_a(it + 1);
            __syncthreads();
        }
    }
    // the pair's partials: waves rh > 0 park theirs in the (now idle) ring, wave rh = 0 adds
    // them in rh order (deterministic)
    f32x4* const part = (f32x4*)sR;  // [NPR][NRS - 1][16 tiles][64 lanes]
    static_assert(NPR * (NRS - 1) * 16 * 64 * 16 <= L::RING, "partials fit in the ring");
    if (rh > 0) {
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    part[((pr * (NRS - 1) + rh - 1) * 16 + u * 8 + i * 4 + j) * 64 + lane] = acc[u][i][j];
    }
    __syncthreads();
    if (rh > 0) return;
#pragma unroll
    for (int q = 1; q < NRS; ++q)
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const f32x4 v = part[((pr * (NRS - 1) + q - 1) * 16 + u * 8 + i * 4 + j) * 64 + lane];
                    acc[u][i][j] += v;
                }
    // C[row = n][col = ci]: n = 16i + 4g + rr, ci = 16j + (lane & 15)
    const int Kw = KH * KW * d.Cin;
    float* const dst = slab ? slab + (long)grp * Cout * Kw : nullptr;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        if (u == 1 && !two) break;
        const int ty = ty0 + u;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int n = 16 * i + 4 * g + rr;
                if (n >= KW * Cout) continue;
                const int tx = n / Cout, co = n - tx * Cout;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const long o = (long)co * Kw + (ty * KW + tx) * d.Cin + chunk * 64 + 16 * j + (lane & 15);
                    if (dst) dst[o] = acc[u][i][j][rr];
                    else atomicAdd(dw + o, acc[u][i][j][rr]);
                }
            }
    }
}

// Ordered two-level reduce of the nb group partials (n floats each; deterministic): level 1
// sums slabs [part*per, (part+1)*per) of index i into tmp[part][i] -- n is small (outc 9408)
// and nb large (512), so one thread per index would be a 512-long dependent load chain --
// level 2 adds the parts into dw in order.
__global__ __launch_bounds__(256) void wgrad_rowspan_reduce1(const float* __restrict__ slab, int nb, int per, long n,
                                                             float* __restrict__ tmp) {
    const long i = blockIdx.x * 256L + threadIdx.x;
    if (i >= n) return;
    const int b0 = blockIdx.y * per, b1 = min(nb, b0 + per);
    float a = 0.f;
    for (int c0 = b0; c0 < b1; c0 += 8) {  // 8 loads in flight, added in order
        float v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = c0 + k < b1 ? slab[(long)(c0 + k) * n + i] : 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (c0 + k < b1) a += v[k];
    }
    tmp[(long)blockIdx.y * n + i] = a;
}
__global__ __launch_bounds__(256) void wgrad_rowspan_reduce2(const float* __restrict__ tmp, int parts, long n,
                                                             float* __restrict__ dw) {
    const long i = blockIdx.x * 256L + threadIdx.x;
    if (i >= n) return;
    float a = dw[i];
    for (int q = 0; q < parts; ++q) a += tmp[(long)q * n + i];
    dw[i] = a;
}

}  // namespace

// Weight gradient of narrow-output stride-1 convs: G outc (7x7, Cin 64) and D's last layer
// (512 -> 1, 4x4: its 64-channel chunks are separate blocks of one group).  bf16, Cin % 64,
// KW * Cout <= 32, ldx / xoff % 8.  dw += the gradient (fp32 [Cout][KH][KW][Cin]); the group
// partials go through ws (ordered reduce) when groups * Cout * KH * KW * Cin <= ws_cap, else
// fp32 atomics.
extern "C" int irgan_conv_wgrad_rowspan(const irgan_conv_desc* d, const void* x, const void* dy, float* dw, float* ws,
                                        long ws_cap, hipStream_t st) {
    if ((long)d->N * d->Ho * d->Wo <= 0 || d->Cout <= 0) return 0;
    static const bool off = getenv("IRGAN_NO_ROWSPAN") != nullptr;
    if (off || d->dtype != IRGAN_BF16 || d->sy != 1 || d->sx != 1 || d->Cin % 64 || d->Cout > 8 ||
        d->KW * d->Cout > 32 || d->KH != d->KW || (d->KH != 7 && d->KH != 4) || d->ldx % 8 || d->xoff % 8 ||
        d->ldy % 8 || d->yoff % 8 || (long)d->N * d->H * d->W * d->ldx * 2 >= (1L << 31) ||
        (long)d->N * d->Ho * d->Wo * d->ldy * 2 >= (1L << 31))
        return IRGAN_EUNSUPPORTED;
    const int seg = d->KH == 7 ? RSW<7, 7>::SEG : RSW<4, 4>::SEG;
    const int nsx = irgan_cdiv(d->Wo, seg), nrb = irgan_cdiv(d->Ho, RS_RB), nchunk = d->Cin / 64;
    const int ng = d->N * nsx * nrb;
    const long n = (long)d->Cout * d->KH * d->KW * d->Cin;
    const int per = 16, parts = irgan_cdiv(ng, per);
    float* slab = (ws && (long)(ng + parts) * n <= ws_cap) ? ws : nullptr;
    if (!slab && irgan_det(d)) return IRGAN_EUNSUPPORTED;  // deterministic: the split kernels cap their splits
    if (d->KH == 7)
        wgrad_rowspan_kernel<7, 7><<<ng * nchunk, 512, 0, st>>>(*d, (const bf16_t*)x, (const bf16_t*)dy, dw, slab, nsx,
                                                                nrb, nchunk);
    else
        wgrad_rowspan_kernel<4, 4><<<ng * nchunk, 512, 0, st>>>(*d, (const bf16_t*)x, (const bf16_t*)dy, dw, slab, nsx,
                                                                nrb, nchunk);
    if (slab) {
        float* tmp = slab + (long)ng * n;
        wgrad_rowspan_reduce1<<<dim3((unsigned)irgan_cdiv(n, 256), parts), 256, 0, st>>>(slab, ng, per, n, tmp);
        wgrad_rowspan_reduce2<<<(unsigned)irgan_cdiv(n, 256), 256, 0, st>>>(tmp, parts, n, dw);
    }
    IRGAN_LAUNCH_CHECK();
    return 0;
}

// Shapes it takes (else IRGAN_EUNSUPPORTED, nothing launched): bf16 operands, stride 1,
// Cin == 64, KW * Cout <= 32 (Cout <= 8), (KH, KW) in {(7,7), (3,3)}, ldx / xoff % 8,
// no mask; any output dtype / activation / accumulate (the caller's conv_epilogue rules).
extern "C" int irgan_conv_fwd_rowspan(const irgan_conv_desc* d, const void* x, const void* w, const float* bias,
                                      void* y, const void* mask, hipStream_t st) {
    if ((long)d->N * d->Ho * d->Wo <= 0 || d->Cout <= 0) return 0;
    static const bool off = getenv("IRGAN_NO_ROWSPAN") != nullptr;
    if (off || d->dtype != IRGAN_BF16 || d->sy != 1 || d->sx != 1 || d->Cin != 64 || d->Cout > 8 ||
        d->KW * d->Cout > 32 || d->ldx % 8 || d->xoff % 8 || mask || d->KH != d->KW ||
        (long)d->N * d->H * d->W * d->ldx * 2 >= (1L << 31))
        return IRGAN_EUNSUPPORTED;
    if (d->KH == 7) launch_rowspan<7, 7>(d, x, w, bias, y, st);
    else if (d->KH == 3) launch_rowspan<3, 3>(d, x, w, bias, y, st);
    else return IRGAN_EUNSUPPORTED;
    IRGAN_LAUNCH_CHECK();
    return 0;
}
