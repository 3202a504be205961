// bf16 backward-weight convolution over row segments with a shared input halo.
//
//   dW[co][ty][tx][ci] += sum_p dY[p][co] * X[iy(p, ty)][ix(p, tx)][ci]
//
// The per-tap wgrad (conv_glds.hip) stages a 64-pixel x 64-channel X tile per
// tap and a dY tile per (tap, channel) block, ~64 FLOP per L2->LDS byte, and is
// bound by that traffic.  Here a block owns (co tile, 64-channel ci chunk, one
// kernel row ty, ALL KW taps of that row) and walks 64-pixel row segments of
// dY: per segment it DMAs the dY tile [64 px][BMC co] and ONE input row span of
// 63*sx + KW pixels x 64 channels; the KW taps are LDS row shifts of that span.
// MFMA operands need 8 consecutive pixels per lane, so both tiles are read with
// ds_read_b64_tr_b16 (pixel rows -> MFMA k).  LDS images are laid out so every
// transposed read is bank-conflict-free:
//   dY, 256-B rows: 16-B chunk XOR 2*((r&3)|((r>>3&1)<<2));
//   dY, 128-B rows and the X span: chunk XOR 2*((r>>1&1)|((r>>3&1)<<1));
//   dY, 32-B rows (Cout <= 8): row r stored at position r ^ ((r>>3&1)<<2);
//   X for stride 2: even input columns in positions [0, 72), odd in [72, 144),
//   so the stride-2 tap rows of consecutive pixels are consecutive positions.
// Pieces (1 KiB = one wave-wide global_load_lds) are dealt round-robin to the
// waves; 3-stage ring, one barrier per segment, fp32 atomics into dW at the end
// (split-K over segments).
#include "common.h"

#ifndef WG_EXP
#define WG_EXP 0  // A/B timing experiments only (tools/build_variant.sh); 0 = the real kernel
#endif
// bits: 1 no MFMA, 2 no DMA in the loop, 4 no fragment reads, 8 no barrier in the loop, 16 no epilogue
#define WGX(b) ((WG_EXP & (b)) != 0)

namespace {

__device__ __attribute__((aligned(4096))) bf16_t g_wgh_zero_page[2048];

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s4;

IRGAN_HD int t128(int r) { return ((r >> 1) & 1) | (((r >> 3) & 1) << 1); }
IRGAN_HD int t256(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }

// byte offset of 16-bit column `col` in LDS row position `pos` of an RB-byte-row image
template <int RB>
IRGAN_HD int img_off(int pos, int col) {
    const int c16 = col >> 3, within = (col & 7) * 2;
    // 512-B rows start on bank 0 like 256-B rows: the same XOR spreads the
    // eight rows of a transposed read over all 64 banks
    if constexpr (RB >= 256) return pos * RB + ((c16 ^ (2 * t256(pos))) << 4) + within;
    else if constexpr (RB == 128) return pos * 128 + ((c16 ^ (2 * t128(pos))) << 4) + within;
    else return pos * RB + c16 * 16 + within;
}

constexpr int XHALF = 72;  // stride-2 span: odd input columns start at this position

IRGAN_HD uint4 tr_pair(const char* lo, const char* hi) {
    const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)lo);
    const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)hi);
    uint4 out;
    __builtin_memcpy(&out, &a, 8);
    __builtin_memcpy((char*)&out + 8, &b, 8);
    return out;
}

template <int BMC, int KW, int SX, int WM, int WN>
__global__ __launch_bounds__(WM * WN * 64, 1) void wgrad_halo_kernel(const irgan_conv_desc d,
                                                                     const bf16_t* __restrict__ x,
                                                                     const bf16_t* __restrict__ dy,
                                                                     float* __restrict__ dw, int segs_per_block,
                                                                     int nseg, int ntco, int nci,
                                                                     const bf16_t* __restrict__ zero, int swz,
                                                                     float* __restrict__ slab) {
    constexpr int NW = WM * WN, STAGES = 3;
    constexpr int RA = BMC * 2;                          // bytes per dY pixel row
    constexpr int APIECES = 64 * RA / 1024;              // dY tile pieces
    constexpr int XROWS = SX == 1 ? 63 + KW : 2 * XHALF; // X span positions
    constexpr int XPIECES = (XROWS + 7) / 8;
    constexpr int TP = APIECES + XPIECES;                // pieces per segment
    constexpr int PW = (TP + NW - 1) / NW;               // max pieces per wave
    constexpr int STAGE = TP * 1024;
    constexpr int MI = BMC / 16 / WM, NJ = KW * 4 / WN;
    static_assert(MI >= 1 && MI * 16 * WM == BMC && NJ * WN == KW * 4, "tile");
    __shared__ __attribute__((aligned(1024))) char smem[STAGES * STAGE];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid / WN, wn = wid % WN;
    // logical block: split-major, (co tile, ci chunk, ty) minor
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
    if (s_beg >= s_end) return;
    const int segs_row = d.Wo / 64;
    const int cout8 = (d.Cout + 7) / 8 * 8;
    const bool reflect = d.pad_mode == IRGAN_PAD_REFLECT;
    const int nrows = 63 * SX + KW;  // input columns in one span

    // issue segment s into ring stage `stage`
    auto issue = [&](int s, int stage) {
        const int rowi = s / segs_row, x0 = (s - rowi * segs_row) * 64;
        const int n = rowi / d.Ho, oy = rowi - n * d.Ho;
        int iy = oy * d.sy + ty + d.c0y;
        if (reflect) iy = reflect_idx(iy, d.H);
        const bool row_ok = (unsigned)iy < (unsigned)d.H;
        const long pix0 = (long)rowi * d.Wo + x0;        // first output pixel of the segment
        const long xrow = ((long)n * d.H + iy) * d.W;    // input row base (pixels)
        char* base = smem + stage * STAGE;
#pragma unroll
        for (int u = 0; u < PW; ++u) {
            const int j = u * NW + wid;  // piece index (wave-uniform)
            if (j >= TP) break;
            const bf16_t* src = zero;
            if (j < APIECES) {
                constexpr int RPP = 1024 / RA, SLOTS = RA / 16;
                const int pos = j * RPP + lane / SLOTS, slot = lane % SLOTS;
                int row, c16;
                if constexpr (RA >= 256) { row = pos; c16 = slot ^ (2 * t256(pos)); }
                else if constexpr (RA == 128) { row = pos; c16 = slot ^ (2 * t128(pos)); }
                else { row = pos ^ (((pos >> 3) & 1) << 2); c16 = slot; }
                if (co0 + c16 * 8 < cout8) src = dy + (pix0 + row) * d.ldy + d.yoff + co0 + c16 * 8;
            } else {
                const int pos = (j - APIECES) * 8 + (lane >> 3), slot = lane & 7;
                const int c16 = slot ^ (2 * t128(pos));
                const int h = SX == 1 ? pos : (pos < XHALF ? 2 * pos : 2 * (pos - XHALF) + 1);
                int ix = x0 * SX + d.c0x + h;
                if (reflect) ix = reflect_idx(ix, d.W);
                const bool ok = row_ok & (h < nrows) & ((unsigned)ix < (unsigned)d.W);
                if (ok) src = x + (xrow + ix) * d.ldx + d.xoff + ci0 + c16 * 8;
            }
            glds16(src, base + j * 1024);
        }
    };

    f32x4 acc[MI][NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // per-lane fragment geometry (ds_read_b64_tr_b16: lane 4q+p of a 16-lane
    // group g supplies row q (and q+4) of its 8-pixel run, columns 4p..4p+3)
    const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
    const int nk = s_end - s_beg;
    const bool more = wid < TP % NW;  // this wave issues PW pieces (else PW-1)
    issue(s_beg, 0);
    if (nk > 1) issue(s_beg + 1, 1);
    for (int kt = 0; kt < nk; ++kt) {
        if (kt + 1 < nk) {
            if constexpr (TP % NW == 0) wait_vmcnt<PW>();
            else { if (more) wait_vmcnt<PW>(); else wait_vmcnt<PW - 1>(); }
        } else {
            wait_vmcnt<0>();
        }
#if !WGX(8)
        lds_barrier();
#endif
        if (kt + 2 < nk && !WGX(2)) issue(s_beg + kt + 2, (kt + 2) % STAGES);
        const char* A = smem + (kt % STAGES) * STAGE;
        const char* X = A + APIECES * 1024;
#pragma unroll
        for (int h = 0; h < 2; ++h) {  // two 32-pixel MFMA k-steps per segment
            const int k_lo = 32 * h + 8 * g + q, k_hi = k_lo + 4;
            uint4 af[MI], bfr[NJ];
#if WGX(4)
            if (kt > 0) {
#pragma unroll
                for (int i = 0; i < MI; ++i) af[i] = make_uint4(kt, h, i, lane);
#pragma unroll
                for (int j = 0; j < NJ; ++j) bfr[j] = make_uint4(kt, j, h, lane);
            } else
#endif
            {
#pragma unroll
            for (int i = 0; i < MI; ++i) {
                const int col = (wm * MI + i) * 16 + 4 * p;
                int plo = k_lo, phi = k_hi;
                if constexpr (RA == 32) {
                    plo = k_lo ^ (((k_lo >> 3) & 1) << 2);
                    phi = k_hi ^ (((k_hi >> 3) & 1) << 2);
                }
                af[i] = tr_pair(A + img_off<RA>(plo, col), A + img_off<RA>(phi, col));
            }
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int jj = wn * NJ + j, tx = jj >> 2, col = (jj & 3) * 16 + 4 * p;
                int plo, phi;
                if constexpr (SX == 1) { plo = k_lo + tx; phi = k_hi + tx; }
                else {
                    const int b = (tx & 1) * XHALF + (tx >> 1);
                    plo = b + k_lo;
                    phi = b + k_hi;
                }
                bfr[j] = tr_pair(X + img_off<128>(plo, col), X + img_off<128>(phi, col));
            }
            }
#pragma unroll
            for (int i = 0; i < MI * !WGX(1); ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[i]),
                                                                        __builtin_bit_cast(bf16x8_t, bfr[j]),
                                                                        acc[i][j], 0, 0, 0);
        }
    }
    // C[row = co][col = ci]: row = (lane>>4)*4 + r, col = lane & 15.  Split-K
    // partials: plain stores into this split's slab (summed in a fixed order by
    // wgrad_slab_reduce) or, without a slab, fp32 atomics into dw.
    const int K = d.KH * KW * d.Cin;
#if WGX(16)
    {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
        if (s == 123.f) dw[0] = s;
        return;
    }
#endif
    float* const dst = slab ? slab + (long)split * d.Cout * K : nullptr;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            const int co = co0 + (wm * MI + i) * 16 + (lane >> 4) * 4 + rr;
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

// dw[i] += sum over splits s (in order) of slab[s][i]: the second stage of the
// split-K reduction (deterministic, no atomics).  n % 4 == 0.
__global__ __launch_bounds__(256) void wgrad_slab_reduce(const float* __restrict__ slab, int splits, long n,
                                                         float* __restrict__ dw) {
    const long n4 = n / 4;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
        slab_sum4(slab, splits, n, dw, i);
    }
}

template <int BMC, int KW, int SX, int WM, int WN>
void launch_t(const irgan_conv_desc* d, const void* x, const void* dy, float* dw, int splitk, hipStream_t st,
              const bf16_t* zero, int swz, float* ws, long ws_cap) {
    constexpr int NW = WM * WN;
    // resident blocks per CU (LDS and VGPR limits, from the runtime) x 256 CUs: the
    // grid is sized to at most one full round -- a grid just above the resident
    // capacity runs a second, nearly empty round
    static int occ = 0;  // resident blocks per CU (a property of the kernel on gfx950)
    if (!occ && (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, wgrad_halo_kernel<BMC, KW, SX, WM, WN>, NW * 64, 0) != hipSuccess || occ < 1))
        occ = 1;
    const int slots = occ * irgan_cu_count();
    const int ntco = irgan_cdiv(d->Cout, BMC), nci = d->Cin / 64;
    const int tiles = ntco * nci * d->KH;
    const int nseg = d->N * d->Ho * (d->Wo / 64);
    if (splitk <= 0) {
        const int maxs = irgan_cdiv(nseg, 4);  // >= 4 segments per split
        splitk = slots / tiles;
        if (splitk < 1) splitk = irgan_cdiv(slots, tiles);  // more tiles than slots: whole rounds anyway
        if (splitk > maxs) splitk = maxs;
        if (splitk < 1) splitk = 1;
        if (swz && (tiles * splitk) % 8) {  // grid multiple of 8 for the XCD remap, within the slots
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
    // slabs pay splitk*n*4 bytes twice (store + reduce); measured on MI355X they beat
    // fp32 atomics only at low split counts (resblock 3x3: 21 splits, -7 %), and
    // lose at 56-170 splits (down1 / up2 at 256^2: +3..12 %)
    // (deterministic mode: slabs at any split count)
    float* slab = (ws && splitk > 1 && (splitk <= 24 || irgan_det(d)) && n % 4 == 0 &&
                   (long)splitk * n <= ws_cap) ? ws : nullptr;
    wgrad_halo_kernel<BMC, KW, SX, WM, WN><<<tiles * splitk, WM * WN * 64, 0, st>>>(
        *d, (const bf16_t*)x, (const bf16_t*)dy, dw, spb, nseg, ntco, nci, zero, swz, slab);
    if (slab) {
        const int blocks = (int)std::min<long>(irgan_cdiv(n / 4, 256), 2048);
        wgrad_slab_reduce<<<blocks, 256, 0, st>>>(slab, splitk, n, dw);
    }
}

}  // namespace

// Preconditions: bf16; Cin % 64 == 0; ldx, xoff, ldy, yoff % 8 == 0; Wo % 64 == 0;
// sx == sy in {1, 2}; (Cout % 64 == 0 and KW in {3, 4}) or (Cout <= 8, KW == 7, stride 1).
extern "C" int irgan_conv_wgrad_halo(const irgan_conv_desc* d, const void* x, const void* dy, float* dw, int splitk,
                                     float* ws, long ws_cap, hipStream_t st) {
    if ((long)d->N * d->Ho * d->Wo <= 0) return 0;
    if (d->Cin % 64 || d->ldx % 8 || d->xoff % 8 || d->ldy % 8 || d->yoff % 8 || d->Wo % 64 || d->sx != d->sy ||
        (d->sx != 1 && d->sx != 2))
        return IRGAN_EUNSUPPORTED;
    static void* zero_cache[IRGAN_MAX_DEVICES];  // the zero page's address per device
    const bf16_t* zero = (const bf16_t*)irgan_symbol(HIP_SYMBOL(g_wgh_zero_page), zero_cache);
    if (!zero) return IRGAN_EUNSUPPORTED;
    const int swz = irgan_xcd_swz();
    const int s2 = d->sx == 2;
    if (d->Cout % 128 == 0 && d->KW == 3 && !s2) {
        // 4 waves of 128 x 48 wave tiles (each A fragment read feeds 3 MFMAs, each B 8):
        // resblock wgrad 124 -> 114 us vs 8 waves of 64 x 48 (profiles/r01_s9_wgrad_ab.txt)
        launch_t<128, 3, 1, 1, 4>(d, x, dy, dw, splitk, st, zero, swz, ws, ws_cap);
    } else if (d->Cout % 128 == 0 && d->KW == 3) {
        if (s2) launch_t<128, 3, 2, 2, 4>(d, x, dy, dw, splitk, st, zero, swz, ws, ws_cap);
        else launch_t<128, 3, 1, 2, 4>(d, x, dy, dw, splitk, st, zero, swz, ws, ws_cap);
    } else if (d->Cout % 128 == 0 && d->KW == 4) {
        if (s2) launch_t<128, 4, 2, 2, 4>(d, x, dy, dw, splitk, st, zero, swz, ws, ws_cap);
        else launch_t<128, 4, 1, 2, 4>(d, x, dy, dw, splitk, st, zero, swz, ws, ws_cap);
    } else if (d->Cout % 64 == 0 && d->KW == 3) {
        if (s2) launch_t<64, 3, 2, 2, 4>(d, x, dy, dw, splitk, st, zero, swz, ws, ws_cap);
        else launch_t<64, 3, 1, 2, 4>(d, x, dy, dw, splitk, st, zero, swz, ws, ws_cap);
    } else if (d->Cout % 64 == 0 && d->KW == 4) {
        if (s2) launch_t<64, 4, 2, 2, 4>(d, x, dy, dw, splitk, st, zero, swz, ws, ws_cap);
        else launch_t<64, 4, 1, 2, 4>(d, x, dy, dw, splitk, st, zero, swz, ws, ws_cap);
    } else if (d->Cout <= 8 && d->KW == 7 && !s2) {
        launch_t<16, 7, 1, 1, 4>(d, x, dy, dw, splitk, st, zero, swz, ws, ws_cap);
    } else {
        return IRGAN_EUNSUPPORTED;
    }
    IRGAN_LAUNCH_CHECK();
    return 0;
}
