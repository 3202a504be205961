// bf16 stride-1 convolution with a resident input halo (forward and the
// stride-1 / per-phase backward-data launches).
//
// The per-tap implicit GEMM of conv_glds.hip streams one 256-pixel x 64-channel
// A tile per tap, so a 3x3 conv moves its input through L2 -> LDS nine times;
// profiled on MI355X that kernel sits at ~20 GB/s/CU of LDS-DMA with the waves
// parked on vmcnt 48% of the time, i.e. it is bound by L2->LDS bytes, not MFMA.
// Here a block owns a 16x16 output patch of one image: per 64-channel chunk it
// DMAs the (16+KH-1)x(16+KW-1) input halo into LDS ONCE (reflect / zero padding
// folded into the source address) and runs all KH*KW taps against it as LDS
// address shifts; only the weight tile (BN x 64 per tap) streams per K-step.
// L2->LDS bytes per chunk drop from taps*48 KiB to ~41 KiB + taps*16 KiB.
//
// 512 threads = 8 waves (4 pixel-row groups x 2 channel halves), block tile
// 256 pixels x BN, K-step = 64 channels of one tap, mfma_f32_16x16x32_bf16.
// Pipeline: K-steps (chunk, tap) flattened; weights of step k+2 are issued
// while k runs, the halo of chunk c+1 as soon as chunk c starts (a whole
// chunk of lead time).  Halo: two buffers (chunk parity), weights: 3-stage
// ring.  Requires taps >= 2.
#include "conv_epilogue.h"

namespace {

// zero page for padded / out-of-range halo rows (this translation unit's own copy)
__device__ __attribute__((aligned(4096))) bf16_t g_halo_zero_page[2048];


IRGAN_HD int lds_off(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }

constexpr int PH = 16, PW = 16;  // output patch

// BN: output-channel tile (128 | 64 | 16); HU: halo pieces per wave (HROWS =
// HU*64 rows: 6 -> 384 >= 19*19 for taps <= 4x4, 8 -> 512 >= 22*22 for 7x7);
// WM x WN waves over (pixels, channels).
template <int BN, int HU, int WM, int WN>
__global__ __launch_bounds__(512, 1) void conv_halo_kernel(const irgan_conv_desc d, const bf16_t* __restrict__ x,
                                                           const bf16_t* __restrict__ w,
                                                           const float* __restrict__ bias, void* __restrict__ y,
                                                           const void* __restrict__ mask,
                                                           const bf16_t* __restrict__ zero, int ntn, int tpx, int tpy,
                                                           int swz) {
    static_assert(WM * WN == 8, "8 waves");
    constexpr int STAGES = 3, HROWS = HU * 64;
    constexpr int HBYTES = HROWS * 128, BBYTES = BN * 128;
    constexpr int MI = 256 / WM / 16, NJ = BN / WN / 16;
    constexpr int BP = BN / 8;                  // weight-tile pieces (1 KiB = 8 channel rows)
    constexpr int BU = BP >= 8 ? BP / 8 : 1;    // pieces per issuing wave
    constexpr int LDS = 2 * HBYTES + STAGES * BBYTES;
    static_assert(MI * 16 * WM == 256 && NJ * 16 * WN == BN, "tile");
    static_assert(256 * (BN + 4) * 4 <= LDS, "epilogue staging fits");
    __shared__ __attribute__((aligned(1024))) char smem[LDS];
    char* const sH = smem;
    char* const sB = smem + 2 * HBYTES;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid / WN, wn = wid % WN;
    const bool bload = BP >= 8 || wid < BP;     // does this wave load weight pieces
    int t = xcd_tile(blockIdx.x, gridDim.x, swz);
    const int nt = t % ntn;
    t /= ntn;
    const int pxi = t % tpx;
    t /= tpx;
    const int pyi = t % tpy;
    const int img = t / tpy;
    const int py0 = pyi * PH, px0 = pxi * PW, n0 = nt * BN;
    const int taps = d.KH * d.KW;
    const int HWd = PW + d.KW - 1;
    const int hrows = (PH + d.KH - 1) * HWd;
    const int Kw = taps * d.Cin;  // weight row stride (Cin % 64 == 0 -> no tap padding)
    const int nk = (d.Cin / 64) * taps;
    const int sub = lane >> 3;
    const int chunk = (lane & 7) ^ sub;  // source chunk for this lane's LDS slot (row & 7 == sub)
    const bool reflect = d.pad_mode == IRGAN_PAD_REFLECT;

    // halo rows this lane loads: piece (wid*HU + u), row sub of the piece
    long h_off[HU];
#pragma unroll
    for (int u = 0; u < HU; ++u) {
        const int h = (wid * HU + u) * 8 + sub;
        const int hy = h / HWd, hx = h - hy * HWd;
        int iy = py0 + hy + d.c0y, ix = px0 + hx + d.c0x;
        if (reflect) {
            iy = reflect_idx(iy, d.H);
            ix = reflect_idx(ix, d.W);
        }
        const bool ok = (h < hrows) & ((unsigned)iy < (unsigned)d.H) & ((unsigned)ix < (unsigned)d.W);
        h_off[u] = ok ? (((long)img * d.H + iy) * d.W + ix) * d.ldx + d.xoff + chunk * 8 : -1;
    }
    const bf16_t* b_src[BU];
#pragma unroll
    for (int u = 0; u < BU; ++u) {
        const int co = n0 + (wid * BU + u) * 8 + sub;
        b_src[u] = co < d.Cout ? w + (long)co * Kw + chunk * 8 : nullptr;
    }

    auto issue_halo = [&](int c) {
        char* dst = sH + (c & 1) * HBYTES + wid * HU * 1024;
#pragma unroll
        for (int u = 0; u < HU; ++u) glds16(h_off[u] >= 0 ? x + h_off[u] + c * 64 : zero, dst + u * 1024);
    };
    auto issue_w = [&](int kt, int stage) {
        if (!bload) return;
        const int c = kt / taps, tp = kt - c * taps;
        const int kcol = tp * d.Cin + c * 64;
#pragma unroll
        for (int u = 0; u < BU; ++u)
            glds16(b_src[u] ? b_src[u] + kcol : zero, sB + stage * BBYTES + (wid * BU + u) * 1024);
    };

    f32x4 acc[MI][NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // Issue order: halo(0), W(0), W(1); then at the top of step kt (after its
    // barrier): halo(c+1) when kt is the first tap of chunk c (its buffer held
    // chunk c-1, retired by that barrier), then W(kt+2).  So the halo of chunk
    // c+1 has a whole chunk of lead time, and the only loads younger than W(kt)
    // are W(kt+1) and a halo issued at step kt-1.
    const int nchunk = d.Cin / 64;
    issue_halo(0);
    issue_w(0, 0);
    if (nk > 1) issue_w(1, 1);
    int c = 0, tp = 0;  // chunk / tap of step kt
    for (int kt = 0; kt < nk; ++kt) {
        if (kt + 1 < nk) {
            const int pk = kt - 1;  // did step kt-1 issue a halo (after W(kt))?
            const bool h = pk >= 0 && pk % taps == 0 && pk / taps + 1 < nchunk;
            if (bload) {
                if (h) wait_vmcnt<BU + HU>(); else wait_vmcnt<BU>();
            } else {
                if (h) wait_vmcnt<HU>(); else wait_vmcnt<0>();
            }
        } else {
            wait_vmcnt<0>();
        }
        lds_barrier();
        if (tp == 0 && c + 1 < nchunk) issue_halo(c + 1);
        if (kt + 2 < nk) issue_w(kt + 2, (kt + 2) % STAGES);
        const char* Hb = sH + (c & 1) * HBYTES;
        const char* B = sB + (kt % STAGES) * BBYTES;
        const int ty = tp / d.KW, tx = tp - ty * d.KW;
        // fragment i covers patch row wm*MI + i, columns lane&15
        const int hbase = (wm * MI + ty) * HWd + (lane & 15) + tx;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            uint4 af[MI], bfr[NJ];
            const int ch = h * 4 + (lane >> 4);
#pragma unroll
            for (int i = 0; i < MI; ++i) af[i] = *(const uint4*)(Hb + lds_off(hbase + i * HWd, ch));
#pragma unroll
            for (int j = 0; j < NJ; ++j)
                bfr[j] = *(const uint4*)(B + lds_off(wn * (BN / WN) + j * 16 + (lane & 15), ch));
#pragma unroll
            for (int i = 0; i < MI; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[i]),
                                                                        __builtin_bit_cast(bf16x8_t, bfr[j]),
                                                                        acc[i][j], 0, 0, 0);
        }
        if (++tp == taps) {
            tp = 0;
            ++c;
        }
    }

    // epilogue: fragment i = patch row wm*MI+i, C row (lane>>4)*4+r = patch column
    conv_epilogue<BN, MI, NJ, WM, WN, 512>(d, acc, smem, wm, wn, n0, bias, y, mask, [&](int m) -> long {
        const int oy = py0 + (m >> 4), ox = px0 + (m & 15);
        if (oy >= d.Ho || ox >= d.Wo) return -1;
        return ((long)img * d.OH + oy * d.omy + d.ooy) * d.OW + ox * d.omx + d.oox;
    });
}

template <int BN, int HU, int WM, int WN>
void launch_halo(const irgan_conv_desc* d, const void* x, const void* w, const float* bias, void* y, const void* mask,
                 hipStream_t st, const bf16_t* zero, int swz) {
    const int tpx = irgan_cdiv(d->Wo, PW), tpy = irgan_cdiv(d->Ho, PH);
    const int ntn = irgan_cdiv(d->Cout, BN);
    conv_halo_kernel<BN, HU, WM, WN><<<d->N * tpy * tpx * ntn, 512, 0, st>>>(
        *d, (const bf16_t*)x, (const bf16_t*)w, bias, y, mask, zero, ntn, tpx, tpy, swz);
}

// ---------------------------------------------------------------------------
// Narrow output (Cout <= 8: G outc 64->3 7x7, VGG conv1_1 backward-data, D's
// last 4x4 layer).  The tile-per-tap pipeline above pays a barrier and a weight
// DMA per K-step for 2 MFMAs per wave; with Cout <= 8 the weights of ALL taps
// of a 64-channel chunk are only taps x 8 rows x 128 B (<= 49 KiB), so they
// land in LDS with the halo and the whole chunk (taps x 2 sub-steps) runs
// without a barrier.  Weight lanes >= 8 of the B fragment are zero registers.
// 8 waves, wave w = patch rows 2w, 2w+1 (2 pixel fragments), NB halo/weight
// buffers: 2 for multi-chunk layers (chunk c+1 streams in under chunk c).
template <int KH, int KW, int HU, int NB>
__global__ __launch_bounds__(512, 1) void conv_narrow_kernel(const irgan_conv_desc d, const bf16_t* __restrict__ x,
                                                             const bf16_t* __restrict__ w,
                                                             const float* __restrict__ bias, void* __restrict__ y,
                                                             const void* __restrict__ mask,
                                                             const bf16_t* __restrict__ zero, int tpx, int tpy,
                                                             int swz) {
    constexpr int TAPS = KH * KW, HWd = PW + KW - 1, HROWS = (PH + KH - 1) * HWd;
    constexpr int WPC = (TAPS * 8 + 7) / 8;             // weight pieces (8 rows of 128 B) per chunk
    constexpr int WPW = (WPC + 7) / 8;                  // weight pieces per wave
    constexpr int HB = HU * 8 * 1024, BUF = HB + WPC * 1024;
    static_assert(HU * 64 >= HROWS && NB * BUF <= 160 * 1024 && 256 * 20 * 4 <= NB * BUF, "lds");
    __shared__ __attribute__((aligned(1024))) char smem[NB * BUF];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    int t = xcd_tile(blockIdx.x, gridDim.x, swz);
    const int pxi = t % tpx;
    t /= tpx;
    const int pyi = t % tpy;
    const int img = t / tpy;
    const int py0 = pyi * PH, px0 = pxi * PW;
    const int Kw = TAPS * d.Cin;
    const int sub = lane >> 3;
    const int chunk = (lane & 7) ^ sub;
    const bool reflect = d.pad_mode == IRGAN_PAD_REFLECT;

    long h_off[HU];
#pragma unroll
    for (int u = 0; u < HU; ++u) {
        const int h = (u * 8 + wid) * 8 + sub;
        const int hy = h / HWd, hx = h - hy * HWd;
        int iy = py0 + hy + d.c0y, ix = px0 + hx + d.c0x;
        if (reflect) {
            iy = reflect_idx(iy, d.H);
            ix = reflect_idx(ix, d.W);
        }
        const bool ok = (h < HROWS) & ((unsigned)iy < (unsigned)d.H) & ((unsigned)ix < (unsigned)d.W);
        h_off[u] = ok ? (((long)img * d.H + iy) * d.W + ix) * d.ldx + d.xoff + chunk * 8 : -1;
    }
    long w_off[WPW];  // weight LDS row r = tap*8 + co
#pragma unroll
    for (int v = 0; v < WPW; ++v) {
        const int r = (v * 8 + wid) * 8 + sub, tp = r >> 3, co = r & 7;
        w_off[v] = (v * 8 + wid < WPC && tp < TAPS && co < d.Cout) ? (long)co * Kw + tp * d.Cin + chunk * 8 : -1;
    }
    auto issue = [&](int c, int buf) {
        char* base = smem + buf * BUF;
#pragma unroll
        for (int u = 0; u < HU; ++u)
            glds16(h_off[u] >= 0 ? x + h_off[u] + c * 64 : zero, base + (u * 8 + wid) * 1024);
#pragma unroll
        for (int v = 0; v < WPW; ++v)
            if (v * 8 + wid < WPC) glds16(w_off[v] >= 0 ? w + w_off[v] + c * 64 : zero, base + HB + (v * 8 + wid) * 1024);
    };

    f32x4 acc[2][1];
    acc[0][0] = acc[1][0] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nchunk = d.Cin / 64;
    const bool wlane = (lane & 15) < 8;
    issue(0, 0);
#pragma unroll 1
    for (int c = 0; c < nchunk; ++c) {
        wait_vmcnt<0>();
        lds_barrier();
        if (NB == 2 && c + 1 < nchunk) issue(c + 1, (c + 1) & 1);
        const char* Hb = smem + (NB == 2 ? (c & 1) : 0) * BUF;
        const char* Wb = Hb + HB;
#pragma unroll 1
        for (int ty = 0; ty < KH; ++ty)
#pragma unroll
        for (int tx = 0; tx < KW; ++tx) {
            const int tp = ty * KW + tx;
            const int hrow = (wid * 2 + ty) * HWd + (lane & 15) + tx;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int ch = h * 4 + (lane >> 4);
                const uint4 a0 = *(const uint4*)(Hb + lds_off(hrow, ch));
                const uint4 a1 = *(const uint4*)(Hb + lds_off(hrow + HWd, ch));
                uint4 b = make_uint4(0u, 0u, 0u, 0u);
                if (wlane) b = *(const uint4*)(Wb + lds_off(tp * 8 + (lane & 15), ch));
                acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a0),
                                                                    __builtin_bit_cast(bf16x8_t, b), acc[0][0], 0, 0, 0);
                acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a1),
                                                                    __builtin_bit_cast(bf16x8_t, b), acc[1][0], 0, 0, 0);
            }
        }
        if (NB == 1 && c + 1 < nchunk) {
            lds_barrier();  // every wave is done with the single buffer
            issue(c + 1, 0);
        }
    }
    conv_epilogue<16, 2, 1, 8, 1, 512>(d, acc, smem, wid, 0, 0, bias, y, mask, [&](int m) -> long {
        const int oy = py0 + (m >> 4), ox = px0 + (m & 15);
        if (oy >= d.Ho || ox >= d.Wo) return -1;
        return ((long)img * d.OH + oy * d.omy + d.ooy) * d.OW + ox * d.omx + d.oox;
    });
}

template <int KH, int KW, int HU, int NB>
void launch_narrow(const irgan_conv_desc* d, const void* x, const void* w, const float* bias, void* y,
                   const void* mask, hipStream_t st, const bf16_t* zero, int swz) {
    const int tpx = irgan_cdiv(d->Wo, PW), tpy = irgan_cdiv(d->Ho, PH);
    conv_narrow_kernel<KH, KW, HU, NB><<<d->N * tpy * tpx, 512, 0, st>>>(*d, (const bf16_t*)x, (const bf16_t*)w, bias,
                                                                        y, mask, zero, tpx, tpy, swz);
}

}  // namespace

extern "C" int irgan_conv_fwd_rowspan(const irgan_conv_desc* d, const void* x, const void* w, const float* bias,
                                      void* y, const void* mask, hipStream_t st);

// Preconditions (checked by the dispatcher in conv.hip): bf16, sy = sx = 1,
// Cin % 64 == 0, ldx % 8 == 0, xoff % 8 == 0, 2 <= KH*KW, KH, KW <= 7 (taps
// beyond 4x4 only for Cout <= 64).
extern "C" int irgan_conv_fwd_halo(const irgan_conv_desc* d, const void* x, const void* w, const float* bias, void* y,
                                   const void* mask, hipStream_t st) {
    if ((long)d->N * d->Ho * d->Wo <= 0 || d->Cout <= 0) return 0;
    if (d->sy != 1 || d->sx != 1 || d->Cin % 64 || d->KH > 7 || d->KW > 7 || d->KH * d->KW < 2)
        return IRGAN_EUNSUPPORTED;
    const bool big = d->KH > 4 || d->KW > 4;
    if (big && d->Cout > 64) return IRGAN_EUNSUPPORTED;
    static void* zero_cache[IRGAN_MAX_DEVICES];  // the zero page's address per device
    const bf16_t* zero = (const bf16_t*)irgan_symbol(HIP_SYMBOL(g_halo_zero_page), zero_cache);
    if (!zero) return IRGAN_EUNSUPPORTED;
    const int swz = irgan_xcd_swz();
    static const bool narrow = !getenv("IRGAN_NO_NARROW");
    if (narrow && d->Cout <= 8) {
        // one 64-channel chunk: the row-span GEMM (conv_rowspan.hip: outc, VGG conv1_1 dgrad)
        if (irgan_conv_fwd_rowspan(d, x, w, bias, y, mask, st) == 0) return 0;
        if (d->KH == 7 && d->KW == 7) { launch_narrow<7, 7, 8, 1>(d, x, w, bias, y, mask, st, zero, swz); IRGAN_LAUNCH_CHECK(); return 0; }
        if (d->KH == 4 && d->KW == 4) { launch_narrow<4, 4, 6, 2>(d, x, w, bias, y, mask, st, zero, swz); IRGAN_LAUNCH_CHECK(); return 0; }
        if (d->KH == 3 && d->KW == 3) { launch_narrow<3, 3, 6, 2>(d, x, w, bias, y, mask, st, zero, swz); IRGAN_LAUNCH_CHECK(); return 0; }
    }
    if (d->Cout > 64) launch_halo<128, 6, 4, 2>(d, x, w, bias, y, mask, st, zero, swz);
    else if (d->Cout > 16) {
        if (big) launch_halo<64, 8, 4, 2>(d, x, w, bias, y, mask, st, zero, swz);
        else launch_halo<64, 6, 4, 2>(d, x, w, bias, y, mask, st, zero, swz);
    } else {
        if (big) launch_halo<16, 8, 8, 1>(d, x, w, bias, y, mask, st, zero, swz);
        else launch_halo<16, 6, 8, 1>(d, x, w, bias, y, mask, st, zero, swz);
    }
    IRGAN_LAUNCH_CHECK();
    return 0;
}
