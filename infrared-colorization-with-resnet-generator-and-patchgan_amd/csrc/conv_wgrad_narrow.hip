// bf16 backward-weight convolution for narrow inputs stored as 8 zero-padded
// channels: the generator's input layer inc (1 -> 64, 7x7 reflect, ir:459-460)
// and the discriminator's model.0 (4 -> 64, 4x4 stride 2, ir:600).
//
//   dW[co][ty][tx][ci] += sum_p dY[p][co] * X[s*oy + ty + c0y][s*ox + tx + c0x][ci]
//
// As a GEMM: M = 64 output channels, K = every output pixel of the batch
// (0.5-1 M), N = the real (tap, channel) pairs -- 49 for inc, 64 for model.0.
// The 64-channel-chunk wgrad kernels would run these at 8x / 2x the work (the
// zero channels).  Here N is packed densely:
//   * CR = 4 channels (model.0): an n-fragment is 4 taps x 4 channels; the input
//     row spans sit in LDS as 8-byte pixel records (the real channels only), so
//     the 4 channels of one tap are one 8-byte transposed-read row;
//   * CR = 1 (inc): an n-fragment is 16 taps of a padded 8-wide tap row (n =
//     ty*8 + tx, tx = 7 discarded); the span is one bf16 per pixel, kept in 4
//     copies shifted by 0..3 elements so that the 4 consecutive taps of any pixel
//     start on an 8-byte boundary in one of them.
// Both MFMA operands come from ds_read_b64_tr_b16 (its 16-lane gather takes an
// arbitrary 8-byte-aligned row address per lane: the stride-2 im2col is only
// addressing).  A block walks 64-pixel output row segments: the dY tile [64 px]
// [64 co] arrives by LDS-DMA, the input spans through registers (compacted to the
// real channels on the way), DIST = 3 segments ahead through a 4-stage LDS ring,
// one barrier per segment.  Wave w owns a (co, n) sub-tile of the
// 64 x NPAD output.  Split-K over segments: each block writes its 64 x NPAD fp32
// partial tile to the caller's slab and wgrad_narrow_reduce sums the slabs in
// block order (deterministic) into dW.
#include "common.h"

namespace {

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s4;

constexpr int NT = 256;  // 4 waves
constexpr int SEG = 64;  // output pixels per segment
constexpr int COT = 64;  // output channels (the whole layer)
constexpr int STG = 4;   // LDS stages
constexpr int DIST = 3;  // segments in flight ahead of the one being multiplied

template <int KH, int KW, int S, int CR>
struct NW {
    static constexpr int TAPS = KH * KW;
    static constexpr int NREAL = CR == 1 ? KH * 8 : TAPS * CR;  // n columns (incl. the tx = 7 pad for CR = 1)
    static constexpr int NFR = (NREAL + 15) / 16;               // n fragments
    static constexpr int NPAD = NFR * 16;
    static constexpr int XW = S * (SEG - 1) + KW;              // input pixels per span row
    static constexpr int XWP = (XW + 8 + 7) / 8 * 8;           // span row pitch (+ tap-row overrun)
    static constexpr int XE = KH * XW;                          // span pixels per segment
    static constexpr int XPASS = (XE + NT - 1) / NT;
    static constexpr int XB = CR == 1 ? 4 * KH * XWP * 2 : KH * XWP * 8;  // X image bytes
    static constexpr int DYB = SEG * COT * 2;
    static constexpr int STAGE = DYB + (XB + 15) / 16 * 16;
    // wave sub-tiles: waves split n fragments first, then co fragments
    static constexpr int NW_N = NFR >= 4 ? 4 : NFR;            // waves along n
    static constexpr int NW_C = 4 / NW_N;                       // waves along co
    static constexpr int FPW = (NFR + NW_N - 1) / NW_N;         // n fragments per wave
    static constexpr int CPW = 4 / NW_C;                        // co fragments per wave
};

IRGAN_HD uint4 tr2(const char* lo, const char* hi) {
    const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)lo);
    const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)hi);
    uint4 out;
    __builtin_memcpy(&out, &a, 8);
    __builtin_memcpy((char*)&out + 8, &b, 8);
    return out;
}

template <int KH, int KW, int S, int CR>
__global__ __launch_bounds__(NT, 2) void wgrad_narrow_kernel(const irgan_conv_desc d, const bf16_t* __restrict__ x,
                                                              const bf16_t* __restrict__ dy, float* __restrict__ ws,
                                                              int segs_per_block, int nseg, int segs_per_row) {
    using C = NW<KH, KW, S, CR>;
    __shared__ __attribute__((aligned(1024))) char smem[STG * C::STAGE];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int sg0 = blockIdx.x * segs_per_block;
    const int sg1 = min(nseg, sg0 + segs_per_block);
    const uint32_t ybytes = (uint32_t)((long)d.N * d.Ho * d.Wo * d.ldy * 2);
    const i32x4 yr = make_rsrc(dy, ybytes);
    const bool reflect = d.pad_mode == IRGAN_PAD_REFLECT;

    auto seg_pos = [&](int sg, int& img, int& oy, int& ox0, int& row) {
        const int xs = sg % segs_per_row;
        row = sg / segs_per_row;  // img * Ho + oy
        img = row / d.Ho;
        oy = row - img * d.Ho;
        ox0 = xs * SEG;
    };
    // dY tile by LDS-DMA: 512 16-byte chunks (pixel e >> 3, chunk e & 7), 2 per thread
    auto issue_dy = [&](int sg, int st) {
        int img, oy, ox0, row;
        seg_pos(sg, img, oy, ox0, row);
        char* base = smem + st * C::STAGE;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int e = u * NT + tid, px = e >> 3, ch = e & 7;
            const bool ok = ox0 + px < d.Wo;
            const uint32_t off = ok ? (uint32_t)((((long)row * d.Wo + ox0 + px) * d.ldy + d.yoff + ch * 8) * 2)
                                    : IRGAN_OOB;
            blds16(yr, off, base + u * NT * 16 + wid * 1024);
        }
    };
    // input span pixels through registers (the first 4 channels of each 16-byte record)
    uint2 xvs[DIST][C::XPASS];
    auto load_x = [&](int sg, uint2 (&xv)[C::XPASS]) {
        int img, oy, ox0, row;
        seg_pos(sg, img, oy, ox0, row);
#pragma unroll
        for (int u = 0; u < C::XPASS; ++u) {
            const int e = u * NT + tid;
            const int ty = e / C::XW, pos = e - ty * C::XW;
            int iy = S * oy + ty + d.c0y, ix = S * ox0 + pos + d.c0x;
            if (reflect) {  // ReflectionPad2d: the padded input is the mirrored pixel
                iy = reflect_idx(iy, d.H);
                ix = reflect_idx(ix, d.W);
            }
            // (the span's tail past the last output pixel may land anywhere: its dY is zero)
            const bool ok = e < C::XE && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W;
            xv[u] = ok ? *(const uint2*)(x + (((long)img * d.H + iy) * d.W + ix) * d.ldx + d.xoff)
                       : make_uint2(0u, 0u);
        }
    };
    auto store_x = [&](int st, const uint2 (&xv)[C::XPASS]) {
        char* xb = smem + st * C::STAGE + C::DYB;
#pragma unroll
        for (int u = 0; u < C::XPASS; ++u) {
            const int e = u * NT + tid;
            if (e >= C::XE) continue;
            const int ty = e / C::XW, pos = e - ty * C::XW;
            if constexpr (CR == 4) {
                *(uint2*)(xb + (ty * C::XWP + pos) * 8) = xv[u];
            } else {  // copy c holds X[pos + c] at element pos: pixel pos goes to copies c <= pos
                const bf16_t v = (bf16_t)(xv[u].x & 0xffffu);
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    if (pos >= c) *(bf16_t*)(xb + ((c * KH + ty) * C::XWP + pos - c) * 2) = v;
            }
        }
    };
    // zero the stages once (the padded tail positions are read by the discarded columns)
    for (int i = tid * 16; i < STG * C::STAGE; i += NT * 16) *(uint4*)(smem + i) = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();

    const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
    const int wn = wid % C::NW_N, wc = wid / C::NW_N;
    f32x4 acc[C::CPW][C::FPW];
#pragma unroll
    for (int i = 0; i < C::CPW; ++i)
#pragma unroll
        for (int f = 0; f < C::FPW; ++f) acc[i][f] = f32x4{0.f, 0.f, 0.f, 0.f};
    // B: column block p of fragment fr -> byte offset (pixel 0 of the segment) in the X image
    int boff[C::FPW];
#pragma unroll
    for (int f = 0; f < C::FPW; ++f) {
        const int fr = wn + C::NW_N * f;
        if constexpr (CR == 4) {
            const int tap = min(4 * fr + p, C::TAPS - 1);  // taps past the last: any valid row (discarded)
            const int ty = tap / KW, tx = tap - (tap / KW) * KW;
            boff[f] = (ty * C::XWP + tx) * 8;
        } else {
            const int n0 = 16 * fr + 4 * p;  // 4 taps ty*8 + tx .. + 3 (same ty)
            const int ty = min(n0 >> 3, KH - 1), tx = n0 & 7;
            boff[f] = ty * C::XWP * 2 + tx * 2;  // + the pixel's element offset, split over the 4 copies
        }
    }

#pragma unroll
    for (int j = 0; j < DIST; ++j)
        if (sg0 + j < sg1) {
            issue_dy(sg0 + j, j);
            load_x(sg0 + j, xvs[j]);
        }
    // iteration k: store_x(k) (its register loads are the oldest the compiler waits for,
    // and dY(k) was issued before them, so it has landed too), barrier, issue k + DIST
    // into the stage segment k-1 used, multiply segment k
#pragma unroll 1
    for (int sg = sg0; sg < sg1; sg += DIST) {
#pragma unroll
        for (int j = 0; j < DIST; ++j) {
        const int k = sg + j;
        if (k >= sg1) break;
        const int st = (k - sg0) % STG;
        store_x(st, xvs[j]);
        wait_vmcnt<(DIST - 1) * (2 + C::XPASS)>();
        __syncthreads();
        if (k + DIST < sg1) {
            issue_dy(k + DIST, (k + DIST - sg0) % STG);
            load_x(k + DIST, xvs[j]);
        }
        const char* ydt = smem + st * C::STAGE;
        const char* xa = ydt + C::DYB;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int pix = ks * 32 + g * 8 + q;  // the first read's row; the second is pix + 4
            uint4 a[C::CPW];
#pragma unroll
            for (int i = 0; i < C::CPW; ++i) {
                const char* r0 = ydt + pix * 128 + ((wc * C::CPW + i) * 16 + 4 * p) * 2;
                a[i] = tr2(r0, r0 + 4 * 128);
            }
#pragma unroll
            for (int f = 0; f < C::FPW; ++f) {
                if (wn + C::NW_N * f >= C::NFR) continue;  // wave-uniform
                uint4 b;
                if constexpr (CR == 4) {
                    const char* r0 = xa + boff[f] + S * pix * 8;
                    b = tr2(r0, r0 + S * 4 * 8);
                } else {
                    const int e0 = S * pix, e1 = S * (pix + 4);  // element offsets of the two rows
                    const char* r0 = xa + ((e0 & 3) * KH * C::XWP) * 2 + boff[f] + (e0 & ~3) * 2;
                    const char* r1 = xa + ((e1 & 3) * KH * C::XWP) * 2 + boff[f] + (e1 & ~3) * 2;
                    b = tr2(r0, r1);
                }
#pragma unroll
                for (int i = 0; i < C::CPW; ++i)
                    acc[i][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a[i]),
                                                                        __builtin_bit_cast(bf16x8_t, b), acc[i][f],
                                                                        0, 0, 0);
            }
        }
        }
    }
    // partial tile -> slab: lane holds D[co = 16 ci + 4(lane >> 4) + r][n = 16 fr + (lane & 15)]
    float* wsb = ws + (long)blockIdx.x * COT * C::NPAD;
#pragma unroll
    for (int f = 0; f < C::FPW; ++f) {
        const int fr = wn + C::NW_N * f;
        if (fr >= C::NFR) continue;
#pragma unroll
        for (int i = 0; i < C::CPW; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                wsb[((wc * C::CPW + i) * 16 + 4 * (lane >> 4) + r) * C::NPAD + fr * 16 + (lane & 15)] = acc[i][f][r];
    }
}

// dW[co][ty][tx][ci] += sum over blocks of slab[b][co][n]; n = ty*8 + tx (CR 1) or
// tap*4 + ci (CR 4); padded columns are skipped
// block = 64 outputs x 16 lanes; lane j sums partials j, j+16, ... then the 16 are
// combined in a fixed order (deterministic)
__global__ __launch_bounds__(1024) void wgrad_narrow_reduce(const float* __restrict__ ws, int nb, int npad, int KH,
                                                           int KW, int cr, int Cin, float* __restrict__ dw) {
    __shared__ float red[16][64];
    const int ol = threadIdx.x & 63, j = threadIdx.x >> 6;
    const int o = blockIdx.x * 64 + ol;
    const bool in = o < COT * npad;
    float s = 0.f;
    if (in)
        for (int b0 = j; b0 < nb; b0 += 16 * 8) {  // 8 loads in flight, added in block order
            float v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = b0 + 16 * k < nb ? ws[(long)(b0 + 16 * k) * COT * npad + o] : 0.f;
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (b0 + 16 * k < nb) s += v[k];
        }
    red[j][ol] = s;
    __syncthreads();
    if (j != 0 || !in) return;
    s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += red[k][ol];
    const int co = o / npad, n = o - co * npad;
    int ty, tx, ci;
    if (cr == 1) {
        ty = n >> 3;
        tx = n & 7;
        ci = 0;
        if (ty >= KH || tx >= KW) return;
    } else {
        const int tap = n / cr;
        ci = n - tap * cr;
        if (tap >= KH * KW || ci >= Cin) return;
        ty = tap / KW;
        tx = tap - ty * KW;
    }
    dw[(((long)co * KH + ty) * KW + tx) * Cin + ci] += s;
}

template <int KH, int KW, int S, int CR>
int launch_narrow(const irgan_conv_desc* d, const void* x, const void* dy, float* dw, float* ws, long ws_cap,
                  hipStream_t st) {
    using C = NW<KH, KW, S, CR>;
    const int segs_per_row = irgan_cdiv(d->Wo, SEG);
    const long nseg = (long)d->N * d->Ho * segs_per_row;
    const long tile = (long)COT * C::NPAD;
    int nb = (int)std::min<long>(irgan_cdiv(nseg, 8), 1024);  // >= 8 segments per block
    if ((long)nb * tile > ws_cap) nb = (int)(ws_cap / tile);
    if (nb < 1) return IRGAN_EUNSUPPORTED;
    const int spb = irgan_cdiv(nseg, nb);
    nb = irgan_cdiv(nseg, spb);
    wgrad_narrow_kernel<KH, KW, S, CR><<<nb, NT, 0, st>>>(*d, (const bf16_t*)x, (const bf16_t*)dy, ws, spb,
                                                          (int)nseg, segs_per_row);
    wgrad_narrow_reduce<<<irgan_cdiv(tile, 64), 1024, 0, st>>>(ws, nb, C::NPAD, KH, KW, CR, d->Cin, dw);
    return 0;
}

}  // namespace

// Narrow-input weight gradient (bf16 operands; x stored with 8 channels, ldx == 8,
// of which Cin = 1 (7x7, stride 1: G inc) or Cin = 4 (4x4, stride 2: D model.0)
// are real; Cout == 64).  ws: caller slab of >= 64 * NPAD floats per block.
// IRGAN_EUNSUPPORTED otherwise.
extern "C" int irgan_conv_wgrad_narrow(const irgan_conv_desc* d, const void* x, const void* dy, float* dw, float* ws,
                                       long ws_cap, hipStream_t st) {
    if ((long)d->N * d->Ho * d->Wo <= 0) return 0;
    if (d->dtype != IRGAN_BF16 || !ws || d->ldx != 8 || d->xoff != 0 || d->Cout != 64 || d->ldy % 8 ||
        d->yoff % 8 || d->sy != d->sx || (long)d->N * d->H * d->W * 8 >= (1L << 30) ||
        (long)d->N * d->Ho * d->Wo * d->ldy >= (1L << 30) || getenv("IRGAN_NO_WGRAD_NARROW"))
        return IRGAN_EUNSUPPORTED;
    int rc = IRGAN_EUNSUPPORTED;
    if (d->KH == 7 && d->KW == 7 && d->sx == 1 && d->Cin == 1)
        rc = launch_narrow<7, 7, 1, 1>(d, x, dy, dw, ws, ws_cap, st);
    else if (d->KH == 4 && d->KW == 4 && d->sx == 2 && d->Cin == 4)
        rc = launch_narrow<4, 4, 2, 4>(d, x, dy, dw, ws, ws_cap, st);
    if (rc) return rc;
    IRGAN_LAUNCH_CHECK();
    return 0;
}
