// fp8 (OCP e4m3) weight gradient of the ResnetBlock 3x3 convs (BASELINE config 5; the
// weight half of the convolution backward of ir:386-411):
//
//   dW[co][ty][tx][ci] += dq_x * dq_dy * sum_p dY8[p][co] * X8[p + (ty, tx)][ci]
//
// on the delayed-scaled e4m3 copies the fp8 path already makes of each conv's input (the IN
// forward apply) and of its output gradient (the IN backward apply), with
// v_mfma_scale_f32_16x16x128_f8f6f4 (unit block scales: twice the bf16 rate).  The same
// producer / consumer schedule as conv_wgrad_pc.hip, on fp8 operands:
//
//  * block = (128-channel co tile, 64-channel ci chunk, kernel row ty, the three tx taps);
//    it walks 128-pixel segments (one MFMA K-step each): two output rows of a 64-wide map
//    or 128 pixels of one row, split-K over segments; partials to an ordered slab;
//  * 8 compute waves (co half wm, 48-column n group wn: 4 x 3 fragments of 16 x 16) and 4
//    loader waves issuing every LDS-DMA piece (16-byte lanes) into a 4-stage ring, one
//    barrier per segment, the DMA two segments ahead;
//  * both MFMA operands come from LDS with ds_read_b64_tr_b8: per 16-lane group a block of
//    8 pixel rows x 16 channel bytes, delivered channel-major (lane i: channel i, 8 pixels) --
//    the pixel (= reduction) index lands in the registers with no VALU.  A fragment is four
//    such reads (32 pixels per lane group); lane group g, byte 8m + q <-> segment pixel
//    32 m + 8 g + q, the same map for both operands.
//
// LDS images (conflict-free for the tr_b8 reads of a 32-lane half):
//   dY tile [128 px][128 co] (128-B rows): 16-B chunk ^ ((row & 7) ^ ((row >> 3) & 1));
//   X span [2 x 72 positions][64 ci] (64-B rows, position 0 = input column x0 - 1):
//   chunk ^ ((row >> 2) & 3).
#include "common.h"

namespace {

typedef int f8v8 __attribute__((ext_vector_type(8)));
typedef int f8v2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) f8v2 lds_f8v2;

constexpr int F8_STAGES = 4;
constexpr int F8_CW = 8, F8_LW = 4, F8_NT = (F8_CW + F8_LW) * 64;
constexpr int DY_PIECES = 16;                 // 128 px x 128 B
constexpr int XPOS = 72;                      // span positions per input row (66 used)
constexpr int X_PIECES = 2 * XPOS * 64 / 1024;  // 144 rows x 64 B = 9 pieces
constexpr int F8_TP = DY_PIECES + X_PIECES;   // 25 pieces per segment
constexpr int F8_STAGE = F8_TP * 1024;
constexpr int F8_PPL = (F8_TP + F8_LW - 1) / F8_LW;  // 7
constexpr int XOFF = DY_PIECES * 1024;        // X span inside a stage
static_assert(F8_TP % F8_LW == 1, "loader 0 takes PPL pieces, the others PPL - 1");

IRGAN_HD int dy_sw(int row) { return (row & 7) ^ ((row >> 3) & 1); }
IRGAN_HD int x_sw(int row) { return (row >> 2) & 3; }

IRGAN_HD f8v2 tr8(const char* p) { return __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_f8v2*)p); }

// wait until at most c segments of this loader's pieces (np per segment) are outstanding
template <int C>
IRGAN_HD void f8_wait(int c, bool full) {
    if constexpr (C == 0) {
        wait_vmcnt<0>();
    } else {
        if (c >= C) {
            if (full) wait_vmcnt<C * F8_PPL>(); else wait_vmcnt<C * (F8_PPL - 1)>();
        } else {
            f8_wait<C - 1>(c, full);
        }
    }
}

// two_rows: a segment is output rows oy0, oy0 + 1 of a 64-wide map (else 128 pixels of one row)
__global__ __launch_bounds__(F8_NT, 1) void wgrad_f8_kernel(const irgan_conv_desc d, const uint8_t* __restrict__ x,
                                                            const uint8_t* __restrict__ dy,
                                                            const float* __restrict__ dqx,
                                                            const float* __restrict__ dqdy, float* __restrict__ dw,
                                                            int segs_per_block, int nseg, int ntco, int nci,
                                                            int two_rows, int swz, float* __restrict__ slab) {
    __shared__ __attribute__((aligned(1024))) char smem[F8_STAGES * F8_STAGE];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int tiles = ntco * nci * d.KH;
    const int t = xcd_tile(blockIdx.x, gridDim.x, swz);
    const int split = t / tiles;
    int r = t - split * tiles;
    const int ty = r % d.KH;
    r /= d.KH;
    const int cic = r % nci, cot = r / nci;
    const int co0 = cot * 128, ci0 = cic * 64;
    const int s_beg = split * segs_per_block;
    const int s_end = min(nseg, s_beg + segs_per_block);
    if (s_beg >= s_end) return;  // block-uniform
    const int nk = s_end - s_beg;
    const int segs_row = two_rows ? 0 : d.Wo / 128, hpair = d.Ho >> 1;

    if (wid >= F8_CW) {
        // ------------------------------------------------------------------ loaders
        const int l = wid - F8_CW;
        const int np = (F8_TP - l + F8_LW - 1) / F8_LW;  // PPL for l = 0, else PPL - 1
        const bool reflect = d.pad_mode == IRGAN_PAD_REFLECT;
        const i32x4 rs_dy = make_rsrc(dy + d.yoff + co0, (uint32_t)((long)d.N * d.Ho * d.Wo * d.ldy - d.yoff - co0));
        const i32x4 rs_x = make_rsrc(x + d.xoff + ci0, (uint32_t)((long)d.N * d.H * d.W * d.ldx - d.xoff - ci0));
        uint32_t voff[F8_PPL];   // dY pieces: lane offset (pixel p of the segment, its source chunk)
        int xh[F8_PPL], xpos[F8_PPL], xc[F8_PPL];
#pragma unroll
        for (int u = 0; u < F8_PPL; ++u) {
            const int j = l + F8_LW * u;
            voff[u] = IRGAN_OOB;
            xh[u] = xpos[u] = xc[u] = 0;
            if (j < DY_PIECES) {
                const int row = j * 8 + (lane >> 3), c = (lane & 7) ^ dy_sw(row);
                // pixel row of the segment: consecutive pixels are consecutive NHWC pixels in
                // both segment forms (two full 64-wide rows, or 128 pixels of one row)
                voff[u] = (uint32_t)(row * d.ldy + c * 16);
            } else if (j < F8_TP) {
                const int row = (j - DY_PIECES) * 16 + (lane >> 2), c = (lane & 3) ^ x_sw(row);
                xh[u] = two_rows ? row / XPOS : 0;
                xpos[u] = two_rows ? row - xh[u] * XPOS : row;
                xc[u] = c * 16;
            }
        }
        auto issue = [&](int s, int stage) {
            int n, oy0, x0;
            if (two_rows) {
                n = s / hpair;
                oy0 = (s - n * hpair) * 2;
                x0 = 0;
            } else {
                const int rowi = s / segs_row;
                x0 = (s - rowi * segs_row) * 128;
                n = rowi / d.Ho;
                oy0 = rowi - n * d.Ho;
            }
            const uint32_t dy_soff = (uint32_t)((((long)n * d.Ho + oy0) * d.Wo + x0) * d.ldy);
            char* base = smem + stage * F8_STAGE;
#pragma unroll
            for (int u = 0; u < F8_PPL; ++u) {
                if (u >= np) break;
                const int j = l + F8_LW * u;
                if (j < DY_PIECES) {
                    blds16(rs_dy, voff[u], dy_soff, base + j * 1024);
                } else {
                    int iy = oy0 + xh[u] + ty + d.c0y, ix = x0 - 1 + xpos[u];
                    if (reflect) {
                        iy = reflect_idx(iy, d.H);
                        ix = reflect_idx(ix, d.W);
                    }
                    const int npos = two_rows ? 66 : 130;
                    const bool ok = xpos[u] < npos && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W;
                    const uint32_t off = ok ? (uint32_t)((((long)n * d.H + iy) * d.W + ix) * d.ldx) + xc[u] : IRGAN_OOB;
                    blds16(rs_x, off, base + j * 1024);
                }
            }
        };
        for (int k = 0; k < F8_STAGES - 1; ++k)
            if (k < nk) issue(s_beg + k, k);
        f8_wait<F8_STAGES - 2>(min(nk - 1, F8_STAGES - 2), np == F8_PPL);
        lds_barrier();
        for (int kt = 0; kt < nk; ++kt) {
            // retire segment kt+1 (kt+2 may stay in flight), then barrier kt
            if (kt + 1 < nk) f8_wait<F8_STAGES - 3>(min(nk - kt - 2, F8_STAGES - 3), np == F8_PPL);
            lds_barrier();
            if (kt + F8_STAGES - 1 < nk) issue(s_beg + kt + F8_STAGES - 1, (kt + F8_STAGES - 1) % F8_STAGES);
        }
        return;
    }

    // ---------------------------------------------------------------------- compute
    // wave (wm, wn): co fragments wm*4 + i (i < 4), n fragments jj = 3 wn + j (j < 3):
    // tap tx = jj >> 2, 16-channel ci group jj & 3
    const int wn = wid & 3, wm = wid >> 2;
    const int g = lane >> 4, q = (lane & 15) >> 1, p = lane & 1;
    // A (dY^T) fragment i, read m: pixel row 32 m + 8 g + q (its swizzle is q ^ (g & 1) for every m),
    // bytes 8 p of co chunk wm*4 + i; + m * 4096
    int aoff[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) aoff[i] = (8 * g + q) * 128 + (((wm * 4 + i) ^ q ^ (g & 1)) << 4) + 8 * p;
    // B (X) fragment j, read m: span row sr = base(m) + 8 g + q + tx with base(m) = 32 m (m < 2)
    // or XPOS + 32 (m - 2) (two rows) / 32 m (one row); the swizzle (sr >> 2) & 3 repeats every 32
    // rows, so two lane offsets per fragment (reads m = 0, 2) plus the +2048 of reads 1, 3
    const int hib = two_rows ? XPOS : 64;
    int boff[3][2];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const int jj = wn * 3 + j, tx = jj >> 2, cg = jj & 3;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int row = h * hib + 8 * g + q + tx;
            boff[j][h] = XOFF + row * 64 + ((cg ^ x_sw(row)) << 4) + 8 * p;
        }
    }
    f32x4 acc[4][3];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto rdA = [&](const char* S, int i) -> f8v8 {
        const f8v2 r0 = tr8(S + aoff[i]), r1 = tr8(S + aoff[i] + 4096), r2 = tr8(S + aoff[i] + 8192),
                   r3 = tr8(S + aoff[i] + 12288);
        return f8v8{r0.x, r0.y, r1.x, r1.y, r2.x, r2.y, r3.x, r3.y};
    };
    auto rdB = [&](const char* S, int j) -> f8v8 {
        const f8v2 r0 = tr8(S + boff[j][0]), r1 = tr8(S + boff[j][0] + 2048), r2 = tr8(S + boff[j][1]),
                   r3 = tr8(S + boff[j][1] + 2048);
        return f8v8{r0.x, r0.y, r1.x, r1.y, r2.x, r2.y, r3.x, r3.y};
    };
    // MFMAs of the current segment with the reads of the next one (stage) rolled in: each
    // fragment register is re-read right after its last MFMA of the segment (b[j] after its
    // 4 MFMAs, a[i] after its third), so one register set serves both segments (the 12-wave
    // block leaves 168 VGPRs per wave); the other compute wave of the SIMD covers the reads'
    // latency
    f8v8 a[4], b[3];
    auto step = [&](int stage) {
        const char* S = smem + stage * F8_STAGE;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[i], b[j], acc[i][j], 0, 0, 0, 127, 0,
                                                                             127);
                if (j == 2) a[i] = rdA(S, i);
            }
            b[j] = rdB(S, j);
        }
    };
    auto barrier = [] {
        __builtin_amdgcn_sched_barrier(0);
        lds_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    barrier();  // prologue barrier: segment 0 landed
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = rdA(smem, i);
#pragma unroll
    for (int j = 0; j < 3; ++j) b[j] = rdB(smem, j);
    for (int kt = 0; kt < nk; ++kt) {
        barrier();                        // barrier kt: segment kt+1 landed, segment kt-1 fully read
        step((kt + 1) % F8_STAGES);       // segment kt | read segment kt+1 (unused past the end)
    }

    // C[row = co][col = n]: co = co0 + (wm*4 + i)*16 + 4g + rr, n = jj*16 + (lane & 15)
    const float sc = *dqx * *dqdy;  // the two per-tensor dequantisation factors (powers of two)
    const int K = d.KH * 3 * d.Cin;
    float* const dst = slab ? slab + (long)split * d.Cout * K : nullptr;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            const int co = co0 + (wm * 4 + i) * 16 + g * 4 + rr;
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const int jj = wn * 3 + j, tx = jj >> 2;
                const int ci = ci0 + (jj & 3) * 16 + (lane & 15);
                const long o = (long)co * K + (ty * 3 + tx) * d.Cin + ci;
                if (dst) dst[o] = acc[i][j][rr] * sc;
                else atomicAdd(dw + o, acc[i][j][rr] * sc);
            }
        }
}

__global__ __launch_bounds__(256) void wgrad_f8_reduce(const float* __restrict__ slab, int splits, long n,
                                                        float* __restrict__ dw) {
    const long n4 = n / 4;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
        slab_sum4(slab, splits, n, dw, i);
    }
}

}  // namespace

extern "C" int irgan_conv_wgrad_fp8(const irgan_conv_desc* d, const void* x8, const void* dy8, const float* dqx,
                                    const float* dqdy, float* dw, float* ws, int64_t ws_floats, irgan_stream_t s) {
    if (!d || !x8 || !dy8 || !dqx || !dqdy || !dw) return IRGAN_EINVAL;
    if ((long)d->N * d->Ho * d->Wo <= 0) return 0;
    const bool two_rows = d->Wo == 64;
    if (d->dtype != IRGAN_FP8 || d->KW != 3 || d->KH < 1 || d->KH > 3 || d->sy != 1 || d->sx != 1 ||
        d->c0x != -1 || d->Cout % 128 || d->Cin % 64 || (!two_rows && d->Wo % 128) || (two_rows && d->Ho % 2) ||
        d->Ho != d->OH || d->Wo != d->OW || d->ldx % 16 || d->xoff % 16 || d->ldy % 16 || d->yoff % 16 ||
        (long)d->N * d->H * d->W * d->ldx >= (1L << 31) || (long)d->N * d->Ho * d->Wo * d->ldy >= (1L << 31))
        return IRGAN_EUNSUPPORTED;
    // reflect_idx() mirrors one pixel past each edge: only the same-size pad-1 3x3 conv
    if (d->pad_mode == IRGAN_PAD_REFLECT && (d->KH != 3 || d->c0y != -1 || d->H != d->Ho || d->W != d->Wo))
        return IRGAN_EUNSUPPORTED;
    hipStream_t st = (hipStream_t)s;
    const int cus = irgan_cu_count();
    const int swz = irgan_xcd_swz();
    const int ntco = d->Cout / 128, nci = d->Cin / 64;
    const int tiles = ntco * nci * d->KH;
    const int nseg = d->N * d->Ho * d->Wo / 128;
    int splitk = cus / tiles;  // one block per CU
    if (splitk < 1) splitk = 1;
    const int maxs = irgan_cdiv(nseg, 4);
    if (splitk > maxs) splitk = maxs;
    if (swz && (tiles * splitk) % 8) {
        for (int s2 = splitk - 1; s2 >= 1 && s2 >= splitk - 8; --s2)
            if ((tiles * s2) % 8 == 0) { splitk = s2; break; }
    }
    const long n = (long)d->Cout * d->KH * 3 * d->Cin;
    if (irgan_det(d)) {  // deterministic: no atomics -- at most the splits the workspace holds
        const long fit = ws ? ws_floats / n : 1;
        if (splitk > fit) splitk = (int)(fit > 1 ? fit : 1);
    }
    const int spb = irgan_cdiv(nseg, splitk);
    splitk = irgan_cdiv(nseg, spb);
    float* slab = (ws && splitk > 1 && (long)splitk * n <= ws_floats) ? ws : nullptr;
    wgrad_f8_kernel<<<tiles * splitk, F8_NT, 0, st>>>(*d, (const uint8_t*)x8, (const uint8_t*)dy8, dqx, dqdy, dw, spb,
                                                      nseg, ntco, nci, two_rows ? 1 : 0, swz, slab);
    if (slab) {
        const int blocks = (int)std::min<long>(irgan_cdiv(n / 4, 256), 2048);
        wgrad_f8_reduce<<<blocks, 256, 0, st>>>(slab, splitk, n, dw);
    }
    IRGAN_LAUNCH_CHECK();
    return 0;
}
