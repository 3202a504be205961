// Border band of the nn.ReflectionPad2d(p) backward-data (ir:381, 402: the
// reflect-padded 3x3 convs of every ResnetBlock), computed and folded in one
// launch.
//
// Backward-data of conv(reflect_pad(x)) is fold(g), g = the zero-padded
// correlation of dy with the flipped weights over the padded (H+2p) x (W+2p)
// domain.  The interior of g maps 1:1 onto dx and is written by the regular
// conv launch (descriptor d: dx[i] = sum_t Wd[t] dy[i + t + c0]).  What is
// left are the ring values of g: g at padded coordinate u is that same
// formula at the "virtual" dx position V = u - p (outside [0, H)), and it folds
// onto the mirrored pixel.  Along one axis dx index i (n = H or W) receives the
// virtual position V = -i when 1 <= i <= p, or V = 2n-2-i when n-1-p <= i <= n-2.
// A band pixel (y, x) therefore gets up to three ring terms: (Vy, x), (y, Vx),
// (Vy, Vx).  One owner per band pixel (no atomics, deterministic):
//   row segments: band rows y (2p of them), all x;
//   column segments: band columns x (2p of them), rows y outside the band rows.
//
// The band is thin (~4 pixel rows per image for 3x3), so the launch is built
// for parallelism rather than operand reuse: block = NPIX band pixels x 64
// output channels, 8 waves that split the K loop (term, tap, 32-channel step)
// round-robin, each holding the full NPIX x 64 tile (NF x 4 fragments of
// mfma_f32_16x16x32_bf16, weights as A: a lane's 4 accumulator rows are 4
// consecutive channels of one pixel).  Operands come straight from L2 (no
// LDS staging); the 4 partial tiles are summed through LDS in a fixed order
// and added into dx with 16-byte read-modify-writes.
#include "common.h"

namespace {

// 64 band pixels per block: each block streams its (taps x Cin) weight slices from L2
// once for 64 pixels instead of 32 -- the launch is bound by those L2 reads
// (32-pixel blocks: ~440 MB per resblock dgrad ring, 35 us)
constexpr int NPIX = 64;  // band pixels per block
constexpr int NF = NPIX / 16;  // pixel fragments
constexpr int NCO = 64;   // output channels per block (4 fragments)
constexpr int NWV = 8;    // waves per block (K split)
constexpr int MAXT = 160; // (term, tap) pairs: 3 terms x KH*KW (7x7: 147)

IRGAN_HD int mirror_pos(int i, int n, int p) {  // virtual position folding onto i, or INT_MIN
    if (i >= 1 && i <= p) return -i;
    if (i >= n - 1 - p && i <= n - 2) return 2 * n - 2 - i;
    return -0x40000000;
}

__global__ __launch_bounds__(NWV * 64) void reflect_ring_kernel(const irgan_conv_desc d, const bf16_t* __restrict__ dy,
                                                           const bf16_t* __restrict__ w, int p, void* __restrict__ dx,
                                                           int segs_row, int segs_col) {
    __shared__ __attribute__((aligned(16))) float red[NWV][NPIX][NCO + 4];  // +4: conflict-free row writes
    __shared__ int tap_list[MAXT];
    __shared__ int ntap_s;
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int H = d.Ho, W = d.Wo;               // dx spatial size (stride 1)
    const int Kw = (d.KH * d.KW * d.Cin + 63) / 64 * 64;  // packed weight row stride
    const int per_img = 2 * p * (segs_row + segs_col);
    const int n = blockIdx.x / per_img;
    int s = blockIdx.x - n * per_img;
    const bool rowseg = s < 2 * p * segs_row;
    int band, seg;
    if (rowseg) {
        band = s / segs_row;
        seg = s - band * segs_row;
    } else {
        s -= 2 * p * segs_row;
        band = s / segs_col;
        seg = s - band * segs_col;
    }
    // band index -> dx row (row segments) or column (column segments): 1..p, n-1-p..n-2
    const int nb = rowseg ? H : W;
    const int bpos = band < p ? band + 1 : nb - 1 - p + (band - p);
    const int co0 = blockIdx.y * NCO;

    // this lane's pixel in fragment f: index q = seg*NPIX + f*16 + (lane & 15) along the band line
    int py[NF], px[NF];
    bool pv[NF];
#pragma unroll
    for (int f = 0; f < NF; ++f) {
        const int q = seg * NPIX + f * 16 + (lane & 15);
        if (rowseg) {
            py[f] = bpos;
            px[f] = q;
            pv[f] = q < W;
        } else {
            py[f] = q;
            px[f] = bpos;
            pv[f] = q < H && mirror_pos(q, H, p) == -0x40000000;  // band rows belong to the row segments
        }
    }
    // block-uniform: which terms can occur.  Row segment: term 0 (Vy, x) for all
    // pixels; terms 1 (y, Vx) and 2 (Vy, Vx) only for pixels in band columns.
    // Column segment: term 1 only.
    const int qlo = seg * NPIX, qhi = min(qlo + NPIX, rowseg ? W : H) - 1;   // the segment's pixels
    const bool has_bandcol = rowseg && (qlo <= p || qhi >= W - 1 - p);
    const int vby = rowseg ? mirror_pos(bpos, H, p) : 0;   // row segments: Vy (uniform)
    const int vbx = rowseg ? 0 : mirror_pos(bpos, W, p);   // column segments: Vx (uniform)

    f32x4 acc[NF][4];
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[f][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // block-uniform list of the DISTINCT (ty, tx) taps that can touch dy, each with the mask
    // of the terms that use it: a tap's weight fragments are loaded once per 32-channel step
    // and shared by its terms (row segments: term 0 needs the taps that reach dy from Vy,
    // terms 1 / 2 only the taps that reach it from a band column's Vx -- 7 of the 15
    // (term, tap) pairs of a 3x3 resblock ring share their weights)
    const int fw0 = seg * NPIX;  // first pixel of the segment along its band line
    if (threadIdx.x == 0) {
        int nt = 0;
        for (int ty = 0; ty < d.KH; ++ty)
            for (int tx = 0; tx < d.KW; ++tx) {
                int m = 0;
                if (rowseg) {
                    const bool rv = (unsigned)(vby + ty + d.c0y) < (unsigned)d.H;       // term 0 / 2 rows
                    const bool r1 = (unsigned)(bpos + ty + d.c0y) < (unsigned)d.H;      // term 1 row
                    bool cv = false;  // some band column of this segment reaches dy through tx
                    if (has_bandcol)
                        for (int k = 0; k < 2 * p; ++k) {  // band columns 1..p, W-1-p..W-2
                            const int q = k < p ? k + 1 : W - 1 - p + (k - p);
                            const int vx = mirror_pos(q, W, p);
                            if (q >= qlo && q <= qhi && (unsigned)(vx + tx + d.c0x) < (unsigned)d.W) cv = true;
                        }
                    if (rv) m |= 1;
                    if (cv && r1) m |= 2;
                    if (cv && rv) m |= 4;
                } else if ((unsigned)(vbx + tx + d.c0x) < (unsigned)d.W) {
                    m = 2;
                }
                if (m) tap_list[nt++] = (m << 8) | (ty << 4) | tx;
            }
        ntap_s = nt;
    }
    __syncthreads();
    const int ntap = ntap_s;

    // mirrored column of fragment f's pixel (terms 1 and 2); fragments that hold no band
    // column skip the term 1 / 2 loads and MFMAs of a row segment (wave-uniform)
    int mxf[NF];
    bool fb[NF];
#pragma unroll
    for (int f = 0; f < NF; ++f) {
        mxf[f] = rowseg ? mirror_pos(px[f], W, p) : vbx;
        const int f0 = fw0 + f * 16, f1 = f0 + 15;
        fb[f] = !rowseg || (f0 <= p && f1 >= 1) || (f0 <= W - 2 && f1 >= W - 1 - p);
    }

    const int kc = (lane >> 4) * 8;  // channel offset of this lane within a 32-deep k step
    const bf16_t* wrow[4];
    bool wok[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int co = co0 + j * 16 + (lane & 15);
        wok[j] = co < d.Cout;
        wrow[j] = w + (long)(wok[j] ? co : 0) * Kw + kc;
    }
    const int nc = d.Cin / 32;
    const int total = ntap * nc;  // flattened K steps (tap, 32-channel step); wave wv takes s = wv mod NWV
    // one K step: the tap's weight fragments once, the dy fragments of each term in its mask
    auto load_step = [&](int q, uint4 (&a)[3][NF], uint4 (&b)[4], int& msk) {
        const int tp = q / nc, c = q - tp * nc;
        const int e = tap_list[tp];
        msk = e >> 8;
        const int ty = (e >> 4) & 15, tx = e & 15;
        const int wb = (ty * d.KW + tx) * d.Cin + c * 32;
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = wok[j] ? *(const uint4*)(wrow[j] + wb) : uint4{0, 0, 0, 0};
#pragma unroll
        for (int term = 0; term < 3; ++term) {
            if (!((msk >> term) & 1)) continue;
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                // term 0: (Vy, x); term 1: (y, Vx); term 2: (Vy, Vx)
                if (term > 0 && !fb[f]) continue;
                const int vy = term == 1 ? py[f] : vby;
                const int vx = term == 0 ? px[f] : mxf[f];
                const bool tv = pv[f] && (term == 0 || mxf[f] != -0x40000000);
                const int r = vy + ty + d.c0y, cc = vx + tx + d.c0x;
                const bool ok = tv && (unsigned)r < (unsigned)d.H && (unsigned)cc < (unsigned)d.W;
                a[term][f] = ok ? *(const uint4*)(dy + (((long)n * d.H + r) * d.W + cc) * d.ldx + d.xoff + kc + c * 32)
                                : uint4{0, 0, 0, 0};
            }
        }
    };
    auto mma = [&](const uint4 (&a)[3][NF], const uint4 (&b)[4], int msk) {
#pragma unroll
        for (int term = 0; term < 3; ++term) {
            if (!((msk >> term) & 1)) continue;
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                if (term > 0 && !fb[f]) continue;
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, b[j]),
                                                                        __builtin_bit_cast(bf16x8_t, a[term][f]),
                                                                        acc[f][j], 0, 0, 0);
            }
        }
    };
    // two steps of operands in flight: step s+NWV loads while step s multiplies
    uint4 a0[3][NF], b0[4], a1[3][NF], b1[4];
    int m0 = 0, m1 = 0;
    int ks = wv;
    if (ks < total) load_step(ks, a0, b0, m0);
    while (ks < total) {
        const int k1 = ks + NWV;
        if (k1 < total) load_step(k1, a1, b1, m1);
        mma(a0, b0, m0);
        if (k1 >= total) break;
        const int k2 = k1 + NWV;
        if (k2 < total) load_step(k2, a0, b0, m0);
        mma(a1, b1, m1);
        ks = k2;
    }
    // partial tiles -> LDS: lane holds pixel f*16 + (lane & 15), channels j*16 + 4*(lane>>4) + r
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            *(float4*)&red[wv][f * 16 + (lane & 15)][j * 16 + 4 * (lane >> 4)] =
                make_float4(acc[f][j][0], acc[f][j][1], acc[f][j][2], acc[f][j][3]);
    __syncthreads();
    // thread -> (pixel, 8 channels): sum the NWV partials in order, add into dx
    static_assert(NPIX * NCO / 8 == NWV * 64, "one (pixel, 8 channels) per thread");
    const int pix_l = threadIdx.x >> 3, cg = (threadIdx.x & 7) * 8;
    const int q = seg * NPIX + pix_l;
    const int yy = rowseg ? bpos : q, xx = rowseg ? q : bpos;
    const bool own = rowseg ? q < W : (q < H && mirror_pos(q, H, p) == -0x40000000);
    const int co = co0 + cg;
    if (!own || co >= d.Cout) return;
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = 0.f;
#pragma unroll
    for (int u = 0; u < NWV; ++u) {
        const float4 lo = *(const float4*)&red[u][pix_l][cg], hi = *(const float4*)&red[u][pix_l][cg + 4];
        v[0] += lo.x; v[1] += lo.y; v[2] += lo.z; v[3] += lo.w;
        v[4] += hi.x; v[5] += hi.y; v[6] += hi.z; v[7] += hi.w;
    }
    const long pix = ((long)n * d.OH + yy * d.omy + d.ooy) * d.OW + xx * d.omx + d.oox;
    const long o = pix * d.ldy + d.yoff + co;
    const bool full = co + 8 <= d.Cout;
    if (d.out_dtype == IRGAN_F32) {
        float* yp = (float*)dx + o;
        if (full && (o & 3) == 0) {
            float4 a = *(float4*)yp, b = *(float4*)(yp + 4);
            a.x += v[0]; a.y += v[1]; a.z += v[2]; a.w += v[3];
            b.x += v[4]; b.y += v[5]; b.z += v[6]; b.w += v[7];
            *(float4*)yp = a;
            *(float4*)(yp + 4) = b;
        } else {
            for (int k = 0; k < 8 && co + k < d.Cout; ++k) yp[k] += v[k];
        }
    } else {
        bf16_t* yp = (bf16_t*)dx + o;
        if (full && (o & 7) == 0) {
            uint4 u = *(uint4*)yp;
            uint32_t wds[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float o0 = __uint_as_float(wds[k] << 16), o1 = __uint_as_float(wds[k] & 0xffff0000u);
                wds[k] = pk_bf16(o0 + v[2 * k], o1 + v[2 * k + 1]);
            }
            *(uint4*)yp = uint4{wds[0], wds[1], wds[2], wds[3]};
        } else {
            for (int k = 0; k < 8 && co + k < d.Cout; ++k) yp[k] = f2bf(bf2f(yp[k]) + v[k]);
        }
    }
}

// ---- Line form of the same fold for the ResnetBlock case (3x3, p = 1, sides <= 64).
// With p = 1 the ring is four 1-D convolutions along the border lines of dy: the padded
// row -1 reads only dy row 0 through tap row ty = 2, row H only dy row H-1 (ty = 0),
// column -1 only dy column 0 (tx = 2), column W only column W-1 (tx = 0):
//   top    g(-1, u) = sum_tx Wd[2][tx] dy(0, u + tx - 1),    u in [-1, W]  -> dx(1, refl(u))
//   bottom g(H, u)  = sum_tx Wd[0][tx] dy(H-1, u + tx - 1),  u in [-1, W]  -> dx(H-2, refl(u))
//   left   g(y, -1) = sum_ty Wd[ty][2] dy(y + ty - 1, 0),    y in [0, H)   -> dx(y, 1)
//   right  g(y, W)  = sum_ty Wd[ty][0] dy(y + ty - 1, W-1),  y in [0, H)   -> dx(y, W-2)
// (the corners are the u = -1 / W ends of the top / bottom lines).  Two launches:
//  * ring_line_gemm_kernel: workgroup = (line, 64 output channels, a group of images).  The
//    line's 3 taps x Cin x 64 weights are loaded once as MFMA fragments into registers (wave =
//    16 channels), the image's dy line (<= 68 positions x Cin) into LDS; per image a [64 co] x
//    [80 positions] x [3 Cin] GEMM (5 position fragments per wave), the next image's line
//    prefetched into registers meanwhile; g (fp32) -> the caller's workspace.
//  * ring_line_fold_kernel: one thread per (owned dx pixel, 8 channels) adds the sum of its
//    ring terms in a fixed order (one read-modify-write, deterministic): rows 1 / H-2 take
//    their line's u plus, at columns 1 / W-2, the corner end and the column line's value.
constexpr int RV_L = 64;            // longest line (H, W)
constexpr int RV_ROWS = RV_L + 4;   // positions per line: dy coordinates -2 .. L+1 (g: u + 1 in [0, 68))
static_assert(RV_ROWS == IRGAN_RING_ROWS, "workspace layout shared with conv_pp_kernel.h");
constexpr int RV_CIN = 256;         // dy channels (LDS row = 512 B)

IRGAN_HD int rv_off(int row, int chunk) { return row * 512 + ((chunk ^ (row & 15)) << 4); }
IRGAN_HD int rv_tap(int line, int k) {  // dgrad-conv tap ty*3 + tx of along-line offset k
    return line == 0 ? 6 + k : (line == 1 ? k : (line == 2 ? 3 * k + 2 : 3 * k));
}

// 512 threads: waves kh = 0 / 1 (wave >> 2) take the dy channel steps cs < ncs / 2 / the rest
// (the K loop halved: one wave per SIMD ran a 3 x 8-step chain with each step's LDS reads
// exposed), then half 1's accumulators are added onto half 0's through LDS in a fixed order
constexpr int RV_NT = 512, RV_CSH = RV_CIN / 64;  // threads; channel steps per half (max)
#ifndef RING_EXP
#define RING_EXP 0  // ablation builds only (tools/build_variant.sh): 1 no weight loads, 2 no MFMA loop,
                    // 4 no line loads, 8 no stores
#endif
// FULL (Cin == RV_CIN, the ResnetBlock): every half has exactly RV_CSH channel steps, so the K
// loop is static and its LDS reads are scheduled ahead of the MFMAs (the dynamic trip count
// exposed each step's reads: 3.8 of the launch's 10.3 us at B = 16, gpurun_out/r05_ringab)
template <bool FULL>
__global__ __launch_bounds__(RV_NT, 1) void ring_line_gemm_kernel(const irgan_conv_desc d, const bf16_t* __restrict__ dy,
                                                                 const bf16_t* __restrict__ w, float* __restrict__ gbuf,
                                                                 int ipb) {
    __shared__ __attribute__((aligned(16))) char smem[RV_ROWS * 512 + 4 * 64 * 5 * 16];
    char* const sL = smem;                                   // [RV_ROWS positions] rows of Cin bf16
    f32x4* const sP = (f32x4*)(smem + RV_ROWS * 512);        // half 1's accumulators [wave][f][lane]
    const int nct = d.Cout / 64;
    const int line = blockIdx.x / nct, ct = blockIdx.x - line * nct;
    const int n0 = blockIdx.y * ipb, n1 = min(d.N, n0 + ipb);
    const int H = d.Ho, W = d.Wo, L = line < 2 ? W : H;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane((tid >> 6) & 3);
    const int kh = __builtin_amdgcn_readfirstlane(tid >> 8);
    const int g = lane >> 4, l16 = lane & 15;
    const int Kw = (9 * d.Cin + 63) / 64 * 64;
    const int c32 = d.Cin / 8;  // 16-byte chunks per row
    const int ncs = FULL ? RV_CIN / 32 : d.Cin / 32;
    const int cs0 = kh * ((ncs + 1) / 2), cs1 = kh ? ncs : (ncs + 1) / 2;  // this half's channel steps

    // this wave's weight fragments straight into registers (16 channels x 32 dy channels per
    // (tap k, channel step cs)): w[ct*64 + wv*16 + l16][rv_tap(line, k) * Cin + 32 cs + 8 g ..],
    // all loads in flight at once -- no LDS staging, no barrier before the first MFMA
    uint4 af[3][RV_CSH];
    {
        const bf16_t* wr = w + (long)(ct * 64 + wv * 16 + l16) * Kw + g * 8;
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
            for (int c = 0; c < RV_CSH; ++c)
                af[k][c] = (FULL || cs0 + c < cs1) && !(RING_EXP & 1)
                               ? *(const uint4*)(wr + rv_tap(line, k) * d.Cin + (cs0 + c) * 32)
                               : make_uint4(0u, 0u, 0u, 0u);
    }
    // the dy line of image n: position p = dy coordinate + 2 along the line
    constexpr int LPER = (RV_ROWS * 32 + RV_NT - 1) / RV_NT;
    auto load_line = [&](int n, uint4 (&v)[LPER]) {
#pragma unroll
        for (int u = 0; u < LPER; ++u) {
            const int e = u * RV_NT + tid, q = (e >> 5) - 2, c = e & 31;
            v[u] = make_uint4(0u, 0u, 0u, 0u);
            if (!(RING_EXP & 4) && e < RV_ROWS * 32 && q >= 0 && q < L && c < c32) {
                const int y = line == 0 ? 0 : (line == 1 ? H - 1 : q);
                const int x = line < 2 ? q : (line == 2 ? 0 : W - 1);
                v[u] = *(const uint4*)(dy + ((long)(n * d.H + y) * d.W + x) * d.ldx + d.xoff + c * 8);
            }
        }
    };
    uint4 lv[LPER];
    if (n0 < n1) load_line(n0, lv);
    const int ub = line < 2 ? -1 : 0;  // position of fragment 0, lane 0
    const int co = ct * 64 + wv * 16 + 4 * g;  // this lane's 4 output channels (C^T rows)
#pragma unroll 1
    for (int n = n0; n < n1; ++n) {
        __syncthreads();  // the previous image's GEMM is done with sL
#pragma unroll
        for (int u = 0; u < LPER; ++u) {
            const int e = u * RV_NT + tid;
            if (e < RV_ROWS * 32) *(uint4*)(sL + rv_off(e >> 5, e & 31)) = lv[u];
        }
        __syncthreads();
            if (n + 1 < n1) load_line(n + 1, lv);  // in flight under this image's GEMM
        f32x4 acc[5];
#pragma unroll
        for (int f = 0; f < 5; ++f) acc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 3 * !(RING_EXP & 2); ++k) {
#pragma unroll
            for (int c = 0; c < RV_CSH; ++c) {
                const int cs = cs0 + c;
                if (!FULL && cs >= cs1) break;
                const uint4 a = af[k][c];
                uint4 b[5];
#pragma unroll
                for (int f = 0; f < 5; ++f)
                    b[f] = *(const uint4*)(sL + rv_off(min(16 * f + l16 + ub + k + 1, RV_ROWS - 1), cs * 4 + g));
#pragma unroll
                for (int f = 0; f < 5; ++f)
                    acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                                     __builtin_bit_cast(bf16x8_t, b[f]), acc[f], 0, 0, 0);
            }
        }
        // half 1 hands its sums to half 0 (one add per element, fixed order)
        if (kh == 1) {
#pragma unroll
            for (int f = 0; f < 5; ++f) sP[(wv * 5 + f) * 64 + lane] = acc[f];
        }
        __syncthreads();
        if (kh == 0) {
            // g[n][line][u + 1][co]: lane = position 16 f + l16 + ub, rows 4g + r = channels
            float* gl = gbuf + ((long)n * 4 + line) * RV_ROWS * d.Cout;
#pragma unroll
            for (int f = 0; f < 5; ++f) {
                const f32x4 o = sP[(wv * 5 + f) * 64 + lane];
                const int pos = 16 * f + l16 + ub + 1;
                if (pos < RV_ROWS && (!(RING_EXP & 8) || acc[f][0] == 1234.5f))
                    *(float4*)(gl + (long)pos * d.Cout + co) =
                        make_float4(acc[f][0] + o[0], acc[f][1] + o[1], acc[f][2] + o[2], acc[f][3] + o[3]);
            }
        }
    }
}

// one thread per (owned dx pixel, 8 channels); targets per image: row 1 (W), row H-2 (W),
// column 1 and column W-2 without those rows (H-2 each)
__global__ __launch_bounds__(256) void ring_line_fold_kernel(const irgan_conv_desc d, const float* __restrict__ gbuf,
                                                             void* __restrict__ dx) {
    const int H = d.Ho, W = d.Wo, C8 = d.Cout / 8;
    const int per_img = (2 * W + 2 * (H - 2)) * C8;
    const long i = blockIdx.x * 256L + threadIdx.x;
    if (i >= (long)d.N * per_img) return;
    const int n = (int)(i / per_img);
    int r = (int)(i - (long)n * per_img);
    const int c = (r % C8) * 8;
    r /= C8;
    int y, x;
    float v[8];
    auto add = [&](int line, int pos) {  // pos = u + 1 (top / bottom) or y + 1 (left / right)
        const float4* q = (const float4*)(gbuf + (((long)n * 4 + line) * RV_ROWS + pos) * d.Cout + c);
        const float4 a = q[0], b = q[1];
        v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
        v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
    };
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = 0.f;
    if (r < 2 * W) {  // rows 1 (top line) / H-2 (bottom line)
        const int line = r / W;
        x = r - line * W;
        y = line == 0 ? 1 : H - 2;
        add(line, x + 1);
        if (x == 1) { add(line, 0); add(2, y + 1); }          // corner end u = -1, left line at y
        if (x == W - 2) { add(line, W + 1); add(3, y + 1); }  // corner end u = W, right line at y
    } else {          // columns 1 (left line) / W-2 (right line), rows other than 1 and H-2
        r -= 2 * W;
        const int side = r / (H - 2);
        int k = r - side * (H - 2);
        y = k == 0 ? 0 : k + 1;                  // rows 0, 2, 3, ..., H-3,
        if (k == H - 3) y = H - 1;               // and H-1
        x = side == 0 ? 1 : W - 2;
        add(2 + side, y + 1);
    }
    const long o = (((long)n * d.OH + y) * d.OW + x) * d.ldy + d.yoff + c;
    if (d.out_dtype == IRGAN_F32) {
        float4* p = (float4*)((float*)dx + o);
        float4 a = p[0], b = p[1];
        a.x += v[0]; a.y += v[1]; a.z += v[2]; a.w += v[3];
        b.x += v[4]; b.y += v[5]; b.z += v[6]; b.w += v[7];
        p[0] = a;
        p[1] = b;
    } else {
        uint4* p = (uint4*)((bf16_t*)dx + o);
        const uint4 u = *p;
        const uint32_t wd[4] = {u.x, u.y, u.z, u.w};
        uint32_t o4[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            o4[k] = pk_bf16(__uint_as_float(wd[k] << 16) + v[2 * k], __uint_as_float(wd[k] & 0xffff0000u) + v[2 * k + 1]);
        *p = make_uint4(o4[0], o4[1], o4[2], o4[3]);
    }
}

}  // namespace

// the line launches' shapes (else the general reflect_ring_kernel): bf16, 3x3, p = 1, output
// = input size with 4 <= H, W <= 64, dy channels % 32 and <= 256, dx channels % 64, 8-aligned
// dy / dx slices, plain (unstrided) output grid, a workspace of N * 4 * 68 * Cout floats
static long ring_line_ws(const irgan_conv_desc* d) { return (long)d->N * 4 * RV_ROWS * d->Cout; }
static bool ring_line_ok(const irgan_conv_desc* d, int p, long ws_floats) {
    static const bool off = getenv("IRGAN_NO_RING_LINE") != nullptr;
    return !off && p == 1 && d->dtype == IRGAN_BF16 && d->KH == 3 && d->KW == 3 && d->c0y == -1 && d->c0x == -1 &&
           d->Cin % 32 == 0 && d->Cin <= RV_CIN && d->Cout % 64 == 0 && d->ldx % 8 == 0 && d->xoff % 8 == 0 &&
           d->ldy % 8 == 0 && d->yoff % 8 == 0 && d->H >= 4 && d->W >= 4 && d->H <= RV_L && d->W <= RV_L &&
           d->Ho == d->H && d->Wo == d->W && d->Ho == d->OH && d->Wo == d->OW && d->omy == 1 && d->omx == 1 &&
           d->ooy == 0 && d->oox == 0 && (d->out_dtype == IRGAN_BF16 || d->out_dtype == IRGAN_F32) &&
           ws_floats >= ring_line_ws(d);
}
// conv_pp.hip's irgan_conv_dgrad_reflect_line: the check, then the line GEMM alone (one
// image per workgroup row); the fold runs in the interior launch's store pass
bool ring_line_check(const irgan_conv_desc* d, int p, long ws_floats) { return ring_line_ok(d, p, ws_floats); }
void ring_line_gemm_launch(const irgan_conv_desc* d, const void* dy, const void* w, float* ws, hipStream_t st) {
    // one image per workgroup row (2 / 4 images per workgroup measured slower: the launch
    // is latency-bound, profiles/r03_ring_gemm_wreg_ab.txt)
    // one image per workgroup row while the grid fits the CUs (2 / 4 images per workgroup
    // measured slower at B = 16: the launch is latency-bound, profiles/r03_ring_gemm_wreg_ab.txt);
    // beyond that (B = 32: two rounds of one block per CU) the images of a row share its weight
    // registers, the next image's line loaded under the current GEMM
    const int per_img = 4 * (d->Cout / 64);
    const int rows_fit = std::max(1, irgan_cu_count() / per_img);
    const int ipb = irgan_cdiv(d->N, rows_fit), groups = irgan_cdiv(d->N, ipb);
    if (d->Cin == RV_CIN)
        ring_line_gemm_kernel<true><<<dim3(per_img, groups), RV_NT, 0, st>>>(*d, (const bf16_t*)dy, (const bf16_t*)w,
                                                                             ws, ipb);
    else
        ring_line_gemm_kernel<false><<<dim3(per_img, groups), RV_NT, 0, st>>>(*d, (const bf16_t*)dy, (const bf16_t*)w,
                                                                              ws, ipb);
}

extern "C" int irgan_reflect_dgrad_ring(const irgan_conv_desc* d, const void* dy, const void* w, int32_t p, void* dx,
                                        irgan_stream_t s) {
    if (!d || !dy || !w || !dx) return IRGAN_EINVAL;
    if ((long)d->N * d->Ho * d->Wo <= 0 || d->Cout <= 0 || p <= 0) return 0;
    if (d->dtype != IRGAN_BF16 || d->Cin % 32 || d->ldx % 8 || d->xoff % 8 || d->sy != 1 || d->sx != 1 ||
        d->Ho != d->H || d->Wo != d->W || d->H < 2 * p + 2 || d->W < 2 * p + 2 || d->accumulate < 0 ||
        d->KH > 15 || d->KW > 15 || 3 * d->KH * d->KW > MAXT)
        return IRGAN_EUNSUPPORTED;
    const int segs_row = irgan_cdiv(d->Wo, NPIX), segs_col = irgan_cdiv(d->Ho, NPIX);
    dim3 grid(d->N * 2 * p * (segs_row + segs_col), irgan_cdiv(d->Cout, NCO));
    reflect_ring_kernel<<<grid, NWV * 64, 0, (hipStream_t)s>>>(*d, (const bf16_t*)dy, (const bf16_t*)w, p, dx, segs_row,
                                                         segs_col);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

// The same fold with a workspace: ResnetBlock shapes (ring_line_ok) run the two line
// launches (GEMM with at most max_blocks workgroups -- for a launch on a second stream beside a
// kernel that leaves that many CUs idle, the ResnetBlock weight gradient: 240 of 256 CUs --
// then the fold); other shapes the general ring launch.
extern "C" int irgan_reflect_dgrad_ring_ws(const irgan_conv_desc* d, const void* dy, const void* w, int32_t p,
                                           void* dx, float* ws, int64_t ws_floats, int32_t max_blocks,
                                           irgan_stream_t s) {
    if (!d || !dy || !w || !dx || max_blocks < 1) return IRGAN_EINVAL;
    if ((long)d->N * d->Ho * d->Wo <= 0 || d->Cout <= 0 || p <= 0) return 0;
    if (!ws || !ring_line_ok(d, p, ws_floats)) return irgan_reflect_dgrad_ring(d, dy, w, p, dx, s);
    hipStream_t st = (hipStream_t)s;
    const int tiles = 4 * (d->Cout / 64);             // (line, 64-channel tile)
    int groups = max_blocks / tiles;                  // image groups
    if (groups < 1) groups = 1;
    if (groups > d->N) groups = d->N;
    const int ipb = irgan_cdiv(d->N, groups);
    groups = irgan_cdiv(d->N, ipb);
    if (d->Cin == RV_CIN)
        ring_line_gemm_kernel<true><<<dim3(tiles, groups), RV_NT, 0, st>>>(*d, (const bf16_t*)dy, (const bf16_t*)w, ws, ipb);
    else
        ring_line_gemm_kernel<false><<<dim3(tiles, groups), RV_NT, 0, st>>>(*d, (const bf16_t*)dy, (const bf16_t*)w, ws, ipb);
    const long threads = (long)d->N * (2 * d->Wo + 2 * (d->Ho - 2)) * (d->Cout / 8);
    ring_line_fold_kernel<<<(unsigned)irgan_cdiv(threads, 256), 256, 0, st>>>(*d, ws, dx);
    IRGAN_LAUNCH_CHECK();
    return 0;
}
