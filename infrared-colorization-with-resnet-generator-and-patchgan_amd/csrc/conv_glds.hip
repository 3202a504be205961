// bf16 implicit-GEMM convolution, LDS-DMA pipeline (forward and backward-data).
//
// 512 threads = 8 waves (4 x 2), block tile 256 pixels x BN output channels,
// K-tile = 64 bf16 (one 128-byte channel run of one tap).  Operands move
// HBM/L2 -> LDS with global_load_lds (16 B per lane, no VGPR staging) into a
// 3-stage ring: tile k+2 is in flight while tile k is multiplied, with one
// counted s_waitcnt vmcnt + one raw s_barrier per K-tile.  Zero padding and
// tails read a zero page, reflect padding is folded into the source address.
// The LDS image keeps the 16-byte-chunk XOR swizzle (chunk ^ (row & 7)) of the
// register-staged kernel; with LDS-DMA the permutation is applied to the
// per-lane SOURCE chunk so the destination stays lane-linear.
#include "conv_epilogue.h"

namespace {

IRGAN_HD int lds_off(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }

template <int BN>
__global__ __launch_bounds__(512, 2) void conv_fwd_glds_kernel(const irgan_conv_desc d, const bf16_t* __restrict__ x,
                                                               const bf16_t* __restrict__ w,
                                                               const float* __restrict__ bias, void* __restrict__ y,
                                                               const void* __restrict__ mask,
                                                               const bf16_t* __restrict__ zero, int ntn, int swz,
                                                               int ksplit, long sstride) {
    constexpr int BM = 256, STAGES = 3;
    constexpr int ABYTES = BM * 128, STAGE = ABYTES + BN * 128;
    constexpr int MI = 4, NJ = BN / 32;  // wave tile 64 x BN/2
    constexpr int AU = BM / 64, BU = BN / 64;  // 1 KiB glds pieces per wave per tile
    __shared__ __attribute__((aligned(1024))) char smem[STAGES * STAGE];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid >> 1, wn = wid & 1;
    const int HoWo = d.Ho * d.Wo;
    const long M = (long)d.N * HoWo;
    const int taps = d.KH * d.KW;
    const int K = (taps * d.Cin + 63) / 64 * 64;  // weight row stride (taps zero-padded)
    // 1-D grid, N-tiles fastest: the tiles of one pixel block are adjacent;
    // K-splits outermost (split ks writes its partial sums at y + ks*sstride)
    int t = xcd_tile(blockIdx.x, gridDim.x, swz);
    const int tiles_mn = gridDim.x / ksplit;
    const int ks = t / tiles_mn;
    t -= ks * tiles_mn;
    const long m0 = (long)(t / ntn) * BM;
    const int n0 = (t % ntn) * BN;
    const int sub = lane >> 3;
    const int chunk = (lane & 7) ^ sub;  // source chunk for this lane's LDS slot (row & 7 == sub)
    // K-tile = 64 channels of one tap (Cin % 64 == 0) or 64/Cin taps of a narrow
    // (8/16/32-channel, zero-padded) input: this lane's chunk -> (tap in tile, channel offset)
    const int cpt = d.Cin >= 64 ? 8 : d.Cin / 8;  // chunks per tap inside a tile
    const int tap_in = chunk / cpt, ch_in = (chunk % cpt) * 8;

    int a_nb[AU], a_iy[AU], a_ix[AU];
#pragma unroll
    for (int u = 0; u < AU; ++u) {
        const long m = m0 + (wid * AU + u) * 8 + sub;
        if (m < M) {
            const int mm = (int)m;
            const int n = mm / HoWo, r = mm - n * HoWo, i = r / d.Wo, j = r - i * d.Wo;
            a_nb[u] = n * d.H;
            a_iy[u] = i * d.sy + d.c0y;
            a_ix[u] = j * d.sx + d.c0x;
        } else {
            a_nb[u] = -1;
            a_iy[u] = 0;
            a_ix[u] = 0;
        }
    }
    const bf16_t* b_src[BU];
#pragma unroll
    for (int u = 0; u < BU; ++u) {
        const int co = n0 + (wid * BU + u) * 8 + sub;
        b_src[u] = co < d.Cout ? w + (long)co * K + chunk * 8 : nullptr;
    }
    const bool reflect = d.pad_mode == IRGAN_PAD_REFLECT;

    auto issue = [&](int kt, int stage) {
        const int k0 = kt * 64;
        int tap, coff;
        if (d.Cin >= 64) {
            tap = k0 / d.Cin;
            coff = d.xoff + (k0 - tap * d.Cin) + chunk * 8;
        } else {
            tap = kt * (8 / cpt) + tap_in;
            coff = d.xoff + ch_in;
        }
        const bool tap_ok = tap < taps;
        const int ty = tap / d.KW, tx = tap - ty * d.KW;
        char* sA = smem + stage * STAGE;
#pragma unroll
        for (int u = 0; u < AU; ++u) {
            int qy = a_iy[u] + ty, qx = a_ix[u] + tx;
            if (reflect) {  // wave-uniform
                qy = reflect_idx(qy, d.H);
                qx = reflect_idx(qx, d.W);
            }
            // branch-free validity (bitwise, no short circuit) -> one v_cndmask on the address
            const bool ok = tap_ok & (a_nb[u] >= 0) & ((unsigned)qy < (unsigned)d.H) & ((unsigned)qx < (unsigned)d.W);
            const long off = ((long)(a_nb[u] + qy) * d.W + qx) * d.ldx;
            const bf16_t* src = ok ? x + off + coff : zero;
            glds16(src, sA + (wid * AU + u) * 1024);
        }
#pragma unroll
        for (int u = 0; u < BU; ++u) {
            const bf16_t* src = b_src[u] ? b_src[u] + k0 : zero;
            glds16(src, sA + ABYTES + (wid * BU + u) * 1024);
        }
    };

    f32x4 acc[MI][NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk_all = K / 64, kper = (nk_all + ksplit - 1) / ksplit;
    const int kb = ks * kper, nk = min(nk_all - kb, kper);  // this split's K-tiles [kb, kb+nk)
    if (nk > 0) issue(kb, 0);
    if (nk > 1) issue(kb + 1, 1);
    for (int kt = 0; kt < nk; ++kt) {
        if (kt + 1 < nk) wait_vmcnt<AU + BU>();
        else wait_vmcnt<0>();
        lds_barrier();
        if (kt + 2 < nk) issue(kb + kt + 2, (kt + 2) % STAGES);
        const char* A = smem + (kt % STAGES) * STAGE;
        const char* B = A + ABYTES;
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
                for (int j = 0; j < NJ; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[i]),
                                                                        __builtin_bit_cast(bf16x8_t, bfr[j]),
                                                                        acc[i][j], 0, 0, 0);
        }
    }

    // epilogue: C[row = (lane>>4)*4 + r][col = lane & 15] of each 16x16 fragment
    void* yk = ks ? (void*)((float*)y + ks * sstride) : y;  // split partials are fp32
    conv_epilogue<BN, MI, NJ, 4, 2, 512>(d, acc, smem, wm, wn, n0, bias, yk, mask, [&](int m) -> long {
        const long mm = m0 + m;
        if (mm >= M) return -1;
        const int n = (int)(mm / HoWo), rr = (int)(mm - (long)n * HoWo), ii = rr / d.Wo, jj = rr - ii * d.Wo;
        return ((long)n * d.OH + ii * d.omy + d.ooy) * d.OW + jj * d.omx + d.oox;
    });
}

}  // namespace

// zero page for padded / out-of-range glds sources (4 KiB, device global)
__device__ __attribute__((aligned(4096))) bf16_t g_irgan_zero_page[2048];

extern "C" int irgan_conv_fwd_glds_split(const irgan_conv_desc* d, const void* x, const void* w, const float* bias,
                                         void* y, const void* mask, int ksplit, long sstride, hipStream_t st) {
    const long M = (long)d->N * d->Ho * d->Wo;
    if (M <= 0 || d->Cout <= 0) return 0;
    static void* zero_cache[IRGAN_MAX_DEVICES];  // the zero page's address per device
    const bf16_t* zero = (const bf16_t*)irgan_symbol(HIP_SYMBOL(g_irgan_zero_page), zero_cache);
    if (!zero) return IRGAN_EUNSUPPORTED;
    const int swz = irgan_xcd_swz();
    if (ksplit < 1) ksplit = 1;
    if (d->Cout > 64) {
        const int ntn = irgan_cdiv(d->Cout, 128);
        conv_fwd_glds_kernel<128><<<irgan_cdiv(M, 256) * ntn * ksplit, 512, 0, st>>>(
            *d, (const bf16_t*)x, (const bf16_t*)w, bias, y, mask, zero, ntn, swz, ksplit, sstride);
    } else {
        const int ntn = irgan_cdiv(d->Cout, 64);
        conv_fwd_glds_kernel<64><<<irgan_cdiv(M, 256) * ntn * ksplit, 512, 0, st>>>(
            *d, (const bf16_t*)x, (const bf16_t*)w, bias, y, mask, zero, ntn, swz, ksplit, sstride);
    }
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_conv_fwd_glds(const irgan_conv_desc* d, const void* x, const void* w, const float* bias, void* y,
                                   const void* mask, hipStream_t st) {
    return irgan_conv_fwd_glds_split(d, x, w, bias, y, mask, 1, 0, st);
}

// ---------------------------------------------------------------------------
// bf16 backward-weight, LDS-DMA + transposed LDS reads.
//   dW[co][tap][ci] += sum_p dY[p][co] * X[q(p, tap)][ci]
// Both operands arrive pixel-major (NHWC rows of channels).  They are DMA'd
// into LDS in that natural layout (one row = the tile's channels of one
// pixel) and the MFMA fragments, which need 8 consecutive PIXELS per lane, are
// read with ds_read_b64_tr_b16 (4 pixel-rows x 16 channels per 16-lane group,
// delivered column-major).  Rows are XOR-swizzled in 16-byte chunks so the
// transposed reads of 8 rows per 32-lane half hit 8 distinct bank groups.
// 512 threads = 8 waves (4 co x 2 ci), tile 128 co x 128 ci (or 64), K-tile 64
// pixels, 3-stage ring, split-K over pixels with one fp32 atomic per element.
// ---------------------------------------------------------------------------
namespace {

typedef __attribute__((ext_vector_type(4))) short s16x4;

// chunk XOR for a pixel row r of an RB-byte LDS row
template <int RB>
IRGAN_HD int wg_swz(int r) {
    if constexpr (RB == 256) return 2 * ((r & 3) | (((r >> 3) & 1) << 2));
    else return 2 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1));
}
template <int RB>
IRGAN_HD int wg_off(int r, int col) {  // byte offset of channel col (16-bit) in pixel row r
    const int c16 = col >> 3, within = (col & 7) * 2;
    return r * RB + ((c16 ^ wg_swz<RB>(r)) << 4) + within;
}

// 8 consecutive pixel rows (k0 + 8*(lane>>4) + [0,8)) of channel (m0 + (lane&15)) -> MFMA operand
template <int RB>
IRGAN_HD uint4 tr_frag(const char* img, int k0, int m0, int lane) {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int r0 = k0 + 8 * g + q;
    typedef __attribute__((address_space(3))) s16x4 lds_s4;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + wg_off<RB>(r0, m0 + 4 * p)));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + wg_off<RB>(r0 + 4, m0 + 4 * p)));
    uint4 out;
    __builtin_memcpy(&out, &lo, 8);
    __builtin_memcpy((char*)&out + 8, &hi, 8);
    return out;
}

template <int BMC, int BNC>  // co tile, ci tile (128 or 64)
__global__ __launch_bounds__(512, 2) void conv_wgrad_glds_kernel(const irgan_conv_desc d, const bf16_t* __restrict__ x,
                                                                 const bf16_t* __restrict__ dy, float* __restrict__ dw,
                                                                 int kchunk, const bf16_t* __restrict__ zero,
                                                                 int ntx, int nty, int swz,
                                                                 float* __restrict__ slab = nullptr) {
    constexpr int KP = 64, STAGES = 3;
    constexpr int RA = BMC * 2, RBB = BNC * 2;          // bytes per pixel row in each image
    constexpr int ABYTES = KP * RA, STAGE = ABYTES + KP * RBB;
    constexpr int WM = 4, WN = 2;                       // wave grid (co x ci)
    constexpr int MI = BMC / WM / 16, NJ = BNC / WN / 16;
    constexpr int AU = ABYTES / 1024 / 8, BU = KP * RBB / 1024 / 8;  // glds pieces per wave per tile
    static_assert(AU >= 1 && BU >= 1, "tile");
    __shared__ __attribute__((aligned(1024))) char smem[STAGES * STAGE];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid / WN, wn = wid % WN;
    const int HoWo = d.Ho * d.Wo;
    const long P = (long)d.N * HoWo;
    const int K = d.KH * d.KW * d.Cin;
    // 1-D grid ordered (split, k-tile, co-tile): the blocks of one pixel range
    // read the same dY / X rows and share an XCD after the remap
    const int t = xcd_tile(blockIdx.x, gridDim.x, swz);
    const int bx = t % ntx, by = (t / ntx) % nty, bz = t / (ntx * nty);
    const int co0 = bx * BMC, n0 = by * BNC;
    const long pb = (long)bz * kchunk;
    const long pe = min(P, pb + kchunk);
    if (pb >= pe) return;
    const int tap = n0 / d.Cin, cin0 = n0 - tap * d.Cin;
    const int ty = tap / d.KW, tx = tap - ty * d.KW;
    const bool reflect = d.pad_mode == IRGAN_PAD_REFLECT;
    const int cout8 = (d.Cout + 7) / 8 * 8;  // dY channels beyond Cout are zero padding

    // lane -> (row within a 1 KiB piece, 16-byte slot) for each image
    constexpr int ARPP = 1024 / RA, BRPP = 1024 / RBB;  // pixel rows per piece
    const int a_sub = lane / (RA / 16), a_slot = lane % (RA / 16);
    const int b_sub = lane / (RBB / 16), b_slot = lane % (RBB / 16);

    auto issue = [&](long p0, int stage) {
        char* sA = smem + stage * STAGE;
        char* sB = sA + ABYTES;
#pragma unroll
        for (int u = 0; u < AU; ++u) {
            const int piece = wid * AU + u;
            const int r = piece * ARPP + a_sub;
            const long p = p0 + r;
            const int c16 = a_slot ^ wg_swz<RA>(r);
            const bool ok = (p < pe) & (co0 + c16 * 8 < cout8);
            const bf16_t* src = ok ? dy + p * d.ldy + d.yoff + co0 + c16 * 8 : zero;
            glds16(src, sA + piece * 1024);
        }
#pragma unroll
        for (int u = 0; u < BU; ++u) {
            const int piece = wid * BU + u;
            const int r = piece * BRPP + b_sub;
            const long p = p0 + r;
            const int c16 = b_slot ^ wg_swz<RBB>(r);
            const int pp = (int)min(p, P - 1);
            const int n = pp / HoWo, rr = pp - n * HoWo, i = rr / d.Wo, j = rr - i * d.Wo;
            int qy = i * d.sy + ty + d.c0y, qx = j * d.sx + tx + d.c0x;
            if (reflect) {
                qy = reflect_idx(qy, d.H);
                qx = reflect_idx(qx, d.W);
            }
            const bool ok = (p < pe) & ((unsigned)qy < (unsigned)d.H) & ((unsigned)qx < (unsigned)d.W);
            const long off = (((long)n * d.H + qy) * d.W + qx) * d.ldx + d.xoff + cin0 + c16 * 8;
            glds16(ok ? x + off : zero, sB + piece * 1024);
        }
    };

    f32x4 acc[MI][NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = (int)((pe - pb + KP - 1) / KP);
    issue(pb, 0);
    if (nk > 1) issue(pb + KP, 1);
    for (int kt = 0; kt < nk; ++kt) {
        if (kt + 1 < nk) wait_vmcnt<AU + BU>();
        else wait_vmcnt<0>();
        lds_barrier();
        if (kt + 2 < nk) issue(pb + (long)(kt + 2) * KP, (kt + 2) % STAGES);
        const char* A = smem + (kt % STAGES) * STAGE;
        const char* B = A + ABYTES;
#pragma unroll
        for (int h = 0; h < 2; ++h) {  // two 32-pixel MFMA k-steps per tile
            uint4 af[MI], bfr[NJ];
#pragma unroll
            for (int i = 0; i < MI; ++i) af[i] = tr_frag<RA>(A, 32 * h, wm * (BMC / WM) + i * 16, lane);
#pragma unroll
            for (int j = 0; j < NJ; ++j) bfr[j] = tr_frag<RBB>(B, 32 * h, wn * (BNC / WN) + j * 16, lane);
#pragma unroll
            for (int i = 0; i < MI; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[i]),
                                                                        __builtin_bit_cast(bf16x8_t, bfr[j]),
                                                                        acc[i][j], 0, 0, 0);
        }
    }
    // split-K partials: plain stores into this split's slab (glds_slab_reduce sums them in
    // a fixed order) or, without a slab, fp32 atomics into dw (order-dependent rounding)
    float* const dst = slab ? slab + (long)bz * d.Cout * K : nullptr;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int co = co0 + wm * (BMC / WM) + i * 16 + (lane >> 4) * 4 + r;
            if (co >= d.Cout) continue;
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int kc = n0 + wn * (BNC / WN) + j * 16 + (lane & 15);
                if (dst) dst[(long)co * K + kc] = acc[i][j][r];
                else atomicAdd(dw + (long)co * K + kc, acc[i][j][r]);
            }
        }
}

// dw[i] += sum over splits s (in order) of slab[s][i]: the deterministic second stage
// of the slab split-K (every element sees the same summation order on every run)
__global__ __launch_bounds__(256) void glds_slab_reduce(const float* __restrict__ slab, int splits, long n,
                                                        float* __restrict__ dw) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n / 4; i += (long)gridDim.x * 256) {
        slab_sum4(slab, splits, n, dw, i);
    }
}

}  // namespace

extern "C" int irgan_conv_wgrad_glds(const irgan_conv_desc* d, const void* x, const void* dy, float* dw, int splitk,
                                     hipStream_t st, float* ws, long ws_cap) {
    const long P = (long)d->N * d->Ho * d->Wo;
    const int K = d->KH * d->KW * d->Cin;
    if (P <= 0) return 0;
    static void* zero_cache[IRGAN_MAX_DEVICES];  // the zero page's address per device
    const bf16_t* zero = (const bf16_t*)irgan_symbol(HIP_SYMBOL(g_irgan_zero_page), zero_cache);
    if (!zero) return IRGAN_EUNSUPPORTED;
    const int BMC = d->Cout % 128 == 0 ? 128 : 64;
    const int BNC = d->Cin % 128 == 0 ? 128 : 64;
    const int tiles = irgan_cdiv(d->Cout, BMC) * (K / BNC);
    if (splitk <= 0) {
        splitk = irgan_cdiv(512, tiles);  // ~2 blocks per CU
        long maxs = (P + 16 * 64 - 1) / (16 * 64);  // >= 16 K-tiles per split
        if (splitk > maxs) splitk = (int)maxs;
        if (splitk < 1) splitk = 1;
    }
    const int swz = irgan_xcd_swz();
    // prefer a split count that makes the grid a multiple of 8 (XCD remap)
    if (swz && splitk > 1 && (tiles * splitk) % 8) {
        for (int s2 = splitk; s2 >= 1 && s2 >= splitk - 7; --s2)
            if ((tiles * s2) % 8 == 0) { splitk = s2; break; }
    }
    if (irgan_det(d)) {  // deterministic: no atomics -- at most the splits the workspace holds
        const long fit = ws ? ws_cap / ((long)d->Cout * d->KH * d->KW * d->Cin) : 1;
        if (splitk > fit) splitk = (int)(fit > 1 ? fit : 1);
    }
    long kc = (P + splitk - 1) / splitk;
    kc = (kc + 63) / 64 * 64;
    splitk = (int)((P + kc - 1) / kc);
    const int ntx = irgan_cdiv(d->Cout, BMC), nty = K / BNC;
    const int nb = ntx * nty * splitk;
    const bf16_t* xp = (const bf16_t*)x;
    const bf16_t* dp = (const bf16_t*)dy;
    const long n = (long)d->Cout * K;
    float* slab = (ws && splitk > 1 && n % 4 == 0 && (long)splitk * n <= ws_cap) ? ws : nullptr;
    if (BMC == 128 && BNC == 128)
        conv_wgrad_glds_kernel<128, 128><<<nb, 512, 0, st>>>(*d, xp, dp, dw, (int)kc, zero, ntx, nty, swz, slab);
    else if (BMC == 128)
        conv_wgrad_glds_kernel<128, 64><<<nb, 512, 0, st>>>(*d, xp, dp, dw, (int)kc, zero, ntx, nty, swz, slab);
    else if (BNC == 128)
        conv_wgrad_glds_kernel<64, 128><<<nb, 512, 0, st>>>(*d, xp, dp, dw, (int)kc, zero, ntx, nty, swz, slab);
    else conv_wgrad_glds_kernel<64, 64><<<nb, 512, 0, st>>>(*d, xp, dp, dw, (int)kc, zero, ntx, nty, swz, slab);
    if (slab) {
        const int blocks = (int)std::min<long>((n / 4 + 255) / 256, 2048);
        glds_slab_reduce<<<blocks, 256, 0, st>>>(slab, splitk, n, dw);
    }
    IRGAN_LAUNCH_CHECK();
    return 0;
}
