// Backward-data of the 4x4 stride-2 pad-1 convolutions (PatchGAN model.0 / .3 / .6,
// ir:600-612) in ONE launch for all four output phases.
//
// dx[2i + py][2j + px] = sum over the 2x2 taps (a, b) of phase (py, px) of
//   Wp[a][b] . dy[i + a + c0y(py)][j + b + c0x(px)]        (c0 in {-1, 0})
// -- the per-phase decomposition ops.PackedConv packs (pc.dg: one flipped / transposed
// [dx channels][2*2*Cin] image per phase).  Four separate launches (conv_halo.hip) re-read
// dy per phase, write every other pixel per launch and, at these shapes (K = 4 taps x
// 64..256, 64-channel outputs), run prologue / epilogue bound at 0.05-0.15 of MFMA peak
// (r03 trace: ~935 us per step on the side stream, D step + GAN-term pass).
//
// Here a block owns a 16x16 dy-space patch = a 32x32 dx patch (1024 pixels, all four
// phases) x BN output channels.  Per 64-channel chunk the 18x18 dy halo is DMA'd into LDS
// once (zero outside dy) and serves all four phases; a K-step = (chunk, tap t): the
// phases' weight tiles for tap t (4 x BN x 64) stream through a 2-stage ring.  Waves are
// WM pixel rows x WN channel columns with each wave row inside one phase, so a wave reads
// one phase's weights per K-step (MFMA: pixels as A, weights as B; the C layout is
// conv_epilogue.h's).  Epilogue: one phase per pass through an fp32 LDS tile, 16-byte
// stores of 8 channels (conv_store8: mask / accumulate / bf16 or fp32 out); the four
// phases of a patch are written by the same block back to back, so L2 merges the
// interleaved pixels into whole lines.
#include "conv_epilogue.h"

namespace {

constexpr int S2P = 16;                          // dy-space patch side
constexpr int S2H = S2P + 2;                     // halo side: dy rows I0-1 .. I0+P
constexpr int S2ROWS = S2H * S2H;                // 324 halo rows of 64 channels
constexpr int S2PIECES = (S2ROWS + 7) / 8;       // 41 pieces of 8 rows (1 KiB)
constexpr int S2HB = S2PIECES * 1024;

IRGAN_HD int s2_off(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }

struct S2Phases {
    const bf16_t* w[4];  // phase images [Cout][4 * Cin]
    int c0y[4], c0x[4];  // dy offset of tap (0, 0)
};

template <int BN, bool ONEC>
struct S2 {
    static constexpr int WM = BN >= 32 ? 4 : 8, WN = 8 / WM;  // wave rows x columns
    static constexpr int MI = 4 * S2P * S2P / WM / 16;        // pixel fragments per wave
    static constexpr int NJ = BN / WN / 16;                   // channel fragments per wave
    static constexpr int BB = BN * 128;                       // one phase's weight tile
    static constexpr int STAGE = 4 * BB;
    static constexpr int RS = BN + 4;                         // epilogue row stride (floats)
    static constexpr int LOOP = (ONEC ? 1 : 2) * S2HB + 2 * STAGE;  // ONEC: one 64-channel chunk, one halo
    static constexpr int EPI = S2P * S2P * RS * 4;            // one phase, fp32
    static constexpr int LDS = LOOP > EPI ? LOOP : EPI;
    static_assert(NJ >= 1 && NJ * 16 * WN == BN && LDS <= 160 * 1024, "tile");
};

template <int BN, bool ONEC>
__global__ __launch_bounds__(512, ONEC ? 2 : 1) void dgrad_s2_kernel(const irgan_conv_desc d, const bf16_t* __restrict__ dy,
                                                          const S2Phases ph, void* __restrict__ dx,
                                                          const void* __restrict__ mask, int tpx, int tpy, int ntn,
                                                          int swz) {
    using G = S2<BN, ONEC>;
    constexpr int WM = G::WM, WN = G::WN, MI = G::MI, NJ = G::NJ, BB = G::BB, STAGE = G::STAGE;
    __shared__ __attribute__((aligned(1024))) char smem[G::LDS];
    char* const sH = smem;
    char* const sW = smem + (ONEC ? 1 : 2) * S2HB;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid / WN, wn = wid % WN;
    const int phs = wm * 4 / WM;                 // this wave row's phase (py << 1 | px)
    const int qb = (wm % (WM / 4)) * MI * 16;    // first pixel (within the phase) of the wave row
    int t = xcd_tile(blockIdx.x, gridDim.x, swz);
    const int nt = t % ntn;
    t /= ntn;
    const int txi = t % tpx;
    t /= tpx;
    const int tyi = t % tpy;
    const int img = t / tpy;
    const int I0 = tyi * S2P, J0 = txi * S2P, n0 = nt * BN;
    const int Kw = 4 * d.Cin, nchunk = d.Cin / 64, nk = 4 * nchunk;

    // ---- DMA: halo of chunk c (piece u = wid + 8k: rows 8u .. 8u+7) and the K-step weights
    const uint32_t dybytes = (uint32_t)((long)d.N * d.H * d.W * d.ldx * 2);
    const int sub = lane >> 3;
    auto issue_halo = [&](int c) {
        const i32x4 rs = make_rsrc(dy + c * 64, dybytes - c * 128);
        char* dst = sH + (ONEC ? 0 : (c & 1) * S2HB);
        for (int u = wid; u < S2PIECES; u += 8) {
            const int r = u * 8 + sub, hy = r / S2H, hx = r - hy * S2H;
            const int iy = I0 - 1 + hy, ix = J0 - 1 + hx;
            const bool ok = r < S2ROWS && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W;
            const uint32_t off = ok ? (uint32_t)((((long)img * d.H + iy) * d.W + ix) * d.ldx + d.xoff) * 2 +
                                          (uint32_t)(((lane & 7) ^ (r & 7)) << 4)
                                    : IRGAN_OOB;
            blds16(rs, off, dst + u * 1024);
        }
    };
    // weights of K-step k (chunk c = k / 4, tap k % 4): phase p's rows n0 .. n0+BN, 64 channels
    const uint32_t wbytes = (uint32_t)((long)d.Cout * Kw * 2);
    auto issue_w = [&](int k) {
        const int c = k >> 2, tp = k & 3;
        char* dst = sW + (k & 1) * STAGE;
        constexpr int PIECES = 4 * BN / 8;  // (phase, 8 rows)
        for (int u = wid; u < PIECES; u += 8) {
            const int p = u / (BN / 8), r = (u - p * (BN / 8)) * 8 + sub;  // row within the phase tile
            const i32x4 rs = make_rsrc(ph.w[p], wbytes);
            const uint32_t off = (uint32_t)(((long)(n0 + r) * Kw + tp * d.Cin + c * 64) * 2) +
                                 (uint32_t)(((lane & 7) ^ (r & 7)) << 4);
            blds16(rs, n0 + r < d.Cout ? off : IRGAN_OOB, dst + p * BB + (u - p * (BN / 8)) * 1024);
        }
    };

    f32x4 acc[MI][NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // pixel fragment i of this wave: phase pixels q = qb + 16 i + (lane & 15), (u, v) = (q / 16, q % 16)
    const int c0y = ph.c0y[phs], c0x = ph.c0x[phs];
    const int row0 = (qb / 16 + c0y + 1) * S2H + (lane & 15) + c0x + 1;  // halo row of fragment 0, tap (0, 0)
    const int g = lane >> 4;
    const int wrow = wn * (BN / WN) + (lane & 15);  // weight row of fragment j = 0 (+16 j)

    issue_halo(0);
    issue_w(0);
    wait_vmcnt<0>();
    __syncthreads();
#pragma unroll 1
    for (int k = 0; k < nk; ++k) {
        const int c = k >> 2, tp = k & 3;
        if (k + 1 < nk) issue_w(k + 1);
        if (tp == 0 && c + 1 < nchunk) issue_halo(c + 1);
        const char* H = sH + (ONEC ? 0 : (c & 1) * S2HB);
        const char* Wt = sW + (k & 1) * STAGE + phs * BB;
        const int tap = (tp >> 1) * S2H + (tp & 1);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            uint4 bfr[NJ], af[MI];
#pragma unroll
            for (int j = 0; j < NJ; ++j) bfr[j] = *(const uint4*)(Wt + s2_off(wrow + 16 * j, g + 4 * h));
#pragma unroll
            for (int i = 0; i < MI; ++i) af[i] = *(const uint4*)(H + s2_off(row0 + i * S2H + tap, g + 4 * h));
#pragma unroll
            for (int i = 0; i < MI; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[i]),
                                                                        __builtin_bit_cast(bf16x8_t, bfr[j]),
                                                                        acc[i][j], 0, 0, 0);
        }
        wait_vmcnt<0>();
        __syncthreads();  // step k+1's weights (and the next chunk's halo) landed; stage k&1 free
    }

    // ---- epilogue: one phase per pass (C: pixel 4 (lane >> 4) + r of the fragment, channel lane & 15)
    constexpr int RS = G::RS;
    float* st = (float*)smem;
    constexpr int LPP = BN / 8, PPP = 512 / LPP;
    const int ch = (tid % LPP) * 8, co = n0 + ch;
    const bool out_f32 = d.out_dtype == IRGAN_F32;
    const bool vec = co + 8 <= d.Cout &&
                     (out_f32 ? (d.ldy % 4 == 0 && d.yoff % 4 == 0) : (d.ldy % 8 == 0 && d.yoff % 8 == 0)) &&
                     (!mask || (d.ldm % 8 == 0 && d.moff % 8 == 0));
    const bool quad = d.Cout == 4 && out_f32 && !mask && d.ldy % 4 == 0 && d.yoff % 4 == 0;
#pragma unroll 1
    for (int p = 0; p < 4; ++p) {
        if (p) __syncthreads();  // the previous phase's tile is stored
        if (phs == p) {
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int i = 0; i < MI; ++i)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        st[(qb + i * 16 + 4 * g + r) * RS + wn * (BN / WN) + j * 16 + (lane & 15)] = acc[i][j][r];
        }
        __syncthreads();
        if (co >= d.Cout) continue;
        const int py = p >> 1, px = p & 1;
        for (int q = tid / LPP; q < S2P * S2P; q += PPP) {
            const int i = I0 + (q >> 4), j = J0 + (q & 15);
            const int oy = 2 * i + py, ox = 2 * j + px;
            if (oy >= d.OH || ox >= d.OW) continue;
            const long pix = ((long)img * d.OH + oy) * d.OW + ox;
            const float4 a0 = *(const float4*)(st + q * RS + ch), a1 = *(const float4*)(st + q * RS + ch + 4);
            if (quad) {  // 4-channel fp32 output (the D input gradient): one 16-byte store
                float4* yp = (float4*)((float*)dx + pix * d.ldy + d.yoff);
                float4 o = a0;
                if (d.accumulate) {
                    const float4 p0 = *yp;
                    o.x += p0.x; o.y += p0.y; o.z += p0.z; o.w += p0.w;
                }
                *yp = o;
                continue;
            }
            float v[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
            conv_store8(d, v, pix, co, vec, out_f32, dx, mask);
        }
    }
}

}  // namespace

extern "C" int irgan_conv_dgrad_s2_pp(const irgan_conv_desc* dd, const void* dy, const void* const* w, void* dx,
                                      const void* mask, hipStream_t st);

// d: the FOUR phase descriptors ops.conv_dgrad builds for a stride-2 layer (in pc.dg order),
// w: their four packed phase images.  Shapes (else IRGAN_EUNSUPPORTED, nothing launched):
// bf16 operands, every phase 2x2 taps with c0y, c0x in {-1, 0}, stride 1 on dy, output pixel
// map omy = omx = 2 with the four (ooy, oox) phases, Cin (dy channels) % 64 == 0, Cout (dx
// channels) <= 16 or % 64 == 0, no bias / activation, dy slice 8-aligned, dy and weights
// below 2^31 bytes; the four descriptors agree on everything else.
extern "C" int irgan_conv_dgrad_s2(const irgan_conv_desc* d, const void* dy, const void* const* w, void* dx,
                                   const void* mask, irgan_stream_t s) {
    if (!d || !dy || !w || !dx) return IRGAN_EINVAL;
    const irgan_conv_desc& a = d[0];
    if ((long)a.N * a.H * a.W <= 0 || a.Cout <= 0) return 0;
    static const bool off = getenv("IRGAN_NO_DGRAD_S2") != nullptr;
    if (off || a.dtype != IRGAN_BF16 || a.Cin % 64 || a.ldx % 8 || a.xoff % 8 || a.act != IRGAN_ACT_NONE ||
        (a.Cout > 16 && a.Cout % 64) || (long)a.N * a.H * a.W * a.ldx * 2 >= (1L << 31) ||
        (long)a.Cout * 4 * a.Cin * 2 >= (1L << 31) || (mask && !a.mask_act))
        return IRGAN_EUNSUPPORTED;
    S2Phases ph;
    int seen = 0;
    for (int k = 0; k < 4; ++k) {
        const irgan_conv_desc& e = d[k];
        if (!w[k] || e.KH != 2 || e.KW != 2 || e.sy != 1 || e.sx != 1 || e.omy != 2 || e.omx != 2 || e.ooy < 0 ||
            e.ooy > 1 || e.oox < 0 || e.oox > 1 || e.c0y < -1 || e.c0y > 0 || e.c0x < -1 || e.c0x > 0 ||
            e.N != a.N || e.H != a.H || e.W != a.W || e.Cin != a.Cin || e.ldx != a.ldx || e.xoff != a.xoff ||
            e.Cout != a.Cout || e.ldy != a.ldy || e.yoff != a.yoff || e.OH != a.OH || e.OW != a.OW ||
            e.accumulate != a.accumulate || e.out_dtype != a.out_dtype || e.mask_act != a.mask_act ||
            e.ldm != a.ldm || e.moff != a.moff || e.act != a.act || e.dtype != a.dtype || e.pad_mode != IRGAN_PAD_ZERO ||
            e.Ho != (a.OH - e.ooy + 1) / 2 || e.Wo != (a.OW - e.oox + 1) / 2)
            return IRGAN_EUNSUPPORTED;
        const int p = e.ooy * 2 + e.oox;
        if (seen & (1 << p)) return IRGAN_EUNSUPPORTED;
        seen |= 1 << p;
        ph.w[p] = (const bf16_t*)w[k];
        ph.c0y[p] = e.c0y;
        ph.c0x[p] = e.c0x;
    }
    // every dx pixel (2i + py, 2j + px) must come from dy position i (< H) of its phase
    if ((a.OH + 1) / 2 > a.H || (a.OW + 1) / 2 > a.W) return IRGAN_EUNSUPPORTED;
    {   // 64-channel dx: the four phases as 2x2 convs on conv_pp (conv_pp.hip)
        const int rc = irgan_conv_dgrad_s2_pp(d, dy, w, dx, mask, (hipStream_t)s);
        if (rc != IRGAN_EUNSUPPORTED) return rc;
    }
    const int swz = irgan_xcd_swz();
    const int tpy = irgan_cdiv((a.OH + 1) / 2, S2P), tpx = irgan_cdiv((a.OW + 1) / 2, S2P);
    hipStream_t st = (hipStream_t)s;
    const bool one = a.Cin == 64;  // one chunk: a single halo buffer (BN 16: two blocks per CU)
#define S2L(BNV, ONEV, NTN) \
    dgrad_s2_kernel<BNV, ONEV><<<a.N * tpy * tpx * (NTN), 512, 0, st>>>(a, (const bf16_t*)dy, ph, dx, mask, tpx, tpy, \
                                                                        NTN, swz)
    if (a.Cout <= 16) {
        if (one) S2L(16, true, 1);
        else S2L(16, false, 1);
    } else {
        if (one) S2L(64, true, a.Cout / 64);
        else S2L(64, false, a.Cout / 64);
    }
#undef S2L
    IRGAN_LAUNCH_CHECK();
    return 0;
}
