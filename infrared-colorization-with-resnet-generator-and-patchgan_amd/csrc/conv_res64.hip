// Resident-weight persistent conv for one 64-channel input chunk (3x3, stride 1):
// VGG conv1_2 / conv2_1 forward, down1 forward (+ fused InstanceNorm statistics) and every
// backward-data conv whose dY has 64 channels (VGG conv1_2, up2_conv).  Entered from
// irgan_conv_fwd_pp / irgan_conv_fwd_stats (conv_pp.hip), which own the C ABI.
#include <type_traits>

#include "conv_epilogue.h"

namespace {

IRGAN_HD int lds_off(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }
constexpr int PH = 16, PW = 16;  // output patch

// ---- resident-weight persistent variant: 3x3 stride 1, Cin == 64 --------------------
// With one 64-channel input chunk a conv_pp block does only 9 K-steps per 16x16 patch, so
// its fixed cost (first DMA latency, per-window barriers, LDS-staged epilogue) outweighs
// the MFMA work: VGG conv1_2 / down1 / up2-dgrad ran at 0.16-0.32 of peak.  Here one
// block per CU loops over the patches of one 64-channel output tile:
//  * all 9 taps x 64 x 64 weights stay in LDS (72 KiB, loaded once per block);
//  * the input halo is double-buffered: patch i+2's halo is DMA'd (buffer_load ... lds)
//    into the buffer patch i just released, so it lands under patch i+1's MFMA loop;
//  * the K loop has no barrier at all (nothing is written into LDS it reads): 8 waves,
//    2 patch rows x 64 channels each, 18 sub-steps of 8 mfma_f32_16x16x32_bf16;
//  * epilogue straight from the C^T accumulators (4 consecutive channels of one pixel
//    per lane: bias, activation, mask, accumulate, one 8-byte store), so a wave that
//    finishes its MFMAs stores while the others still multiply; STATS: per-wave channel
//    sums by a 4-step reduce-scatter across the 16 pixel lanes, 8 wave rows summed in
//    fixed order into the same per-(image, patch, channel) partials as conv_pp;
//  * two barriers per patch: halo landed (counted vmcnt: the next patch's pieces are
//    the only younger loads) and halo released.
// LDS: 73728 (weights) + 2 x 41984 (halos) + 4096 (stats rows) = 161792 bytes.
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
// s_waitcnt vmcnt(n) for a wave-uniform n in [0, 31] (the immediate is an encoding field)
IRGAN_HD void wait_vm_dyn(int n) {
    switch (n) {
#define WV(k) case k: wait_vmcnt<k>(); break;
        WV(0) WV(1) WV(2) WV(3) WV(4) WV(5) WV(6) WV(7) WV(8) WV(9) WV(10) WV(11) WV(12) WV(13) WV(14) WV(15)
        WV(16) WV(17) WV(18) WV(19) WV(20) WV(21) WV(22) WV(23) WV(24) WV(25) WV(26) WV(27) WV(28) WV(29) WV(30)
#undef WV
        default: wait_vmcnt<31>(); break;
    }
}
// R64_EXP (ablation builds only, tools/build_variant.sh): bit 0 no MFMA, bit 1 no output
// stores, bit 2 no halo DMA after the first two patches, bit 3 no fragment reads from LDS
#ifndef R64_EXP
#define R64_EXP 0
#endif
constexpr int R64_HP = 41;               // halo pieces: 18 x 18 rows of 128 B
constexpr int R64_HB = R64_HP * 1024;
constexpr int R64_WB = 9 * 64 * 128;
constexpr int R64_LDS = R64_WB + 2 * R64_HB + 8 * 64 * 8;

// ONEB: one barrier per patch -- the next-but-one halo is issued at the top of the following
// iteration instead of after a second, post-K-loop barrier.
// RUN (round 6): the block walks a CONTIGUOUS run of `runk` patches (q0 .. q0 + runk - 1) instead
// of every qs-th patch.  With STATS each lane then keeps its two reduce-scattered channel sums
// (sum, sum of squares) in registers over the whole run; they are summed across the 8 waves
// (stats rows in LDS) only where the run ends or crosses into the next image -- one partial
// row per (image, run) instead of per patch -- so the per-patch stats rows and the post-K-loop
// barrier are gone and STATS runs the ONEB schedule.  Runs align with the
// images (runk divides the patches per image, or is a multiple of them): row = run index, or
// the image when a run covers whole images.
// POOL (round 6): the epilogue also writes the 2x2 max-pool of the activated output (VGG
// conv1_2 -> pool, ir:664 features[:16]): a wave's two patch rows are one pooled row, the two
// columns of a window sit in lanes px and px ^ 1.  y == nullptr: the pooled map alone (the
// real images' half, whose pre-pool activations nothing reads).  Max of the fp32 values then
// one bf16 rounding == max of the rounded values (rounding is monotone): the bits of
// irgan_maxpool_fwd over the stored map.
template <bool ACC, bool STATS, bool ONEB = false, bool RUN = false, bool POOL = false>
__global__ __launch_bounds__(512, 1) void conv_res64_kernel(const irgan_conv_desc d, const bf16_t* __restrict__ x,
                                                           const bf16_t* __restrict__ w,
                                                           const float* __restrict__ bias, bf16_t* __restrict__ y,
                                                           const bf16_t* __restrict__ mask, int ntn, int tpx,
                                                           int tpy, float2* __restrict__ part, int xcdg, int runk,
                                                           bf16_t* __restrict__ ypool) {
    constexpr int TAPS = 9, HWd = PW + 2, HROWS = (PH + 2) * HWd, MI = 2, NJ = 4, Kw = TAPS * 64;
    static_assert(HROWS <= R64_HP * 8 && R64_HP * 8 - HROWS < 8, "halo pieces");
    static_assert(!(ONEB && STATS && !RUN), "per-patch stats rows need the post-loop barrier");
    static_assert(!RUN || ONEB, "runs use the one-barrier schedule");
    static_assert(!POOL || (ONEB && !ACC && !STATS), "pooling: plain forward");
    __shared__ __attribute__((aligned(1024))) char smem[R64_LDS];
    char* const sW = smem;
    char* const sH = smem + R64_WB;
    float2* const sR = (float2*)(smem + R64_WB + 2 * R64_HB);  // [8 waves][64 channels]

    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    // block -> (channel tile, patch sequence).  With gridDim % (8 ntn) == 0 the ntn tiles of one
    // patch sequence sit on the same XCD (blocks b, b+8, ...: workgroups are dealt to the 8
    // XCDs round-robin), so the second tile's halo reads hit the L2 the first one filled
    int nt, q0;
    const int qs = gridDim.x / ntn;
    if (xcdg) {
        const int x = blockIdx.x & 7, sl = blockIdx.x >> 3;
        nt = sl % ntn;
        q0 = (sl / ntn) * 8 + x;
    } else {
        nt = blockIdx.x % ntn;
        q0 = blockIdx.x / ntn;
    }
    const int P = d.N * tpy * tpx;
    const int tpi = tpx * tpy;
    const int pstep = RUN ? 1 : qs;                          // patch sequence q0, q0 + pstep, ...
    const int pend = RUN ? min(P, (q0 + 1) * runk) : P;
    if (RUN) q0 *= runk;                                     // run index -> its first patch
    const int n0 = nt * 64;
    const int nh = (R64_HP - wid + 7) >> 3;  // halo pieces of this wave: 6 (wave 0) or 5
    const int sub = lane >> 3;
    const bool reflect = d.pad_mode == IRGAN_PAD_REFLECT;
    const i32x4 xr = make_rsrc(x, (uint32_t)((long)d.N * d.H * d.W * d.ldx * 2));

    auto issue_halo = [&](int p, int buf) {
        if ((R64_EXP & 4) && p >= q0 + 2 * qs) return;
        const int pxi = p % tpx, pyi = (p / tpx) % tpy, img = p / (tpx * tpy);
        const int py0 = pyi * PH + d.c0y, px0 = pxi * PW + d.c0x;
        char* dst = sH + buf * R64_HB;
        int lsub = sub;
        asm volatile("" : "+v"(lsub));
#pragma unroll
        for (int u = 0; u < 6; ++u) {
            if (u < nh) {
                const int h = (u * 8 + wid) * 8 + lsub;
                const int hy = h / HWd, hx = h - hy * HWd;
                int iy = py0 + hy, ix = px0 + hx;
                if (reflect) {
                    iy = reflect_idx(iy, d.H);
                    ix = reflect_idx(ix, d.W);
                }
                const bool ok = (h < HROWS) & ((unsigned)iy < (unsigned)d.H) & ((unsigned)ix < (unsigned)d.W);
                const uint32_t off = ok ? (uint32_t)((((img * d.H + iy) * d.W + ix) * d.ldx + d.xoff) * 2 +
                                                     ((lane & 7) ^ lsub) * 16)
                                        : IRGAN_OOB;
                blds16(xr, off, dst + (u * 8 + wid) * 1024);
            }
        }
    };

    // prologue: the block's weight tile (piece u*8 + wid = tap u, channels wid*8 .. +8),
    // then the first two halos
    {
        const i32x4 wr = make_rsrc(w, (uint32_t)((long)d.Cout * Kw * 2));
        const uint32_t off = (uint32_t)((n0 + wid * 8 + sub) * Kw * 2 + ((lane & 7) ^ sub) * 16);
#pragma unroll
        for (int u = 0; u < TAPS; ++u) blds16(wr, off, (uint32_t)(u * 128), sW + (u * 8 + wid) * 1024);
    }
    if (q0 < pend) issue_halo(q0, 0);
    if (q0 + pstep < pend) issue_halo(q0 + pstep, 1);

    const int prow = wid * 2;
    const int g0 = lane >> 4;
    const int arow0 = prow * HWd + (lane & 15);
    const int bb0 = lds_off(lane & 15, g0), bb1 = lds_off(lane & 15, 4 + g0);
    int tsw[8];
#pragma unroll
    for (int k8 = 0; k8 < 8; ++k8) tsw[k8] = (g0 ^ ((arow0 + k8) & 7)) << 4;
    const int cl0 = 4 * g0;  // tile-local channel of r = 0, j = 0
    float4 b4[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
        b4[j] = bias ? *(const float4*)(bias + n0 + cl0 + j * 16) : make_float4(0.f, 0.f, 0.f, 0.f);
    const bool vmask = mask != nullptr;

    // output through a raw buffer resource: exactly MI * NJ store instructions per wave and
    // patch (a pixel outside the image gets the out-of-range offset and is dropped), so the
    // counted vmcnt at the top of the loop knows how many of its ops are younger than a halo
    const bool yfull = !POOL || y != nullptr;
    const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(
        yfull ? y : ypool, (short)0, yfull ? (int)((long)d.N * d.OH * d.OW * d.ldy * 2) : 0, 0x00020000);
    // pooled map: [N][Ho / 2][Wo / 2][Cout] bf16, dense
    const __amdgpu_buffer_rsrc_t pr = __builtin_amdgcn_make_buffer_rsrc(
        POOL ? ypool : y, (short)0, POOL ? (int)((long)d.N * (d.Ho / 2) * (d.Wo / 2) * d.Cout * 2) : 0, 0x00020000);
    // stores per wave and patch (the counted vmcnt at the top of the loop)
    const int NST = (yfull ? MI * NJ : 0) + (POOL ? NJ : 0);
    int it = 0;
    int flushed = 0;          // RUN && STATS: the previous patch ended with a partial-row store
    float2 racc = make_float2(0.f, 0.f);  // RUN && STATS: this lane's two sums over the run so far
#pragma unroll 1
    for (int p = q0; p < pend; p += pstep, ++it) {
        const int buf = it & 1;
        // VMEM ops issued after this patch's halo, in issue order: (it >= 2) the stats
        // store of patch it-2 (made at the top of it-1), the stores of patch it-1, the halo
        // of patch it+1 (it == 0: only that halo)
        // (ONEB: halo it+1 was issued at the top of iteration it-1, so only patch it-1's stores
        // are younger from it == 1 on)
        {
            const int nxt = p + pstep < pend ? nh : 0;
            const int younger = it == 0 ? nxt
                                        : (ONEB ? NST + flushed
                                                : (it == 1 ? NST + nxt : (STATS ? 1 : 0) + NST + nxt));
            wait_vm_dyn(__builtin_amdgcn_readfirstlane(younger));
        }
        lds_barrier();  // every wave's pieces of this patch's halo (and the weights) landed
        // this patch's epilogue operands (backward mask, accumulate's old values) are loaded
        // now, ahead of the next halo and the K loop, so their latency hides under the MFMAs
        // (loaded at the epilogue they stalled every patch: VGG conv1_2 backward-data 130 us
        // against its forward's 81)
        const int pxi = p % tpx, pyi = (p / tpx) % tpy, img = p / (tpx * tpy);
        uint2 old[MI][NJ], mk[MI][NJ];
        long pixs[MI];
        bool oks[MI];
#pragma unroll
        for (int i = 0; i < MI; ++i) {
            const int oy = pyi * PH + prow + i, ox = pxi * PW + (lane & 15);
            oks[i] = oy < d.Ho && ox < d.Wo;
            pixs[i] = oks[i] ? ((long)img * d.OH + oy * d.omy + d.ooy) * d.OW + ox * d.omx + d.oox : 0;
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int co = n0 + cl0 + j * 16;
                old[i][j] = mk[i][j] = make_uint2(0u, 0u);
                if (ACC && oks[i]) old[i][j] = *(const uint2*)(y + pixs[i] * d.ldy + d.yoff + co);
                if (vmask && oks[i]) mk[i][j] = *(const uint2*)(mask + pixs[i] * d.ldm + d.moff + co);
            }
        }
        // ONEB: every wave has also finished patch it-1 (K loop and stores), so its halo buffer
        // takes patch it+1's halo now
        const bool halo_next = ONEB && it > 0 && p + pstep < pend;
        if (halo_next) issue_halo(p + pstep, buf ^ 1);
        if constexpr (STATS && !RUN) {
            // patch it-1's partials: its 8 wave rows are complete (written before this barrier)
            if (it > 0 && lane < 8) {
                const int c = wid * 8 + lane;
                float a = 0.f, b = 0.f;
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    const float2 e = sR[r * 64 + c];
                    a += e.x;
                    b += e.y;
                }
                part[(long)(p - qs) * d.Cout + n0 + c] = make_float2(a, b);
            }
        }

        f32x4 acc[MI][NJ];
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int hb = arow0 * 128 + buf * R64_HB;
#pragma unroll
        for (int tp = 0; tp < TAPS; ++tp) {
            const int ty = tp / 3, tx = tp % 3;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                uint4 af[MI], bfr[NJ];
#pragma unroll
                for (int j = 0; j < NJ; ++j)
                    bfr[j] = (R64_EXP & 8) ? make_uint4(lane + j, tp, h, 1) : *(const uint4*)(sW + tp * 8192 + (h ? bb1 : bb0) + j * 2048);
#pragma unroll
                for (int i = 0; i < MI; ++i) {
                    const int K = (i + ty) * HWd + tx;
                    af[i] = (R64_EXP & 8) ? make_uint4(lane + i, K, h, 2) : *(const uint4*)(sH + (hb + (tsw[K & 7] ^ (h * 64))) + K * 128);
                }
#pragma unroll
                for (int i = 0; i < MI; ++i)
#pragma unroll
                    for (int j = 0; j < NJ; ++j)
                        if (!(R64_EXP & 1)) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, bfr[j]),
                                                                            __builtin_bit_cast(bf16x8_t, af[i]),
                                                                            acc[i][j], 0, 0, 0);
            }
        }
        // every wave is done with this halo buffer; the stats rows were read.  ONEB: no barrier
        // here -- a wave that finishes its MFMAs stores while the others still multiply
        if (!ONEB) lds_barrier();

        // ---- epilogue from the accumulators (the prefetched operands are older than the
        // halo pieces issued after them: only those may stay in flight)
        if (ACC || vmask) wait_vm_dyn(__builtin_amdgcn_readfirstlane(halo_next ? nh : 0));
        float st[2 * NJ * 4];  // STATS: (sum, sum of squares) of channel (j, r) at [2 (4j + r) + {0, 1}]
#pragma unroll
        for (int k = 0; k < 2 * NJ * 4; ++k) st[k] = 0.f;
        float pmx[POOL ? NJ : 1][4];  // POOL: row prow's activated values, per (j, r)
        auto body = [&](auto actc) {
            constexpr int A = decltype(actc)::value;
#pragma unroll
            for (int i = 0; i < MI; ++i) {
                const bool ok = oks[i];
                const long pix = pixs[i];
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    const int co = n0 + cl0 + j * 16;
                    const float bb[4] = {b4[j].x, b4[j].y, b4[j].z, b4[j].w};
                    float v[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        v[r] = conv_act(acc[i][j][r] + bb[r], A);
                        if (vmask) {
                            const uint32_t mw = r < 2 ? mk[i][j].x : mk[i][j].y;
                            v[r] *= mask_mul(__uint_as_float((r & 1) ? (mw & 0xffff0000u) : (mw << 16)), d.mask_act);
                        }
                        if (ACC) {
                            const uint32_t ow = r < 2 ? old[i][j].x : old[i][j].y;
                            v[r] += __uint_as_float((r & 1) ? (ow & 0xffff0000u) : (ow << 16));
                        }
                    }
                    u32x2_t pk;
                    pk.x = pk_bf16(v[0], v[1]);
                    pk.y = pk_bf16(v[2], v[3]);
                    const int off = ok && !(R64_EXP & 2) ? (int)((pix * d.ldy + d.yoff + co) * 2) : (int)IRGAN_OOB;
                    if (yfull) __builtin_amdgcn_raw_buffer_store_b64(pk, yr, off, 0, 0);
                    if constexpr (POOL) {
                        // rows prow, prow + 1 (i = 0, 1) then columns px, px ^ 1 (lane ^ 1)
                        if (i == 0) {
#pragma unroll
                            for (int r = 0; r < 4; ++r) pmx[j][r] = v[r];
                        } else {
                            float m[4];
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                m[r] = fmaxf(pmx[j][r], v[r]);
                                m[r] = fmaxf(m[r], dpp_xor16<1>(m[r]));
                            }
                            u32x2_t pp;
                            pp.x = pk_bf16(m[0], m[1]);
                            pp.y = pk_bf16(m[2], m[3]);
                            const int oy = pyi * PH + prow, ox = pxi * PW + (lane & 15);
                            const bool pok = ((lane & 1) == 0) && oy + 1 < d.Ho && ox + 1 < d.Wo;
                            const long ppix = ((long)img * (d.Ho / 2) + (oy >> 1)) * (d.Wo / 2) + (ox >> 1);
                            __builtin_amdgcn_raw_buffer_store_b64(pp, pr, pok ? (int)((ppix * d.Cout + co) * 2)
                                                                              : (int)IRGAN_OOB, 0, 0);
                        }
                    }
                    if constexpr (STATS) {
                        if (ok) {
                            const float q[4] = {__uint_as_float(pk.x << 16), __uint_as_float(pk.x & 0xffff0000u),
                                                __uint_as_float(pk.y << 16), __uint_as_float(pk.y & 0xffff0000u)};
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                st[2 * (4 * j + r)] += q[r];
                                st[2 * (4 * j + r) + 1] += q[r] * q[r];
                            }
                        }
                    }
                }
            }
        };
        switch (d.act) {
            case IRGAN_ACT_RELU: body(std::integral_constant<int, IRGAN_ACT_RELU>()); break;
            case IRGAN_ACT_LRELU: body(std::integral_constant<int, IRGAN_ACT_LRELU>()); break;
            default: body(std::integral_constant<int, IRGAN_ACT_NONE>()); break;
        }
        if constexpr (STATS) {
            // reduce-scatter over the 16 pixel lanes (lane & 15): 32 values -> 2 per lane;
            // lane (g0, k) ends with channel (j, r) = (k >> 2, k & 3) of its lane group.  The
            // partner values move by DPP (dpp_xor16): no LDS round trips in the epilogue
            auto level = [&](auto mc) {
                constexpr int m = decltype(mc)::value, n = 4 * m;  // xor distance, values held
                const bool hi = (lane & m) != 0;
#pragma unroll
                for (int k = 0; k < n / 2; ++k) {
                    const float keep = hi ? st[n / 2 + k] : st[k];
                    const float send = hi ? st[k] : st[n / 2 + k];
                    st[k] = keep + dpp_xor16<m>(send);
                }
            };
            level(std::integral_constant<int, 8>());
            level(std::integral_constant<int, 4>());
            level(std::integral_constant<int, 2>());
            level(std::integral_constant<int, 1>());
        }
        const int sk = lane & 15;
        float2* const srow = sR + wid * 64 + (sk >> 2) * 16 + cl0 + (sk & 3);
        if constexpr (STATS && !RUN) *srow = make_float2(st[0], st[1]);
        if constexpr (STATS && RUN) {
            racc.x += st[0];
            racc.y += st[1];
            // the run ends, or the next patch is another image's: this (image, run)'s partial row
            const int img_p = p / tpi;
            flushed = 0;
            if (p + pstep >= pend || (p + pstep) / tpi != img_p) {
                *srow = racc;
                lds_barrier();  // every wave's row of the run's sums
                if (lane < 8) {
                    const int c = wid * 8 + lane;
                    float a = 0.f, b = 0.f;
#pragma unroll
                    for (int r = 0; r < 8; ++r) {
                        const float2 e = sR[r * 64 + c];
                        a += e.x;
                        b += e.y;
                    }
                    const long row = runk <= tpi ? (long)(p / runk) : (long)img_p;
                    part[row * d.Cout + n0 + c] = make_float2(a, b);
                }
                lds_barrier();  // the rows were read before the next flush rewrites them
                racc = make_float2(0.f, 0.f);
                flushed = 1;
            }
        }
        if (!ONEB && p + 2 * qs < P) issue_halo(p + 2 * qs, buf);
    }
    if constexpr (STATS && !RUN) {
        lds_barrier();  // the last patch's stats rows
        if (lane < 8) {
            const int c = wid * 8 + lane;
            float a = 0.f, b = 0.f;
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const float2 e = sR[r * 64 + c];
                a += e.x;
                b += e.y;
            }
            part[(long)(q0 + (it - 1) * qs) * d.Cout + n0 + c] = make_float2(a, b);
        }
    }
    wait_vmcnt<0>();
}

}  // namespace

namespace irgan_res64 {

bool ok(const irgan_conv_desc* d) {
    static const bool on = !getenv("IRGAN_NO_RES64");
    return on && d->Cin == 64 && d->KH == 3 && d->KW == 3 && d->sy == 1 && d->sx == 1 && d->Cout % 64 == 0 &&
           d->dtype == IRGAN_BF16 && d->out_dtype == IRGAN_BF16 && d->act != IRGAN_ACT_TANH && d->ldy % 4 == 0 &&
           d->yoff % 4 == 0 && d->ldx % 8 == 0 && d->xoff % 8 == 0 && (long)d->N * d->H * d->W * d->ldx < (1L << 30) &&
           (long)d->N * d->OH * d->OW * d->ldy * 2 < (1L << 31);
}

static int grid_for(int ntn, int tiles) {
    const int cus = irgan_cu_count();
    const int g = (cus / ntn) * ntn;
    return g < tiles ? (g > 0 ? g : ntn) : tiles;
}

// The statistics variant's run length: the smallest k >= the patches one block must take for
// the grid to fit the CUs, with k | P and (k | patches per image or patches per image | k)
static int run_len(int P, int tpi, int ntn) {
    const int cus = irgan_cu_count();
    const int per = cus / ntn > 0 ? cus / ntn : 1;
    for (int k = irgan_cdiv(P, per); k < P; ++k)
        if (P % k == 0 && (tpi % k == 0 || k % tpi == 0)) return k;
    return P;
}

// mask: NULL or the bf16 backward mask (8-byte aligned slices: checked by the caller).
// Returns the InstanceNorm partial rows per image written into part (0 without part).
int launch(const irgan_conv_desc* d, const void* x, const void* w, const float* bias, void* y, const void* mask,
           float2* part, hipStream_t st, void* ypool) {
    const int tpx = irgan_cdiv(d->Wo, PW), tpy = irgan_cdiv(d->Ho, PH), ntn = d->Cout / 64;
    const int P = d->N * tpx * tpy, tpi = tpx * tpy;
    static const bool per_patch = getenv("IRGAN_R64_PATCH_STATS") != nullptr;  // A/B: round-5 schedule
    const int runk = part && !per_patch ? run_len(P, tpi, ntn) : 0;
    const int grid = runk ? ntn * (P / runk) : grid_for(ntn, P * ntn);
    const int xcdg = ntn > 1 && grid % (8 * ntn) == 0;
#define R64(ACCV, STV, OB, RN, ...)                                                                                 \
    conv_res64_kernel<ACCV, STV, OB, RN, ##__VA_ARGS__><<<grid, 512, 0, st>>>(                                        \
        *d, (const bf16_t*)x, (const bf16_t*)w, bias, (bf16_t*)y, (const bf16_t*)mask, ntn, tpx, tpy, part, xcdg,      \
        runk, (bf16_t*)ypool)
    if (ypool) R64(false, false, true, false, true);
    else if (part && runk) R64(false, true, true, true);
    else if (part) R64(false, true, false, false);
    else if (d->accumulate) R64(true, false, true, false);
    else R64(false, false, true, false);
#undef R64
    if (!part) return 0;
    return runk ? (runk <= tpi ? tpi / runk : 1) : tpi;
}

}  // namespace irgan_res64

