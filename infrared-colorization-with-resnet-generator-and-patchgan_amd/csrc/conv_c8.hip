// bf16 stride-1 convolution for 8-channel inputs (the zero-padded narrow layers:
// G inc 1->64 7x7, G outc backward-data 3->64 7x7, VGG conv1_1 3->64 3x3).
//
// With Cin = 8 a tap contributes only 8 of the 32 k-values an
// mfma_f32_16x16x32_bf16 consumes, so a per-tap K-step wastes 3/4 of the MFMA.
// Here the K axis is (tap, channel) flattened, exactly the packed weight row
// [co][tap][8]: one 32-deep K-step covers 4 taps, and lane group g (lane >> 4)
// of a pixel fragment reads its 8 channels (16 bytes) at the pixel shifted by
// tap 4s + g.  The input halo of a 16x16 output patch is (16+KH-1)(16+KW-1)
// pixels x 16 B (7.6 KiB for 7x7) and the whole weight matrix (64 x 416 bf16 for
// 7x7) stays resident in LDS, so the block is persistent: it loads the weights
// once and walks patches blockIdx.x, +gridDim.x, ..., double-buffering the
// halo (global loads of patch p+1 are in flight while patch p multiplies).
//
// C^T orientation (weights are the MFMA A operand): a lane's 4 accumulator
// rows are 4 consecutive output channels of one pixel, stored as one 8-byte
// (bf16) or 16-byte (fp32) write straight from registers -- no staging.
// 4 waves; wave w owns patch rows 4w..4w+3 (4 pixel fragments) x 64 channels.
// Stride 2 (D's first layer, 4x4): the halo is the 34x34 input span and output
// pixel (r, c) of tap t reads span pixel (2r + ty, 2c + tx).
#include <type_traits>

#include "conv_epilogue.h"

#ifndef C8_EXP
#define C8_EXP 0  // A/B timing experiments only (tools/build_variant.sh); 0 = the real kernel
#endif
// bits: 1 no output stores, 2 no MFMA, 4 no halo loads (zeros)
#define C8X(b) ((C8_EXP & (b)) != 0)
#ifndef C8_MINB
#define C8_MINB 2  // resident blocks per CU the register allocation is held to
#endif

namespace {

constexpr int PH = 16, PW = 16;

template <int KH, int KW, int S>
struct C8 {
    // stride S: the patch's input span is (16 S + K - S) pixels per axis
    static constexpr int TAPS = KH * KW, HWd = PW * S + KW - S, HPIX = (PH * S + KH - S) * HWd;
    static constexpr int KS = (TAPS * 8 + 31) / 32;  // 32-deep K-steps
    static constexpr int KP = KS * 32;
    // weight row stride: KP*2 + 16 bytes keeps the 16 rows of a fragment read on
    // distinct banks (row stride = 4 dwords mod 64 apart for KP*2 % 256 in {64, 192, 0})
    static constexpr int WS = KP * 2 + 16;
    static constexpr int HBYTES = HPIX * 16;
    static constexpr int HPT = (HPIX + 255) / 256;   // halo pixels per thread
    static constexpr int LDS = 64 * WS + 2 * HBYTES;
    // two resident blocks per CU (more spill: the 4x4 accumulator tile needs ~200 VGPRs)
    static_assert(2 * LDS <= 160 * 1024, "resident blocks per CU");
};

template <int KH, int KW, int S>
__global__ __launch_bounds__(256, C8_MINB) void conv_c8_kernel(const irgan_conv_desc d, const bf16_t* __restrict__ x,
                                                         const bf16_t* __restrict__ w, const float* __restrict__ bias,
                                                         void* __restrict__ y, int tpx, int tpy, int npatch) {
    using G = C8<KH, KW, S>;
    constexpr int TAPS = G::TAPS, HWd = G::HWd, HPIX = G::HPIX, KS = G::KS, KP = G::KP, WS = G::WS;
    __shared__ __attribute__((aligned(16))) char smem[G::LDS];
    char* const sW = smem;
    char* const sH = smem + 64 * WS;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, c16 = lane & 15;
    const bool reflect = d.pad_mode == IRGAN_PAD_REFLECT;
    const bool out_f32 = d.out_dtype == IRGAN_F32;

    // ---- weights: rows co < Cout, k < TAPS*8 from the packed [co][tap][8] rows (row
    // stride rounded up to the 64-element K-tile, include/irgan.h); zero elsewhere
    {
        constexpr int Kw = (TAPS * 8 + 63) / 64 * 64;
        for (int e = tid; e < 64 * (KP / 8); e += 256) {
            const int co = e / (KP / 8), k8 = e - co * (KP / 8);
            uint4 v = make_uint4(0u, 0u, 0u, 0u);
            if (co < d.Cout && k8 * 8 < TAPS * 8) v = *(const uint4*)(w + (long)co * Kw + k8 * 8);
            *(uint4*)(sW + co * WS + k8 * 16) = v;
        }
    }
    // per-lane halo offset (pixels) of tap 4s + g; taps past the end read pixel 0
    // (their weights are zero)
    int toff[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
        const int t = s * 4 + g;
        toff[s] = t < TAPS ? (t / KW) * HWd + t % KW : 0;
    }

    auto load_halo = [&](int p, uint4 (&hv)[G::HPT]) {
        const int pxi = p % tpx, r = p / tpx, pyi = r % tpy, img = r / tpy;
#pragma unroll
        for (int u = 0; u < G::HPT; ++u) {
            const int h = u * 256 + tid;
            hv[u] = make_uint4(0u, 0u, 0u, 0u);
            if (h < HPIX) {
                const int hy = h / HWd, hx = h - hy * HWd;
                int iy = pyi * PH * S + hy + d.c0y, ix = pxi * PW * S + hx + d.c0x;
                if (reflect) {
                    iy = reflect_idx(iy, d.H);
                    ix = reflect_idx(ix, d.W);
                }
                if ((unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W && !C8X(4))
                    hv[u] = *(const uint4*)(x + (((long)img * d.H + iy) * d.W + ix) * d.ldx + d.xoff);
            }
        }
    };
    auto store_halo = [&](int buf, const uint4 (&hv)[G::HPT]) {
#pragma unroll
        for (int u = 0; u < G::HPT; ++u) {
            const int h = u * 256 + tid;
            if (h < HPIX) *(uint4*)(sH + buf * G::HBYTES + h * 16) = hv[u];
        }
    };

    const bool vec = d.ldy % 4 == 0 && d.yoff % 4 == 0;
    float bv[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int co = j * 16 + 4 * g + r;
            bv[j][r] = (bias && co < d.Cout) ? bias[co] : 0.f;
        }

    uint4 hv[G::HPT];
    int p = blockIdx.x;
    if (p < npatch) {
        load_halo(p, hv);
        store_halo(0, hv);
    }
    __syncthreads();
#pragma unroll 1
    for (int it = 0; p < npatch; ++it, p += gridDim.x) {
        const int pn = p + gridDim.x;
        if (pn < npatch) load_halo(pn, hv);  // in flight under this patch's MFMAs
        const char* H = sH + (it & 1) * G::HBYTES;
        f32x4 acc[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            uint4 a[4], b[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) b[j] = *(const uint4*)(sW + (j * 16 + c16) * WS + s * 64 + g * 16);
#pragma unroll
            for (int i = 0; i < 4; ++i)
                a[i] = *(const uint4*)(H + ((wid * 4 + i) * S * HWd + c16 * S + toff[s]) * 16);
#pragma unroll
            for (int i = 0; i < 4 * !C8X(2); ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, b[j]),
                                                                        __builtin_bit_cast(bf16x8_t, a[i]),
                                                                        acc[i][j], 0, 0, 0);
        }
        // ---- epilogue: pixel (row wid*4+i, column c16), channels j*16 + 4g + r
        {
            const int pxi = p % tpx, r0 = p / tpx, pyi = r0 % tpy, img = r0 / tpy;
            const int ox = pxi * PW + c16;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int oy = pyi * PH + wid * 4 + i;
                if (oy >= d.Ho || ox >= d.Wo || C8X(1)) continue;
                const long pix = ((long)img * d.OH + oy * d.omy + d.ooy) * d.OW + ox * d.omx + d.oox;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int co = j * 16 + 4 * g;
                    if (co >= d.Cout) continue;
                    float v[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = conv_act(acc[i][j][r] + bv[j][r], d.act);
                    const bool full = co + 4 <= d.Cout;
                    if (out_f32) {
                        float* yp = (float*)y + pix * d.ldy + d.yoff + co;
                        if (full && vec) {
                            float4 o = make_float4(v[0], v[1], v[2], v[3]);
                            if (d.accumulate) {
                                const float4 q = *(const float4*)yp;
                                o.x += q.x; o.y += q.y; o.z += q.z; o.w += q.w;
                            }
                            *(float4*)yp = o;
                        } else {
                            for (int r = 0; r < 4 && co + r < d.Cout; ++r) yp[r] = d.accumulate ? yp[r] + v[r] : v[r];
                        }
                    } else {
                        bf16_t* yp = (bf16_t*)y + pix * d.ldy + d.yoff + co;
                        if (full && vec) {
                            if (d.accumulate) {
                                const uint2 q = *(const uint2*)yp;
                                v[0] += bf2f((bf16_t)(q.x & 0xffffu)); v[1] += bf2f((bf16_t)(q.x >> 16));
                                v[2] += bf2f((bf16_t)(q.y & 0xffffu)); v[3] += bf2f((bf16_t)(q.y >> 16));
                            }
                            uint2 o;
                            o.x = pk_bf16(v[0], v[1]);
                            o.y = pk_bf16(v[2], v[3]);
                            *(uint2*)yp = o;
                        } else {
                            for (int r = 0; r < 4 && co + r < d.Cout; ++r)
                                yp[r] = f2bf(d.accumulate ? bf2f(yp[r]) + v[r] : v[r]);
                        }
                    }
                }
            }
        }
        if (pn < npatch) store_halo((it + 1) & 1, hv);
        __syncthreads();
    }
}

template <int KH, int KW, int S>
void launch_c8(const irgan_conv_desc* d, const void* x, const void* w, const float* bias, void* y, hipStream_t st) {
    static int occ = 0;  // resident blocks per CU (a property of the kernel on gfx950)
    if (!occ && (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, conv_c8_kernel<KH, KW, S>, 256, 0) != hipSuccess || occ < 1))
        occ = 1;
    const int slots = occ * irgan_cu_count();
    const int tpx = irgan_cdiv(d->Wo, PW), tpy = irgan_cdiv(d->Ho, PH);
    const int npatch = d->N * tpx * tpy;
    const int grid = npatch < slots ? npatch : slots;
    conv_c8_kernel<KH, KW, S><<<grid, 256, 0, st>>>(*d, (const bf16_t*)x, (const bf16_t*)w, bias, y, tpx, tpy, npatch);
}


// ---- dense-K variant: the REAL input channels only (d.cin_real = CR of the 8): G inc
// (CR 1), VGG conv1_1 (3), D model.0 (4), G outc backward-data (dY of 3 channels).  The
// K axis is (tap, channel) over CR channels, padded to 32: inc 49 -> 64 instead of 392 ->
// 416, conv1_1 27 -> 32 instead of 96.  Per patch the block builds the im2col tile
// [256 pixels][64-deep K chunk] in LDS from the resident halo (one 8-byte halo read per
// tap per pixel), multiplies it with the dense weight rows, and stages the bf16 output
// tile [256][64] in the same LDS to store it as whole 128-byte pixel rows, 16 bytes per
// lane: the plain kernel's 8-byte stores straight from the accumulators (16 pixels x 32 B
// per instruction) held it at ~2 TB/s -- without them it ran 4-5x faster
// (profiles/r03_k_c8_ablation.txt).  One halo buffer (the halo is dead once the last K
// chunk's tile is built; the next one is staged through registers meanwhile).  No
// accumulate (the staged tile is rounded to bf16 before it could be added).
template <int KH, int KW, int S, int CR>
struct C8R {
    static constexpr int TAPS = KH * KW, HWd = PW * S + KW - S, HPIX = (PH * S + KH - S) * HWd;
    static constexpr int KR = TAPS * CR, KP = (KR + 31) / 32 * 32, NCH = (KP + 63) / 64;
    static constexpr int WS = KP * 2 + 16;           // weight row stride (bytes)
    static constexpr int TS = 144;                   // tile row stride: 64 K (or 64 co) bf16 + 16 B
    static constexpr int HPT = (HPIX + 255) / 256;
    static constexpr int HBYTES = HPT * 256 * 16;    // whole DMA pieces (the tail lanes land in the pad)
    static constexpr int LDS = 64 * WS + HBYTES + 256 * TS + 64 * 4;  // + the bias
    static_assert(2 * LDS <= 160 * 1024, "two resident blocks per CU");
};

// STATS (irgan_conv_fwd_stats, the G inc layer's reflect-pad 7x7 conv -> InstanceNorm, ir:458-463):
// each patch also writes its per-channel (sum, sum of squares) of the stored bf16 outputs, one
// float2 per (image, patch, channel) in finalize_kernel's layout (norm.hip) -- the separate
// statistics pass over the 134 MB output is gone.
template <int KH, int KW, int S, int CR, bool STATS = false>
__global__ __launch_bounds__(256, 2) void conv_c8r_kernel(const irgan_conv_desc d, const bf16_t* __restrict__ x,
                                                          const bf16_t* __restrict__ w,
                                                          const float* __restrict__ bias, bf16_t* __restrict__ y,
                                                          int tpx, int tpy, int npatch,
                                                          float2* __restrict__ part = nullptr) {
    using G = C8R<KH, KW, S, CR>;
    constexpr int TAPS = G::TAPS, HWd = G::HWd, HPIX = G::HPIX, KR = G::KR, KP = G::KP, WS = G::WS, TS = G::TS;
    __shared__ __attribute__((aligned(16))) char smem[G::LDS];
    char* const sW = smem;
    char* const sH = smem + 64 * WS;
    char* const sT = sH + G::HBYTES;
    float* const sBias = (float*)(sT + 256 * TS);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, c16 = lane & 15;
    const bool reflect = d.pad_mode == IRGAN_PAD_REFLECT;

    // dense weight rows: k = tap * CR + c <- packed [co][tap][8] element tap*8 + c
    {
        constexpr int Kw = (TAPS * 8 + 63) / 64 * 64;
        for (int e = tid; e < 64 * KP; e += 256) {
            const int co = e / KP, k = e - co * KP;
            bf16_t v = 0;
            if (co < d.Cout && k < KR) v = w[(long)co * Kw + (k / CR) * 8 + (k % CR)];
            *(bf16_t*)(sW + co * WS + k * 2) = v;
        }
    }
    // The halo goes HBM -> LDS by DMA (buffer_load ... lds, out-of-range pixels as zeros), the
    // output through unconditional raw buffer stores (out-of-range pixels dropped), so the loop
    // issues exactly HPT DMA pieces and 8 stores per patch and waits by count: the next patch's
    // halo lands while this patch's MFMAs, staging and stores run.  (Loaded through registers
    // with predicated loads / stores, the compiler waited vmcnt(0) at the top of each patch and
    // ahead of the epilogue, which serialised halo, compute and stores: inc forward 70 us for
    // 150 MB.)
    const i32x4 xrs = make_rsrc(x, (uint32_t)((long)d.N * d.H * d.W * d.ldx * 2));
    const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)y, (short)0, (int)((long)d.N * d.OH * d.OW * d.ldy * 2), 0x00020000);
    auto issue_halo = [&](int p) {
        const int pxi = p % tpx, r = p / tpx, pyi = r % tpy, img = r / tpy;
        const int wid64 = wid * 64;
#pragma unroll
        for (int u = 0; u < G::HPT; ++u) {
            const int h = u * 256 + tid;
            const int hy = h / HWd, hx = h - hy * HWd;
            int iy = pyi * PH * S + hy + d.c0y, ix = pxi * PW * S + hx + d.c0x;
            if (reflect) {
                iy = reflect_idx(iy, d.H);
                ix = reflect_idx(ix, d.W);
            }
            const bool ok = h < HPIX && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W;
            const uint32_t off = ok ? (uint32_t)((((long)img * d.H + iy) * d.W + ix) * d.ldx + d.xoff) * 2 : IRGAN_OOB;
            blds16(xrs, off, sH + (u * 256 + wid64) * 16);  // lane-linear: pixel h at sH + 16 h
        }
    };
    // im2col row of this thread's pixel (patch row pr, column pc) for K chunk kc: one 8-byte
    // halo read (channels 0-3) per tap the chunk touches, the bf16 halves moved by bit ops
    const int pr = tid >> 4, pcol = tid & 15;
    auto build = [&](auto kcc) {
        constexpr int kc = decltype(kcc)::value;
        constexpr int k0 = kc * 64, k1 = (k0 + 64 < KR ? k0 + 64 : KR);
        constexpr int t0 = k0 / CR, t1 = (k1 - 1) / CR;   // taps of this chunk
        uint2 tv[t1 - t0 + 1];
#pragma unroll
        for (int t = t0; t <= t1; ++t) {
            const int ty = t / KW, tx = t % KW;
            tv[t - t0] = *(const uint2*)(sH + ((pr * S + ty) * HWd + pcol * S + tx) * 16);
        }
        auto half = [&](int kk) -> uint32_t {   // bf16 bits of K index kk (0 past KR)
            if (kk >= KR) return 0u;
            const int t = kk / CR, c = kk % CR;
            const uint2 v = tv[t - t0];
            const uint32_t wd = c < 2 ? v.x : v.y;
            return (c & 1) ? (wd >> 16) : (wd & 0xffffu);
        };
#pragma unroll
        for (int k8 = 0; k8 < 8; ++k8) {
            if (k0 + k8 * 8 >= KP) break;
            uint32_t wds[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) wds[k] = half(k0 + k8 * 8 + 2 * k) | (half(k0 + k8 * 8 + 2 * k + 1) << 16);
            *(uint4*)(sT + tid * TS + k8 * 16) = make_uint4(wds[0], wds[1], wds[2], wds[3]);
        }
    };

    // bias through LDS (read in the epilogue by ds_read: no global load for the waits to track)
    if (tid < 64) sBias[tid] = (bias && tid < d.Cout) ? bias[tid] : 0.f;
    int p = blockIdx.x;
    if (p < npatch) issue_halo(p);
#pragma unroll 1
    for (int it = 0; p < npatch; p += gridDim.x, ++it) {
        // halo p landed: its DMA pieces are older than the 8 stores of patch p - 1
        if (it == 0) wait_vmcnt<0>();
        else wait_vmcnt<8>();
        __syncthreads();  // every wave's halo pieces (and the bias / weights) visible
        const int pn = p + gridDim.x;
        f32x4 acc[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        auto chunk = [&](auto kcc) {
            constexpr int kc = decltype(kcc)::value;
            if (kc) __syncthreads();  // the previous chunk's tile consumed
            build(kcc);
            __syncthreads();
            // the last chunk's tile is built: the halo buffer takes the next patch's DMA
            if (kc == G::NCH - 1 && pn < npatch) issue_halo(pn);
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                if (kc * 64 + s * 32 >= KP) break;
                uint4 a[4], b[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) b[j] = *(const uint4*)(sW + (j * 16 + c16) * WS + (kc * 64 + s * 32) * 2 + g * 16);
#pragma unroll
                for (int i = 0; i < 4; ++i) a[i] = *(const uint4*)(sT + ((wid * 4 + i) * 16 + c16) * TS + s * 64 + g * 16);
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, b[j]),
                                                                            __builtin_bit_cast(bf16x8_t, a[i]),
                                                                            acc[i][j], 0, 0, 0);
            }
        };
        chunk(std::integral_constant<int, 0>());
        if constexpr (G::NCH > 1) chunk(std::integral_constant<int, 1>());
        if constexpr (G::NCH > 2) chunk(std::integral_constant<int, 2>());
        static_assert(G::NCH <= 3, "K chunks");
        __syncthreads();  // every wave done with the tile: it becomes the output staging
        // pixel (row wid*4+i, column c16), channels j*16 + 4g + r -> staging row (4w+i)*16 + c16
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float v[4];
                const float4 bb = *(const float4*)(sBias + j * 16 + 4 * g);
                const float bj[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = conv_act(acc[i][j][r] + bj[r], d.act);
                uint2 o;
                o.x = pk_bf16(v[0], v[1]);
                o.y = pk_bf16(v[2], v[3]);
                *(uint2*)(sT + ((wid * 4 + i) * 16 + c16) * TS + (j * 16 + 4 * g) * 2) = o;
            }
        __syncthreads();
        // whole pixel rows: 8 lanes x 16 B per pixel, 8 pixels per wave instruction
        {
            const int pxi = p % tpx, r0 = p / tpx, pyi = r0 % tpy, img = r0 / tpy;
            float s1[8], s2[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) s1[k] = s2[k] = 0.f;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int e = u * 256 + tid, px = e >> 3, ch = e & 7;
                const int oy = pyi * PH + (px >> 4), ox = pxi * PW + (px & 15);
                const long pix = ((long)img * d.OH + oy * d.omy + d.ooy) * d.OW + ox * d.omx + d.oox;
                const bool in = oy < d.Ho && ox < d.Wo;
                const int off = in ? (int)((pix * d.ldy + d.yoff + ch * 8) * 2) : (int)IRGAN_OOB;
                const uint4 o = *(const uint4*)(sT + px * TS + ch * 16);
                __builtin_amdgcn_raw_buffer_store_b128(
                    __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, o), yr, off, 0, 0);
                if constexpr (STATS) {
                    if (in) {
                        const uint32_t wv[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            const float lo = __uint_as_float(wv[k] << 16), hi = __uint_as_float(wv[k] & 0xffff0000u);
                            s1[2 * k] += lo; s2[2 * k] += lo * lo;
                            s1[2 * k + 1] += hi; s2[2 * k + 1] += hi * hi;
                        }
                    }
                }
            }
            if constexpr (STATS) {
                // this thread's channels (tid & 7) * 8 .. +7 over its 8 pixels; the 32 threads of a
                // channel group add through LDS in a fixed order (the staging tile is free again)
                __syncthreads();
                float2* red = (float2*)sT;  // [32 pixel groups][64 channels]
                const int ch8 = (tid & 7) * 8, grp = tid >> 3;
#pragma unroll
                for (int k = 0; k < 8; ++k) red[grp * 64 + ch8 + k] = make_float2(s1[k], s2[k]);
                __syncthreads();
                if (tid < 64) {
                    float a = 0.f, b = 0.f;
                    for (int r = 0; r < 32; ++r) {
                        const float2 v = red[r * 64 + tid];
                        a += v.x;
                        b += v.y;
                    }
                    part[((long)img * (tpx * tpy) + pyi * tpx + pxi) * 64 + tid] = make_float2(a, b);
                }
            }
        }
    }
}

template <int KH, int KW, int S, int CR, bool STATS = false>
void launch_c8r(const irgan_conv_desc* d, const void* x, const void* w, const float* bias, void* y, hipStream_t st,
                float2* part = nullptr) {
    static int occ = 0;  // resident blocks per CU (a property of the kernel on gfx950)
    if (!occ && (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, conv_c8r_kernel<KH, KW, S, CR, STATS>, 256, 0) !=
                     hipSuccess || occ < 1))
        occ = 1;
    const int slots = occ * irgan_cu_count();
    const int tpx = irgan_cdiv(d->Wo, PW), tpy = irgan_cdiv(d->Ho, PH);
    const int npatch = d->N * tpx * tpy;
    const int grid = npatch < slots ? npatch : slots;
    conv_c8r_kernel<KH, KW, S, CR, STATS><<<grid, 256, 0, st>>>(*d, (const bf16_t*)x, (const bf16_t*)w, bias,
                                                               (bf16_t*)y, tpx, tpy, npatch, part);
}

// the dense-K launch for (KH, KW, S, cin_real); false: no instance (the caller runs conv_c8)
bool try_c8r(const irgan_conv_desc* d, const void* x, const void* w, const float* bias, void* y, hipStream_t st) {
    static const bool off = getenv("IRGAN_NO_C8R") != nullptr;
    // (accumulate: the staged bf16 tile would round before the add)
    if (off || d->cin_real <= 0 || d->cin_real >= 8 || d->Cout != 64 || d->out_dtype != IRGAN_BF16 || d->ldy % 8 ||
        d->yoff % 8 || d->accumulate)
        return false;
    const int cr = d->cin_real, k = d->KH, s = d->sy;
    if (k == 7 && s == 1 && cr == 1) launch_c8r<7, 7, 1, 1>(d, x, w, bias, y, st);
    else if (k == 7 && s == 1 && cr == 3) launch_c8r<7, 7, 1, 3>(d, x, w, bias, y, st);
    else if (k == 3 && s == 1 && cr == 3) launch_c8r<3, 3, 1, 3>(d, x, w, bias, y, st);
    else if (k == 4 && s == 2 && cr == 4) launch_c8r<4, 4, 2, 4>(d, x, w, bias, y, st);
    else return false;
    return true;
}

}  // namespace

// conv_pp.hip's irgan_conv_fwd_stats for the 8-channel-input convs: the G inc layer (7x7,
// stride 1, one real input channel, 64 outputs) with the InstanceNorm partials fused (STATS);
// returns the partials per image, 0 when this kernel does not take the layer (nothing ran)
int c8r_fwd_stats(const irgan_conv_desc* d, const void* x, const void* w, const float* bias, void* y, void* part,
                  hipStream_t st) {
    static const bool off = getenv("IRGAN_NO_C8R") != nullptr || getenv("IRGAN_NO_C8R_STATS") != nullptr;
    if (off || d->dtype != IRGAN_BF16 || d->Cin != 8 || d->ldx % 8 || d->xoff % 8 || d->cin_real != 1 ||
        d->KH != 7 || d->KW != 7 || d->sy != 1 || d->sx != 1 || d->Cout != 64 || d->out_dtype != IRGAN_BF16 ||
        d->ldy % 8 || d->yoff % 8 || d->accumulate || d->act != IRGAN_ACT_NONE || d->Ho != d->OH || d->Wo != d->OW ||
        d->omy != 1 || d->omx != 1 || d->ooy || d->oox)
        return 0;
    const int tpx = irgan_cdiv(d->Wo, PW), tpy = irgan_cdiv(d->Ho, PH);
    if (tpx * tpy > IRGAN_IN_PARTS || (long)d->N * d->Ho * d->Wo <= 0) return 0;
    launch_c8r<7, 7, 1, 1, true>(d, x, w, bias, y, st, (float2*)part);
    return tpx * tpy;
}

// Preconditions: bf16 input and weights, Cin == 8, ldx % 8 == 0, xoff % 8 == 0,
// sy = sx = 1 with (KH, KW) in {(7,7), (4,4), (3,3)} or sy = sx = 2 with 4x4 (D's first
// layer), Cout <= 64, no mask.
extern "C" int irgan_conv_fwd_c8(const irgan_conv_desc* d, const void* x, const void* w, const float* bias, void* y,
                                 const void* mask, hipStream_t st) {
    if ((long)d->N * d->Ho * d->Wo <= 0 || d->Cout <= 0) return 0;
    if (d->dtype != IRGAN_BF16 || d->Cin != 8 || d->ldx % 8 || d->xoff % 8 || d->sy != d->sx || d->Cout > 64 ||
        mask)
        return IRGAN_EUNSUPPORTED;
    if (d->KH == d->KW && try_c8r(d, x, w, bias, y, st)) {
        IRGAN_LAUNCH_CHECK();
        return 0;
    }
    if (d->sy == 2) {
        if (d->KH == 4 && d->KW == 4) launch_c8<4, 4, 2>(d, x, w, bias, y, st);
        else return IRGAN_EUNSUPPORTED;
    } else if (d->sy == 1) {
        if (d->KH == 7 && d->KW == 7) launch_c8<7, 7, 1>(d, x, w, bias, y, st);
        else if (d->KH == 4 && d->KW == 4) launch_c8<4, 4, 1>(d, x, w, bias, y, st);
        else if (d->KH == 3 && d->KW == 3) launch_c8<3, 3, 1>(d, x, w, bias, y, st);
        else return IRGAN_EUNSUPPORTED;
    } else {
        return IRGAN_EUNSUPPORTED;
    }
    IRGAN_LAUNCH_CHECK();
    return 0;
}
