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

}  // namespace

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
