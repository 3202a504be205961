// Launchers of conv_pp_kernel (conv_pp_kernel.h): bf16 stride-1 3x3 / 4x4 convolutions,
// the fused InstanceNorm-statistics epilogue, the fp8 ResnetBlock path.
#include "conv_pp_kernel.h"

// conv_res64.hip: the resident-weight persistent kernel for one input chunk (Cin == 64)
namespace irgan_res64 {
bool ok(const irgan_conv_desc* d);
int launch(const irgan_conv_desc* d, const void* x, const void* w, const float* bias, void* y, const void* mask,
           float2* part, hipStream_t st, void* ypool = nullptr);
}  // namespace irgan_res64

namespace {

// BN-64 tiles take the single-halo buffer (two blocks per CU), and Cout % 128 (not % 256)
// layers run as BN-64 single-halo tiles: two blocks per CU beat one BN-128 block on every
// such layer of the step (down1 / up1 / VGG conv2, profiles/r02_s5_pp_one_ab.txt)
constexpr bool use_one(int) { return true; }
constexpr bool split128(int) { return true; }

// Output-channel tile for a Cout % 256 == 0 layer: 256 unless that leaves most CUs idle
// (the PatchGAN 4x4 layers at 32x32: D model.8 backward-data at B = 16 is 64 BN-256 blocks
// for 256 CUs) -- then 128 or the 64-channel single-halo tile (two blocks per CU)
//
// Round 6: also when BN-256 blocks fill the CUs but end in a mostly empty last round -- the
// 128 x 160 ResnetBlock maps of 512 x 640 at B = 4 (config 4) are 320 BN-256 blocks, two
// rounds for 1.25 rounds of work.  Rounds are priced as measured at B = 16 / 32
// (a round of BN-128 blocks, or of two BN-64 blocks per CU, takes 0.575
// of a BN-256 round); BN-128 is taken when it is >= 10 % cheaper.  PP_BN_MODEL=0 builds the
// round-5 rule alone (A/B variants).
#ifndef PP_BN_MODEL
#define PP_BN_MODEL 1
#endif
int narrow_bn(const irgan_conv_desc* d) {
    const long patches = (long)d->N * irgan_cdiv(d->Ho, PH) * irgan_cdiv(d->Wo, PW);
    if (patches * (d->Cout / 256) >= 160) {
        if (PP_BN_MODEL) {
            const long cus = irgan_cu_count();
            const long r256 = irgan_cdiv(patches * (d->Cout / 256), cus);
            const long r128 = irgan_cdiv(patches * (d->Cout / 128), cus);
            if (r128 * 0.575 <= 0.9 * r256) return 128;
        }
        return 256;
    }
    return patches * (d->Cout / 128) >= 160 ? 128 : 64;
}

template <int KH, int KW, int BN, bool S2D = false>
void launch_pp(const irgan_conv_desc* d, const void* x, const void* w, const float* bias, void* y, const void* mask,
               hipStream_t st, int swz) {
    const int tpx = irgan_cdiv(d->Wo, PW), tpy = irgan_cdiv(d->Ho, PH);
    const int ntn = irgan_cdiv(d->Cout, BN);
    const int nb = d->N * tpy * tpx * ntn;
    if constexpr (BN == 64) {
        if (use_one(d->Cin)) {  // single halo buffer: two blocks per CU
            if (d->accumulate)
                conv_pp_kernel<KH, KW, BN, true, false, false, true, S2D><<<nb, 512, 0, st>>>(
                    *d, (const bf16_t*)x, (const bf16_t*)w, bias, y, mask, ntn, tpx, tpy, swz);
            else
                conv_pp_kernel<KH, KW, BN, false, false, false, true, S2D><<<nb, 512, 0, st>>>(
                    *d, (const bf16_t*)x, (const bf16_t*)w, bias, y, mask, ntn, tpx, tpy, swz);
            return;
        }
    }
    if (d->accumulate)
        conv_pp_kernel<KH, KW, BN, true, false, false, false, S2D><<<nb, 512, 0, st>>>(
            *d, (const bf16_t*)x, (const bf16_t*)w, bias, y, mask, ntn, tpx, tpy, swz);
    else
        conv_pp_kernel<KH, KW, BN, false, false, false, false, S2D><<<nb, 512, 0, st>>>(
            *d, (const bf16_t*)x, (const bf16_t*)w, bias, y, mask, ntn, tpx, tpy, swz);
}

}  // namespace

extern "C" int irgan_conv_fwd_pp(const irgan_conv_desc* d, const void* x, const void* w, const float* bias, void* y,
                                 const void* mask, hipStream_t st) {
    if ((long)d->N * d->Ho * d->Wo <= 0 || d->Cout <= 0) return 0;
    const bool k33 = d->KH == 3 && d->KW == 3, k44 = d->KH == 4 && d->KW == 4;
    const bool s2d = k44 && d->sy == 2 && d->sx == 2;  // 4x4 stride 2 as a space-to-depth 2x2 conv
    if (d->dtype != IRGAN_BF16 || d->act == IRGAN_ACT_TANH || ((d->sy != 1 || d->sx != 1) && !s2d) || d->Cin % 64 ||
        !(k33 || k44) || d->Cout % 64 || d->ldx % 8 || d->xoff % 8 || (long)d->N * d->H * d->W * d->ldx >= (1L << 30) ||
        (long)d->Cout * d->KH * d->KW * d->Cin >= (1L << 30))
        return IRGAN_EUNSUPPORTED;
    const int swz = irgan_xcd_swz();
    if (irgan_res64::ok(d) && (!mask || (d->ldm % 4 == 0 && d->moff % 4 == 0))) {  // one input chunk: resident weights
        irgan_res64::launch(d, x, w, bias, y, mask, nullptr, st);
        IRGAN_LAUNCH_CHECK();
        return 0;
    }
    const int nbn = d->Cout % 256 == 0 ? narrow_bn(d) : 0;
    if (s2d) {
        if (nbn == 256) launch_pp<2, 2, 256, true>(d, x, w, bias, y, mask, st, swz);
        else if (nbn == 128 || (nbn == 0 && d->Cout % 128 == 0 && !split128(d->Cin)))
            launch_pp<2, 2, 128, true>(d, x, w, bias, y, mask, st, swz);
        else launch_pp<2, 2, 64, true>(d, x, w, bias, y, mask, st, swz);
    } else if (nbn == 256) {
        if (k33) launch_pp<3, 3, 256>(d, x, w, bias, y, mask, st, swz);
        else launch_pp<4, 4, 256>(d, x, w, bias, y, mask, st, swz);
    } else if (nbn == 128 || (nbn == 0 && d->Cout % 128 == 0 && !split128(d->Cin))) {
        if (k33) launch_pp<3, 3, 128>(d, x, w, bias, y, mask, st, swz);
        else launch_pp<4, 4, 128>(d, x, w, bias, y, mask, st, swz);
    } else {  // BN-64 single-halo tiles (up2_conv's Cout-192 backward-data: three of them, 350 -> 323 us)
        if (k33) launch_pp<3, 3, 64>(d, x, w, bias, y, mask, st, swz);
        else launch_pp<4, 4, 64>(d, x, w, bias, y, mask, st, swz);
    }
    IRGAN_LAUNCH_CHECK();
    return 0;
}

// conv_ring.hip: the line-form reflect ring's shape check and its GEMM launch
bool ring_line_check(const irgan_conv_desc* d, int p, long ws_floats);
void ring_line_gemm_launch(const irgan_conv_desc* d, const void* dy, const void* w, float* ws, hipStream_t st);

// Reflect-padded ResnetBlock backward-data (ir:386-411) as the ring's line GEMM into ws, then
// the interior conv_pp launch whose store pass adds the ring terms onto dx's rows 1 / H-2 and
// columns 1 / W-2 (ring_line_add): the fold launch of irgan_reflect_dgrad_ring_ws and its
// read-modify-write of dx's border band are gone, dx is bit-identical.
extern "C" int irgan_conv_dgrad_reflect_line(const irgan_conv_desc* d, const void* dy, const void* w, int32_t p,
                                             void* dx, float* ws, int64_t ws_floats, irgan_stream_t s) {
    if (!d || !dy || !w || !dx || !ws) return IRGAN_EINVAL;
    if ((long)d->N * d->Ho * d->Wo <= 0 || d->Cout <= 0) return 0;
    if (!ring_line_check(d, p, ws_floats) || d->out_dtype != IRGAN_BF16 || d->act != IRGAN_ACT_NONE ||
        d->sy != 1 || d->sx != 1 || d->Cin % 64 || d->Cout % 256 || narrow_bn(d) != 256 || irgan_res64::ok(d) ||
        (long)d->N * d->H * d->W * d->ldx >= (1L << 30) || (long)d->Cout * 9 * d->Cin >= (1L << 30))
        return IRGAN_EUNSUPPORTED;
    hipStream_t st = (hipStream_t)s;
    ring_line_gemm_launch(d, dy, w, ws, st);
    const int swz = irgan_xcd_swz();
    const int tpx = irgan_cdiv(d->Wo, PW), tpy = irgan_cdiv(d->Ho, PH), ntn = d->Cout / 256;
    const int nb = d->N * tpy * tpx * ntn;
    if (d->accumulate)
        conv_pp_kernel<3, 3, 256, true><<<nb, 512, 0, st>>>(*d, (const bf16_t*)dy, (const bf16_t*)w, nullptr, dx,
                                                            nullptr, ntn, tpx, tpy, swz, nullptr, nullptr, nullptr, ws);
    else
        conv_pp_kernel<3, 3, 256, false><<<nb, 512, 0, st>>>(*d, (const bf16_t*)dy, (const bf16_t*)w, nullptr, dx,
                                                             nullptr, ntn, tpx, tpy, swz, nullptr, nullptr, nullptr, ws);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

// The fp8 path's ResnetBlock backward-data (config 5): the ring's line GEMM on the bf16 dY and
// bf16 flipped weights (d, dy, w: as irgan_conv_dgrad_reflect_line), then the interior on the
// e4m3 operands (d8: d with dtype FP8 and dy8's ld / offset; dqy, dqw: their dequantisation
// factors) whose store pass folds the ring in -- the interior launch + ring launch + fold of
// before in one pass over dx, with the same terms and roundings.
extern "C" int irgan_conv_dgrad_reflect_line_fp8(const irgan_conv_desc* d, const void* dy, const void* w,
                                                 const irgan_conv_desc* d8, const void* dy8, const void* w8,
                                                 const float* dqy, const float* dqw, int32_t p, void* dx, float* ws,
                                                 int64_t ws_floats, irgan_stream_t s) {
    if (!d || !dy || !w || !d8 || !dy8 || !w8 || !dqy || !dqw || !dx || !ws) return IRGAN_EINVAL;
    if ((long)d->N * d->Ho * d->Wo <= 0 || d->Cout <= 0) return 0;
    if (!ring_line_check(d, p, ws_floats) || d->dtype != IRGAN_BF16 || d->out_dtype != IRGAN_BF16 ||
        d->act != IRGAN_ACT_NONE || d->sy != 1 || d->sx != 1 || d->Cin % 128 || d->Cout % 256 || d->mask_act ||
        d8->dtype != IRGAN_FP8 || d8->out_dtype != IRGAN_BF16 || d8->ldx % 16 || d8->xoff % 16 || d8->N != d->N ||
        d8->H != d->H || d8->W != d->W || d8->Cin != d->Cin || d8->Cout != d->Cout || d8->Ho != d->Ho ||
        d8->Wo != d->Wo || d8->ldy != d->ldy || d8->yoff != d->yoff || d8->c0y != d->c0y || d8->c0x != d->c0x ||
        d8->accumulate != d->accumulate || d8->KH != 3 || d8->KW != 3 || d8->act != IRGAN_ACT_NONE ||
        (long)d->N * d->H * d->W * d8->ldx >= (1L << 30) || (long)d->Cout * 9 * d->Cin >= (1L << 30))
        return IRGAN_EUNSUPPORTED;
    hipStream_t st = (hipStream_t)s;
    ring_line_gemm_launch(d, dy, w, ws, st);
    const int swz = irgan_xcd_swz();
    const int tpx = irgan_cdiv(d->Wo, PW), tpy = irgan_cdiv(d->Ho, PH), ntn = d->Cout / 256;
    const int nb = d->N * tpy * tpx * ntn;
    if (d->accumulate)
        conv_pp_kernel<3, 3, 256, true, false, true><<<nb, 512, 0, st>>>(
            *d8, (const bf16_t*)dy8, (const bf16_t*)w8, nullptr, dx, nullptr, ntn, tpx, tpy, swz, nullptr, dqy, dqw, ws);
    else
        conv_pp_kernel<3, 3, 256, false, false, true><<<nb, 512, 0, st>>>(
            *d8, (const bf16_t*)dy8, (const bf16_t*)w8, nullptr, dx, nullptr, ntn, tpx, tpy, swz, nullptr, dqy, dqw, ws);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

// The four-phase backward-data of a 4x4 stride-2 layer (irgan_conv_dgrad_s2's descriptors and
// phase images) as ONE conv_pp launch of 2x2 stride-1 phase convs (PH4): dx channels % 64, dY
// channels % 64, every phase the same Ho x Wo (even dx sides).  IRGAN_EUNSUPPORTED otherwise
// (the caller then runs dgrad_s2_kernel).
extern "C" int irgan_conv_dgrad_s2_pp(const irgan_conv_desc* dd, const void* dy, const void* const* w, void* dx,
                                      const void* mask, hipStream_t st) {
    const irgan_conv_desc& a = dd[0];
    if (a.Cout % 64 || a.Cin % 64 || a.OH % 2 || a.OW % 2 || a.ldy % 8 || a.yoff % 8 ||
        (mask && (a.ldm % 4 || a.moff % 4)) || (long)a.N * a.H * a.W * a.ldx >= (1L << 30) ||
        (long)a.Cout * 4 * a.Cin >= (1L << 30))
        return IRGAN_EUNSUPPORTED;
    PhaseTab tab;
    for (int k = 0; k < 4; ++k) {
        const irgan_conv_desc& e = dd[k];
        if (e.Ho != a.OH / 2 || e.Wo != a.OW / 2) return IRGAN_EUNSUPPORTED;
        const int p = e.ooy * 2 + e.oox;
        tab.w[p] = (const bf16_t*)w[k];
        tab.c0y[p] = e.c0y;
        tab.c0x[p] = e.c0x;
        tab.ooy[p] = e.ooy;
        tab.oox[p] = e.oox;
    }
    irgan_conv_desc d = a;  // the per-phase fields come from tab
    d.Ho = a.OH / 2;
    d.Wo = a.OW / 2;
    const int swz = irgan_xcd_swz();
    const int tpx = irgan_cdiv(d.Wo, PW), tpy = irgan_cdiv(d.Ho, PH);
    const int bn = d.Cout % 256 == 0 ? narrow_bn(&d) : 64;
    const int ntn = d.Cout / bn;
    const int nb = d.N * tpy * tpx * 4 * ntn;
#define PH4L(BNV, ACCV, ONEV)                                                                                     \
    conv_pp_kernel<2, 2, BNV, ACCV, false, false, ONEV, false, true><<<nb, 512, 0, st>>>(                           \
        d, (const bf16_t*)dy, (const bf16_t*)w[0], nullptr, dx, mask, ntn, tpx, tpy, swz, nullptr, nullptr, nullptr, \
        nullptr, tab)
    if (bn == 256) { if (d.accumulate) PH4L(256, true, false); else PH4L(256, false, false); }
    else if (bn == 128) { if (d.accumulate) PH4L(128, true, false); else PH4L(128, false, false); }
    else { if (d.accumulate) PH4L(64, true, true); else PH4L(64, false, true); }
#undef PH4L
    IRGAN_LAUNCH_CHECK();
    return 0;
}

// Forward conv with the InstanceNorm statistics of its output fused into the
// epilogue (replaces the separate irgan_in_stats pass over y; ir:154-165, 392, 417).
// part: float2[N * nb * Cout] partials, nb (out) = 16x16 patches per image; reduce
// them with irgan_in_finalize.  IRGAN_EUNSUPPORTED when the layer is not a plain
// bf16 ping-pong conv with Cout % 64 == 0, Cout != 192 (the caller then runs conv +
// in_stats).
// conv_c8.hip: the 8-channel-input (G inc) conv with fused statistics; 0 = not taken
int c8r_fwd_stats(const irgan_conv_desc* d, const void* x, const void* w, const float* bias, void* y, void* part,
                  hipStream_t st);

extern "C" int irgan_conv_fwd_stats(const irgan_conv_desc* d, const void* x, const void* w, const float* bias, void* y,
                                    void* part, int32_t* nb, irgan_stream_t s) {
    if (!d || !x || !w || !y || !part || !nb) return IRGAN_EINVAL;
    if (d->Cin == 8) {
        const int n = c8r_fwd_stats(d, x, w, bias, y, part, (hipStream_t)s);
        if (!n) return IRGAN_EUNSUPPORTED;
        IRGAN_LAUNCH_CHECK();
        *nb = n;
        return 0;
    }
    const bool k33 = d->KH == 3 && d->KW == 3, k44 = d->KH == 4 && d->KW == 4;
    const bool s2d = k44 && d->sy == 2 && d->sx == 2;  // as irgan_conv_fwd_pp
    if (d->dtype != IRGAN_BF16 || d->out_dtype != IRGAN_BF16 || d->accumulate || d->act != IRGAN_ACT_NONE ||
        ((d->sy != 1 || d->sx != 1) && !s2d) || d->Cin % 64 || !(k33 || k44) || d->Cout % 64 || d->Cout == 192 || d->ldx % 8 ||
        d->xoff % 8 ||
        d->ldy % 8 || d->yoff % 8 || d->Ho != d->OH || d->Wo != d->OW || d->omy != 1 || d->omx != 1 || d->ooy ||
        d->oox || (long)d->N * d->H * d->W * d->ldx >= (1L << 30) ||
        (long)d->Cout * d->KH * d->KW * d->Cin >= (1L << 30))
        return IRGAN_EUNSUPPORTED;
    const int tpx = irgan_cdiv(d->Wo, PW), tpy = irgan_cdiv(d->Ho, PH);
    if (tpx * tpy > IRGAN_IN_PARTS) return IRGAN_EUNSUPPORTED;
    if ((long)d->N * d->Ho * d->Wo <= 0) return IRGAN_EUNSUPPORTED;
    const int swz = irgan_xcd_swz();
    const int bn = d->Cout % 256 == 0 ? narrow_bn(d)
                                      : (d->Cout % 128 == 0 && !split128(d->Cin) ? 128 : 64);  // as irgan_conv_fwd_pp
    const int ntn = d->Cout / bn;
    const int blocks = d->N * tpy * tpx * ntn;
    hipStream_t st = (hipStream_t)s;
    if (irgan_res64::ok(d)) {
        *nb = irgan_res64::launch(d, x, w, bias, y, nullptr, (float2*)part, st);
        IRGAN_LAUNCH_CHECK();
        return 0;
    }
#define PPS(KHV, BNV, ONEV, ...)                                                                                   \
    conv_pp_kernel<KHV, KHV, BNV, false, true, false, ONEV, ##__VA_ARGS__><<<blocks, 512, 0, st>>>(                  \
        *d, (const bf16_t*)x, (const bf16_t*)w, bias, y, nullptr, ntn, tpx, tpy, swz, (float2*)part)
    const bool one = bn == 64 && use_one(d->Cin);
    if (s2d) {
        if (bn == 256) PPS(2, 256, false, true);
        else if (bn == 128) PPS(2, 128, false, true);
        else PPS(2, 64, true, true);
    } else if (k33) {
        if (bn == 256) PPS(3, 256, false);
        else if (bn == 128) PPS(3, 128, false);
        else { if (one) PPS(3, 64, true); else PPS(3, 64, false); }
    } else {
        if (bn == 256) PPS(4, 256, false);
        else if (bn == 128) PPS(4, 128, false);
        else { if (one) PPS(4, 64, true); else PPS(4, 64, false); }
    }
#undef PPS
    IRGAN_LAUNCH_CHECK();
    *nb = tpx * tpy;
    return 0;
}

// Forward conv + activation + 2x2 max-pool in one launch (the VGG features[:16] conv1_2 ->
// MaxPool2d(2), ir:664): y (may be NULL: the pooled map alone) gets the activated map, yp the
// pooled one, dense [N][Ho / 2][Wo / 2][Cout] bf16 -- the bits of irgan_conv_fwd +
// irgan_maxpool_fwd.  IRGAN_EUNSUPPORTED unless the layer takes the resident-weight kernel
// (one 64-channel input chunk, 3x3 stride 1) with even Ho, Wo and a plain output.
extern "C" int irgan_conv_fwd_pool(const irgan_conv_desc* d, const void* x, const void* w, const float* bias, void* y,
                                   void* yp, irgan_stream_t s) {
    if (!d || !x || !w || !yp) return IRGAN_EINVAL;
    if ((long)d->N * d->Ho * d->Wo <= 0) return 0;
    if (!irgan_res64::ok(d) || d->accumulate || d->mask_act || d->Ho % 2 || d->Wo % 2 || d->Ho != d->OH ||
        d->Wo != d->OW || d->omy != 1 || d->omx != 1 || d->ooy || d->oox ||
        (long)d->N * (d->Ho / 2) * (d->Wo / 2) * d->Cout * 2 >= (1L << 31))
        return IRGAN_EUNSUPPORTED;
    irgan_res64::launch(d, x, w, bias, y, nullptr, nullptr, (hipStream_t)s, yp);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

// fp8 e4m3 operands (x: NHWC, w: the packed [Cout][taps][Cin] image, both OCP
// e4m3 with per-tensor scales): y = act(conv(x, w) * dqx[0] * dqw[0] + bias), bf16
// out, and with part != NULL the InstanceNorm partials of y as irgan_conv_fwd_stats.
extern "C" int irgan_conv_fwd_fp8(const irgan_conv_desc* d, const void* x, const void* w, const float* dqx,
                                  const float* dqw, const float* bias, void* y, void* part, int32_t* nb,
                                  irgan_stream_t s) {
    if (!d || !x || !w || !dqx || !dqw || !y || (part && !nb)) return IRGAN_EINVAL;
    if ((long)d->N * d->Ho * d->Wo <= 0 || d->Cout <= 0) return 0;
    const bool k33 = d->KH == 3 && d->KW == 3;
    if (d->dtype != IRGAN_FP8 || d->out_dtype != IRGAN_BF16 || d->act == IRGAN_ACT_TANH || d->sy != 1 || d->sx != 1 ||
        d->Cin % 128 || !k33 || d->Cout % 64 || d->Cout == 192 || d->ldx % 16 || d->xoff % 16 || d->mask_act ||
        (long)d->N * d->H * d->W * d->ldx >= (1L << 30) || (long)d->Cout * 9 * d->Cin >= (1L << 30))
        return IRGAN_EUNSUPPORTED;
    if (part && (d->accumulate || d->act != IRGAN_ACT_NONE || d->ldy % 8 || d->yoff % 8 || d->Ho != d->OH ||
                 d->Wo != d->OW || d->omy != 1 || d->omx != 1 || d->ooy || d->oox))
        return IRGAN_EUNSUPPORTED;
    const int tpx = irgan_cdiv(d->Wo, PW), tpy = irgan_cdiv(d->Ho, PH);
    if (part && tpx * tpy > IRGAN_IN_PARTS) return IRGAN_EUNSUPPORTED;
    const int swz = irgan_xcd_swz();
    const int bn = d->Cout % 256 == 0 ? 256 : (d->Cout % 128 == 0 ? 128 : 64);
    const int ntn = d->Cout / bn;
    const int blocks = d->N * tpy * tpx * ntn;
    hipStream_t st = (hipStream_t)s;
#define PP8(BNV, ACCV, STV)                                                                                        \
    conv_pp_kernel<3, 3, BNV, ACCV, STV, true><<<blocks, 512, 0, st>>>(*d, (const bf16_t*)x, (const bf16_t*)w, bias, \
                                                                       y, nullptr, ntn, tpx, tpy, swz, (float2*)part, dqx, dqw)
    if (part) {
        if (bn == 256) PP8(256, false, true); else if (bn == 128) PP8(128, false, true); else PP8(64, false, true);
        *nb = tpx * tpy;
    } else if (d->accumulate) {
        if (bn == 256) PP8(256, true, false); else if (bn == 128) PP8(128, true, false); else PP8(64, true, false);
    } else {
        if (bn == 256) PP8(256, false, false); else if (bn == 128) PP8(128, false, false); else PP8(64, false, false);
    }
#undef PP8
    IRGAN_LAUNCH_CHECK();
    return 0;
}
