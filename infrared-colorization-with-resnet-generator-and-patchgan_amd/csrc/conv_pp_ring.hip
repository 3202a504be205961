// Reflect-padded ResnetBlock backward-data in ONE launch (ir:381-392, 401-411): the
// interior correlation AND the fold of the reflect-pad ring, conv_pp_kernel<..., RING>
// (conv_pp_kernel.h).  Replaces the interior launch + reflect_ring_kernel pair
// (conv_ring.hip) on the shapes it takes: the ring rows ride as one extra fragment in
// the top / bottom patches' K loop (added straight into the mirrored row's
// accumulators), the ring columns are a 17-row GEMM in the left / right patches'
// epilogue; every dx pixel is rounded to bf16 once.
#include "conv_pp_kernel.h"

namespace {

template <bool ACC, bool STATS>
void launch_ring(const irgan_conv_desc* d, const void* dy, const void* w, void* dx, hipStream_t st, int swz,
                 float2* part, const InBwdStats& ib) {
    const int tpx = d->Wo / PW, tpy = d->Ho / PH;
    const int blocks = d->N * tpy * tpx * (d->Cout / 256);
    conv_pp_kernel<3, 3, 256, ACC, STATS, false, false, true><<<blocks, 512, 0, st>>>(
        *d, (const bf16_t*)dy, (const bf16_t*)w, nullptr, dx, nullptr, d->Cout / 256, tpx, tpy, swz, part, nullptr,
        nullptr, ib);
}

}  // namespace

// Opt-in (irgan_set_ring_fold / IRGAN_RING_FOLD=1): on the bench step the fold measured no
// faster than interior + ring (the border patches' extra K-loop rows and epilogue GEMM
// lengthen the one-block-per-CU launch by about what the separate ring launch costs).
// Shapes the one-launch fold takes (else the caller runs interior + ring): bf16, 3x3, stride
// 1, p = 1, dY / dx channels % 64 / 256, an output the size of the input whose sides are
// multiples of 16 with >= 2 patches each (a mirrored row / column then lies in its own
// patch), plain (unstrided) output grid, no mask / activation / bias.
static int g_ring_fold = -1;  // -1: not yet read from IRGAN_RING_FOLD

extern "C" int irgan_set_ring_fold(int32_t on) {
    const int old = g_ring_fold < 0 ? (getenv("IRGAN_RING_FOLD") != nullptr) : g_ring_fold;
    g_ring_fold = on ? 1 : 0;
    return old;
}

bool irgan_ring_fold_ok(const irgan_conv_desc* d, int p) {
    if (g_ring_fold < 0) g_ring_fold = getenv("IRGAN_RING_FOLD") != nullptr;
    return g_ring_fold && p == 1 && d->dtype == IRGAN_BF16 && d->KH == 3 && d->KW == 3 && d->sy == 1 && d->sx == 1 &&
           d->Cin % 64 == 0 && d->Cout % 256 == 0 && d->ldx % 8 == 0 && d->xoff % 8 == 0 && d->Ho == d->H &&
           d->Wo == d->W && d->H % 16 == 0 && d->W % 16 == 0 && d->H >= 32 && d->W >= 32 && d->Ho == d->OH &&
           d->Wo == d->OW && d->omy == 1 && d->omx == 1 && d->ooy == 0 && d->oox == 0 &&
           d->act == IRGAN_ACT_NONE && d->mask_act == 0 && d->pad_mode == IRGAN_PAD_ZERO &&
           (d->out_dtype == IRGAN_BF16 || d->out_dtype == IRGAN_F32) &&
           (long)d->N * d->H * d->W * d->ldx < (1L << 30) && (long)d->Cout * 9 * d->Cin < (1L << 30);
}

// irgan_conv_dgrad_in_stats's fused path: the same launch with the IN-backward partials
int irgan_ring_fold_in_stats(const irgan_conv_desc* d, const void* dy, const void* w, void* dx, const void* z,
                             int ldz, int zoff, int act, int pstride, const float* mr, void* part, hipStream_t st) {
    const InBwdStats ib{(const bf16_t*)z, ldz, zoff, act, pstride, mr};
    static const int swz = getenv("IRGAN_NO_XCD_SWZ") ? 0 : 1;
    if (d->accumulate) launch_ring<true, true>(d, dy, w, dx, st, swz, (float2*)part, ib);
    else launch_ring<false, true>(d, dy, w, dx, st, swz, (float2*)part, ib);
    IRGAN_LAUNCH_CHECK();
    return 0;
}

extern "C" int irgan_conv_dgrad_reflect(const irgan_conv_desc* d, const void* dy, const void* w, int32_t p, void* dx,
                                        irgan_stream_t s) {
    if (!d || !dy || !w || !dx) return IRGAN_EINVAL;
    if ((long)d->N * d->Ho * d->Wo <= 0 || d->Cout <= 0) return 0;
    hipStream_t st = (hipStream_t)s;
    if (irgan_ring_fold_ok(d, p)) {
        static const int swz = getenv("IRGAN_NO_XCD_SWZ") ? 0 : 1;
        if (d->accumulate) launch_ring<true, false>(d, dy, w, dx, st, swz, nullptr, InBwdStats{});
        else launch_ring<false, false>(d, dy, w, dx, st, swz, nullptr, InBwdStats{});
        IRGAN_LAUNCH_CHECK();
        return 0;
    }
    // interior, then the ring launch (conv_ring.hip)
    int rc = irgan_conv_fwd(d, dy, w, nullptr, dx, nullptr, s);
    if (rc) return rc;
    return p > 0 ? irgan_reflect_dgrad_ring(d, dy, w, p, dx, s) : 0;
}
