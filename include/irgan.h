/*
 * irgan.h -- C ABI of the MI355X (gfx950) kernels for the IR->RGB GAN train step.
 *
 * The reference (/root/reference/Code/ir_colorization.py, cited ir:LINE) has no
 * FFI: its hot path (the train-step body ir:1636-1681) dispatches PyTorch ATen
 * ops.  Each entry point below replaces the ATen work of one reference layer
 * type; the Python host package (ir_colorization.py in the *_amd package)
 * binds them with ctypes exactly as INTEGRATION.md shows.
 *
 * Conventions
 *  - Activations are NHWC.  A tensor "slice" is (pointer, ld, off): pixel p,
 *    channel c lives at ptr[p*ld + off + c], so torch.cat along channels
 *    (ir:557, 564, 1639-1640) is free: producers write into channel slices.
 *  - Conv weights are K-major "KRSC": w[cout][ky][kx][cin].
 *  - dtype codes: IRGAN_F32 (exact-fp32 parity mode, f32 MFMA) or IRGAN_BF16
 *    (bf16 MFMA, fp32 accumulate).  Bias / statistics / losses are fp32.
 *  - All calls are asynchronous on the given HIP stream (hipStream_t passed as
 *    void*), allocate nothing, and return 0 or a hipError_t / IRGAN_E* code.
 *    The caller owns every buffer (PyTorch caching allocator on the host side).
 */
#ifndef IRGAN_H
#define IRGAN_H
#include <stdint.h>
#include <stddef.h>

/* Every entry point below is exported from libirgan.so; everything else in the library is
 * hidden (built with -fvisibility=hidden). */
#if defined(__GNUC__) || defined(__clang__)
#define IRGAN_API __attribute__((visibility("default")))
#else
#define IRGAN_API
#endif

#ifdef __cplusplus
extern "C" {
#endif

typedef void* irgan_stream_t;

/* The source id this library was built from: a hash of the csrc .hip / .h sources and this header
 * (computed by pkg/_build.py, baked in at compile time), NUL-terminated into buf[len].
 * pkg/_lib.py refuses a library whose id differs from the tree it is loaded from.  No
 * reference counterpart (build provenance of the drop-in library). */
IRGAN_API int irgan_build_id(char* buf, int32_t len);

enum { IRGAN_F32 = 0, IRGAN_BF16 = 1, IRGAN_FP8 = 2 };  /* FP8: OCP e4m3 (e4m3fn) */
enum { IRGAN_PAD_ZERO = 0, IRGAN_PAD_REFLECT = 1 };
/* forward activations (epilogues / IN apply) */
enum { IRGAN_ACT_NONE = 0, IRGAN_ACT_RELU = 1, IRGAN_ACT_LRELU = 2, IRGAN_ACT_TANH = 3 };
enum { IRGAN_OK = 0, IRGAN_EINVAL = 1001, IRGAN_EUNSUPPORTED = 1002 };

/* Implicit-GEMM convolution descriptor.  Launch domain: N x Ho x Wo output
 * positions (i, j); the input coordinate of tap (ty, tx) is
 * (i*sy + ty + c0y, j*sx + tx + c0x), zero- or reflect-mapped into H x W; the
 * result lands at output pixel (i*omy + ooy, j*omx + oox) of an N x OH x OW
 * tensor.  A forward conv with stride s and padding p is sy=s, c0y=-p,
 * omy=1, ooy=0.  Backward-data and ConvTranspose2d use the same descriptor on
 * re-packed weights (irgan_weight_pack) and, for stride 2, one launch per
 * output phase (omy=2, ooy=phase). */
typedef struct irgan_conv_desc {
    int32_t N, H, W, Cin, ldx, xoff;      /* input slice */
    int32_t Ho, Wo, Cout, ldy, yoff;      /* launch domain + output slice */
    int32_t OH, OW, omy, ooy, omx, oox;   /* output tensor + pixel mapping */
    int32_t KH, KW, sy, sx, c0y, c0x;     /* taps / input mapping */
    int32_t pad_mode;                     /* IRGAN_PAD_* */
    int32_t act;                          /* IRGAN_ACT_* applied in the epilogue */
    int32_t accumulate;                   /* 1: y += result (fp32 output only) */
    int32_t dtype;                        /* input/weight dtype IRGAN_F32|IRGAN_BF16|IRGAN_FP8 */
    int32_t out_dtype;                    /* output dtype */
    int32_t mask_act;                     /* backward mask: 0 none, 1 relu, 2 lrelu(0.2) */
    int32_t ldm, moff;                    /* mask slice (same pixel grid as output) */
    int32_t cin_real;                     /* nonzero input channels of a zero-padded input (0: Cin) */
    int32_t flags;                        /* IRGAN_CONV_* bits */
} irgan_conv_desc;
/* flags: IRGAN_CONV_DETERMINISTIC -- a split-K weight gradient (irgan_conv_wgrad_ws) reduces
 * its partials through the caller's workspace in a fixed order and never through fp32
 * atomics: it lowers its split count to what the workspace holds (fp32 parity mode: one
 * split, so each output element takes a single atomic add) (torch's
 * use_deterministic_algorithms analogue; bit-identical gradients run to run and under any
 * stream schedule).  Without it the atomics are kept where they are faster (high split
 * counts: up2 / down1-class layers at 256^2). */
enum { IRGAN_CONV_DETERMINISTIC = 1 };

/* y = act(conv(x, w) + bias) [* mask'(m)]   -- replaces nn.Conv2d forward
 * (ir:460, 470, 478, 390, 411, 504, 521, 529, 600-629, vgg 664) and, on
 * re-packed weights, conv backward-data and nn.ConvTranspose2d (ir:496, 513). */
IRGAN_API int irgan_conv_fwd(const irgan_conv_desc* d, const void* x, const void* w,
                   const float* bias, void* y, const void* mask, irgan_stream_t s);

/* irgan_conv_fwd (bf16, stride 1, 3x3 / 4x4, no activation) that
 * also writes the InstanceNorm statistics of its output -- the conv -> IN pairs of
 * ResnetBlock and the encoder / D (ir:386-392, 405-411, 468-470, 606-624) -- as
 * float2 (sum, sum of squares) partials part[n][b][c], b < *nb (16x16 patches per
 * image, <= IRGAN_IN_PARTS; Cout % 64 == 0 except 192); irgan_in_finalize turns them
 * into {mean, rstd}.  Also the G inc layer (ir:458-463): 7x7 stride 1, Cin = 8 with
 * cin_real = 1 (the zero-padded IR channel), Cout = 64.
 * Returns IRGAN_EUNSUPPORTED (nothing launched) for other layers. */
IRGAN_API int irgan_conv_fwd_stats(const irgan_conv_desc* d, const void* x, const void* w,
                         const float* bias, void* y, void* part, int32_t* nb, irgan_stream_t s);

/* irgan_conv_fwd_stats / irgan_conv_fwd on fp8 operands (BASELINE config 5): x and
 * w OCP e4m3 (d->dtype = IRGAN_FP8; x NHWC with ldx, xoff % 16 == 0, w the packed
 * [Cout][3][3][Cin] image), 3x3, stride 1, Cin % 128 == 0, Cout % 64 == 0 (not
 * 192), bf16 output y = act(conv * dqx[0] * dqw[0] + bias) -- the dequantisation
 * multipliers of the per-tensor scales, read on the device.  part != NULL: also the
 * InstanceNorm partials of y (as irgan_conv_fwd_stats; act none, no accumulate).
 * Replaces the ResnetBlock convs (ir:386-411) forward and backward-data in the fp8
 * path.  IRGAN_EUNSUPPORTED (nothing launched) for other layers. */
IRGAN_API int irgan_conv_fwd_fp8(const irgan_conv_desc* d, const void* x, const void* w, const float* dqx,
                       const float* dqw, const float* bias, void* y, void* part, int32_t* nb,
                       irgan_stream_t s);

/* Weight gradient of a 3x3 stride-1 conv on fp8 operands (BASELINE config 5: the ResnetBlock
 * convs, ir:386-411): dw[co][ky][kx][ci] += dqx[0] * dqdy[0] * sum_p dy8[p][co] x8[p + tap][ci]
 * with x8 / dy8 the OCP e4m3 copies of the conv's input and output gradient (d->dtype =
 * IRGAN_FP8, NHWC, ld / off % 16 == 0) and dqx / dqdy their per-tensor dequantisation factors
 * (device).  d is the FORWARD descriptor (pad 1: c0x == -1, zero or reflect).  Cout % 128,
 * Cin % 64, Wo == 64 (then Ho even) or Wo % 128 == 0.  ws (ws_floats, nullable): the split-K
 * slab as irgan_conv_wgrad_ws.  IRGAN_EUNSUPPORTED (nothing launched) for other layers. */
IRGAN_API int irgan_conv_wgrad_fp8(const irgan_conv_desc* d, const void* x8, const void* dy8, const float* dqx,
                         const float* dqdy, float* dw, float* ws, int64_t ws_floats, irgan_stream_t s);

/* fp8 amax slots: each slot is IRGAN_FP8_AMAX_PARTS uint32 partial maxima (bits of
 * non-negative floats); a kernel's block b raises part b % IRGAN_FP8_AMAX_PARTS of
 * the slot it records into, irgan_fp8_scale takes the max over the parts. */
enum { IRGAN_FP8_AMAX_PARTS = 256 };

/* fp8 quantisation of an NHWC slice: y[p][yoff + c] = e4m3(clamp(x * q[0], +-448))
 * (round to nearest even; x bf16 or fp32 by dt; C, ld, off % 8 == 0), and the
 * max |x| recorded into the amax slot when amax != NULL.  y == NULL: the max only.
 * q == NULL: q = 1. */
IRGAN_API int irgan_fp8_quant(const void* x, int32_t dt, int64_t P, int32_t C, int32_t ldx, int32_t xoff,
                    void* y, int32_t ldy, int32_t yoff, const float* q, uint32_t* amax,
                    irgan_stream_t s);
/* Per-tensor scales from recorded maxima, for n slots (amax: n x IRGAN_FP8_AMAX_PARTS):
 * q = 2^floor(log2(448 / amax)) (1 if amax is 0), dq = 1 / q; reset != 0 clears the
 * slots afterwards. */
IRGAN_API int irgan_fp8_scale(uint32_t* amax, int32_t n, float* q, float* dq, int32_t reset, irgan_stream_t s);
/* A table of njobs irgan_fp8_job records (device memory; n % 8 == 0, bf16 src,
 * n <= max_n): amax != NULL -> max |src| into amax slot `slot` only; otherwise
 * dst = e4m3(clamp(src * q[slot], +-448)).  The per-step re-quantisation of the
 * packed fp8 weights: one amax launch, irgan_fp8_scale, one quantise launch. */
typedef struct irgan_fp8_job {
    const void* src;
    void* dst;
    int64_t n;
    int32_t slot, reserved;
} irgan_fp8_job;
IRGAN_API int irgan_fp8_quant_batch(const void* jobs, int32_t njobs, int64_t max_n, const float* q,
                          uint32_t* amax, irgan_stream_t s);

/* Split-K partial sums of irgan_conv_fwd (fp32 out; no bias, activation, mask or
 * accumulate): the K range is cut into ksplit parts and part ks lands at
 * y + ks*split_stride.  The consumer sums the parts (e.g. irgan_reflect_ring_fold).
 * bf16 LDS-DMA path; other dtypes support ksplit == 1 only. */
IRGAN_API int irgan_conv_fwd_splitk(const irgan_conv_desc* d, const void* x, const void* w, float* y,
                          int32_t ksplit, int64_t split_stride, irgan_stream_t s);

/* dw[cout][ky][kx][cin] += sum_pixels dy * im2col(x)  (fp32 atomics, split-K
 * over pixels) -- replaces the weight half of convolution_backward.  d is the
 * FORWARD descriptor (x = forward input, dy = grad at the forward output with
 * slice ldy/yoff); dw must be zeroed by the caller for a fresh gradient. */
IRGAN_API int irgan_conv_wgrad(const irgan_conv_desc* d, const void* x, const void* dy,
                     float* dw, int32_t splitk, irgan_stream_t s);

/* Same as irgan_conv_wgrad with a caller-owned fp32 workspace of ws_floats
 * floats: when it holds splitk x (Cout*KH*KW*Cin) floats, the split-K partials
 * are written there with plain stores and summed into dw by a second launch in
 * a fixed order (deterministic, no atomics); otherwise identical to
 * irgan_conv_wgrad.  ws may be NULL. */
IRGAN_API int irgan_conv_wgrad_ws(const irgan_conv_desc* d, const void* x, const void* dy, float* dw,
                        int32_t splitk, float* ws, int64_t ws_floats, irgan_stream_t s);

/* Weight re-pack: dst rows [R][Kp] (dtype) from the fp32 KRSC master
 * src[Cout][KH][KW][Cin], Kp = roundup(taps*Cp, kalign), taps and channels
 * zero-padded (Cp = max(cpad, channels)).  transpose=0: R = Cout, row =
 * [ky][kx][ci] (plain cast).  transpose=1: R = Cin, row = [a][b][co] with
 * (ky, kx) = (tyr + s*(Ay-1-a), txr + s*(Ax-1-b)) -- the flipped / per-phase
 * weights of backward-data and ConvTranspose2d.  A ConvTranspose2d weight
 * [Cin][Cout][K][K] is handed over as the KRSC master of the conv it transposes.
 * Narrow inputs (1/3/4 channels) are zero-padded to cpad = 8 so the bf16
 * LDS-DMA conv takes 64/8 = 8 taps per K-tile (kalign = 64). */
IRGAN_API int irgan_weight_pack(const float* src, void* dst, int32_t dtype, int32_t Cout, int32_t KH,
                      int32_t KW, int32_t Cin, int32_t transpose, int32_t s, int32_t tyr,
                      int32_t Ay, int32_t txr, int32_t Ax, int32_t cpad, int32_t kalign,
                      irgan_stream_t st);

/* One weight re-pack job (the arguments of irgan_weight_pack as a POD record). */
typedef struct irgan_pack_desc {
    const float* src;
    void* dst;
    int32_t dtype, Cout, KH, KW, Cin, transpose, s, tyr, Ay, txr, Ax, cpad, kalign, reserved;
} irgan_pack_desc;
/* n irgan_weight_pack jobs in ONE launch (a network's post-Adam re-pack: ~50
 * small launches -> 1).  descs: device array of n records. */
IRGAN_API int irgan_weight_pack_batch(const irgan_pack_desc* descs, int32_t n, irgan_stream_t st);

/* ---- InstanceNorm (ir:154-165), per-(n,c) over H*W, eps 1e-5, no affine ---- */
/* Reductions are two-level and atomic-free: <= IRGAN_IN_PARTS block partials per
 * (n, c) summed in fp64 in a fixed order. */
enum { IRGAN_IN_PARTS = 256 };
/* mr[n][c] = {mean, rstd} from nb float2 (sum, sum of squares) partials per (n, c)
 * written by irgan_conv_fwd_stats (the reduction half of irgan_in_stats). */
IRGAN_API int irgan_in_finalize(const void* part, int32_t N, int32_t HW, int32_t C, int32_t nb, float* mr,
                      irgan_stream_t s);
/* mr[n][c] = {mean, rstd}; work: IRGAN_IN_PARTS*N*C doubles of scratch (a reduce launch,
 * then a fixed-order finalize launch). */
IRGAN_API int irgan_in_stats(const void* x, int32_t dtype, int32_t N, int32_t HW, int32_t C,
                   int32_t ld, int32_t off, double* work, float* mr, irgan_stream_t s);
/* y = act((x - mean) * rstd) [+ res];  optional xhat output ([P][C], dtype). */
IRGAN_API int irgan_in_apply(const void* x, int32_t dtype, int32_t N, int32_t HW, int32_t C, int32_t ldx,
                   int32_t xoff, const float* mr, int32_t act, const void* res, int32_t ldr,
                   int32_t roff, void* y, int32_t ldy, int32_t yoff, void* xhat, irgan_stream_t s);
/* Backward of y = act(IN(x)) [+ res] given the PRE-norm input x and its
 * (mean, rstd): xhat = (x - mean)*rstd, g = (dy [+ dy2]) * act'(xhat),
 * red[n][c] = {mean g, mean g*xhat}.  work: IRGAN_IN_PARTS*N*C doubles of scratch. */
IRGAN_API int irgan_in_bwd_reduce(const void* dy, int32_t dy_dtype, int32_t lddy, int32_t dyoff,
                        const void* dy2, int32_t dy2_dtype, int32_t lddy2, int32_t dy2off,
                        const void* x, int32_t x_dtype, int32_t ldx, int32_t xoff, int32_t act,
                        int32_t N, int32_t HW, int32_t C, const float* mr, double* work,
                        float* red, irgan_stream_t s);
/* dx = rstd*(g - mean(g) - xhat*mean(g*xhat)); also db[c] += sum dx (fp32 bias
 * grad of the producing conv, caller zeroes) when db != NULL.  dx may alias dy. */
IRGAN_API int irgan_in_bwd_apply(const void* dy, int32_t dy_dtype, int32_t lddy, int32_t dyoff,
                       const void* dy2, int32_t dy2_dtype, int32_t lddy2, int32_t dy2off,
                       const void* x, int32_t x_dtype, int32_t ldx, int32_t xoff, int32_t act,
                       int32_t N, int32_t HW, int32_t C, const float* mr, const float* red,
                       void* dx, int32_t dx_dtype, int32_t lddx, int32_t dxoff, float* db,
                       irgan_stream_t s);

/* irgan_in_apply (bf16 x, res, y) / irgan_in_bwd_apply (bf16, no db) that also
 * write y8 = e4m3(clamp(bf16(y) * q[0], +-448)) (an NHWC fp8 slice) and record
 * max |bf16(y)| into the amax slot (IRGAN_FP8_AMAX_PARTS partials): the producers
 * of the fp8 path's ResnetBlock conv operands, so no separate quantise pass runs.
 * IRGAN_EUNSUPPORTED when C, the strides or offsets are not multiples of 8. */
IRGAN_API int irgan_in_apply_fp8(const void* x, int32_t N, int32_t HW, int32_t C, int32_t ldx, int32_t xoff,
                       const float* mr, int32_t act, const void* res, int32_t ldr, int32_t roff, void* y,
                       int32_t ldy, int32_t yoff, void* y8, int32_t ld8, int32_t off8, const float* q,
                       uint32_t* amax, irgan_stream_t s);
IRGAN_API int irgan_in_bwd_apply_fp8(const void* dy, int32_t lddy, int32_t dyoff, const void* dy2, int32_t lddy2,
                           int32_t dy2off, const void* x, int32_t ldx, int32_t xoff, int32_t act, int32_t N,
                           int32_t HW, int32_t C, const float* mr, const float* red, void* dx, int32_t lddx,
                           int32_t dxoff, void* y8, int32_t ld8, int32_t off8, const float* q,
                           uint32_t* amax, irgan_stream_t s);
/* db[c] += sum over pixels of g[p][c] (bias gradient), g slice (dtype, ld, off).
 * work: 16*IRGAN_IN_PARTS*C doubles of scratch. */
IRGAN_API int irgan_channel_sum(const void* g, int32_t dtype, int32_t P, int32_t C, int32_t ld,
                      int32_t off, float* db, double* work, irgan_stream_t s);

/* ---- resampling (ir:269-355 and reflection-pad backward) ---- */
/* Per-axis tables of a separable resampling map (host only, no GPU work).
 * kind 0: Downsample = reflect pad 1 + [1,2,1]/4 taps, stride 2 (ir:269-310);
 * kind 1: UpsampleAA = bilinear x2 (align_corners) + reflect pad 1 + blur (ir:313-355);
 * kind 2: nn.ReflectionPad2d(p).  transpose=1 gives the adjoint (rows = the
 * forward map's input coordinates).  Fills idx/w [rows][tmax] and returns rows,
 * or a negative IRGAN_E* code. */
IRGAN_API int irgan_resample_table(int32_t kind, int32_t n_in, int32_t p, int32_t transpose, int32_t* idx,
                         float* w, int32_t tmax, int32_t rows_cap);
/* Border half of the nn.ReflectionPad2d(p) backward (ir:381, 402, 459, 528).
 * The backward-data result g over the padded (H+2p) x (W+2p) domain has its
 * interior written straight to dx; its RING arrives as nsplit fp32 split-K
 * partials in two compact NHWC buffers: rows[ks][N][2p][W+2p][C] (padded rows
 * k and H+p+k at compact rows k and p+k) and cols[ks][N][H][2p][C] (padded
 * columns k and W+p+k of the interior rows).  dx[band] += every mirrored ring
 * value (a gather: deterministic).  Together: dx = fold(g). */
IRGAN_API int irgan_reflect_ring_fold(const float* rows, const float* cols, int32_t nsplit, int32_t N, int32_t H,
                            int32_t W, int32_t C, int32_t p, void* dx, int32_t dx_dtype, int32_t lddx,
                            int32_t dxoff, irgan_stream_t s);
/* Same fold in one launch, without the fp32 partials (bf16, stride-1 reflect
 * convs, dY channels % 32 == 0, H, W >= 2p+2): d is the descriptor of the
 * interior backward-data launch (irgan_conv_fwd on the flipped weights w,
 * Ho = H, Wo = W, c0 shifted by p), which must already have written dx; this
 * evaluates every ring value of g with MFMA and adds it onto its mirrored
 * border pixel of dx (one owner per pixel, no atomics). */
IRGAN_API int irgan_reflect_dgrad_ring(const irgan_conv_desc* d, const void* dy, const void* w, int32_t p, void* dx,
                             irgan_stream_t s);
/* irgan_reflect_dgrad_ring with a caller workspace ws of ws_floats floats.  ResnetBlock
 * shapes (3x3, p = 1, 4 <= H, W <= 64, dY channels % 32 and <= 256, dx channels % 64, bf16,
 * ws_floats >= N * 4 * 68 * dx channels) run as two launches: the four border lines as
 * GEMMs with LDS-resident weights (at most max_blocks workgroups, each walking a group of
 * images) into ws, then the fold onto dx (one read-modify-write per owned pixel); other
 * shapes: irgan_reflect_dgrad_ring.  max_blocks bounds the first launch for a second stream
 * beside a kernel that leaves that many CUs idle). */
IRGAN_API int irgan_reflect_dgrad_ring_ws(const irgan_conv_desc* d, const void* dy, const void* w, int32_t p, void* dx,
                                float* ws, int64_t ws_floats, int32_t max_blocks, irgan_stream_t s);
/* Reflect-padded ResnetBlock backward-data (ir:386-411; replaces torch autograd's
 * ReflectionPad2d + Conv2d backward) in two launches: the ring's line GEMM into ws (as
 * irgan_reflect_dgrad_ring_ws), then the interior conv whose store pass adds the ring terms
 * onto dx's border band -- the same dx, bit for bit, as irgan_conv_fwd (interior) followed by
 * irgan_reflect_dgrad_ring_ws, one launch and one dx read-modify-write fewer.  d: the interior
 * descriptor (ops.conv_dgrad).  IRGAN_EUNSUPPORTED (nothing launched) unless the line-ring
 * shapes hold (irgan_reflect_dgrad_ring_ws), dx is bf16 without activation, and dx channels
 * % 256 == 0 take the 256-channel conv tile. */
IRGAN_API int irgan_conv_dgrad_reflect_line(const irgan_conv_desc* d, const void* dy, const void* w, int32_t p, void* dx,
                                  float* ws, int64_t ws_floats, irgan_stream_t s);
/* The fp8 path's ResnetBlock backward-data (config 5): the ring's line GEMM on the bf16 dy
 * and bf16 flipped weights w (d: as irgan_conv_dgrad_reflect_line), then the interior on e4m3
 * operands -- d8 = d with dtype IRGAN_FP8 and dy8's ld / offset, w8 the e4m3 flipped image,
 * dqy / dqw their device dequantisation factors -- whose store pass folds the ring in: the
 * same dx as irgan_conv_fwd_fp8 (interior) followed by irgan_reflect_dgrad_ring_ws.  dy
 * channels % 128, dx channels % 256, dy8 ld / offset % 16; else IRGAN_EUNSUPPORTED. */
IRGAN_API int irgan_conv_dgrad_reflect_line_fp8(const irgan_conv_desc* d, const void* dy, const void* w,
                                      const irgan_conv_desc* d8, const void* dy8, const void* w8,
                                      const float* dqy, const float* dqw, int32_t p, void* dx, float* ws,
                                      int64_t ws_floats, irgan_stream_t s);
/* Backward-data of a 4x4 stride-2 pad-1 conv (PatchGAN model.0 / .3 / .6, ir:600-612) in
 * ONE launch for all four output phases: d = the four per-phase descriptors (2x2 taps on
 * dy, omy = omx = 2, (ooy, oox) the phase, c0y / c0x in {-1, 0}; otherwise identical), w =
 * their four packed phase images.  dx (+)= result, with the optional backward mask as
 * irgan_conv_fwd.  bf16, dy channels % 64, dx channels <= 16 or % 64, no bias / activation;
 * else IRGAN_EUNSUPPORTED (nothing launched; the caller runs the four phase launches). */
IRGAN_API int irgan_conv_dgrad_s2(const irgan_conv_desc* d, const void* dy, const void* const* w, void* dx,
                        const void* mask, irgan_stream_t s);
/* out = (Wy (x) Wx) in on NHWC slices, tables from irgan_resample_table (device
 * copies, rows [Hout][Ty] and [Wout][Tx]: the host may drop trailing all-zero
 * tap columns); accumulate: out += result.  Downsample / UpsampleAA forward
 * and backward, and the reflect-pad fold, are all this one launch. */
IRGAN_API int irgan_sep_resample(const void* in, int32_t in_dtype, int32_t N, int32_t Hin, int32_t Win,
                       int32_t C, int32_t ldi, int32_t offi, void* out, int32_t out_dtype,
                       int32_t Hout, int32_t Wout, int32_t ldo, int32_t offo, const int32_t* ty,
                       const float* wy, int32_t Ty, const int32_t* tx, const float* wx,
                       int32_t Tx, int32_t accumulate, irgan_stream_t s);
/* irgan_sep_resample (no accumulate) of act(InstanceNorm(in)): mr = the per-(n, c)
 * {mean, rstd} pairs of in (irgan_in_finalize / irgan_in_stats), act IRGAN_ACT_*.
 * The IN apply + ReLU of down1 / down2 / up1_conv (ir:469-482, 557-558) fused into the
 * Downsample / UpsampleAA that consumes it.  IRGAN_EUNSUPPORTED unless 8-channel-aligned
 * slices and at most 8 taps per axis (then apply + resample separately). */
IRGAN_API int irgan_sep_resample_in(const void* in, int32_t in_dtype, int32_t N, int32_t Hin, int32_t Win,
                          int32_t C, int32_t ldi, int32_t offi, const float* mr, int32_t act,
                          void* out, int32_t out_dtype, int32_t Hout, int32_t Wout, int32_t ldo,
                          int32_t offo, const int32_t* ty, const float* wy, int32_t Ty,
                          const int32_t* tx, const float* wx, int32_t Tx, irgan_stream_t s);
/* The fp8 path's producers of the down2 / up1_conv operands (config 5; ir:469-482, 554-558):
 * irgan_sep_resample (mr == NULL) or irgan_sep_resample_in (mr != NULL) into a bf16 out (no
 * accumulate) that also writes y8 = e4m3(clamp(bf16(out) * q[0], +-448)) (an NHWC slice, ld8 /
 * off8) and raises max |bf16(out)| into the amax slot (IRGAN_FP8_AMAX_PARTS partials) -- the
 * bytes irgan_fp8_quant makes from the stored out, with no pass reading it back.
 * IRGAN_EUNSUPPORTED (nothing launched) unless the LDS form takes the shapes (8-channel-aligned
 * slices, ld8 / off8 % 8, at most 8 taps per axis). */
IRGAN_API int irgan_sep_resample_fp8(const void* in, int32_t in_dtype, int32_t N, int32_t Hin, int32_t Win,
                           int32_t C, int32_t ldi, int32_t offi, const float* mr, int32_t act,
                           void* out, int32_t out_dtype, int32_t Hout, int32_t Wout, int32_t ldo,
                           int32_t offo, const int32_t* ty, const float* wy, int32_t Ty,
                           const int32_t* tx, const float* wx, int32_t Tx, void* y8, int32_t ld8,
                           int32_t off8, const float* q, uint32_t* amax, irgan_stream_t s);
/* 2x2 max pool (VGG features) forward / backward (first max wins, as ATen). */
/* VGG conv + ReLU + MaxPool2d(2) in one launch (ir:664: vgg16.features[:16] conv1_2 -> pool):
 * y (NULL: not written) = act(conv(x) + bias) as irgan_conv_fwd, yp = its 2x2 max-pool, dense
 * NHWC [N][Ho/2][Wo/2][Cout] bf16 -- bit-identical to irgan_conv_fwd + irgan_maxpool_fwd.
 * IRGAN_EUNSUPPORTED (nothing launched) unless bf16 3x3 stride 1 with Cin == 64, even Ho, Wo,
 * no accumulate / mask. */
IRGAN_API int irgan_conv_fwd_pool(const irgan_conv_desc* d, const void* x, const void* w, const float* bias,
                                  void* y, void* yp, irgan_stream_t s);
IRGAN_API int irgan_maxpool_fwd(const void* x, int32_t dtype, int32_t N, int32_t H, int32_t W, int32_t C,
                      void* y, irgan_stream_t s);
IRGAN_API int irgan_maxpool_bwd(const void* x, const void* dy, int32_t dtype, int32_t N, int32_t H,
                      int32_t W, int32_t C, void* dx, int32_t relu_mask, irgan_stream_t s);

/* ---- layout / elementwise ---- */
/* NCHW fp32 -> NHWC slice (dtype), optional affine y = x*scale[c] + shift[c]. */
IRGAN_API int irgan_nchw_to_nhwc(const float* x, int32_t N, int32_t C, int32_t H, int32_t W, void* y,
                       int32_t dtype, int32_t ldy, int32_t yoff, const float* scale,
                       const float* shift, irgan_stream_t s);
/* NHWC slice (dtype) -> NCHW fp32, y = x*scale (+= when accumulate). */
IRGAN_API int irgan_nhwc_to_nchw(const void* x, int32_t dtype, int32_t ldx, int32_t xoff, int32_t N,
                       int32_t C, int32_t H, int32_t W, float* y, float scale, int32_t accumulate,
                       irgan_stream_t s);
/* y[p][c] = a*x[p][c] (+ b*y) on slices; dtype conversion allowed. */
IRGAN_API int irgan_axpby(const void* x, int32_t xdtype, int32_t ldx, int32_t xoff, float a, void* y,
                int32_t ydtype, int32_t ldy, int32_t yoff, float b, int32_t P, int32_t C,
                irgan_stream_t s);
/* y[p][c] = x[p][c]*scale[c] (+ shift[c]) (+ y when accumulate): VGG input
 * normalisation (ir:679-682) and its backward. */
IRGAN_API int irgan_affine(const void* x, int32_t xdt, int32_t ldx, int32_t xoff, const float* scale,
                 const float* shift, void* y, int32_t ydt, int32_t ldy, int32_t yoff,
                 int32_t accumulate, int32_t P, int32_t C, irgan_stream_t s);
/* dx = dy * act'(a): 1 relu (a>0), 2 lrelu (a>0 ? 1 : 0.2), 3 tanh (1 - a^2). */
IRGAN_API int irgan_act_bwd(const void* dy, int32_t dy_dtype, int32_t lddy, int32_t dyoff, const void* a,
                  int32_t a_dtype, int32_t lda, int32_t aoff, int32_t act, void* dx,
                  int32_t dx_dtype, int32_t lddx, int32_t dxoff, int32_t P, int32_t C,
                  irgan_stream_t s);

/* ---- losses (ir:1647-1679, 686-750) ; images NHWC fp32 (B,H,W,3) ---- */
/* Hinge for D on a [real; fake] patch map (ir:1647-1649) and for G (ir:1662).
 * mode 0: loss = 0.5*(mean relu(1-p[:n]) + mean relu(1+p[n:])), grad written;
 * mode 1: loss = -mean p, grad = -scale/cnt.  Other modes: IRGAN_EINVAL.
 * loss accumulated into *loss (fp64). */
IRGAN_API int irgan_hinge(const float* pred, int32_t n_half, int32_t mode, float scale, float* grad,
                double* loss, irgan_stream_t s);
/* Pixel / feature L1: loss += w*mean|a-b|; ga = w*sign(a-b)/cnt (dtype of ga). */
IRGAN_API int irgan_l1(const void* a, const void* b, int32_t dtype, int64_t count, float w, void* ga,
             int32_t ga_dtype, int32_t accumulate, double* loss, irgan_stream_t s);
/* TV (ir:686-694) on NHWC fp32 x: loss += w*tv(x), g += grad. */
IRGAN_API int irgan_tv(const float* x, int32_t N, int32_t H, int32_t W, int32_t C, float w, float* g,
             double* loss, irgan_stream_t s);
/* SSIM loss w*(1 - mean ssim((a+1)/2, (b+1)/2)) (ir:714-750, 1675-1677);
 * grad wrt a accumulated into g.  work: 10*N*H*W*C floats of scratch. */
IRGAN_API int irgan_ssim(const float* a, const float* b, int32_t N, int32_t H, int32_t W, int32_t C, float w,
               float* g, double* loss, float* work, irgan_stream_t s);
/* irgan_ssim with ssim_loss_torch's window_size (ir:714-736): any odd size 1..15
 * (Gaussian sigma 1.5, zero padding window / 2); IRGAN_EUNSUPPORTED otherwise. */
IRGAN_API int irgan_ssim_ws(const float* a, const float* b, int32_t N, int32_t H, int32_t W, int32_t C, float w,
                  float* g, double* loss, float* work, int32_t window, irgan_stream_t s);

/* ---- optimizer (torch.optim.Adam, ir:1601-1604) over a flat fp32 buffer ---- */
/* step_size = lr/(1-beta1^t), bc2_sqrt = sqrt(1-beta2^t) (host, fp64 -> fp32). */
IRGAN_API int irgan_adam(float* p, const float* g, float* m, float* v, int64_t n, float step_size,
               float beta1, float beta2, float bc2_sqrt, float eps, irgan_stream_t s);
/* The same update with the step count on the device (a captured train step replays with
 * the right bias corrections): irgan_adam_prep advances *count (int32, device) and writes
 * prm[0] = step_size, prm[1] = bc2_sqrt for the new count (the host formula above, fp64 on
 * the device, then fp32); irgan_adam_dev reads them from prm. */
IRGAN_API int irgan_adam_prep(int32_t* count, double lr, double beta1, double beta2, float* prm, irgan_stream_t s);
IRGAN_API int irgan_adam_dev(float* p, const float* g, float* m, float* v, int64_t n, const float* prm, float beta1,
                   float beta2, float eps, irgan_stream_t s);

/* ---- inference / evaluation ---- */
/* out[p][c] = uint8(clip((x + 1) / 2, 0, 1) * 255) for every pixel p and
 * channel c of an NHWC fp32 slice (x, ldx, xoff), out dense [N][H][W][C]
 * (16-byte aligned) -- the float32 pipeline of tensor_to_rgb_image
 * (ir:865-876) for a whole batch, on the device; truncation as numpy astype. */
IRGAN_API int irgan_to_rgb_u8(const float* x, int32_t N, int32_t H, int32_t W, int32_t C, int32_t ldx,
                    int32_t xoff, void* out, irgan_stream_t s);
/* Per-image error sums of compute_metrics (ir:1184-1206) over uint8 images
 * (as run_test feeds it, ir:1412-1415): d = pred/255 - gt/255 in fp32,
 * sums[2n] = sum |d|, sums[2n+1] = sum d^2 over the per_image bytes of image n
 * (MAE = sums[2n]/per_image, MSE = sums[2n+1]/per_image).  work: >= 128*N
 * doubles of scratch (work_cap = its size in doubles). */
IRGAN_API int irgan_image_metrics_u8(const void* pred, const void* gt, int32_t N, int64_t per_image,
                           double* work, int64_t work_cap, double* sums, irgan_stream_t s);

/* ---- KAIST data pipeline (KAISTPairDataset ir:1132-1177) ---- */
/* cv2.resize(..., INTER_AREA) of a batch of uint8 images src [N][Hin][Win][C]
 * (C <= 4, image stride img_stride bytes) to out_u8 [N][C][Hout][Wout] (NCHW),
 * as OpenCV's general area path computes it (resizeArea_: per destination
 * pixel, source rows reduced horizontally with the x-table weights, then summed
 * with the y-table weights, float32, round half to even, clamp).  Tables are
 * CSR over destination indices: entries yptr[y]..yptr[y+1]-1 of (ysrc, yw), and
 * the same for x (host: computeResizeAreaTab's recurrence).  flip (nullable,
 * uint8 per image): 1 = horizontal flip (np.fliplr, ir:1166-1168).  img_max
 * (nullable, zeroed int32 per image): max destination byte of each image. */
IRGAN_API int irgan_area_resize_u8(const void* src, int32_t N, int32_t Hin, int32_t Win, int32_t C, int64_t img_stride,
                         const int32_t* yptr, const int32_t* ysrc, const float* yw, int32_t Hout,
                         const int32_t* xptr, const int32_t* xsrc, const float* xw, int32_t Wout,
                         const void* flip, void* out_u8, int32_t* img_max, irgan_stream_t s);
/* cv2.resize(INTER_AREA) when an axis UPscales (img_size above the source, ir:818,
 * 1139, 1156): OpenCV's linear resampler with area-mode coefficients in 8-bit fixed
 * point.  Tables (data.linear_area_table): yofs [Hout], ycoef [Hout][2], xofs [Wout],
 * xcoef [Wout][2] (int, x 2048), xlim = first destination column with a single tap.
 * Layouts, flip and img_max as irgan_area_resize_u8. */
IRGAN_API int irgan_linear_area_resize_u8(const void* src, int32_t N, int32_t Hin, int32_t Win, int32_t C,
                                int64_t img_stride, const int32_t* yofs, const int32_t* ycoef, int32_t Hout,
                                const int32_t* xofs, const int32_t* xcoef, int32_t xlim, int32_t Wout,
                                const void* flip, void* out_u8, int32_t* img_max, irgan_stream_t s);
/* out[n][i] = float32(in[n][i]) / 255 * 2 - 1 for per_image bytes per image (the
 * [-1, 1] tensors of ir:1157, 1175-1176); max_rule = 1: the IR rule of ir:1142 --
 * images whose img_max[n] <= 1 are not divided by 255. */
IRGAN_API int irgan_u8_to_unit(const void* in, int32_t N, int64_t per_image, const int32_t* img_max, int32_t max_rule,
                     float* out, irgan_stream_t s);

/* The SSIM of compute_metrics (ir:1208-1213): skimage.metrics.structural_similarity(
 * gt, pred, data_range=1.0, channel_axis=2) for N uint8 image pairs [N][H][W][C]
 * standing for v / 255 -- per channel 7x7 uniform windows, sample covariance,
 * C1 = 0.01^2, C2 = 0.03^2, map averaged over pixels >= 3 from the border, then over
 * channels; fp64.  ssim[n] out.  work: >= N doubles (more = more blocks). */
IRGAN_API int irgan_ssim_eval_u8(const void* pred, const void* gt, int32_t N, int32_t H, int32_t W, int32_t C,
                       double* work, int64_t work_cap, double* ssim, irgan_stream_t s);

/* nn.Dropout(p) in training mode (ResnetBlock use_dropout, ir:394-395) on NHWC slices:
 * y = keep ? x / (1 - p) : 0, keep decided per element (pixel * C + channel) by a
 * counter-based hash of seed; the backward is the same call on the gradient (same seed).
 * x and y may alias. */
IRGAN_API int irgan_dropout(const void* x, int32_t xdt, int32_t P, int32_t C, int32_t ldx, int32_t xoff, void* y,
                  int32_t ydt, int32_t ldy, int32_t yoff, uint64_t seed, float p, irgan_stream_t s);

/* PatchGAN head: NLayerDiscriminator's last layer, Conv2d(C, 1, 4, stride 1, padding 1)
 * (ir:625-627), as GEMMs over the 16 taps on v_mfma_f32_16x16x32_bf16 (bf16 products, fp32
 * sums, fixed order).  Forward: x bf16 NHWC [N][H][W] (ldx, xoff), w the forward pack row
 * [16 taps][C] bf16 (tap = ky * 4 + kx), y fp32 [N][H-1][W-1] = conv + bias[0] (bias may be
 * NULL); ws holds the per-pixel tap products (16 x N*H*W rounded up to 16 floats; smaller ->
 * IRGAN_EUNSUPPORTED).  Backward-data: g = dL/dy fp32, pixel stride ldg floats (split into two
 * bf16 parts, so not rounded to bf16); dx bf16 NHWC [N][H][W] (lddx, dxoff) is written (not
 * accumulated).  C must be 512 and ldx / xoff / lddx / dxoff multiples of 8, else
 * IRGAN_EUNSUPPORTED (nothing launched). */
IRGAN_API int irgan_patch_head_fwd(const void* x, int32_t N, int32_t H, int32_t W, int32_t C, int32_t ldx,
                         int32_t xoff, const void* w, const float* bias, float* y, float* ws, int64_t ws_floats,
                         irgan_stream_t s);
IRGAN_API int irgan_patch_head_dgrad(const float* g, int32_t ldg, const void* w, void* dx, int32_t N, int32_t H,
                           int32_t W, int32_t C, int32_t lddx, int32_t dxoff, irgan_stream_t s);
/* Weight gradient of the same layer (its Conv2d weight grad under loss_D.backward(),
 * ir:1650): dw fp32 [16 taps][C] += sum over pixels of x * g (g = dL/dy fp32 as above, split
 * into bf16 hi + lo).  Block partials (<= 256) go to ws and one ordered pass adds them into dw
 * (deterministic); ws_floats too small for the launch's partials -> IRGAN_EUNSUPPORTED. */
IRGAN_API int irgan_patch_head_wgrad(const void* x, int32_t N, int32_t H, int32_t W, int32_t C, int32_t ldx,
                           int32_t xoff, const float* g, int32_t ldg, float* dw, float* ws, int64_t ws_floats,
                           irgan_stream_t s);

/* MFMA throughput probe (bench.py's measured MFMA peak): blocks x 256 threads,
 * each wave iters x 8 back-to-back v_mfma_f32_16x16x32_bf16 (16384 FLOP each) on operands
 * read once from src (>= 4096 x 16 bytes of random bf16); one float per thread to out
 * (blocks * 256 floats).  FLOP = blocks * 4 * iters * 8 * 16384; time it with events. */
IRGAN_API int irgan_mfma_probe(const void* src, float* out, int32_t blocks, int32_t iters, irgan_stream_t s);

/* Version / capability probe (no GPU work). */
IRGAN_API int irgan_version(void);

#ifdef __cplusplus
}
#endif
#endif /* IRGAN_H */
