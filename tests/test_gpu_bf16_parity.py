"""Tight parity for the bf16 kernels the benchmark actually runs.

bf16 mode = bf16 operands, exact bf16 x bf16 products, fp32 accumulation.  So the
HIP result is compared with an fp64 reference computed on the SAME bf16-quantised
operands (x, w, dY), not with an unquantised fp32 conv:

    |got - ref64| <= r_out * |ref64| + 2e-5 * absref   (every element)

* ``absref`` is the same op on |x|, |w|, |dY| (the sum of |terms| of each output):
  2e-5 of it bounds fp32 accumulation-order error with margin (sqrt(K) * eps32 is
  3e-6 at K = 2304 and 5e-6 at K = 8192 pixels);
* ``r_out`` = 2^-8 for bf16 outputs (the unit roundoff of an 8-bit significand),
  0 for fp32.  The reflect-pad dgrad writes its interior first and folds the ring
  onto the border band afterwards, so a bf16 border pixel is rounded twice: there
  the bound is 2^-8 * (|ref| + |interior part|).

A kernel that drops, duplicates or misplaces even one output element fails this,
as do writes outside the output channel slice (checked separately).  Cases cover
every family the dispatch reaches on the train step: conv_pp (BN 256/192/128/64,
plain / accumulate / fused-IN-stats), the reflect ring, conv_c8 (incl. stride 2),
conv_narrow, conv_halo, conv_glds (stride 2, per-phase dgrad), wgrad_halo (row
segments, slab split-K), wgrad_pc, wgrad_narrow (8-channel inputs), wgrad_glds and the
generic fallbacks, with ragged tiles.
"""
import pytest
import torch
import torch.nn.functional as F

from conftest import pkg
from test_gpu_kernels import CONV_CASES

pytestmark = pytest.mark.gpu
DEV = "cuda"
R_BF16 = 2.0 ** -8
R_ACC = 2e-5

EXTRA_CASES = [
    # cin, cout, k, s, p, mode, H : the G / D / VGG layers at odd sizes (ragged 16x16 patches)
    (256, 256, 3, 1, 1, 1, 37),    # resblock: pp BN256 fwd, ring + pp dgrad
    (128, 256, 3, 1, 1, 0, 33),    # down2: BN256 fwd, BN128 (accumulating) dgrad
    (64, 128, 3, 1, 1, 0, 40),     # down1: BN128 fwd, BN64 dgrad
    (384, 128, 3, 1, 1, 0, 24),    # up1_conv: BN128 fwd, 384-ch dgrad
    (192, 64, 3, 1, 1, 0, 40),     # up2_conv: BN64 fwd, BN192 dgrad
    (64, 64, 3, 1, 1, 0, 24),      # VGG conv1_2
    (256, 512, 4, 1, 1, 0, 13),    # D model.8
    (128, 256, 4, 2, 1, 0, 34),    # D model.5 (stride 2: glds fwd, per-phase dgrad)
    (8, 64, 4, 2, 1, 0, 66),       # D model.0 with the 8-channel padded input
    # 8-channel-input weight gradient (conv_wgrad_narrow.hip): inc 7x7 reflect, D model.0 s2, ragged rows
    (1, 64, 7, 1, 3, 1, 37),
    (1, 64, 7, 1, 3, 1, 130),
    (4, 64, 4, 2, 1, 0, 258),
    # Wo % 64 == 0, Cout % 128 == 0: the producer/consumer wgrad (conv_wgrad_pc.hip, 128-channel co tiles)
    (128, 256, 3, 1, 1, 0, 64),    # down2 shape, zero pad, 2 co tiles
    (384, 128, 3, 1, 1, 0, 64),    # up1_conv shape, 6 ci chunks
    (64, 128, 3, 1, 1, 0, 128),    # down1 shape, 2 segments per row
    (256, 256, 3, 1, 1, 1, 128),   # resblock conv, reflect, interior + edge segments
    # 4x4 stride 1 with Wo <= 32: wgrad_pc on paired-row segments (two output rows of 32 per
    # 64-pixel segment; odd Ho masks the last pair's second row): D model.8 at its own shape
    (256, 512, 4, 1, 1, 0, 32),
    (128, 256, 4, 1, 1, 0, 33),
    # Cout % 128 != 0 (Cout % 64 == 0): wgrad_pc with 64-channel co tiles (128-B dY rows)
    (192, 64, 3, 1, 1, 0, 64),     # up2_conv shape, 3 ci chunks
    (64, 64, 3, 1, 1, 1, 128),     # reflect, 2 segments per row
    # one 64-channel input chunk: the resident-weight persistent kernel (conv_res64) takes the
    # bf16 forward and every dgrad whose dY has 64 channels (ragged patches, reflect, 3 co tiles)
    (64, 64, 3, 1, 1, 1, 37),
    (192, 64, 3, 1, 1, 1, 21),
    (64, 192, 3, 1, 1, 0, 50),
    # the PatchGAN head (Cout 1 forward / one-channel-dY backward-data / weight gradient):
    # n_layers = 2's 256-channel head and a larger 512-channel one
    (256, 1, 4, 1, 1, 0, 21),
    (512, 1, 4, 1, 1, 0, 40),
    # non-square maps (H, W): the ResnetBlock at 512 x 640's 128 x 160 (config 4, scaled down in
    # H) and widths that are not a multiple of 64 -- the wide-n weight gradient's partial segments
    (256, 256, 3, 1, 1, 1, 16, 160),
    (128, 256, 3, 1, 1, 0, 12, 96),
    (384, 128, 3, 1, 1, 0, 8, 40),
]


def q(t):
    """bf16-representable copy (fp32 storage)."""
    return t.bfloat16().float()


def nhwc(x, dt=torch.bfloat16):
    return x.permute(0, 2, 3, 1).contiguous().to(DEV, dt)


def nchw64(x):
    return x.double().cpu().permute(0, 3, 1, 2).contiguous()


def ref_conv(x, w, b, k, s, p, mode):
    if mode == 1:
        x = F.pad(x, (p, p, p, p), mode="reflect")
        p = 0
    return F.conv2d(x, w, b, stride=s, padding=p)


def references(x, w, b, gy, k, s, p, mode):
    """fp64 y, dx, dw on the given operands, and the interior part of dx (reflect
    mode: the padded-domain gradient before the ring is folded back; else dx)."""
    xr, wr = x.double().requires_grad_(True), w.double().requires_grad_(True)
    y = ref_conv(xr, wr, None if b is None else b.double(), k, s, p, mode)
    y.backward(gy.double())
    interior = xr.grad
    if mode == 1:
        xp = F.pad(x.double(), (p, p, p, p), mode="reflect").requires_grad_(True)
        F.conv2d(xp, w.double(), stride=s).backward(gy.double())
        interior = xp.grad[..., p:-p, p:-p]
    return y.detach(), xr.grad, wr.grad, interior


def check(got, ref, aref, r_out, what, partial=None):
    """partial: an intermediate that a bf16 output is rounded to before the rest is
    added (the reflect dgrad's interior, written before the ring is folded onto the
    border band): its rounding enters the bound too."""
    err = (got - ref).abs()
    mag = ref.abs()
    if partial is not None:   # pixels that received a ring term were rounded twice
        twice = (partial - ref).abs() > 1e-9 * aref
        mag = mag + torch.where(twice, partial.abs(), torch.zeros_like(mag))
    bound = r_out * mag + R_ACC * aref + 1e-30
    ratio = (err / bound).max().item()
    assert ratio <= 1.0, f"{what}: worst |err|/bound = {ratio:.3g}, max |err| {err.max().item():.3g}"


@pytest.fixture(scope="module")
def ops():
    return pkg().ops


@pytest.mark.parametrize("case", CONV_CASES + EXTRA_CASES)
def test_bf16_conv_family_tight(ops, case):
    cin, cout, k, s, p, mode, H = case[:7]
    W = case[7] if len(case) > 7 else H
    torch.manual_seed(0)
    N = 2
    x = q(torch.randn(N, cin, H, W))
    w = q(torch.randn(cout, cin, k, k) * (1.0 / (cin * k * k) ** 0.5))
    b = torch.randn(cout) * 0.1
    spec = ops.ConvSpec(cin, cout, k, s, p, mode)
    Ho, Wo = spec.out_hw(H, W)
    gy = q(torch.randn(N, cout, Ho, Wo))
    y64, dx64, dw64, dxi = references(x, w, b, gy, k, s, p, mode)
    ya, dxa, dwa, _ = references(x.abs(), w.abs(), b.abs(), gy.abs(), k, s, p, mode)

    master = w.permute(0, 2, 3, 1).contiguous().reshape(-1).to(DEV)
    pc = ops.PackedConv(spec, master, b.to(DEV), ops.BF16)
    pc.pack()
    xd = torch.zeros(N, H, W, pc.cin_eff, device=DEV, dtype=torch.bfloat16)
    xd[..., :cin] = nhwc(x)

    # forward, bf16 output into a channel slice (ld = cout + 8, off 8) -- the step's layout
    yb = torch.zeros(N, Ho, Wo, cout + 8, device=DEV, dtype=torch.bfloat16)
    ops.conv_fwd(pc, ops.Feat(xd), ops.Feat(yb, 8, cout))
    check(nchw64(yb[..., 8:]), y64, ya, R_BF16, "fwd bf16")
    assert not yb[..., :8].any(), "fwd wrote outside its channel slice"
    # forward, fp32 output
    yf = torch.zeros(N, Ho, Wo, cout, device=DEV, dtype=torch.float32)
    ops.conv_fwd(pc, ops.Feat(xd), ops.Feat(yf))
    check(nchw64(yf), y64, ya, 0.0, "fwd fp32")

    # backward-data: dY zero-padded to cout_eff channels
    gyd = torch.zeros(N, Ho, Wo, pc.cout_eff, device=DEV, dtype=torch.bfloat16)
    gyd[..., :cout] = nhwc(gy)
    pad = torch.empty(N * (H + 2 * p) * (W + 2 * p) * cin, device=DEV) if mode == 1 else None
    for out_dt, r_out in ((torch.float32, 0.0), (torch.bfloat16, R_BF16)):
        dx = torch.zeros(N, H, W, cin, device=DEV, dtype=out_dt)
        ops.conv_dgrad(pc, ops.Feat(gyd), ops.Feat(dx), pad_buf=pad)
        check(nchw64(dx), dx64, dxa, r_out, f"dgrad {out_dt}", partial=dxi)
    # backward-data accumulating onto another branch's gradient (bf16, the step's
    # resblock / down2 / down1 skip paths), into a channel slice when aligned
    sl = 8 if cin % 8 == 0 else 0
    old = q(torch.randn(N, cin, H, W))
    dxb = torch.zeros(N, H, W, cin + sl, device=DEV, dtype=torch.bfloat16)
    dxb[..., sl:] = nhwc(old)
    ops.conv_dgrad(pc, ops.Feat(gyd), ops.Feat(dxb, sl, cin), accumulate=True, pad_buf=pad)
    check(nchw64(dxb[..., sl:]), dx64 + old.double(), dxa + old.double().abs(), R_BF16, "dgrad accumulate",
          partial=dxi + old.double())
    assert not dxb[..., :sl].any(), "dgrad wrote outside its channel slice"

    # backward-weight (fp32, split-K slab workspace), accumulated onto an existing value
    dw0 = torch.randn(cout * k * k * cin, device=DEV)
    dw = dw0.clone()
    ops.conv_wgrad(spec, ops.Feat(xd), ops.Feat(gyd, 0, cout), dw, ops.BF16)
    got = (dw - dw0).view(cout, k, k, cin).permute(0, 3, 1, 2).double().cpu()
    check(got, dw64, dwa + dw0.abs().max().item() * 1e-2, 0.0, "wgrad")


@pytest.mark.parametrize("case", [(256, 256, 3, 1, 64, 2), (256, 256, 3, 1, 37, 2), (128, 256, 3, 0, 33, 2),
                                  (64, 128, 3, 0, 40, 2), (384, 128, 3, 0, 24, 2), (256, 512, 4, 0, 13, 2),
                                  (192, 64, 3, 0, 64, 1), (64, 64, 3, 1, 37, 3), (64, 128, 3, 0, 64, 2)])
def test_bf16_fused_in_stats_tight(ops, case):
    """conv_pp with the fused InstanceNorm-statistics epilogue: the bf16 output holds
    the tight bound, and {mean, rstd} equal the fp64 statistics OF THAT bf16 OUTPUT
    (which is what the IN apply normalises) to fp32 rounding."""
    cin, cout, k, mode, H, N = case
    torch.manual_seed(4)
    spec = ops.ConvSpec(cin, cout, k, 1, 1, mode)
    x = q(torch.randn(N, cin, H, H))
    w = q(torch.randn(cout, cin, k, k) * (1.0 / (cin * k * k) ** 0.5))
    b = torch.randn(cout) * 0.1
    pc = ops.PackedConv(spec, w.permute(0, 2, 3, 1).contiguous().reshape(-1).to(DEV), b.to(DEV), ops.BF16)
    pc.pack()
    Ho, Wo = spec.out_hw(H, H)
    y = ops.Feat(torch.empty(N, Ho, Wo, cout, device=DEV, dtype=torch.bfloat16))
    work = torch.empty(ops.IN_PARTS * N * cout, dtype=torch.float64, device=DEV)
    nb = ops.conv_fwd_stats(pc, ops.Feat(nhwc(x)), y, work)
    assert nb > 0, "layer did not take the fused-statistics kernel"
    mr = torch.empty(N * cout * 2, device=DEV)
    ops.in_finalize(y, work, nb, mr)
    y64 = ref_conv(x.double(), w.double(), b.double(), k, 1, 1, mode)
    ya = ref_conv(x.abs().double(), w.abs().double(), b.abs().double(), k, 1, 1, mode)
    yg = nchw64(y.t)
    check(yg, y64, ya, R_BF16, "fwd+stats")
    mean = yg.mean(dim=(2, 3))
    rstd = (yg.var(dim=(2, 3), unbiased=False) + 1e-5).rsqrt()
    got = mr.view(N, cout, 2).double().cpu()
    torch.testing.assert_close(got[..., 0], mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(got[..., 1], rstd, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("cout,H,mode", [(64, 37, 1), (192, 24, 0), (128, 16, 0)])
def test_bf16_res64_act_mask_tight(ops, cout, H, mode):
    """The Cin = 64 resident-weight kernel's epilogue: ReLU / LeakyReLU activations and the
    backward ReLU / LeakyReLU masks (VGG conv1_2 / conv2_1, ir:664) on the bf16 path, into a
    channel slice, held to the tight bf16 bound."""
    torch.manual_seed(7)
    N, cin = 2, 64
    spec = ops.ConvSpec(cin, cout, 3, 1, 1, mode)
    x = q(torch.randn(N, cin, H, H))
    w = q(torch.randn(cout, cin, 3, 3) * (1.0 / (cin * 9) ** 0.5))
    b = torch.randn(cout) * 0.1
    m = q(torch.randn(N, cout, H, H))
    pc = ops.PackedConv(spec, w.permute(0, 2, 3, 1).contiguous().reshape(-1).to(DEV), b.to(DEV), ops.BF16)
    pc.pack()
    y64 = ref_conv(x.double(), w.double(), b.double(), 3, 1, 1, mode)
    ya = ref_conv(x.abs().double(), w.abs().double(), b.abs().double(), 3, 1, 1, mode)
    for act, fn in ((ops.ACT_RELU, F.relu), (ops.ACT_LRELU, lambda t: F.leaky_relu(t, 0.2))):
        y = torch.zeros(N, H, H, cout + 8, device=DEV, dtype=torch.bfloat16)
        ops.conv_fwd(pc, ops.Feat(nhwc(x)), ops.Feat(y, 8, cout), act=act)
        check(nchw64(y[..., 8:]), fn(y64), ya, R_BF16, f"act {act}")
        assert not y[..., :8].any()
    for mact, slope in ((1, 0.0), (2, 0.2)):
        y = torch.zeros(N, H, H, cout, device=DEV, dtype=torch.bfloat16)
        ops.conv_fwd(pc, ops.Feat(nhwc(x)), ops.Feat(y), mask=ops.Feat(nhwc(m)), mask_act=mact)
        mm = torch.where(m > 0, 1.0, slope).double()
        check(nchw64(y), y64 * mm, ya, R_BF16, f"mask {mact}")


@pytest.mark.parametrize("cin,cout,H", [(128, 128, 40), (256, 256, 24), (128, 64, 33), (256, 128, 16)])
def test_bf16_pp_mask_tight(ops, cin, cout, H):
    """conv_pp (Cin > 64) with a backward mask (the VGG backward-data chain, ir:664, and D's
    LeakyReLU masks): the ReLU mask is applied in the store pass on the rounded values, the
    LeakyReLU mask and accumulate in registers.  Mask slices with an offset and exact / signed
    zeros in the mask; the ReLU-masked output must also equal the unmasked output with the
    masked-off elements zeroed, bit for bit."""
    torch.manual_seed(11)
    N = 2
    spec = ops.ConvSpec(cin, cout, 3, 1, 1, 0)
    x = q(torch.randn(N, cin, H, H))
    w = q(torch.randn(cout, cin, 3, 3) * (1.0 / (cin * 9) ** 0.5))
    m = q(torch.randn(N, cout, H, H))
    m[:, :, ::3] = 0.0
    m[:, :, 1::5] = -0.0
    pc = ops.PackedConv(spec, w.permute(0, 2, 3, 1).contiguous().reshape(-1).to(DEV), None, ops.BF16)
    pc.pack()
    y64 = ref_conv(x.double(), w.double(), None, 3, 1, 1, 0)
    ya = ref_conv(x.abs().double(), w.abs().double(), None, 3, 1, 1, 0)
    md = torch.zeros(N, H, H, cout + 16, device=DEV, dtype=torch.bfloat16)
    md[..., 8:8 + cout] = nhwc(m)
    xd = nhwc(x)
    plain = torch.zeros(N, H, H, cout, device=DEV, dtype=torch.bfloat16)
    ops.conv_fwd(pc, ops.Feat(xd), ops.Feat(plain), bias=False)
    for mact, slope in ((1, 0.0), (2, 0.2)):
        y = torch.zeros(N, H, H, cout, device=DEV, dtype=torch.bfloat16)
        ops.conv_fwd(pc, ops.Feat(xd), ops.Feat(y), bias=False, mask=ops.Feat(md, 8, cout), mask_act=mact)
        mm = torch.where(m > 0, 1.0, slope).double()
        check(nchw64(y), y64 * mm, ya, R_BF16, f"mask {mact}")
        if mact == 1:
            keep = (md[..., 8:8 + cout].float() > 0)
            assert torch.equal(y.view(torch.int16), torch.where(keep, plain, plain * 0).view(torch.int16))
        # accumulate onto a prior gradient (the register path for both masks)
        base = q(torch.randn(N, cout, H, H))
        ya2 = nhwc(base)
        ops.conv_fwd(pc, ops.Feat(xd), ops.Feat(ya2), bias=False, accumulate=True, mask=ops.Feat(md, 8, cout),
                     mask_act=mact)
        check(nchw64(ya2), y64 * mm + base.double(), ya + base.abs().double(), R_BF16, f"acc mask {mact}")


@pytest.mark.parametrize("cin,cout,H", [(64, 128, 32), (128, 256, 18), (64, 128, 17)])
def test_bf16_s2_dgrad_mask_tight(ops, cin, cout, H):
    """Backward-data of the PatchGAN's 4x4 stride-2 layers (ir:607-615) with the LeakyReLU mask
    of the layer below (D model.2's dgrad folds model.0's LReLU): the four phase convs in one
    conv_pp launch (even dx sides) or dgrad_s2_kernel (odd), plain and accumulating."""
    torch.manual_seed(5)
    N = 2
    spec = ops.ConvSpec(cin, cout, 4, 2, 1, 0)
    x = q(torch.randn(N, cin, H, H))
    w = q(torch.randn(cout, cin, 4, 4) * (1.0 / (cin * 16) ** 0.5))
    Ho = spec.out_hw(H, H)[0]
    gy = q(torch.randn(N, cout, Ho, Ho))
    m = q(torch.randn(N, cin, H, H))
    _, dx64, _, _ = references(x, w, None, gy, 4, 2, 1, 0)
    _, dxa, _, _ = references(x.abs(), w.abs(), None, gy.abs(), 4, 2, 1, 0)
    pc = ops.PackedConv(spec, w.permute(0, 2, 3, 1).contiguous().reshape(-1).to(DEV), None, ops.BF16)
    pc.pack()
    mm = torch.where(m > 0, 1.0, 0.2).double()
    dx = torch.zeros(N, H, H, cin, device=DEV, dtype=torch.bfloat16)
    ops.conv_dgrad(pc, ops.Feat(nhwc(gy)), ops.Feat(dx), mask=ops.Feat(nhwc(m)), mask_act=2)
    check(nchw64(dx), dx64 * mm, dxa, R_BF16, "s2 dgrad mask")
    base = q(torch.randn(N, cin, H, H))
    dxb = nhwc(base)
    ops.conv_dgrad(pc, ops.Feat(nhwc(gy)), ops.Feat(dxb), accumulate=True)
    check(nchw64(dxb), dx64 + base.double(), dxa + base.abs().double(), R_BF16, "s2 dgrad acc")


@pytest.mark.parametrize("N,H,W", [(2, 32, 48), (1, 64, 64), (3, 48, 32), (2, 16, 64), (1, 37, 64)])
def test_reflect_dgrad_ring_tight(ops, N, H, W):
    """ResnetBlock backward-data (ir:386-411) through ops.conv_dgrad: the interior conv_pp launch
    plus the reflect-pad ring (line GEMM folded into the interior's store pass on the bf16
    line shapes, else the ring launch) against fp64, for plain / accumulating bf16 and fp32
    outputs, non-square and multi-image shapes (every corner / edge patch kind).  The band
    pixels are rounded twice (interior, then + ring): the bound allows the partial sum."""
    C = 256
    torch.manual_seed(12)
    x = q(torch.randn(N, C, H, W))
    w = q(torch.randn(C, C, 3, 3) * (1.0 / (C * 9) ** 0.5))
    spec = ops.ConvSpec(C, C, 3, 1, 1, 1)
    gy = q(torch.randn(N, C, H, W))
    _, dx64, _, dxi = references(x, w, None, gy, 3, 1, 1, 1)
    _, dxa, _, _ = references(x.abs(), w.abs(), None, gy.abs(), 3, 1, 1, 1)
    pc = ops.PackedConv(spec, w.permute(0, 2, 3, 1).contiguous().reshape(-1).to(DEV), None, ops.BF16)
    pc.pack()
    gyd = nhwc(gy)
    for out_dt, r_out in ((torch.bfloat16, R_BF16), (torch.float32, 0.0)):
        dx = torch.zeros(N, H, W, C, device=DEV, dtype=out_dt)
        ops.conv_dgrad(pc, ops.Feat(gyd), ops.Feat(dx))
        check(nchw64(dx), dx64, dxa, r_out, f"ring {out_dt}", partial=dxi)
    old = q(torch.randn(N, C, H, W))
    dxb = torch.zeros(N, H, W, C + 8, device=DEV, dtype=torch.bfloat16)
    dxb[..., 8:] = nhwc(old)
    ops.conv_dgrad(pc, ops.Feat(gyd), ops.Feat(dxb, 8, C), accumulate=True)
    check(nchw64(dxb[..., 8:]), dx64 + old.double(), dxa + old.double().abs(), R_BF16, "ring accumulate",
          partial=dxi + old.double())
    assert not dxb[..., :8].any()


@pytest.mark.parametrize("N,H,W,cout,keep", [(2, 32, 48, 64, True), (2, 32, 48, 64, False), (3, 20, 36, 128, True),
                                             (1, 256, 256, 64, False)])
def test_conv_pool_fused_bit_identical(ops, N, H, W, cout, keep):
    """irgan_conv_fwd_pool (the VGG conv1_2 -> ReLU -> MaxPool2d(2), ir:664, in one launch of the
    resident-weight kernel) against irgan_conv_fwd + irgan_maxpool_fwd: the activated map (when
    kept) and the pooled map bit-identical; ragged 16x16 patches (20 x 36), two co tiles, the
    full 256 x 256 VGG map; an odd size is refused (nothing launched)."""
    torch.manual_seed(2)
    cin = 64
    spec = ops.ConvSpec(cin, cout, 3, 1, 1, 0)
    w = q(torch.randn(cout, cin, 3, 3) * (1.0 / (cin * 9) ** 0.5))
    pc = ops.PackedConv(spec, w.permute(0, 2, 3, 1).contiguous().reshape(-1).to(DEV),
                        (torch.randn(cout) * 0.1).to(DEV), ops.BF16)
    pc.pack()
    x = torch.randn(N, H, W, cin, device=DEV).bfloat16()
    y_ref = torch.empty(N, H, W, cout, device=DEV, dtype=torch.bfloat16)
    p_ref = torch.empty(N, H // 2, W // 2, cout, device=DEV, dtype=torch.bfloat16)
    ops.conv_fwd(pc, ops.Feat(x), ops.Feat(y_ref), act=ops.ACT_RELU)
    ops.maxpool(ops.Feat(y_ref), ops.Feat(p_ref))
    y = torch.full_like(y_ref, 7.0)
    p = torch.full_like(p_ref, 7.0)
    assert ops.conv_fwd_pool(pc, ops.Feat(x), ops.Feat(y) if keep else None, ops.Feat(p))
    torch.cuda.synchronize()
    assert torch.equal(p.view(torch.int16), p_ref.view(torch.int16)), "pooled map"
    if keep:
        assert torch.equal(y.view(torch.int16), y_ref.view(torch.int16)), "activated map"
    else:
        assert bool((y == 7.0).all()), "y written although not kept"
    xo = torch.randn(1, 21, 32, cin, device=DEV).bfloat16()
    assert not ops.conv_fwd_pool(pc, ops.Feat(xo), None,
                                 ops.Feat(torch.empty(1, 10, 16, cout, device=DEV, dtype=torch.bfloat16)))
