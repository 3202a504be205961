"""Tight parity for the bf16 NON-conv kernels of the benchmarked step.

Companion of test_gpu_bf16_parity.py (the convs): every elementwise / reduction /
resampling kernel that the bf16 train step launches (profiles/r02_s10_summary.md)
is checked here on bf16 operands against an fp64 reference computed on the SAME
bf16 values, with the bound of that file:

    |got - ref64| <= r_out * |ref64| + r_acc * absref      (every element)

* ``r_out`` = 2^-8 for a bf16 output (one rounding of an 8-bit significand), 0 for
  fp32 outputs / statistics;
* ``absref`` = the same op on the absolute values of its terms; ``r_acc`` bounds the
  kernel's fp32 arithmetic: 2e-5 where fp32 sums run over many terms (statistics,
  reductions), 1e-5 for the short fixed-length expressions.

Kernels covered (reference ops ir:154-165 InstanceNorm, ir:269-355 Downsample /
UpsampleAA, ir:664 VGG max-pool + input normalisation, ir:1664-1669 L1):
  rows8_kernel<0,8> + finalize_kernel  (irgan_in_stats)
  apply_kernel<8>                      (irgan_in_apply, with / without residual)
  rows8_kernel<1,4> + finalize mode 1  (irgan_in_bwd_reduce), rows8_kernel<2,4>
                                       (irgan_in_bwd_apply, in place as the step runs it)
  sep_lds_kernel<2|4|6>                (Downsample, UpsampleAA and their adjoints)
  sep_lds_kernel<4|6, NORM>            (irgan_sep_resample_in: IN apply + ReLU fused
                                        into the Downsample / UpsampleAA loads)
  maxpool_fwd/bwd_kernel<8>, affine_kernel, nchw_to_nhwc_kernel (VGG affine pack),
  act_bwd_kernel, axpby_kernel, l1_kernel<bf16>
Layouts follow the step: channel slices (ld > C, off > 0) wherever the step has them.
"""
import pytest
import torch
import torch.nn.functional as F

from conftest import pkg

pytestmark = pytest.mark.gpu
DEV = "cuda"
R_BF16 = 2.0 ** -8


@pytest.fixture(scope="module")
def ops():
    return pkg().ops


def q(t):
    """bf16-representable copy (fp32 storage, CPU)."""
    return t.bfloat16().float()


def to_slice(x, ld_extra=0, off=0, fill=0.0):
    """NCHW CPU -> NHWC bf16 device tensor of width C + ld_extra, x in channels [off, off + C)."""
    N, C, H, W = x.shape
    t = torch.full((N, H, W, C + ld_extra), fill, device=DEV, dtype=torch.bfloat16)
    t[..., off:off + C] = x.permute(0, 2, 3, 1).to(DEV, torch.bfloat16)
    return t


def from_slice(t, off, C):
    return t[..., off:off + C].double().cpu().permute(0, 3, 1, 2).contiguous()


def check(got, ref, aref, r_out, r_acc, what):
    err = (got.double() - ref).abs()
    bound = r_out * ref.abs() + r_acc * aref + 1e-30
    ratio = (err / bound).max().item()
    assert ratio <= 1.0, f"{what}: worst |err|/bound = {ratio:.3g}, max |err| {err.max().item():.3g}"


def act64(h, act):
    if act == 1:
        return h.clamp_min(0.0)
    if act == 2:
        return torch.where(h > 0, h, 0.2 * h)
    return h


def act_grad32(xh32, act):
    """act'(xhat) with xhat evaluated exactly as the kernels do: fp32 (x - mean) * rstd."""
    if act == 1:
        return (xh32 > 0).double()
    if act == 2:
        return torch.where(xh32 > 0, 1.0, 0.2).double()
    return torch.ones_like(xh32, dtype=torch.float64)


IN_SHAPES = [(2, 256, 64, 64), (2, 128, 96, 80), (3, 64, 45, 38), (1, 192, 33, 17)]


def _stats(ops, x, ld_extra, off):
    N, C, H, W = x.shape
    xd = to_slice(x, ld_extra, off, fill=7.0)   # neighbouring channels hold junk
    work = torch.empty(ops.IN_PARTS * N * C, dtype=torch.float64, device=DEV)
    mr = torch.empty(2 * N * C, device=DEV)
    ops.in_stats(ops.Feat(xd, off, C), work, mr)
    return xd, mr


@pytest.mark.parametrize("shape", IN_SHAPES)
def test_in_stats_bf16(ops, shape):
    """rows8_kernel<0,8> partials + finalize_kernel: (mean, rstd) of the bf16 tensor."""
    torch.manual_seed(1)
    N, C, H, W = shape
    x = q(torch.randn(shape) * 2 + 0.7)
    _, mr = _stats(ops, x, 16, 8)
    x64 = x.double()
    mean = x64.mean(dim=(2, 3))
    var = x64.var(dim=(2, 3), unbiased=False)
    e_abs, e_sq = x64.abs().mean(dim=(2, 3)), (x64 * x64).mean(dim=(2, 3))
    got = mr.view(N, C, 2).double().cpu()
    check(got[..., 0], mean, e_abs, 0.0, 2e-5, "mean")
    # var = E[x^2] - mean^2 from fp32 partial sums: its error is <= 2e-5 * (E[x^2] + 2|mean| E|x|)
    dvar = 2e-5 * (e_sq + 2 * mean.abs() * e_abs)
    rstd = (var + 1e-5).rsqrt()
    check(got[..., 1], rstd, rstd * 0.5 * dvar / (var + 1e-5), 2.0 ** -23, 1.0, "rstd")


@pytest.mark.parametrize("shape", IN_SHAPES)
@pytest.mark.parametrize("act,res", [(0, True), (1, False), (2, False), (0, False)])
def test_in_apply_bf16(ops, shape, act, res):
    """apply_kernel<8>: y = act((x - mean) * rstd) [+ res] into a channel slice."""
    torch.manual_seed(2)
    N, C, H, W = shape
    x = q(torch.randn(shape) * 1.5 - 0.3)
    xd, mr = _stats(ops, x, 8, 0)
    r = q(torch.randn(shape)) if res else None
    rd = to_slice(r, 8, 8) if res else None
    y = torch.zeros(N, H, W, C + 16, device=DEV, dtype=torch.bfloat16)
    ops.in_apply(ops.Feat(xd, 0, C), mr, ops.Feat(y, 8, C), act=act, res=ops.Feat(rd, 8, C) if res else None)
    m = mr.view(N, C, 2).double().cpu()
    mean, rstd = m[..., 0, None, None], m[..., 1, None, None]
    h = (x.double() - mean) * rstd
    ref = act64(h, act) + (r.double() if res else 0.0)
    aref = h.abs() + (r.double().abs() if res else 0.0)
    check(from_slice(y, 8, C), ref, aref, R_BF16, 1e-5, f"in_apply act={act} res={res}")
    assert not y[..., :8].any() and not y[..., 8 + C:].any(), "apply wrote outside its channel slice"


@pytest.mark.parametrize("shape", IN_SHAPES)
@pytest.mark.parametrize("act,dy2,inplace", [(1, False, True), (0, False, True), (2, False, False),
                                             (1, True, False)])
def test_in_backward_bf16(ops, shape, act, dy2, inplace):
    """rows8_kernel<1,4> + finalize (mean g, mean g*xhat), then rows8_kernel<2,4>:
    dx = rstd * (g - mean g - xhat * mean g*xhat), g = (dy [+ dy2]) * act'(xhat);
    in place (dx aliases dy) as GeneratorEngine.backward runs it."""
    torch.manual_seed(3)
    N, C, H, W = shape
    z = q(torch.randn(shape) * 2 + 0.5)
    zd, mr = _stats(ops, z, 0, 0)
    dy = q(torch.randn(shape))
    d2 = q(torch.randn(shape) * 0.5) if dy2 else None
    dyd = to_slice(dy, 8, 8)
    d2d = to_slice(d2, 0, 0) if dy2 else None
    work = torch.empty(ops.IN_PARTS * N * C, dtype=torch.float64, device=DEV)
    red = torch.empty(2 * N * C, device=DEV)
    if inplace:
        dxd, dx_off = dyd, 8
    else:
        dxd, dx_off = torch.zeros(N, H, W, C, device=DEV, dtype=torch.bfloat16), 0
    ops.in_backward(ops.Feat(dyd, 8, C), ops.Feat(zd), act, mr, work, red, ops.Feat(dxd, dx_off, C),
                    dy2=ops.Feat(d2d) if dy2 else None)
    m = mr.view(N, C, 2).cpu()
    m32, r32 = m[..., 0, None, None], m[..., 1, None, None]
    xh32 = (z - m32) * r32                                  # the kernels' fp32 xhat (mask decisions)
    mean, rstd = m32.double(), r32.double()
    xh = (z.double() - mean) * rstd
    g = (dy.double() + (d2.double() if dy2 else 0.0)) * act_grad32(xh32, act)
    HW = H * W
    mg, mgx = g.mean(dim=(2, 3)), (g * xh).mean(dim=(2, 3))
    got_red = red.view(N, C, 2).double().cpu()
    check(got_red[..., 0], mg, g.abs().mean(dim=(2, 3)), 0.0, 2e-5, "mean g")
    check(got_red[..., 1], mgx, (g * xh).abs().mean(dim=(2, 3)), 0.0, 2e-5, "mean g*xhat")
    kg, kgx = got_red[..., 0, None, None], got_red[..., 1, None, None]
    ref = rstd * (g - kg - xh * kgx)
    aref = rstd * (g.abs() + kg.abs() + (xh * kgx).abs())
    check(from_slice(dxd, dx_off, C), ref, aref, R_BF16, 1e-5, f"in_bwd_apply act={act} dy2={dy2}")
    assert HW > 0


# ---------------------------------------------------------------------------
# resampling (sep_lds_kernel): the step's own shapes and slices at N = 1, and odd sizes
# ---------------------------------------------------------------------------

def _filt(C):
    from oracle import step as O
    return O.binomial_filter(3)[None, None].repeat(C, 1, 1, 1).double()


def _down64(x):
    from oracle import step as O
    return O.blur_down(x, _filt(x.shape[1]))


def _up64(x, size=None):
    from oracle import step as O
    y = O.up_aa(x, _filt(x.shape[1]))
    if size is not None and tuple(y.shape[-2:]) != tuple(size):
        y = F.interpolate(y, size=size, mode="bilinear", align_corners=True)
    return y


def _adjoint(fwd, dy, in_shape):
    x = torch.zeros(in_shape, dtype=torch.float64, requires_grad=True)
    fwd(x).backward(dy)
    return x.grad


# name, C, Hin, Win, (in ld_extra, in off), (out ld_extra, out off): the step's layers
RESAMPLE_CASES = [
    ("down", 256, 128, 128, (0, 0), (0, 0)),        # down2: z2 -> h0
    ("down", 128, 256, 256, (0, 0), (256, 256)),    # down1: z1 -> x1 = cat1[..., 256:384]
    ("up", 256, 64, 64, (0, 0), (128, 0)),          # up1_up: h9 -> cat1[..., :256]
    ("up", 128, 128, 128, (0, 0), (64, 0)),         # up2_up: a3 -> cat2[..., :128]
    ("down_adj", 256, 128, 128, (0, 0), (0, 0)),    # blur_down_bwd: dh -> dz2
    ("down_adj", 128, 256, 256, (256, 256), (0, 0)),  # dcat1[..., 256:] -> dz1
    ("up_adj", 256, 64, 64, (128, 0), (0, 0)),      # dcat1[..., :256] -> dh
    ("up_adj", 128, 128, 128, (64, 0), (0, 0)),     # dcat2[..., :128] -> da3
    ("down", 64, 45, 38, (8, 8), (0, 0)),           # odd sizes
    ("up", 64, 23, 19, (0, 0), (8, 8)),
    ("up_resize", 64, 11, 9, (0, 0), (0, 0)),       # odd skip sizes: UpsampleAA + bilinear resize
]


@pytest.mark.parametrize("case", RESAMPLE_CASES, ids=lambda c: f"{c[0]}-{c[1]}x{c[2]}x{c[3]}")
def test_resample_bf16(ops, case):
    name, C, Hin, Win, (lxi, oxi), (lxo, oxo) = case
    torch.manual_seed(4)
    N = 1
    if name in ("down", "up", "up_resize"):
        x = q(torch.randn(N, C, Hin, Win))
        if name == "down":
            fn = _down64
        elif name == "up":
            fn = _up64
        else:
            size = (2 * Hin - 1, 2 * Win - 3)
            fn = lambda t: _up64(t, size)   # noqa: E731
        ref, aref = fn(x.double()), fn(x.double().abs())
        Ho, Wo = ref.shape[-2:]
        xd = to_slice(x, lxi, oxi, fill=5.0)
        y = torch.zeros(N, Ho, Wo, C + lxo, device=DEV, dtype=torch.bfloat16)
        xf, yf = ops.Feat(xd, oxi, C), ops.Feat(y, oxo, C)
        {"down": ops.blur_down, "up": ops.upsample, "up_resize": ops.upsample}[name](xf, yf)
    else:
        # adjoints: Hin x Win is the forward input (the gradient's output) size
        fwd = _down64 if name == "down_adj" else _up64
        Ho, Wo = fwd(torch.zeros(1, 1, Hin, Win, dtype=torch.float64)).shape[-2:]
        dy = q(torch.randn(N, C, Ho, Wo))
        ref = _adjoint(fwd, dy.double(), (N, C, Hin, Win))
        aref = _adjoint(fwd, dy.double().abs(), (N, C, Hin, Win))
        dyd = to_slice(dy, lxi, oxi, fill=5.0)
        y = torch.zeros(N, Hin, Win, C + lxo, device=DEV, dtype=torch.bfloat16)
        (ops.blur_down_bwd if name == "down_adj" else ops.upsample_bwd)(ops.Feat(dyd, oxi, C), ops.Feat(y, oxo, C))
    check(from_slice(y, oxo, C), ref, aref, R_BF16, 1e-5, name)
    if lxo:
        rest = torch.cat([y[..., :oxo], y[..., oxo + C:]], dim=-1)
        assert not rest.any(), "resample wrote outside its channel slice"


NORM_CASES = [
    ("down", 128, 256, 256, 1, (256, 256)),   # down1: IN + ReLU fused into the blur-down, into cat1
    ("down", 256, 128, 128, 1, (0, 0)),       # down2 -> h0
    ("up", 128, 128, 128, 1, (64, 0)),        # up1_conv's IN + ReLU fused into UpsampleAA, into cat2
    ("down", 64, 45, 38, 2, (8, 8)),          # LeakyReLU, odd size
    ("up", 64, 23, 19, 0, (0, 0)),            # no activation
]


@pytest.mark.parametrize("case", NORM_CASES, ids=lambda c: f"{c[0]}-{c[1]}x{c[2]}x{c[3]}-act{c[4]}")
def test_resample_in_bf16(ops, case):
    """sep_lds_kernel<T, NORM> (irgan_sep_resample_in): resample(act((z - mean) * rstd))."""
    name, C, Hin, Win, act, (lxo, oxo) = case
    torch.manual_seed(5)
    N = 1
    z = q(torch.randn(N, C, Hin, Win) * 2 + 0.4)
    zd, mr = _stats(ops, z, 0, 0)
    m = mr.view(N, C, 2).double().cpu()
    mean, rstd = m[..., 0, None, None], m[..., 1, None, None]
    h = act64((z.double() - mean) * rstd, act)
    habs = z.double().abs() * rstd + (mean * rstd).abs()   # the kernel forms z*rstd - mean*rstd
    fn = _down64 if name == "down" else _up64
    ref, aref = fn(h), fn(habs)
    Ho, Wo = ref.shape[-2:]
    y = torch.zeros(N, Ho, Wo, C + lxo, device=DEV, dtype=torch.bfloat16)
    ok = (ops.blur_down_in if name == "down" else ops.upsample_in)(ops.Feat(zd), mr, act, ops.Feat(y, oxo, C))
    assert ok, "the fused kernel did not take the shape"
    check(from_slice(y, oxo, C), ref, aref, R_BF16, 1e-5, f"{name}_in act={act}")
    if lxo:
        rest = torch.cat([y[..., :oxo], y[..., oxo + C:]], dim=-1)
        assert not rest.any(), "resample_in wrote outside its channel slice"


# ---------------------------------------------------------------------------
# VGG pieces: max-pool, the affine input pack, L1 on features; act_bwd / axpby
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("C,H,W", [(64, 256, 256), (128, 128, 128), (64, 37, 30)])
def test_maxpool_bf16_exact(ops, C, H, W):
    """maxpool_fwd/bwd_kernel<8> on ReLU'd bf16 features (VGG pools 1 and 2): the max is a
    copy and the gradient a routed copy, so both must be bit-exact vs torch (first argmax
    on ties, as torch; gradient through the pool input's ReLU)."""
    torch.manual_seed(6)
    N = 1
    x = q(torch.randn(N, C, H, W)).relu()
    xr = x.clone().requires_grad_(True)
    y = F.max_pool2d(xr, 2)
    gy = q(torch.randn_like(y))
    y.backward(gy)
    gx_ref = xr.grad * (x > 0)   # relu' of the pool input (the conv's ReLU output)
    xd = to_slice(x)
    yd = torch.empty(N, H // 2, W // 2, C, device=DEV, dtype=torch.bfloat16)
    ops.maxpool(ops.Feat(xd), ops.Feat(yd))
    assert torch.equal(from_slice(yd, 0, C), y.detach().double())
    dx = torch.full((N, H, W, C), 3.0, device=DEV, dtype=torch.bfloat16)
    if H % 2 or W % 2:
        dx.zero_()
    ops.maxpool_bwd(ops.Feat(xd), ops.Feat(to_slice(gy)), ops.Feat(dx), relu_mask=True)
    assert torch.equal(from_slice(dx, 0, C), gx_ref.double())


def test_vgg_affine_pack_bf16(ops):
    """nchw_to_nhwc_kernel with (scale, shift) and affine_kernel: the ImageNet
    normalisation ((x+1)/2 - mean)/std (ir:672-675) written as bf16 VGG input into the
    8-channel padded buffer, and the input-gradient affine accumulated in fp32."""
    eng = pkg().engine
    torch.manual_seed(7)
    N, H, W = 2, 64, 48
    x = torch.rand(N, 3, H, W) * 2 - 1
    scale = (0.5 / torch.tensor(eng.IMAGENET_STD)).float()
    shift = ((0.5 - torch.tensor(eng.IMAGENET_MEAN)) / torch.tensor(eng.IMAGENET_STD)).float()
    ref = x.double() * scale.double()[:, None, None] + shift.double()[:, None, None]
    aref = (x.double() * scale.double()[:, None, None]).abs() + shift.double().abs()[:, None, None]
    buf = torch.zeros(N, H, W, 8, device=DEV, dtype=torch.bfloat16)
    ops.nchw_to_nhwc(x.to(DEV), ops.Feat(buf, 0, 3), scale.to(DEV), shift.to(DEV))
    check(from_slice(buf, 0, 3), ref, aref, R_BF16, 1e-6, "nchw_to_nhwc affine")
    assert not buf[..., 3:].any()
    # affine_kernel: fp32 NHWC -> bf16 slice (the fake half of the VGG input), and the
    # backward's bf16 -> fp32 accumulate
    xn = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    buf2 = torch.zeros(N, H, W, 8, device=DEV, dtype=torch.bfloat16)
    ops.affine(ops.Feat(xn), scale.to(DEV), shift.to(DEV), ops.Feat(buf2, 0, 3))
    check(from_slice(buf2, 0, 3), ref, aref, R_BF16, 1e-6, "affine fwd")
    dv = q(torch.randn(N, 3, H, W))
    acc0 = torch.randn(N, H, W, 3)
    acc = acc0.clone().to(DEV)
    ops.affine(ops.Feat(to_slice(dv, 5, 0), 0, 3), scale.to(DEV), None, ops.Feat(acc), accumulate=True)
    want = dv.double() * scale.double()[:, None, None] + acc0.double().permute(0, 3, 1, 2)
    aw = (dv.double() * scale.double()[:, None, None]).abs() + acc0.double().permute(0, 3, 1, 2).abs()
    check(acc.double().cpu().permute(0, 3, 1, 2), want, aw, 0.0, 2 ** -22, "affine accumulate")


@pytest.mark.parametrize("act", [1, 2, 3])
def test_act_bwd_and_axpby_bf16(ops, act):
    """act_bwd_kernel (tanh' of outc into the zero-padded bf16 dz; ReLU / LReLU masks)
    and axpby_kernel (the D-input concat and the GAN-term d fake)."""
    torch.manual_seed(8)
    N, H, W, C = 2, 40, 36, 3
    dy = torch.randn(N, C, H, W)
    a = torch.tanh(torch.randn(N, C, H, W)) if act == 3 else torch.randn(N, C, H, W)
    f = {1: (a > 0).double(), 2: torch.where(a > 0, 1.0, 0.2).double(), 3: 1 - a.double() ** 2}[act]
    ref = dy.double() * f
    dyn, an = dy.permute(0, 2, 3, 1).contiguous().to(DEV), a.permute(0, 2, 3, 1).contiguous().to(DEV)
    out = torch.zeros(N, H, W, 8, device=DEV, dtype=torch.bfloat16)
    ops.act_bwd(ops.Feat(dyn), ops.Feat(an), act, ops.Feat(out, 0, C))
    check(from_slice(out, 0, C), ref, (dy.double() * f).abs(), R_BF16, 1e-6, f"act_bwd {act}")
    assert not out[..., C:].any()
    # axpby: y[slice] = a*x + b*y (bf16 out), the D input built from fp32 NHWC sources
    x = torch.randn(N, C, H, W)
    y0 = q(torch.randn(N, C, H, W))
    yd = to_slice(y0, 5, 1)
    ops.axpby(ops.Feat(x.permute(0, 2, 3, 1).contiguous().to(DEV)), 0.75, ops.Feat(yd, 1, C), -1.5)
    want = 0.75 * x.double() - 1.5 * y0.double()
    check(from_slice(yd, 1, C), want, (0.75 * x.double()).abs() + (1.5 * y0.double()).abs(), R_BF16, 1e-6, "axpby")


@pytest.mark.parametrize("count", [16 * 256 * 64 * 64, 1001])
def test_l1_bf16_features_tight(ops, count):
    """l1_kernel<bf16, bf16>: the perceptual L1 on relu3_3 features (ir:1669): fp64 block
    sums of fp32 |a - b| terms, gradient sign(a - b) * w / count stored in bf16."""
    torch.manual_seed(9)
    a = q(torch.randn(count))
    b = q(torch.randn(count))
    ga = torch.zeros(count, dtype=torch.bfloat16, device=DEV)
    loss = torch.zeros(1, dtype=torch.float64, device=DEV)
    ops.l1(a.to(DEV, torch.bfloat16), b.to(DEV, torch.bfloat16), 30.0, ga, loss)
    d = a.double() - b.double()
    ref = d.abs().mean() * 30
    check(loss.cpu(), ref.view(1), ref.view(1), 0.0, 2e-5, "l1 loss")
    want = torch.sign(d) * 30 / count
    check(ga.cpu().double(), want, want.abs(), R_BF16, 1e-7, "l1 grad")
