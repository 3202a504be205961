"""fp32 PyTorch-CPU restatement of the reference hot path (test oracle only).

Every function cites the reference line range it restates
(``ir:N`` = ``/root/reference/Code/ir_colorization.py`` line N).  Parameters
are plain ``{state_dict_key: tensor}`` dicts in the reference's OIHW layout and
key order, so a reference checkpoint loads here unchanged.

Parity pinning: ``tests/test_oracle_golden.py`` checks this module against
``tests/golden/step_*.npz``, which ``tests/golden/make_golden.py`` produced by
executing the reference's own modules in the build container.
"""
from __future__ import annotations

import math
from collections import OrderedDict

import torch
import torch.nn.functional as F

__all__ = [
    "binomial_filter", "g_param_shapes", "d_param_shapes", "vgg_param_shapes",
    "seeded_params", "g_forward", "d_forward", "vgg_features", "tv_loss",
    "ssim_loss", "adam_update", "AdamState", "train_step", "PRE_IN_BIAS_G",
    "PRE_IN_BIAS_D", "pre_in_bias_keys", "lr_lambda", "fp8_q",
]

IN_EPS = 1e-5                       # nn.InstanceNorm2d default (ir:161)
LRELU = 0.2                         # ir:601, 614, 624
IMAGENET_MEAN = (0.485, 0.456, 0.406)   # ir:672
IMAGENET_STD = (0.229, 0.224, 0.225)    # ir:673


# ----------------------------------------------------------------------------
# parameter layout (state_dict keys / shapes / order)
# ----------------------------------------------------------------------------

def binomial_filter(n: int = 3) -> torch.Tensor:
    """Normalised binomial kernel a a^T / sum (ir:240-266)."""
    rows = {1: [1.], 2: [1., 1.], 3: [1., 2., 1.], 4: [1., 3., 3., 1.],
            5: [1., 4., 6., 4., 1.], 6: [1., 5., 10., 10., 5., 1.],
            7: [1., 6., 15., 20., 15., 6., 1.]}
    if n not in rows:
        raise ValueError("filt_size must be 1-7")
    a = torch.tensor(rows[n], dtype=torch.float32)
    f = a[:, None] * a[None, :]
    return f / f.sum()


def res_conv_keys(padding_type="reflect", use_dropout=False):
    """Indices of the two convs in ResnetBlock.conv_block (ir:375-411): pad modules only
    for reflect / replicate, the Dropout only with use_dropout."""
    first = 0 if padding_type == "zero" else 1
    return first, first + 3 + int(bool(use_dropout)) + (0 if padding_type == "zero" else 1)


def g_param_shapes(input_nc=1, output_nc=3, ngf=64, n_blocks=9,
                   no_antialias=False, no_antialias_up=False, use_bias=True, padding_type="reflect",
                   use_dropout=False):
    """Generator state_dict layout (ir:443-531); buffers 'filt' included.
    use_bias = (norm_layer == nn.InstanceNorm2d) (ir:450-455): norm 'none' drops every
    conv bias but outc's."""
    s = OrderedDict()
    b = lambda key, c: s.__setitem__(key, (c,)) if use_bias else None   # noqa: E731
    s["inc.1.weight"] = (ngf, input_nc, 7, 7); b("inc.1.bias", ngf)
    s["down1.0.weight"] = (2 * ngf, ngf, 3, 3); b("down1.0.bias", 2 * ngf)
    if not no_antialias:
        s["down1_down.filt"] = (2 * ngf, 1, 3, 3)
    s["down2.0.weight"] = (4 * ngf, 2 * ngf, 3, 3); b("down2.0.bias", 4 * ngf)
    if not no_antialias:
        s["down2_down.filt"] = (4 * ngf, 1, 3, 3)
    for blk in range(n_blocks):
        for c in res_conv_keys(padding_type, use_dropout):
            s[f"resblocks.{blk}.conv_block.{c}.weight"] = (4 * ngf, 4 * ngf, 3, 3)
            b(f"resblocks.{blk}.conv_block.{c}.bias", 4 * ngf)
    if no_antialias_up:
        s["up1_up.weight"] = (4 * ngf, 4 * ngf, 3, 3); b("up1_up.bias", 4 * ngf)
    else:
        s["up1_up.filt"] = (4 * ngf, 1, 3, 3)
    s["up1_conv.0.weight"] = (2 * ngf, 6 * ngf, 3, 3); b("up1_conv.0.bias", 2 * ngf)
    if no_antialias_up:
        s["up2_up.weight"] = (2 * ngf, 2 * ngf, 3, 3); b("up2_up.bias", 2 * ngf)
    else:
        s["up2_up.filt"] = (2 * ngf, 1, 3, 3)
    s["up2_conv.0.weight"] = (ngf, 3 * ngf, 3, 3); b("up2_conv.0.bias", ngf)
    s["outc.1.weight"] = (output_nc, ngf, 7, 7); s["outc.1.bias"] = (output_nc,)
    return s


def d_param_shapes(input_nc=4, ndf=64, n_layers=3, use_bias=True):
    """PatchGAN state_dict layout (ir:585-632)."""
    s = OrderedDict()
    s["model.0.weight"] = (ndf, input_nc, 4, 4); s["model.0.bias"] = (ndf,)
    idx, mult = 2, 1
    for n in range(1, n_layers):
        prev, mult = mult, min(2 ** n, 8)
        s[f"model.{idx}.weight"] = (ndf * mult, ndf * prev, 4, 4)
        if use_bias:
            s[f"model.{idx}.bias"] = (ndf * mult,)
        idx += 3
    prev, mult = mult, min(2 ** n_layers, 8)
    s[f"model.{idx}.weight"] = (ndf * mult, ndf * prev, 4, 4)
    if use_bias:
        s[f"model.{idx}.bias"] = (ndf * mult,)
    idx += 3
    s[f"model.{idx}.weight"] = (1, ndf * mult, 4, 4); s[f"model.{idx}.bias"] = (1,)
    return s


VGG_CONVS = ((0, 3, 64), (2, 64, 64), (5, 64, 128), (7, 128, 128),
             (10, 128, 256), (12, 256, 256), (14, 256, 256))


def vgg_param_shapes():
    """torchvision vgg16.features[:16] conv layout (ir:664)."""
    s = OrderedDict()
    for i, ci, co in VGG_CONVS:
        s[f"{i}.weight"] = (co, ci, 3, 3); s[f"{i}.bias"] = (co,)
    return s


def seeded_params(shapes, seed, weight_std=0.02, bias_std=0.0, kaiming=False):
    """Deterministic parameter dict from a seed (test/bench init spec).

    weights ~ N(0, weight_std) (ir:181 uses N(0, 0.02)) or kaiming-normal
    (std = sqrt(2/fan_in), used for the synthetic VGG), biases ~ N(0, bias_std),
    blur buffers = binomial filter (ir:300-304).  Generated in key order on CPU.
    """
    g = torch.Generator().manual_seed(seed)
    out = OrderedDict()
    for k, shp in shapes.items():
        if k.endswith(".filt"):
            out[k] = binomial_filter(shp[-1])[None, None].repeat(shp[0], 1, 1, 1).contiguous()
        elif len(shp) == 4:
            std = math.sqrt(2.0 / (shp[1] * shp[2] * shp[3])) if kaiming else weight_std
            out[k] = torch.randn(shp, generator=g) * std
        else:
            out[k] = torch.randn(shp, generator=g) * bias_std if bias_std else torch.zeros(shp)
    return out


def pre_in_bias_keys(keys):
    """Biases of convs followed by InstanceNorm: their gradient is exactly 0 in
    exact arithmetic (IN subtracts the channel mean), so fp32 values are noise.
    Not normalised: outc, the ConvTranspose2d ups, the PatchGAN's first and last conv
    (the last is the highest model.N, whatever n_layers is)."""
    keys = list(keys)
    dix = [int(k.split(".")[1]) for k in keys if k.startswith("model.")]
    last = f"model.{max(dix)}." if dix else None
    free = ("outc.", "model.0.", "up1_up.", "up2_up.") + ((last,) if last else ())
    return [k for k in keys if k.endswith(".bias") and not k.startswith(free)]


PRE_IN_BIAS_G = pre_in_bias_keys(g_param_shapes().keys())
PRE_IN_BIAS_D = pre_in_bias_keys(d_param_shapes().keys())


# ----------------------------------------------------------------------------
# building blocks
# ----------------------------------------------------------------------------

def _rpad(x, p):
    return F.pad(x, (p, p, p, p), mode="reflect")


def _inorm(x):
    # per-(n,c) mean / biased var over HxW, no affine, no running stats (ir:154-165)
    return F.instance_norm(x, eps=IN_EPS)


def blur_down(x, filt):
    """Downsample: reflect pad 1 + depthwise binomial, stride 2 (ir:269-310)."""
    return F.conv2d(_rpad(x, 1), filt, stride=2, groups=x.shape[1])


def up_aa(x, filt):
    """UpsampleAA: bilinear x2 (align_corners) + reflect pad 1 + blur (ir:313-355)."""
    y = F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=True)
    return F.conv2d(_rpad(y, 1), filt, stride=1, groups=x.shape[1])


def fp8_q(t):
    """Per-tensor e4m3 fake-quantisation with the product's power-of-two scale rule
    (csrc/fp8.hip): q = 2^floor(log2(448 / max|t|)), e4m3(clamp(t * q)) / q."""
    a = float(t.detach().abs().max())
    q = 2.0 ** math.floor(math.log2(448.0 / a)) if a > 0 else 1.0
    return (t.detach() * q).clamp(-448.0, 448.0).to(torch.float8_e4m3fn).to(t.dtype) / q


class _Fp8ResConv(torch.autograd.Function):
    """The fp8 path's ResnetBlock conv (reflect pad 1, 3x3; GeneratorEngine(fp8=True)):
    forward on e4m3(x), e4m3(bf16(w)); backward-data on e4m3(dY) x e4m3(bf16(w)) over
    the padded interior, the reflect ring folded from the unquantised dY and bf16(w);
    the weight gradient on e4m3(x) x e4m3(dY) (irgan_conv_wgrad_fp8), the bias gradient
    on the unquantised dY.  Not a reference
    function: the emulation the fp8 step is checked against (ir:390-411 otherwise)."""

    @staticmethod
    def forward(ctx, x, w, b):
        wb = w.to(torch.bfloat16).to(w.dtype)
        ctx.save_for_backward(x, w, wb)
        return F.conv2d(_rpad(fp8_q(x), 1), fp8_q(wb), b)

    @staticmethod
    def backward(ctx, gy):
        x, w, wb = ctx.saved_tensors
        gq = fp8_q(gy)
        with torch.autocast("cpu", enabled=False):   # e4m3 operands: exact in fp32
            dw = torch.nn.grad.conv2d_weight(_rpad(fp8_q(x).float(), 1), w.shape, gq.float()).to(w.dtype)
        H, W = x.shape[-2:]
        xp = torch.zeros(x.shape[0], x.shape[1], H + 2, W + 2, dtype=x.dtype, device=x.device)
        g8 = torch.nn.grad.conv2d_input(xp.shape, fp8_q(wb), gq)
        gb = torch.nn.grad.conv2d_input(xp.shape, wb, gy)
        xf = torch.zeros_like(x, requires_grad=True)
        with torch.enable_grad():
            ring = torch.autograd.grad(_rpad(xf, 1), xf, gb)[0] - gb[..., 1:-1, 1:-1]
        return g8[..., 1:-1, 1:-1] + ring, dw, gy.sum(dim=(0, 2, 3))


class _Fp8ZeroConv(torch.autograd.Function):
    """The fp8 path's down2 / up1_conv (zero pad 1, 3x3; GeneratorEngine(fp8=True) with the
    anti-aliased resamplers): forward on e4m3(x) x e4m3(bf16(w)), backward-data on e4m3(dY)
    x e4m3(bf16(w)), the weight gradient on e4m3(x) x e4m3(dY), the bias gradient on the
    unquantised dY.  Not a reference function: the emulation the fp8 step is checked against
    (ir:477-482, 557-558 otherwise)."""

    @staticmethod
    def forward(ctx, x, w, b):
        wb = w.to(torch.bfloat16).to(w.dtype)
        ctx.save_for_backward(x, w, wb)
        return F.conv2d(fp8_q(x), fp8_q(wb), b, padding=1)

    @staticmethod
    def backward(ctx, gy):
        x, w, wb = ctx.saved_tensors
        gq = fp8_q(gy)
        with torch.autocast("cpu", enabled=False):   # e4m3 operands: exact in fp32
            dw = torch.nn.grad.conv2d_weight(fp8_q(x).float(), w.shape, gq.float(), padding=1).to(w.dtype)
        dx = torch.nn.grad.conv2d_input(x.shape, fp8_q(wb), gq, padding=1)
        return dx, dw, gy.sum(dim=(0, 2, 3))


def _res_conv(h, w, b, padding_type):
    """[ReflectionPad2d(1) | ReplicationPad2d(1) | -] + Conv2d(3, padding 0 | 0 | 1) (ir:380-411)."""
    if padding_type == "reflect":
        return F.conv2d(_rpad(h, 1), w, b)
    if padding_type == "replicate":
        return F.conv2d(F.pad(h, (1, 1, 1, 1), mode="replicate"), w, b)
    if padding_type == "zero":
        return F.conv2d(h, w, b, padding=1)
    raise NotImplementedError(f"Padding [{padding_type}] is not implemented")


def g_forward(P, x, no_antialias=False, no_antialias_up=False, n_blocks=9, acts=None, fp8=False, norm="instance",
              padding_type="reflect", dropout_masks=None):
    """ResnetUNetGenerator.forward (ir:533-569); returns the tanh image.
    fp8=True: the ResnetBlock convs as the fp8 path computes them (_Fp8ResConv), and with the
    anti-aliased resamplers down2 / up1_conv too (_Fp8ZeroConv).
    norm 'none': Identity norm layers and no conv biases (ir:162-163, 450-455: absent
    keys read as None).  padding_type: the ResnetBlock padding (ir:380-411).
    dropout_masks: per block a tensor of keep / (1 - p) factors multiplied after the
    ResnetBlock's ReLU -- nn.Dropout(0.5) in training mode with given masks (ir:394-395);
    None = no dropout layer or eval mode."""
    nrm = _inorm if norm == "instance" else (lambda t: t)   # noqa: E731
    bias = lambda k: P.get(k)                                # noqa: E731
    k1, k2 = res_conv_keys(padding_type, dropout_masks is not None)

    def rec(name, t):
        if acts is not None:
            acts[name] = t
        return t
    x0 = rec("x0", F.relu(nrm(F.conv2d(_rpad(x, 3), P["inc.1.weight"], bias("inc.1.bias")))))
    s = 2 if no_antialias else 1
    x1 = F.relu(nrm(F.conv2d(x0, P["down1.0.weight"], bias("down1.0.bias"), stride=s, padding=1)))
    if not no_antialias:
        x1 = blur_down(x1, P["down1_down.filt"])
    rec("x1", x1)
    fp8_ud = fp8 and not no_antialias and not no_antialias_up
    if fp8_ud:
        x2 = F.relu(nrm(_Fp8ZeroConv.apply(x1, P["down2.0.weight"], bias("down2.0.bias"))))
    else:
        x2 = F.relu(nrm(F.conv2d(x1, P["down2.0.weight"], bias("down2.0.bias"), stride=s, padding=1)))
    if not no_antialias:
        x2 = blur_down(x2, P["down2_down.filt"])
    h = rec("x2", x2)
    for b in range(n_blocks):
        pre = f"resblocks.{b}.conv_block."
        w1, b1, w2, b2 = P[f"{pre}{k1}.weight"], bias(f"{pre}{k1}.bias"), P[f"{pre}{k2}.weight"], bias(f"{pre}{k2}.bias")
        if fp8:
            t = F.relu(nrm(_Fp8ResConv.apply(h, w1, b1)))
            t = nrm(_Fp8ResConv.apply(t, w2, b2))
        else:
            t = F.relu(nrm(_res_conv(h, w1, b1, padding_type)))
            if dropout_masks is not None:
                t = t * dropout_masks[b]
            t = nrm(_res_conv(t, w2, b2, padding_type))
        h = h + t                                              # ir:417-418
    rec("x3", h)
    if no_antialias_up:
        y = F.conv_transpose2d(h, P["up1_up.weight"], bias("up1_up.bias"), stride=2,
                               padding=1, output_padding=1)    # ir:495-500
    else:
        y = up_aa(h, P["up1_up.filt"])
    if y.shape[-2:] != x1.shape[-2:]:                          # ir:555-556
        y = F.interpolate(y, size=x1.shape[-2:], mode="bilinear", align_corners=True)
    if fp8_ud:
        y = F.relu(nrm(_Fp8ZeroConv.apply(torch.cat([y, x1], 1), P["up1_conv.0.weight"], bias("up1_conv.0.bias"))))
    else:
        y = F.relu(nrm(F.conv2d(torch.cat([y, x1], 1), P["up1_conv.0.weight"],
                                bias("up1_conv.0.bias"), padding=1)))
    rec("u1", y)
    if no_antialias_up:
        y = F.conv_transpose2d(y, P["up2_up.weight"], bias("up2_up.bias"), stride=2,
                               padding=1, output_padding=1)
    else:
        y = up_aa(y, P["up2_up.filt"])
    if y.shape[-2:] != x0.shape[-2:]:
        y = F.interpolate(y, size=x0.shape[-2:], mode="bilinear", align_corners=True)
    y = F.relu(nrm(F.conv2d(torch.cat([y, x0], 1), P["up2_conv.0.weight"],
                            bias("up2_conv.0.bias"), padding=1)))
    rec("u2", y)
    return torch.tanh(F.conv2d(_rpad(y, 3), P["outc.1.weight"], P["outc.1.bias"]))


def d_forward(P, x, n_layers=3, norm="instance"):
    """NLayerDiscriminator.forward (ir:585-635): conv s2 + LReLU, n_layers - 1 conv s2 +
    norm + LReLU, conv s1 + norm + LReLU, conv s1 to one channel."""
    nrm = _inorm if norm == "instance" else (lambda t: t)   # noqa: E731
    h = F.leaky_relu(F.conv2d(x, P["model.0.weight"], P["model.0.bias"], stride=2, padding=1), LRELU)
    stages = [(2 + 3 * i, 2) for i in range(n_layers - 1)] + [(2 + 3 * (n_layers - 1), 1)]
    for idx, s in stages:
        h = F.leaky_relu(nrm(F.conv2d(h, P[f"model.{idx}.weight"], P.get(f"model.{idx}.bias"),
                                      stride=s, padding=1)), LRELU)
    last = 2 + 3 * n_layers
    return F.conv2d(h, P[f"model.{last}.weight"], P[f"model.{last}.bias"], stride=1, padding=1)


def vgg_features(V, x):
    """VGGPerceptual.forward (ir:677-683): [-1,1] -> ImageNet-normalised -> relu3_3."""
    mean = torch.tensor(IMAGENET_MEAN, dtype=x.dtype, device=x.device).view(1, 3, 1, 1)
    std = torch.tensor(IMAGENET_STD, dtype=x.dtype, device=x.device).view(1, 3, 1, 1)
    h = ((x + 1.0) / 2.0 - mean) / std
    for i, _, _ in VGG_CONVS:
        h = F.relu(F.conv2d(h, V[f"{i}.weight"], V[f"{i}.bias"], padding=1))
        if i in (2, 7):
            h = F.max_pool2d(h, 2)
    return h


def tv_loss(x):
    """Total variation (ir:686-694)."""
    return (x[:, :, 1:, :] - x[:, :, :-1, :]).abs().mean() + (x[:, :, :, 1:] - x[:, :, :, :-1]).abs().mean()


def gaussian_window(n=11, sigma=1.5, dtype=torch.float32):
    """1-D normalised Gaussian (ir:699-703)."""
    c = torch.arange(n, dtype=dtype) - (n - 1) / 2.0
    g = torch.exp(-(c ** 2) / (2 * sigma ** 2))
    return g / g.sum()


def ssim_loss(a, b, window_size=11, size_average=True):
    """1 - mean SSIM with a window_size^2 Gaussian (sigma 1.5), zero pad window_size // 2,
    C1=1e-4, C2=9e-4 (ir:714-750); size_average=False: the per-image vector (ir:746-747)."""
    c = a.shape[1]
    g = gaussian_window(window_size, 1.5, a.dtype).to(a.device)[:, None]
    w = (g @ g.t()).expand(c, 1, window_size, window_size).contiguous()
    p = window_size // 2
    blur = lambda t: F.conv2d(t, w, padding=p, groups=c)   # noqa: E731
    mu1, mu2 = blur(a), blur(b)
    s11 = blur(a * a) - mu1 * mu1
    s22 = blur(b * b) - mu2 * mu2
    s12 = blur(a * b) - mu1 * mu2
    C1, C2 = 0.01 ** 2, 0.03 ** 2
    m = ((2 * mu1 * mu2 + C1) * (2 * s12 + C2)) / ((mu1 * mu1 + mu2 * mu2 + C1) * (s11 + s22 + C2))
    return 1.0 - (m.mean() if size_average else m.mean(dim=[1, 2, 3]))


def lr_lambda(epoch, lr_decay_start_epoch=40, epochs=50):
    """LambdaLR factor (ir:212-233); epoch is 0-based as LambdaLR passes it."""
    e = epoch + 1
    if e <= lr_decay_start_epoch:
        return 1.0
    if e >= epochs:
        return 0.0
    frac = float(e - lr_decay_start_epoch) / float(max(1, epochs - lr_decay_start_epoch))
    return max(0.0, 1.0 - frac)


# ----------------------------------------------------------------------------
# optimizer + step
# ----------------------------------------------------------------------------

class AdamState:
    """torch.optim.Adam single-tensor state (ir:1601-1604: betas (0.5, 0.999), eps 1e-8)."""

    def __init__(self, params, lr=2e-4, betas=(0.5, 0.999), eps=1e-8):
        self.lr, self.b1, self.b2, self.eps = lr, betas[0], betas[1], eps
        self.step = 0
        self.m = {k: torch.zeros_like(v) for k, v in params.items()}
        self.v = {k: torch.zeros_like(v) for k, v in params.items()}


def adam_update(params, grads, st: AdamState, lr_scale=1.0):
    """One Adam step in torch's single-tensor order (lerp, addcmul, addcdiv)."""
    st.step += 1
    bc1 = 1 - st.b1 ** st.step
    bc2 = 1 - st.b2 ** st.step
    step_size = st.lr * lr_scale / bc1
    bc2s = math.sqrt(bc2)
    with torch.no_grad():
        for k, g in grads.items():
            if g is None:
                continue
            m, v = st.m[k], st.v[k]
            m.lerp_(g, 1 - st.b1)
            v.mul_(st.b2).addcmul_(g, g, value=1 - st.b2)
            denom = (v.sqrt() / bc2s).add_(st.eps)
            params[k].addcdiv_(m, denom, value=-step_size)


LAMBDAS = dict(lambda_L1=30.0, lambda_perc=30.0, lambda_tv=1e-4, lambda_ssim=2.0, lambda_gan=0.1)  # ir:100-104


def _trainable(P):
    return [k for k in P if not k.endswith(".filt")]


def train_step(G, D, V, ir, rgb, optG, optD, lam=None, no_antialias=False,
               no_antialias_up=False, n_blocks=9, grad_hook=None, fp8=False, as_written=False):
    """One train step, minimal form of ir:1636-1681.

    D step: hinge on D(cat[ir,rgb]) and D(cat[ir,G(ir)]) (G detached), D Adam.
    G step: loss = l_gan*(-mean D(cat[ir,fake])) + 30*L1 + 30*L1(VGG) + 1e-4*TV
            + 2*(1-SSIM); only G grads are taken (D is not stepped by loss_G).
    The reference runs G forward twice with identical weights (ir:1638, 1657);
    one forward is mathematically the same.  Mutates G, D, opt states.
    Returns a dict of losses, outputs and grads (for parity checks).
    ``grad_hook(name, grads)`` (name "D" or "G") may rewrite the grad dict in
    place before the Adam update -- the data-parallel tests use it to insert
    the product's gradient all-reduce.
    ``as_written=True`` does the work of ir:1636-1681 exactly as written (the CPU
    baseline's second leg): a separate no-grad G forward for the D step (ir:1638-1639),
    a second G forward for the G step (ir:1657), and loss_G.backward() also producing
    the (unused) D weight gradients, since D's parameters still require grad (ir:1680).
    Same values, more work.
    """
    lam = dict(LAMBDAS, **(lam or {}))
    out = {}
    gk = {k: G[k].detach().clone().requires_grad_(k in _trainable(G)) for k in G}
    if as_written:
        with torch.no_grad():
            fake_d = g_forward(gk, ir, no_antialias, no_antialias_up, n_blocks, fp8=fp8)
    fake = g_forward(gk, ir, no_antialias, no_antialias_up, n_blocks, fp8=fp8)
    out["fake"] = fake.detach().clone()

    # ---- D step (ir:1636-1651)
    dk = {k: D[k].detach().clone().requires_grad_(True) for k in D}
    pred_real = d_forward(dk, torch.cat([ir, rgb], 1))
    pred_fake = d_forward(dk, torch.cat([ir, (fake_d if as_written else fake).detach()], 1))
    loss_D = 0.5 * (F.relu(1.0 - pred_real).mean() + F.relu(1.0 + pred_fake).mean())
    gD = torch.autograd.grad(loss_D, [dk[k] for k in D])
    out.update(pred_real=pred_real.detach(), pred_fake=pred_fake.detach(), loss_D=loss_D.detach())
    out["gradD"] = {k: g for k, g in zip(D, gD)}
    if grad_hook is not None:
        grad_hook("D", out["gradD"])
    adam_update(D, out["gradD"], optD)

    # ---- G step (ir:1656-1681), D frozen at its updated weights
    dg = {k: D[k].detach().clone().requires_grad_(True) for k in D} if as_written else D
    pred_fake_G = d_forward(dg, torch.cat([ir, fake], 1))
    l_gan = -pred_fake_G.mean()
    l_l1 = (fake - rgb).abs().mean() * lam["lambda_L1"]
    l_perc = (vgg_features(V, fake) - vgg_features(V, rgb)).abs().mean() * lam["lambda_perc"]
    l_tv = tv_loss(fake) * lam["lambda_tv"]
    l_ssim = ssim_loss((fake + 1.0) / 2.0, (rgb + 1.0) / 2.0) * lam["lambda_ssim"]
    loss_G = lam["lambda_gan"] * l_gan + l_l1 + l_perc + l_tv + l_ssim
    keys = _trainable(G)
    if as_written:   # loss_G.backward() also fills D's .grad (ir:1680); discarded
        gG = torch.autograd.grad(loss_G, [gk[k] for k in keys] + [dg[k] for k in D])[:len(keys)]
    else:
        gG = torch.autograd.grad(loss_G, [gk[k] for k in keys])
    out.update(pred_fake_G=pred_fake_G.detach(), loss_G=loss_G.detach(), loss_G_GAN=l_gan.detach(),
               loss_G_L1=l_l1.detach(), loss_G_perc=l_perc.detach(), loss_G_TV=l_tv.detach(),
               loss_G_ssim=l_ssim.detach())
    out["gradG"] = {k: g for k, g in zip(keys, gG)}
    if grad_hook is not None:
        grad_hook("G", out["gradG"])
    adam_update(G, out["gradG"], optG)
    return out
