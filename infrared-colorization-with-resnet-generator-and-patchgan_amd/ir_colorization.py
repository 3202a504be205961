"""Public API: the reference's names and signatures, backed by the HIP engine.

Mirrors /root/reference/Code/ir_colorization.py (cited ir:LINE) for the hot
path and the pieces a train/test driver touches:

    Config (ir:32-142), get_norm_layer (ir:154), init_weights / init_net
    (ir:168-209), get_lr_lambda (ir:212), get_filter (ir:240),
    ResnetUNetGenerator (ir:425), NLayerDiscriminator (ir:576),
    VGGPerceptual (ir:642), tv_loss (ir:686), ssim_loss_torch (ir:714),
    IRColorizationModel (ir:757), validate_kaist (ir:1521), train_kaist (ir:1549),
    and the test-mode names re-exported from inference.py / evaluation.py:
    ir_to_tensor, tensor_to_rgb_image, compute_metrics, save_best_k_outputs,
    make_comparison_collage, save_comparison_image, run_test (ir:855-1514)

Modules keep the reference ``state_dict`` keys and OIHW shapes (checkpoints
``netG_*.pth`` load unchanged), but their parameters are views into flat
device buffers used by the HIP kernels; forward/backward always run on the
GPU kernels (autograd.Function wrappers), and there is no CPU fallback.
``GANTrainer.step`` is the fused train step used by ``train_kaist`` and
``bench.py``.
"""
from __future__ import annotations

import functools
import math
import os
import random
import time

import numpy as np
import torch
import torch.nn as nn

from . import ops
from .engine import (Buffers, DiscriminatorEngine, GANStep, GeneratorEngine, ParamStore, VGGEngine, d_layers,
                     d_param_shapes, g_param_shapes, res_conv_keys, vgg_param_shapes)
from .ops import BF16, F32, Feat

__all__ = ["Config", "Identity", "get_norm_layer", "init_weights", "init_net", "get_lr_lambda", "get_filter",
           "ResnetUNetGenerator", "NLayerDiscriminator", "VGGPerceptual", "tv_loss", "ssim_loss_torch",
           "IRColorizationModel", "GANTrainer", "validate_kaist", "train_kaist", "SyntheticPairDataset",
           "g_param_shapes", "d_param_shapes", "vgg_param_shapes", "seeded_state", "dp_loaders", "val_shard",
           "compute_metrics", "save_best_k_outputs", "run_test", "make_comparison_collage", "save_comparison_image",
           "float01_to_uint8_rgb", "save_rgb", "ir_to_tensor", "tensor_to_rgb_image", "HAVE_SKIMAGE", "main"]


# =============================================================================
# 0) Configuration (ir:32-142) -- same attribute names and defaults
# =============================================================================

class Config:
    def __init__(self):
        self.mode = "test"
        self.device = "cuda" if torch.cuda.is_available() else "cpu"
        self.img_size = 256
        self.input_nc = 1
        self.output_nc = 3
        self.ngf = 64
        self.norm = "instance"
        self.no_antialias = False
        self.no_antialias_up = False
        self.save_every = 5
        self.save_dir = os.path.join(".", "Weights", "trained_w_night", "checkpoints_kaist")
        self.output_dir = os.path.join(".", "results")
        self.test_G_weights = os.path.join(self.save_dir, "netG_best.pth")
        self.train_roots = [os.path.join("kaist-dataset", "versions", "1", s) for s in ("set00", "set01", "set03", "set04")]
        self.kaist_root = self.train_roots[0]
        self.batch_size = 4
        self.epochs = 50
        self.lr_G = 2e-4
        self.lr_D = 2e-4
        self.beta1 = 0.5
        self.beta2 = 0.999
        self.lambda_L1 = 30.0
        self.lambda_perc = 30.0
        self.lambda_tv = 1e-4
        self.lambda_ssim = 2.0
        self.lambda_gan = 0.1
        self.num_workers = 4
        self.val_ratio = 0.1
        self.lr_decay_start_epoch = 40
        self.init_G_weights = None
        self.test_roots = [os.path.join("kaist-dataset", "versions", "1", s) for s in ("set02", "set05")]
        self.save_comparisons = True
        self.comparison_dirname = "Comparisons"
        self.comparison_add_text = False
        self.comparison_pad = 8
        self.comparison_font_scale = 0.6
        self.comparison_thickness = 2
        self.best50_copy_preds = True
        self.best50_copy_collages = True
        self.best50_preds_subdir = "colored"
        self.best50_collages_subdir = "collages"
        self.topk = 50
        self.best50_dirname = "Best_50_colored_images"
        # --- MI355X additions (new names only; nothing above is renamed)
        self.compute_dtype = "bf16"      # "bf16" (MFMA bf16, fp32 accumulate), "fp8" (bf16 + e4m3 ResnetBlock
                                         # convs, BASELINE config 5) or "fp32" (exact parity mode)
        self.vgg_weights = None          # local path to vgg16 features weights (ImageNet); None -> seeded synthetic
        self.vgg_seed = 3
        self.log_every = 50
        self.test_batch = 16             # run_test: frames per generator call (the reference runs one)
        self.deterministic = False       # ops.set_deterministic: bitwise-reproducible weight gradients


# =============================================================================
# 1) helpers (ir:148-266)
# =============================================================================

class Identity(nn.Module):
    def forward(self, x):
        return x


def get_norm_layer(norm_type="instance"):
    """ir:154-165.  The HIP path implements 'instance' (the reference default)."""
    if norm_type == "batch":
        return nn.BatchNorm2d
    if norm_type == "instance":
        return nn.InstanceNorm2d
    if norm_type == "none" or norm_type is None:
        return lambda num_features: Identity()
    raise NotImplementedError(f"Normalization type [{norm_type}] not supported")


def _norm_name(norm_layer):
    """The engine norm for a reference norm_layer (ir:154-165): nn.InstanceNorm2d ->
    'instance', get_norm_layer('none')'s Identity factory -> 'none'.  nn.BatchNorm2d
    needs cross-sample statistics (SyncBN under data parallelism): out of scope."""
    f = norm_layer.func if isinstance(norm_layer, functools.partial) else norm_layer
    if f is nn.InstanceNorm2d:
        return "instance"
    if f is nn.BatchNorm2d:
        raise NotImplementedError("norm='batch' is out of scope for the HIP engines (SURVEY.md 8e); "
                                  "use 'instance' (the reference default) or 'none'")
    try:
        probe = norm_layer(4)
    except Exception:
        probe = None
    if isinstance(probe, (Identity, nn.Identity)):
        return "none"
    raise NotImplementedError(f"unsupported norm_layer {norm_layer!r}")


def init_weights(net, init_type="normal", init_gain=0.02, generator=None):
    """ir:168-198: conv weights ~ N(0, gain) (normal), bias 0.  Writes through the
    OIHW parameter views into the flat device buffers."""
    with torch.no_grad():
        for name, p in net.named_parameters():
            if name.endswith(".weight") and p.dim() == 4:
                w = torch.empty(p.shape)
                if init_type == "normal":
                    w.normal_(0.0, init_gain, generator=generator)
                elif init_type == "xavier":
                    nn.init.xavier_normal_(w, gain=init_gain)
                elif init_type == "kaiming":
                    nn.init.kaiming_normal_(w, a=0, mode="fan_in")
                elif init_type == "orthogonal":
                    nn.init.orthogonal_(w, gain=init_gain)
                else:
                    raise NotImplementedError(f"init method [{init_type}] is not implemented")
                p.copy_(w)
            elif name.endswith(".bias"):
                p.zero_()
    if hasattr(net, "repack"):
        net.repack()


def init_net(net, init_type="normal", init_gain=0.02, device=None, initialize_weights=True):
    """ir:201-209 (the network is created on its device already)."""
    if initialize_weights:
        init_weights(net, init_type, init_gain)
    return net


def get_lr_lambda(cfg: Config):
    """ir:212-233."""
    def lr_lambda(epoch):
        e = epoch + 1
        if e <= cfg.lr_decay_start_epoch:
            return 1.0
        if e >= cfg.epochs:
            return 0.0
        frac = float(e - cfg.lr_decay_start_epoch) / float(max(1, cfg.epochs - cfg.lr_decay_start_epoch))
        return max(0.0, 1.0 - frac)
    return lr_lambda


def get_filter(filt_size=3):
    """ir:240-266 binomial filter."""
    rows = {1: [1.], 2: [1., 1.], 3: [1., 2., 1.], 4: [1., 3., 3., 1.], 5: [1., 4., 6., 4., 1.],
            6: [1., 5., 10., 10., 5., 1.], 7: [1., 6., 15., 20., 15., 6., 1.]}
    if filt_size not in rows:
        raise ValueError("filt_size must be 1-7")
    a = np.array(rows[filt_size], dtype=np.float32)
    f = a[:, None] * a[None, :]
    return torch.from_numpy(f / f.sum())


def seeded_state(shapes, seed, weight_std=0.02, bias_std=0.0, kaiming=False):
    """Deterministic OIHW state dict from a seed (same spec as the test oracle)."""
    g = torch.Generator().manual_seed(seed)
    out = {}
    for k, shp in shapes.items():
        if k.endswith(".filt"):
            out[k] = get_filter(shp[-1])[None, None].repeat(shp[0], 1, 1, 1).contiguous()
        elif len(shp) == 4:
            std = math.sqrt(2.0 / (shp[1] * shp[2] * shp[3])) if kaiming else weight_std
            out[k] = torch.randn(shp, generator=g) * std
        else:
            out[k] = torch.randn(shp, generator=g) * bias_std if bias_std else torch.zeros(shp)
    return out


def _require_cuda(t: torch.Tensor, what: str):
    if not t.is_cuda:
        raise RuntimeError(f"{what}: the MI355X path runs only on HIP device tensors (got {t.device}); "
                           "there is no CPU fallback")


def _dtype_code(name):
    """compute_dtype -> engine dtype.  "fp8": the bf16 engines with the generator's
    ResnetBlock convs on e4m3 operands (GeneratorEngine(fp8=True))."""
    return {"bf16": BF16, "fp8": BF16, "fp32": F32, "f32": F32}[name]


# =============================================================================
# module skeletons with reference state_dict keys
# =============================================================================

class _Slot(nn.Module):
    """Holds the weight/bias Parameters (OIHW views into a ParamStore)."""

    def __init__(self, store: ParamStore, key: str):
        super().__init__()
        self.weight = nn.Parameter(store.oihw(key + ".weight"))
        if key + ".bias" in store.shapes:   # use_bias (ir:450-455, 588-593)
            self.bias = nn.Parameter(store.oihw(key + ".bias"))


class _Filt(nn.Module):
    def __init__(self, channels, device):
        super().__init__()
        self.register_buffer("filt", get_filter(3)[None, None].repeat(channels, 1, 1, 1).to(device))


def _seq(*mods):
    return nn.Sequential(*[m if m is not None else nn.Identity() for m in mods])


class _StoreModule(nn.Module):
    """Common plumbing: device pinning, grad views, repack after external writes."""

    def _apply(self, fn, recurse=True):  # .to()/.cuda()/.float() must not detach params from the store
        probe = fn(torch.zeros(1, device=self.store.device))
        if probe.device != self.store.device or probe.dtype != torch.float32:
            raise RuntimeError("MI355X modules live on their HIP device in fp32 master precision; "
                               "pick the compute dtype with Config.compute_dtype instead of .to()")
        return self

    def _load_from_state_dict(self, *args, **kw):
        super()._load_from_state_dict(*args, **kw)
        self._dirty = True

    def repack(self):
        self.engine.pack()
        self._dirty = False

    def _maybe_repack(self):
        if getattr(self, "_dirty", True):
            self.repack()

    def flat_grad_to_params(self):
        """Expose the flat gradient buffer as .grad of the OIHW parameters."""
        for k, p in self.named_parameters():
            p.grad = self.store.oihw(k, self.store.grad)


# =============================================================================
# 3-4) Generator (ir:425-569)
# =============================================================================

# Every autograd-recorded forward below runs on its OWN engine buffer set
# (engine.Buffers), held by its ctx until the backward: the reference interleaves
# calls before one backward (netD(real), netD(fake), loss_D.backward() ir:1642-1650;
# vgg_perc(fake), vgg_perc(rgb) ir:1667-1668), so each call must back-propagate
# through its own activations, ReLU/LReLU masks, maxpool argmaxes and IN statistics.

class _GFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mod, *params):
        bufs = Buffers(x.device)
        fake = mod.engine.forward(x.float(), bufs=bufs)
        ctx.mod, ctx.bufs = mod, bufs
        out = torch.empty(fake.shape[0], fake.shape[3], fake.shape[1], fake.shape[2], device=x.device)
        ops.nhwc_to_nchw(Feat(fake), out)
        return out

    @staticmethod
    def backward(ctx, dout):
        mod, bufs = ctx.mod, ctx.bufs
        ctx.bufs = None
        dnhwc = torch.empty(dout.shape[0], dout.shape[2], dout.shape[3], dout.shape[1], device=dout.device)
        ops.nchw_to_nhwc(dout.contiguous().float(), Feat(dnhwc))
        mod.store.zero_grad()
        mod.engine.backward(dnhwc, bufs=bufs)
        grads = [mod.store.oihw(k, mod.store.grad).clone() for k, _ in mod.named_parameters()]
        return (None, None, *grads)


class ResnetUNetGenerator(_StoreModule):
    """ir:425-569.  forward(x) -> (out, None).  Input (B, input_nc, H, W) in
    [-1,1] on the HIP device, any H, W >= 2: when H or W is not divisible by 4 the
    decoder resizes the up-sampled map to the skip's size as the reference does
    (ir:555-556, 562-563)."""

    def __init__(self, input_nc, output_nc, ngf=64, norm_layer=nn.InstanceNorm2d, use_dropout=False, n_blocks=9,
                 padding_type="reflect", no_antialias=False, no_antialias_up=False, device=None,
                 compute_dtype="bf16"):
        super().__init__()
        assert n_blocks >= 0
        norm = _norm_name(norm_layer)
        k1, k2 = res_conv_keys(padding_type, use_dropout)   # raises on an unknown padding (ir:380-386)
        device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
        self.store = ParamStore(g_param_shapes(input_nc, output_nc, ngf, n_blocks, no_antialias, no_antialias_up,
                                               use_bias=norm == "instance", padding_type=padding_type,
                                               use_dropout=use_dropout), device)
        S = self.store
        self.inc = _seq(None, _Slot(S, "inc.1"), None, None)
        self.down1 = _seq(_Slot(S, "down1.0"), None, None)
        self.down1_down = None if no_antialias else _Filt(2 * ngf, device)
        self.down2 = _seq(_Slot(S, "down2.0"), None, None)
        self.down2_down = None if no_antialias else _Filt(4 * ngf, device)
        blocks = []
        nmods = k2 + 2   # [pad] conv norm relu [dropout] [pad] conv norm (ir:375-411)
        for b in range(n_blocks):
            blk = nn.Module()
            blk.conv_block = _seq(*[_Slot(S, f"resblocks.{b}.conv_block.{i}") if i in (k1, k2) else None
                                    for i in range(nmods)])
            blocks.append(blk)
        self.resblocks = nn.Sequential(*blocks)
        self.up1_up = _Slot(S, "up1_up") if no_antialias_up else _Filt(4 * ngf, device)
        self.up1_conv = _seq(_Slot(S, "up1_conv.0"), None, None)
        self.up2_up = _Slot(S, "up2_up") if no_antialias_up else _Filt(2 * ngf, device)
        self.up2_conv = _seq(_Slot(S, "up2_conv.0"), None, None)
        self.outc = _seq(None, _Slot(S, "outc.1"), None)
        self.engine = GeneratorEngine(S, _dtype_code(compute_dtype), ngf=ngf, input_nc=input_nc,
                                      output_nc=output_nc, n_blocks=n_blocks, no_antialias=no_antialias,
                                      no_antialias_up=no_antialias_up, fp8=compute_dtype == "fp8", norm=norm,
                                      padding_type=padding_type, use_dropout=use_dropout)
        self._dirty = True

    def forward(self, x, layers=None, encode_only=False):
        _require_cuda(x, "ResnetUNetGenerator")
        self.repack()  # parameters may have been changed in place by any optimizer
        self.engine.training = self.training   # nn.Dropout follows train() / eval() (ir:394-395)
        params = [p for _, p in self.named_parameters()]
        if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in params)):
            return _GFn.apply(x, self, *params), None
        fake = self.engine.forward(x.float())
        out = torch.empty(fake.shape[0], fake.shape[3], fake.shape[1], fake.shape[2], device=x.device)
        ops.nhwc_to_nchw(Feat(fake), out)
        return out, None


# =============================================================================
# 5) Discriminator (ir:576-635)
# =============================================================================

def _nhwc_input(x, pc, tdt, scale=None, shift=None):
    """NCHW fp32 -> NHWC compute-dtype conv input, narrow channels zero-padded to 8."""
    B, C, H, W = x.shape
    buf = torch.zeros(B, H, W, max(8, C), device=x.device, dtype=tdt)
    ops.nchw_to_nhwc(x.contiguous().float(), Feat(buf, 0, C), scale, shift)
    return Feat(buf, 0, pc.cin_eff)


class _DFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mod, *params):
        bufs = Buffers(x.device)
        out = mod.engine.forward(_nhwc_input(x, mod.engine.packs[0], mod.engine.tdt), tag="api", bufs=bufs)
        ctx.mod, ctx.bufs = mod, bufs
        return out.permute(0, 3, 1, 2).contiguous()

    @staticmethod
    def backward(ctx, dout):
        mod, bufs = ctx.mod, ctx.bufs
        ctx.bufs = None
        mod.store.zero_grad()
        dn = dout.permute(0, 2, 3, 1).contiguous().float()
        dx = mod.engine.backward(dn, want_wgrad=True, want_dinput=True, tag="api", bufs=bufs)
        B, H, W, C = dx.t.shape
        gx = torch.empty(B, C, H, W, device=dout.device)
        ops.nhwc_to_nchw(dx, gx)
        grads = [mod.store.oihw(k, mod.store.grad).clone() for k, _ in mod.named_parameters()]
        return (gx, None, *grads)


class NLayerDiscriminator(_StoreModule):
    """ir:576-635: any n_layers >= 1 (train_kaist builds 3), norm 'instance' or 'none'."""

    def __init__(self, input_nc, ndf=64, n_layers=3, norm_layer=nn.InstanceNorm2d, device=None,
                 compute_dtype="bf16"):
        super().__init__()
        assert n_layers >= 1
        norm = _norm_name(norm_layer)
        device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
        self.store = ParamStore(d_param_shapes(input_nc, ndf, n_layers, use_bias=norm == "instance"), device)
        S = self.store
        keys = [k for k, _, _ in d_layers(n_layers)]
        last = int(keys[-1].split(".")[1])
        self.model = _seq(*[_Slot(S, f"model.{i}") if f"model.{i}" in keys else None for i in range(last + 1)])
        self.engine = DiscriminatorEngine(S, _dtype_code(compute_dtype), input_nc=input_nc, ndf=ndf,
                                          n_layers=n_layers, norm=norm)
        self._dirty = True

    def forward(self, x):
        _require_cuda(x, "NLayerDiscriminator")
        self.repack()
        params = [p for _, p in self.named_parameters()]
        if torch.is_grad_enabled():
            return _DFn.apply(x, self, *params)
        din = _nhwc_input(x, self.engine.packs[0], self.engine.tdt)
        return self.engine.forward(din, tag="api").permute(0, 3, 1, 2).contiguous()


# =============================================================================
# 6) Perceptual / TV / SSIM losses (ir:642-750)
# =============================================================================

class _VFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mod):
        bufs = Buffers(x.device)
        feat = mod._features(x, bufs)
        ctx.mod, ctx.bufs = mod, bufs
        ctx.n = x.shape[0]
        return feat.t.permute(0, 3, 1, 2).float().contiguous()

    @staticmethod
    def backward(ctx, dfeat):
        mod, bufs = ctx.mod, ctx.bufs
        ctx.bufs = None
        dn = dfeat.permute(0, 2, 3, 1).contiguous().to(mod.engine.tdt)
        dv = mod.engine.backward_input(Feat(dn), ctx.n, bufs=bufs)
        dimg = torch.zeros(dv.N, dv.H, dv.W, dv.C, device=dfeat.device)
        ops.affine(dv, mod.engine.scale, None, Feat(dimg))
        out = torch.empty(dv.N, dv.C, dv.H, dv.W, device=dfeat.device)
        ops.nhwc_to_nchw(Feat(dimg), out)
        return out, None


class VGGPerceptual(_StoreModule):
    """ir:642-683: frozen VGG-16 features[:16] on ImageNet-normalised input.

    ImageNet weights cannot be downloaded here: pass ``weights`` (a local
    state_dict path or dict with keys '0.weight'...'14.bias' or
    'features.N.*') or get the seeded synthetic stack (``seed``)."""

    def __init__(self, device=None, weights=None, seed=3, compute_dtype="bf16"):
        super().__init__()
        device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
        self.store = ParamStore(vgg_param_shapes(), device, with_grad=False, with_adam=False)
        if weights is None:
            self.store.load(seeded_state(vgg_param_shapes(), seed, kaiming=True), strict=True)
        else:
            sd = torch.load(weights, map_location="cpu", weights_only=True) if isinstance(weights, str) else weights
            sd = {k[len("features."):] if k.startswith("features.") else k: v for k, v in sd.items()}
            self.store.load(sd, strict=True)
        S = self.store
        mods = []
        for i in range(16):
            mods.append(_Slot(S, str(i)) if f"{i}.weight" in S.shapes else None)
        self.features = _seq(*mods)
        for p in self.features.parameters():
            p.requires_grad = False
        self.register_buffer("mean", torch.tensor([0.485, 0.456, 0.406], device=device).view(1, 3, 1, 1))
        self.register_buffer("std", torch.tensor([0.229, 0.224, 0.225], device=device).view(1, 3, 1, 1))
        self.engine = VGGEngine(S, _dtype_code(compute_dtype))
        self._dirty = True

    def _features(self, x, bufs=None):
        _require_cuda(x, "VGGPerceptual")
        self._maybe_repack()
        vin = _nhwc_input(x, self.engine.packs[0], self.engine.tdt, self.engine.scale, self.engine.shift)
        return self.engine.forward(vin, bufs=bufs)

    def forward(self, x):
        if torch.is_grad_enabled() and x.requires_grad:
            return _VFn.apply(x, self)
        return self._features(x).t.permute(0, 3, 1, 2).float().contiguous()


def _nhwc32(x):
    B, C, H, W = x.shape
    t = torch.empty(B, H, W, C, device=x.device)
    ops.nchw_to_nhwc(x.contiguous().float(), Feat(t))
    return t


class _TVFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        xn = _nhwc32(x)
        g = torch.zeros_like(xn)
        loss = torch.zeros(1, dtype=torch.float64, device=x.device)
        ops.tv(Feat(xn), 1.0, g, loss)
        ctx.save_for_backward(g)
        return loss.float()[0]

    @staticmethod
    def backward(ctx, gl):
        (g,) = ctx.saved_tensors
        out = torch.empty(g.shape[0], g.shape[3], g.shape[1], g.shape[2], device=g.device)
        ops.nhwc_to_nchw(Feat(g), out)
        return out * gl


def tv_loss(x):
    """ir:686-694 on the HIP kernel."""
    _require_cuda(x, "tv_loss")
    return _TVFn.apply(x)


class _SSIMFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, size_average, window):
        # kernel takes [-1,1] images and maps (x+1)/2 itself; feed 2x-1 of the [0,1] inputs
        an, bn = _nhwc32(a * 2 - 1), _nhwc32(b * 2 - 1)
        g = torch.zeros_like(an)
        if size_average:   # 1 - mean over B*C*H*W (ir:744-745): one launch over the batch
            loss = torch.zeros(1, dtype=torch.float64, device=a.device)
            work = torch.empty(10 * an.numel(), device=a.device)
            ops.ssim(Feat(an), Feat(bn), 1.0, g, loss, work, window)
        else:              # 1 - per-image mean over C*H*W (ir:746-747): one launch per image
            B = an.shape[0]
            loss = torch.zeros(B, dtype=torch.float64, device=a.device)
            work = torch.empty(10 * an[0].numel(), device=a.device)
            for i in range(B):
                ops.ssim(Feat(an[i:i + 1]), Feat(bn[i:i + 1]), 1.0, g[i:i + 1], loss[i:i + 1], work, window)
        ctx.save_for_backward(g)
        ctx.size_average = size_average
        out = loss.float()
        return out[0] if size_average else out

    @staticmethod
    def backward(ctx, gl):
        (g,) = ctx.saved_tensors
        out = torch.empty(g.shape[0], g.shape[3], g.shape[1], g.shape[2], device=g.device)
        ops.nhwc_to_nchw(Feat(g), out, scale=2.0)  # d/d(img01) = 2 * d/d(img[-1,1])
        if not ctx.size_average:
            gl = gl.view(-1, 1, 1, 1)
        return out * gl, None, None, None


def ssim_loss_torch(img1, img2, window_size=11, size_average=True):
    """ir:714-750: 1 - SSIM of [0,1] images (window_size^2 Gaussian, sigma 1.5, zero
    padding window_size // 2); a scalar, or with size_average=False the per-image
    vector (B,) of ir:746-747.  Odd window sizes 1..15 (default 11)."""
    assert img1.shape == img2.shape, "SSIM images must have the same shape"
    if window_size % 2 == 0 or not 1 <= window_size <= 15:
        raise NotImplementedError("HIP SSIM implements odd window sizes 1..15 (an even window's padding changes "
                                  "the map size)")
    _require_cuda(img1, "ssim_loss_torch")
    return _SSIMFn.apply(img1, img2, bool(size_average), int(window_size))


# =============================================================================
# 7) Model wrapper (ir:757-796)
# =============================================================================

class IRColorizationModel(nn.Module):
    def __init__(self, cfg: Config):
        super().__init__()
        norm_layer = get_norm_layer(cfg.norm)
        self.device = torch.device(cfg.device)
        self.netG = ResnetUNetGenerator(cfg.input_nc, cfg.output_nc, cfg.ngf, norm_layer=norm_layer,
                                        use_dropout=False, n_blocks=9, padding_type="reflect",
                                        no_antialias=cfg.no_antialias, no_antialias_up=cfg.no_antialias_up,
                                        device=self.device, compute_dtype=getattr(cfg, "compute_dtype", "bf16"))
        init_net(self.netG, init_type="normal", init_gain=0.02, device=self.device, initialize_weights=True)

    def load_weights(self, path):
        """Raw state_dict or {'state_dict': ...}, strict=False (ir:781-789)."""
        state = torch.load(path, map_location="cpu", weights_only=True)
        if isinstance(state, dict) and "state_dict" in state:
            state = state["state_dict"]
        self.netG.load_state_dict(state, strict=False)
        self.netG.repack()

    def forward(self, ir_tensor):
        fake_b, _ = self.netG(ir_tensor)
        return fake_b


# =============================================================================
# fused train step (the hot path) + train / validation drivers (ir:1521-1723)
# =============================================================================

class GANTrainer:
    """Owns G (through the model), D, VGG and both Adams; ``step(ir, rgb)`` runs
    the fused HIP train step and returns the device loss vector (no host sync)."""

    def __init__(self, cfg: Config, model: IRColorizationModel = None, netD: NLayerDiscriminator = None,
                 vgg: VGGPerceptual = None, process_group=None, force_reduce=False):
        """force_reduce: the data-parallel gradient collectives run even at world size 1
        (engine.BucketedAllreduce; needs an initialised process group)."""
        self.cfg = cfg
        dev = torch.device(cfg.device)
        dt = getattr(cfg, "compute_dtype", "bf16")
        if getattr(cfg, "deterministic", False):
            ops.set_deterministic(True)
        self.model = model or IRColorizationModel(cfg)
        self.netD = netD or init_net(NLayerDiscriminator(cfg.input_nc + cfg.output_nc, 64, 3,
                                                         get_norm_layer(cfg.norm), device=dev, compute_dtype=dt))
        self.vgg = vgg or VGGPerceptual(dev, weights=getattr(cfg, "vgg_weights", None),
                                        seed=getattr(cfg, "vgg_seed", 3), compute_dtype=dt)
        self.netG = self.model.netG
        self.netG._maybe_repack()
        self.netD._maybe_repack()
        self.vgg._maybe_repack()
        # the fused step drives the networks' own engines (shared packed weights / buffers)
        self.core = GANStep(self.netG.store, self.netD.store, self.vgg.store, cfg, _dtype_code(dt),
                            process_group=process_group, gen=self.netG.engine, dis=self.netD.engine,
                            vgg=self.vgg.engine, force_reduce=force_reduce)
        self.lr_lambda = get_lr_lambda(cfg)
        self.epoch_index = 0

    def step(self, ir, rgb):
        _require_cuda(ir, "GANTrainer.step")
        return self.core.step(ir, rgb)

    def losses(self, L):
        return GANStep.loss_dict(L, self.cfg)

    def scheduler_step(self):
        """Both LambdaLR schedulers (ir:1718-1719)."""
        self.epoch_index += 1
        self.core.lr_scale = self.lr_lambda(self.epoch_index)

    @property
    def current_lr_G(self):
        return self.cfg.lr_G * self.core.lr_scale

    # ---- full training state.  The reference checkpoints G only
    # (ir:1708); this adds D, both Adams (torch.optim.Adam.state_dict() layout) and
    # the LambdaLR position, so an interrupted run resumes bit-exactly.
    def state_dict(self):
        c, s = self.cfg, self.core
        return {"netG": {k: v.detach().cpu().clone() for k, v in self.netG.store.state().items()},
                "netD": {k: v.detach().cpu().clone() for k, v in self.netD.store.state().items()},
                "optimizer_G": self.netG.store.adam_state_dict(c.lr_G * s.lr_scale, (c.beta1, c.beta2), 1e-8, c.lr_G),
                "optimizer_D": self.netD.store.adam_state_dict(c.lr_D * s.lr_scale, (c.beta1, c.beta2), 1e-8, c.lr_D),
                "epoch_index": self.epoch_index, "lr_scale": s.lr_scale}

    def load_state_dict(self, sd):
        self.netG.store.load(sd["netG"], strict=True)
        self.netD.store.load(sd["netD"], strict=True)
        self.netG.store.load_adam_state_dict(sd["optimizer_G"])
        self.netD.store.load_adam_state_dict(sd["optimizer_D"])
        self.epoch_index = int(sd["epoch_index"])
        self.core.lr_scale = float(sd["lr_scale"])
        for net in (self.netG, self.netD):
            net.repack()

    def save_checkpoint(self, path):
        torch.save(self.state_dict(), path)

    def load_checkpoint(self, path):
        self.load_state_dict(torch.load(path, map_location="cpu", weights_only=True))


def _dp():
    """(rank, world) of the data-parallel job, (0, 1) when not distributed."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


@torch.no_grad()
def validate_kaist(model: IRColorizationModel, val_loader, device):
    """ir:1521-1542 (under no_grad, ir:1532): batch-size-weighted mean L1 of G(ir)
    vs rgb.  Under data parallelism each rank scores its val shard (disjoint, no
    padding duplicates: dp_loaders) and (sum, count) is all-reduced."""
    total, count = 0.0, 0
    mode = hasattr(model, "eval")   # an nn.Module (a bare callable has no train/eval state)
    if mode:
        model.eval()   # ir:1527
    with torch.no_grad():
        for batch in val_loader:
            ir = batch["ir"].to(device)
            rgb = batch["rgb"].to(device)
            fake = model(ir)
            total += float((fake - rgb).abs().mean()) * ir.size(0)
            count += ir.size(0)
    if mode:
        model.train()  # ir:1541
    rank, world = _dp()
    if world > 1:
        import torch.distributed as dist
        dev = device if dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([total, float(count)], dtype=torch.float64, device=dev)
        dist.all_reduce(t)
        total, count = float(t[0]), int(t[1])
    return total / max(count, 1)


def dp_loaders(train_ds, val_ds, batch_size, seed=0):
    """Train/val loaders (ir:1575-1581).  With world > 1 every rank gets an equal
    shard of whole per-rank batches (DistributedSampler, drop_last) so that the
    gradient all-reduce (engine.BucketedAllreduce) averages equal-sized batch means:
    ``batch_size`` is per rank, the global batch is batch_size * world."""
    rank, world = _dp()
    if world == 1:
        tl = torch.utils.data.DataLoader(train_ds, batch_size=batch_size, shuffle=True, num_workers=0,
                                         pin_memory=True, drop_last=True)
        vl = torch.utils.data.DataLoader(val_ds, batch_size=batch_size, shuffle=False, num_workers=0,
                                         pin_memory=True, drop_last=False)
        return tl, vl, None
    from torch.utils.data.distributed import DistributedSampler
    ts = DistributedSampler(train_ds, num_replicas=world, rank=rank, shuffle=True, seed=seed, drop_last=True)
    tl = torch.utils.data.DataLoader(train_ds, batch_size=batch_size, sampler=ts, num_workers=0,
                                     pin_memory=True, drop_last=True)
    # validation: a strided, disjoint shard per rank WITHOUT DistributedSampler's
    # padding duplicates, so the all-reduced (sum, count) is exactly the
    # single-process val L1 (ir:1538-1542) whatever len(val) % world is
    vl = torch.utils.data.DataLoader(val_shard(val_ds, rank, world), batch_size=batch_size, shuffle=False,
                                     num_workers=0, pin_memory=True, drop_last=False)
    return tl, vl, ts


def val_shard(val_ds, rank, world):
    """Rank ``rank``'s disjoint strided share of the validation set (no padding)."""
    return torch.utils.data.Subset(val_ds, list(range(rank, len(val_ds), world)))


class SyntheticPairDataset(torch.utils.data.Dataset):
    """KAISTPairDataset item contract (ir:1171-1177): {'ir': 1xHxW, 'rgb': 3xHxW}
    in [-1,1]; seeded uniform data (the KAIST dataset is not shipped)."""

    def __init__(self, n, img_size=256, seed=7, input_nc=1, output_nc=3):
        g = torch.Generator().manual_seed(seed)
        self.ir = torch.rand(n, input_nc, img_size, img_size, generator=g) * 2 - 1
        self.rgb = torch.rand(n, output_nc, img_size, img_size, generator=g) * 2 - 1

    def __len__(self):
        return self.ir.shape[0]

    def __getitem__(self, i):
        return {"ir": self.ir[i], "rgb": self.rgb[i]}


def train_kaist(cfg: Config, dataset=None, log=print, trainer_hook=None):
    """ir:1549-1723 with the fused HIP step.  ``dataset=None`` trains on the KAIST
    pairs under ``cfg.train_roots`` (data.KAISTPairDataset: decode on the host,
    INTER_AREA resize + paired flip + normalisation on the device); any dataset
    yielding {'ir','rgb'} (e.g. SyntheticPairDataset) may be passed instead.
    ``trainer_hook(trainer)`` (optional) runs once after the networks are built
    (e.g. to load D / VGG weights from files)."""
    device = torch.device(cfg.device)
    log(f"[TRAIN] Device: {device}")
    log(f"KAIST root (V000, V001, ...): {cfg.kaist_root}")
    rank, world = _dp()
    if dataset is None:
        from .data import KAISTPairDataset, kaist_loader
        N = len(KAISTPairDataset(cfg.train_roots, img_size=cfg.img_size, augment=False, verbose=rank == 0))
    else:
        N = len(dataset)
    val_size = max(1, int(N * cfg.val_ratio))
    train_size = N - val_size
    log(f"Total pairs: {N}, train: {train_size}, val: {val_size}")
    idxs = list(range(N))
    random.seed(42)
    random.shuffle(idxs)
    if dataset is None:
        train_ds = KAISTPairDataset(cfg.train_roots, img_size=cfg.img_size, augment=True, indices=idxs[:train_size],
                                    verbose=rank == 0)
        val_ds = KAISTPairDataset(cfg.train_roots, img_size=cfg.img_size, augment=False,
                                  indices=idxs[train_size:][rank::world], verbose=rank == 0)
        sampler = None
        if world > 1:
            from torch.utils.data.distributed import DistributedSampler
            sampler = DistributedSampler(train_ds, num_replicas=world, rank=rank, shuffle=True, seed=0, drop_last=True)
        train_loader = kaist_loader(train_ds, cfg.batch_size, device, shuffle=True, drop_last=True,
                                    num_workers=cfg.num_workers, sampler=sampler)
        val_loader = kaist_loader(val_ds, cfg.batch_size, device, num_workers=cfg.num_workers)
    else:
        train_ds = torch.utils.data.Subset(dataset, idxs[:train_size])
        val_ds = torch.utils.data.Subset(dataset, idxs[train_size:])
        train_loader, val_loader, sampler = dp_loaders(train_ds, val_ds, cfg.batch_size)
    model = IRColorizationModel(cfg)
    if cfg.init_G_weights is not None and os.path.isfile(cfg.init_G_weights):
        log(f"Initializing generator from: {cfg.init_G_weights}")
        model.load_weights(cfg.init_G_weights)
    trainer = GANTrainer(cfg, model=model)
    if trainer_hook is not None:
        trainer_hook(trainer)
    if rank == 0:
        os.makedirs(cfg.save_dir, exist_ok=True)
    best_val = float("inf")
    best_path = os.path.join(cfg.save_dir, "netG_best.pth")
    history = []
    for epoch in range(1, cfg.epochs + 1):
        if sampler is not None:
            sampler.set_epoch(epoch)
        acc = torch.zeros(8, dtype=torch.float64, device=device)
        steps = 0
        for i, batch in enumerate(train_loader, start=1):
            ir = batch["ir"].to(device, non_blocking=True)
            rgb = batch["rgb"].to(device, non_blocking=True)
            L = trainer.step(ir, rgb)
            acc += L
            steps += 1
            if i % cfg.log_every == 0 or i == 1:
                d = trainer.losses(L)
                log(f"Epoch [{epoch}/{cfg.epochs}] Step [{i}/{len(train_loader)}] "
                    f"D: {d['loss_D']:.4f} | G: {d['loss_G']:.4f} "
                    f"(GAN {d['loss_G_GAN']:.4f} + L1 {d['loss_G_L1']:.4f} "
                    f"+ Perc {d['loss_G_perc']:.4f} + TV {d['loss_G_TV']:.6f} "
                    f"+ SSIM {d['loss_G_ssim']:.4f})")
        avg = trainer.losses(acc / max(steps, 1))
        val_l1 = validate_kaist(model, val_loader, device)
        log(f"Epoch [{epoch}/{cfg.epochs}] DONE | avg D: {avg['loss_D']:.4f} | avg G: {avg['loss_G']:.4f} | "
            f"val L1: {val_l1:.4f}")
        history.append(dict(epoch=epoch, val_l1=val_l1, **avg))
        if rank == 0 and ((epoch % cfg.save_every == 0) or (epoch == cfg.epochs)):
            path = os.path.join(cfg.save_dir, f"netG_epoch_{epoch:03d}.pth")
            torch.save(_cpu_state(model.netG), path)
            log(f"Saved generator checkpoint to {path}")
        if val_l1 < best_val:
            best_val = val_l1
            if rank == 0:
                torch.save(_cpu_state(model.netG), best_path)
            log(f"New best model saved to {best_path} (val L1={best_val:.4f})")
        trainer.scheduler_step()
        log(f"Current LR (G): {trainer.current_lr_G:.6e}")
    log(f"Training finished. Best val L1: {best_val:.4f}, best model: {best_path}")
    return history


def _cpu_state(net):
    """state_dict in the reference layout: contiguous OIHW fp32 (ir:1708)."""
    return type(net.state_dict())((k, v.detach().contiguous().cpu()) for k, v in net.state_dict().items())


# test-mode names (ir:855-1514); evaluation imports this module lazily, so bind them last
from .evaluation import (HAVE_SKIMAGE, float01_to_uint8_rgb, make_comparison_collage, run_test,  # noqa: E402
                         save_best_k_outputs, save_comparison_image, save_rgb)
from .inference import compute_metrics, ir_to_tensor, tensor_to_rgb_image  # noqa: E402


def main(cfg: Config = None, log=print):
    """ir:1730-1752: train or test according to cfg.mode (``python -m <package>``)."""
    cfg = cfg or Config()
    log(f"Config mode: {cfg.mode}")
    log(f"SAVE_DIR: {cfg.save_dir}")
    log(f"OUTPUT_DIR: {cfg.output_dir}")
    log(f"TEST_G_WEIGHTS: {cfg.test_G_weights}")
    if cfg.mode == "train":
        return train_kaist(cfg, log=log)
    if cfg.mode == "test":
        return run_test(cfg, log=log)
    raise ValueError("cfg.mode must be 'train' or 'test'")
