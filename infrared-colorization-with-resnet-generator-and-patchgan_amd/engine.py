"""The fused GAN train step on HIP kernels (the product hot path).

One ``GANStep.step(ir, rgb)`` = the reference's inner-loop body
(ir:1636-1681) in its minimal form: one G forward reused (detached) for the D
step; D forward/backward on the batched [real; fake] pair; D Adam; D forward on
fake with the updated D; hinge + L1 + VGG-perceptual + TV + SSIM losses with
their gradients written directly; G backward; G Adam.  No autograd tape: every
backward is an explicit HIP kernel sequence over activations kept in static
NHWC buffers (capturable in a HIP graph).

Parameters live in flat fp32 buffers (one per network) whose per-key slices are
KRSC conv weights; the reference's OIHW ``state_dict`` tensors are permuted
*views* of those slices (``ParamStore.oihw``), so checkpoints load/save in the
reference layout while the kernels and the single-launch Adam read the flat
buffer.  Data-parallel: each rank owns a batch shard and all-reduces the flat
gradient buffers (RCCL) before each Adam.
"""
from __future__ import annotations

import math
import os
from collections import OrderedDict
from contextlib import nullcontext as _nullcontext

import torch

from . import ops
from .ops import (ACT_LRELU, ACT_NONE, ACT_RELU, ACT_TANH, BF16, F32, PAD_REFLECT, PAD_ZERO, ConvSpec, Feat,
                  PackedConv)

IMAGENET_MEAN = (0.485, 0.456, 0.406)   # ir:672
IMAGENET_STD = (0.229, 0.224, 0.225)    # ir:673


# ----------------------------------------------------------------------------
# parameter layout (reference state_dict keys / OIHW shapes / order)
# ----------------------------------------------------------------------------

def g_param_shapes(input_nc=1, output_nc=3, ngf=64, n_blocks=9, no_antialias=False, no_antialias_up=False,
                   use_bias=True, padding_type="reflect", use_dropout=False):
    """ResnetUNetGenerator state_dict layout (ir:443-531), buffers included.  use_bias:
    the reference's ``norm_layer == nn.InstanceNorm2d`` (ir:450-455); without it (norm
    'none') every conv but outc, and the ConvTranspose2d, has no bias."""
    s = OrderedDict()

    def conv(key, shape):
        s[key + ".weight"] = shape
        if use_bias:
            s[key + ".bias"] = (shape[0],)
    conv("inc.1", (ngf, input_nc, 7, 7))
    conv("down1.0", (2 * ngf, ngf, 3, 3))
    if not no_antialias:
        s["down1_down.filt"] = (2 * ngf, 1, 3, 3)
    conv("down2.0", (4 * ngf, 2 * ngf, 3, 3))
    if not no_antialias:
        s["down2_down.filt"] = (4 * ngf, 1, 3, 3)
    for b in range(n_blocks):
        for c in res_conv_keys(padding_type, use_dropout):
            conv(f"resblocks.{b}.conv_block.{c}", (4 * ngf, 4 * ngf, 3, 3))
    for name, ch, cat in (("up1", 4 * ngf, 6 * ngf), ("up2", 2 * ngf, 3 * ngf)):
        if no_antialias_up:
            conv(f"{name}_up", (ch, ch, 3, 3))
        else:
            s[f"{name}_up.filt"] = (ch, 1, 3, 3)
        conv(f"{name}_conv.0", (ch // 2, cat, 3, 3))
    s["outc.1.weight"] = (output_nc, ngf, 7, 7); s["outc.1.bias"] = (output_nc,)
    return s


def d_layers(n_layers=3):
    """PatchGAN layer table (ir:585-632): (state key, stride, normalised) per conv.
    model.0 (s2, LeakyReLU), n_layers - 1 s2 conv/norm/LeakyReLU blocks, one s1
    conv/norm/LeakyReLU, the s1 1-channel output conv."""
    out = [("model.0", 2, False)]
    idx = 2
    for _ in range(1, n_layers):
        out.append((f"model.{idx}", 2, True))
        idx += 3
    out.append((f"model.{idx}", 1, True))
    out.append((f"model.{idx + 3}", 1, False))
    return out


def d_channels(input_nc=4, ndf=64, n_layers=3):
    """Channel counts along the PatchGAN (ir:598-632): ndf * min(2^n, 8)."""
    return [input_nc] + [ndf * min(2 ** n, 8) for n in range(n_layers + 1)] + [1]


def d_param_shapes(input_nc=4, ndf=64, n_layers=3, use_bias=True):
    """NLayerDiscriminator layout (ir:585-632); the first and last convs always carry a
    bias, the normalised ones only with InstanceNorm (use_bias, ir:588-593)."""
    s = OrderedDict()
    ch = d_channels(input_nc, ndf, n_layers)
    for i, (key, _, normed) in enumerate(d_layers(n_layers)):
        s[key + ".weight"] = (ch[i + 1], ch[i], 4, 4)
        if use_bias or not normed:
            s[key + ".bias"] = (ch[i + 1],)
    return s


VGG_CONVS = ((0, 3, 64), (2, 64, 64), (5, 64, 128), (7, 128, 128), (10, 128, 256), (12, 256, 256), (14, 256, 256))


def vgg_param_shapes():
    s = OrderedDict()
    for i, ci, co in VGG_CONVS:
        s[f"{i}.weight"] = (co, ci, 3, 3); s[f"{i}.bias"] = (co,)
    return s


class ParamStore:
    """Flat fp32 parameter / gradient / Adam-moment buffers for one network."""

    def __init__(self, shapes: "OrderedDict[str, tuple]", device, with_grad=True, with_adam=True):
        self.shapes = OrderedDict((k, tuple(v)) for k, v in shapes.items() if not k.endswith(".filt"))
        self.offsets, off = {}, 0
        for k, shp in self.shapes.items():
            self.offsets[k] = off
            off += math.prod(shp)
            off = (off + 63) // 64 * 64  # 256-byte aligned slices
        self.numel = off
        self.device = device
        self.flat = torch.zeros(off, device=device)
        self.grad = torch.zeros(off, device=device) if with_grad else None
        self.m = torch.zeros(off, device=device) if with_adam else None
        self.v = torch.zeros(off, device=device) if with_adam else None
        self.step_count = 0
        self.dev_adam = False   # GANStep: step count on the device (irgan_adam_prep)
        self._count = self._prm = None
        self._count_host = 0

    def krsc(self, k, buf=None):
        buf = self.flat if buf is None else buf
        o = self.offsets[k]
        return buf[o:o + math.prod(self.shapes[k])]

    def oihw(self, k, buf=None):
        """The reference-layout view: OIHW shape over KRSC storage."""
        shp = self.shapes[k]
        t = self.krsc(k, buf)
        if len(shp) == 4:
            O, I, KH, KW = shp
            return t.view(O, KH, KW, I).permute(0, 3, 1, 2)
        return t.view(shp)

    @torch.no_grad()
    def load(self, state: dict, strict=False):
        """Copy OIHW tensors (reference checkpoint / state_dict) into the store."""
        missing = []
        for k in self.shapes:
            if k not in state:
                missing.append(k)
                continue
            src = state[k]
            dst = self.oihw(k)
            if tuple(src.shape) != tuple(dst.shape):
                raise RuntimeError(f"size mismatch for {k}: copying {tuple(src.shape)} into {tuple(dst.shape)}")
            dst.copy_(src.to(self.device, torch.float32))
        if strict and missing:
            raise RuntimeError(f"missing keys {missing}")
        return missing

    def state(self, buf=None):
        return OrderedDict((k, self.oihw(k, buf)) for k in self.shapes)

    def zero_grad(self):
        self.grad.zero_()

    def adam_state_dict(self, lr, betas=(0.5, 0.999), eps=1e-8, initial_lr=None):
        """The Adam moments as a ``torch.optim.Adam.state_dict()`` (ir:1601-1609):
        parameter indices follow the module's ``parameters()`` order (the
        state_dict order without buffers), tensors in OIHW fp32 on the CPU, so the
        file loads into the reference's optimizer unchanged."""
        state = {}
        if self.step_count > 0:
            for i, k in enumerate(self.shapes):
                state[i] = {"step": torch.tensor(float(self.step_count)),
                            "exp_avg": self.oihw(k, self.m).detach().cpu().contiguous(),
                            "exp_avg_sq": self.oihw(k, self.v).detach().cpu().contiguous()}
        group = {"lr": lr, "betas": tuple(betas), "eps": eps, "weight_decay": 0, "amsgrad": False,
                 "maximize": False, "foreach": None, "capturable": False, "differentiable": False, "fused": None,
                 "params": list(range(len(self.shapes)))}
        if initial_lr is not None:
            group["initial_lr"] = initial_lr   # LambdaLR's key (ir:1606-1609)
        return {"state": state, "param_groups": [group]}

    @torch.no_grad()
    def load_adam_state_dict(self, sd):
        """Inverse of adam_state_dict (also accepts a reference optimizer file)."""
        st = sd["state"]
        if not st:
            self.m.zero_()
            self.v.zero_()
            self.step_count = 0
            return
        steps = set()
        for i, k in enumerate(self.shapes):
            e = st[i]
            self.oihw(k, self.m).copy_(e["exp_avg"].to(self.device, torch.float32))
            self.oihw(k, self.v).copy_(e["exp_avg_sq"].to(self.device, torch.float32))
            steps.add(int(float(e["step"])))
        if len(steps) != 1:
            raise RuntimeError(f"per-parameter Adam step counts differ: {sorted(steps)}")
        self.step_count = steps.pop()

    def adam_step(self, lr, b1=0.5, b2=0.999, eps=1e-8):
        self.adam_begin(lr, b1, b2, eps)(0, self.numel)

    def adam_begin(self, lr, b1=0.5, b2=0.999, eps=1e-8):
        """Count one optimizer step and return apply(start, end), the Adam update of
        the flat slice [start, end): a step may be applied bucket by bucket as each
        bucket's gradient all-reduce completes (BucketedAllreduce.finish)."""
        self.step_count += 1
        t = self.step_count
        if self.dev_adam:
            # the count and the bias corrections on the device (a captured step replays with
            # the right t); the device count is resynced to the host's after a state load
            if self._count is None:
                self._count = torch.zeros(1, dtype=torch.int32, device=self.device)
                self._prm = torch.zeros(2, dtype=torch.float32, device=self.device)
                self._count_host = 0
            if self._count_host != t - 1:
                self._count.fill_(t - 1)
            ops.adam_prep(self._count, lr, b1, b2, self._prm)
            self._count_host = t

            def apply_dev(a, b):
                ops.adam_dev(self.flat[a:b], self.grad[a:b], self.m[a:b], self.v[a:b], self._prm, b1, b2, eps)
            return apply_dev

        def apply(a, b):
            ops.adam(self.flat[a:b], self.grad[a:b], self.m[a:b], self.v[a:b], t, lr, b1, b2, eps)
        return apply


def _pc(store: ParamStore, key: str, spec: ConvSpec, dtype, need_dgrad=True):
    """Packed conv of state key ``key``; its bias only if the layout has one (use_bias)."""
    bias = store.krsc(key + ".bias") if key + ".bias" in store.shapes else None
    return PackedConv(spec, store.krsc(key + ".weight"), bias, dtype, need_dgrad=need_dgrad)


class Buffers:
    """Device buffers keyed by name (allocated once per shape) plus the forward
    state a backward needs (``state``: activation lists, the input shape).

    The fused step reuses one long-lived set per engine.  The module API
    (autograd.Function wrappers) gives every forward call a fresh set that its
    ctx keeps until the backward, so interleaved calls -- netD(real), netD(fake),
    then backward (ir:1642-1650) -- each back-propagate through their own
    activations and InstanceNorm statistics."""

    def __init__(self, device):
        self.device, self.d, self.state = device, {}, {}

    def get(self, name, shape, dtype):
        t = self.d.get(name)
        if t is None or tuple(t.shape) != tuple(shape) or t.dtype != dtype:
            t = torch.empty(shape, dtype=dtype, device=self.device)
            self.d[name] = t
        return t

    def zeros(self, name, shape, dtype):
        """Like get(), zero-filled when (re)allocated: padding channels stay 0."""
        t = self.d.get(name)
        if t is None or tuple(t.shape) != tuple(shape) or t.dtype != dtype:
            t = torch.zeros(shape, dtype=dtype, device=self.device)
            self.d[name] = t
        return t

    def flat(self, name, numel, dtype=torch.float32):
        t = self.d.get(name)
        if t is None or t.numel() < numel or t.dtype != dtype:
            t = torch.empty(numel, dtype=dtype, device=self.device)
            self.d[name] = t
        return t


class INLayer:
    """Per-layer InstanceNorm statistics kept from forward to backward.

    The conv bias in front of an InstanceNorm has an exactly-zero gradient
    (IN subtracts the per-channel mean, so the bias never reaches any output);
    the reference's fp32 autograd produces rounding noise there.
    By default the exact zero is kept (no reduction, no atomics); set
    ``INLayer.sum_bias_grad = True`` to accumulate the fp32 sum of dx instead.
    ``fused_stats``: take the forward statistics from the producing conv's epilogue
    where a fused kernel exists (irgan_conv_fwd_stats) instead of a separate pass.
    """
    fused_stats = True
    fused_resample = True
    sum_bias_grad = False

    def fwd(self, bufs: Buffers, name: str, x: Feat, y: Feat, act, res: Feat = None, xhat=None, nb=0, q8=None):
        """nb > 0: x's statistics partials are already in the shared work buffer
        (written by the producing conv, conv_fwd); only the reduction runs.
        The {mean, rstd} table stays in ``bufs`` under ``name`` for bwd().
        q8: also write y's fp8 copy (ops.in_apply)."""
        N, C = x.N, x.C
        work = bufs.flat("in_work", ops.IN_PARTS * N * C, torch.float64)
        mr = bufs.get("mr_" + name, (N * C * 2,), torch.float32)
        if nb:
            ops.in_finalize(x, work, nb, mr)
        else:
            ops.in_stats(x, work, mr)
        ops.in_apply(x, mr, y, act=act, res=res, xhat=xhat, q8=q8)

    def conv_fwd8(self, bufs: Buffers, name: str, pc, w8, dqw, x8: Feat, dqx, z: Feat, y: Feat, act,
                  res: Feat = None, q8=None):
        """conv_fwd on fp8 operands (ops.conv_fwd_fp8) with the fused statistics."""
        work = bufs.flat("in_work", ops.IN_PARTS * z.N * z.C, torch.float64)
        nb = ops.conv_fwd_fp8(pc, w8, dqw, x8, dqx, z, part=work)
        self.fwd(bufs, name, z, y, act, res=res, nb=nb, q8=q8)

    def conv_fwd(self, bufs: Buffers, name: str, pc, x: Feat, z: Feat, y: Feat, act, res: Feat = None):
        """z = conv(x) (kept for the backward), y = act(IN(z) [+ res]): the IN statistics
        come from the conv's epilogue when it has a fused kernel (ops.conv_fwd_stats)."""
        work = bufs.flat("in_work", ops.IN_PARTS * z.N * z.C, torch.float64)
        nb = ops.conv_fwd_stats(pc, x, z, work) if INLayer.fused_stats else 0
        if not nb:
            ops.conv_fwd(pc, x, z)
        self.fwd(bufs, name, z, y, act, res=res, nb=nb)

    def conv_stats(self, bufs: Buffers, name: str, pc, x: Feat, z: Feat, conv8=None):
        """z = conv(x) and z's {mean, rstd} table (returned, kept for bwd()) -- no apply:
        the consumer normalises on load (ops.blur_down_in / ops.upsample_in).
        conv8 = (w8, dqw, x8, dqx): the conv on fp8 operands (ops.conv_fwd_fp8)."""
        work = bufs.flat("in_work", ops.IN_PARTS * z.N * z.C, torch.float64)
        mr = bufs.get("mr_" + name, (z.N * z.C * 2,), torch.float32)
        if conv8 is not None:
            w8, dqw, x8, dqx = conv8
            ops.in_finalize(z, work, ops.conv_fwd_fp8(pc, w8, dqw, x8, dqx, z, part=work), mr)
            return mr
        nb = ops.conv_fwd_stats(pc, x, z, work) if INLayer.fused_stats else 0
        if nb:
            ops.in_finalize(z, work, nb, mr)
        else:
            ops.conv_fwd(pc, x, z)
            ops.in_stats(z, work, mr)
        return mr

    def resample_fwd(self, bufs: Buffers, name: str, pc, x: Feat, z: Feat, a_name: str, act, y: Feat, fused, plain,
                     conv8=None, q8=None):
        """y = resample(act(IN(conv(x)))): the IN apply fused into the resample when
        ``fused(z, mr, act, y)`` takes the shapes, else apply into bufs[a_name] + ``plain``.
        conv8: the conv on fp8 operands (conv_stats); q8: also y's e4m3 copy (Fp8Acts.spec)."""
        mr = self.conv_stats(bufs, name, pc, x, z, conv8=conv8)
        if INLayer.fused_resample and (fused(z, mr, act, y, q8=q8) if q8 is not None else fused(z, mr, act, y)):
            return
        a = Feat(bufs.get(a_name, (z.N, z.H, z.W, z.C), z.t.dtype))
        ops.in_apply(z, mr, a, act=act)
        plain(a, y)
        if q8 is not None:
            ops.fp8_quant(y, *q8)

    def bwd(self, bufs: Buffers, name: str, dy: Feat, z: Feat, act, dx: Feat, db=None, dy2: Feat = None, q8=None):
        """z: the PRE-norm input kept from forward; act: the activation after IN.
        q8: also write dx's fp8 copy (ops.in_backward)."""
        N, C = z.N, z.C
        work = bufs.flat("in_work", ops.IN_PARTS * N * C, torch.float64)
        red = bufs.flat("in_red", 2 * N * C)
        mr = bufs.d["mr_" + name]
        ops.in_backward(dy, z, act, mr, work, red, dx, db=db if INLayer.sum_bias_grad else None, dy2=dy2,
                        q8=q8 if not INLayer.sum_bias_grad else None)

class NoNorm(INLayer):
    """norm='none' (ir:162-163: ``lambda num_features: Identity()``): the layer is just its
    activation, y = act(z) [+ res], and the conv in front has no bias (use_bias is False,
    ir:450-455, 588-593).  Same interface as INLayer: the forward applies an identity
    {mean 0, rstd 1} table through the same apply / fused-resample kernels ((z - 0) * 1 = z
    exactly), the backward is the activation's derivative."""

    def _ident(self, bufs: Buffers, name: str, N: int, C: int) -> torch.Tensor:
        mr = bufs.get("mr_" + name, (N * C * 2,), torch.float32)
        if bufs.state.get("ident_" + name) is not mr:
            mr.view(-1, 2)[:, 0] = 0.0
            mr.view(-1, 2)[:, 1] = 1.0
            bufs.state["ident_" + name] = mr
        return mr

    def fwd(self, bufs, name, x, y, act, res=None, xhat=None, nb=0, q8=None):
        if q8 is not None:
            raise NotImplementedError("the fp8 path runs with InstanceNorm (norm='instance')")
        ops.in_apply(x, self._ident(bufs, name, x.N, x.C), y, act=act, res=res)

    def conv_fwd8(self, *a, **kw):
        raise NotImplementedError("the fp8 path runs with InstanceNorm (norm='instance')")

    def conv_fwd(self, bufs, name, pc, x, z, y, act, res=None):
        ops.conv_fwd(pc, x, z, bias=pc.bias is not None)
        self.fwd(bufs, name, z, y, act, res=res)

    def conv_stats(self, bufs, name, pc, x, z, conv8=None):
        if conv8 is not None:
            raise NotImplementedError("the fp8 path runs with InstanceNorm (norm='instance')")
        ops.conv_fwd(pc, x, z, bias=pc.bias is not None)
        return self._ident(bufs, name, z.N, z.C)

    def bwd(self, bufs, name, dy, z, act, dx, db=None, dy2=None, q8=None):
        if dy2 is not None or q8 is not None:
            raise NotImplementedError("NoNorm.bwd: dy2 / q8 are InstanceNorm-path features")
        if act == ACT_NONE and dx.t.data_ptr() == dy.t.data_ptr() and dx.off == dy.off:
            pass                                   # identity, in place
        else:
            ops.act_bwd(dy, z, act, dx)            # z > 0 <=> act(z) > 0 for ReLU / LeakyReLU
        if db is not None:
            ops.channel_sum(dx, db)

def make_norm(norm: str) -> INLayer:
    """The engine's per-layer norm for Config.norm (ir:154-165): 'instance' or 'none'
    ('batch' needs cross-sample statistics (SyncBN under DP): out of scope)."""
    if norm == "instance":
        return INLayer()
    if norm in ("none", None):
        return NoNorm()
    raise NotImplementedError(f"norm '{norm}': the HIP engines implement 'instance' and 'none'")


def res_conv_keys(padding_type="reflect", use_dropout=False):
    """Indices of the two convs inside ResnetBlock.conv_block (ir:375-411): the pad
    modules exist only for reflect / replicate, the Dropout only with use_dropout."""
    if padding_type not in ("reflect", "replicate", "zero"):
        raise NotImplementedError(f"Padding [{padding_type}] is not implemented")
    first = 0 if padding_type == "zero" else 1
    second = first + 3 + (1 if use_dropout else 0) + (0 if padding_type == "zero" else 1)
    return first, second


# ----------------------------------------------------------------------------
# generator  (ir:425-569)
# ----------------------------------------------------------------------------

class GeneratorEngine:
    _pack_batch = None  # ops.PackBatch of self.packs, built on the first pack()

    def __init__(self, store: ParamStore, dtype=BF16, ngf=64, input_nc=1, output_nc=3, n_blocks=9,
                 no_antialias=False, no_antialias_up=False, fp8=False, norm="instance", padding_type="reflect",
                 use_dropout=False, dropout_seed=0):
        """fp8: the ResnetBlock convs and, with the anti-aliased resamplers (the default),
        down2 and up1_conv run on OCP e4m3 operands (BASELINE config 5: forward, backward-
        data interior, weight gradient): per-tensor power-of-two scales, current scaling
        for the re-packed weights, delayed scaling for the activations and gradients they
        read; everything else stays bf16.
        norm / padding_type / use_dropout: the reference's constructor options (ir:154-165,
        375-411, 443-447); the ResnetBlock convs of padding 'replicate' read an explicitly
        padded copy of their input (ops.pad) and fold their input gradient back (ops.pad_fold)."""
        self.store, self.dtype, self.ngf = store, dtype, ngf
        self.fp8 = bool(fp8)
        if self.fp8 and (dtype != BF16 or 4 * ngf % 128):
            raise ValueError("the fp8 path runs on the bf16 engine with 4*ngf % 128 == 0")
        if self.fp8 and (norm != "instance" or padding_type != "reflect" or use_dropout):
            raise ValueError("the fp8 path runs the default ResnetBlock (InstanceNorm, reflect, no dropout)")
        self.norm_type, self.padding_type, self.use_dropout = norm, padding_type, bool(use_dropout)
        self.dropout_seed, self.dropout_calls = int(dropout_seed), 0
        self.training = True
        self.input_nc, self.output_nc, self.n_blocks = input_nc, output_nc, n_blocks
        self.no_aa, self.no_aa_up = no_antialias, no_antialias_up
        self.tdt = ops.TORCH_DT[dtype]
        c0, c1, c2 = ngf, 2 * ngf, 4 * ngf
        sd = 2 if no_antialias else 1
        S = store
        self.inc = _pc(S, "inc.1", ConvSpec(input_nc, c0, 7, 1, 3, PAD_REFLECT), dtype, need_dgrad=False)
        self.down1 = _pc(S, "down1.0", ConvSpec(c0, c1, 3, sd, 1, PAD_ZERO), dtype)
        self.down2 = _pc(S, "down2.0", ConvSpec(c1, c2, 3, sd, 1, PAD_ZERO), dtype)
        k1, k2 = res_conv_keys(padding_type, use_dropout)
        self.res_keys = (k1, k2)
        rspec = {"reflect": ConvSpec(c2, c2, 3, 1, 1, PAD_REFLECT), "zero": ConvSpec(c2, c2, 3, 1, 1, PAD_ZERO),
                 "replicate": ConvSpec(c2, c2, 3, 1, 0, PAD_ZERO)}[padding_type]   # replicate: on the padded copy
        self.res = [(_pc(S, f"resblocks.{b}.conv_block.{k1}", rspec, dtype),
                     _pc(S, f"resblocks.{b}.conv_block.{k2}", rspec, dtype)) for b in range(n_blocks)]
        if no_antialias_up:
            # ConvTranspose2d(C, C, 3, s2, p1, op1) == backward-data of conv(3, s2, p1)
            self.up1_up = _pc(S, "up1_up", ConvSpec(c2, c2, 3, 2, 1, PAD_ZERO), dtype)
            self.up2_up = _pc(S, "up2_up", ConvSpec(c1, c1, 3, 2, 1, PAD_ZERO), dtype)
        self.up1 = _pc(S, "up1_conv.0", ConvSpec(c2 + c1, c1, 3, 1, 1, PAD_ZERO), dtype)
        self.up2 = _pc(S, "up2_conv.0", ConvSpec(c1 + c0, c0, 3, 1, 1, PAD_ZERO), dtype)
        self.outc = _pc(S, "outc.1", ConvSpec(c0, output_nc, 7, 1, 3, PAD_REFLECT), dtype)
        self.packs = [self.inc, self.down1, self.down2, self.up1, self.up2, self.outc] + \
            [p for pr in self.res for p in pr] + ([self.up1_up, self.up2_up] if no_antialias_up else [])
        # fp8 on down2 / up1_conv too (ir:477-482, 557-558): their operands come from the
        # fused resamplers (x1 from down1's Downsample, the up-sampled bottleneck)
        # (their kernels take 128-channel K chunks: down2's Cin = 2*ngf must be a multiple of 128)
        self.fp8_ud = self.fp8 and not no_antialias and not no_antialias_up and c1 % 128 == 0
        if self.fp8:
            # weight images 4b..4b+3: conv1 fwd, conv1 dgrad, conv2 fwd, conv2 dgrad of block b;
            # 4n..4n+3: down2 fwd, down2 dgrad, up1_conv fwd, up1_conv dgrad.
            # activation slots: forward inputs 2b (conv1), 2b+1 (conv2); backward-data inputs
            # 2n+2b (conv2's dY), 2n+2b+1 (conv1's dY); 4n: up1_conv's concat [up(h) | x1] (x1
            # is down2's input: one scale for both), 4n+1 / 4n+2: up1_conv's / down2's dY
            ud = [self.down2.fwd, self.down2.dg[0][2], self.up1.fwd, self.up1.dg[0][2]] if self.fp8_ud else []
            self.f8w = ops.Fp8Weights([im for p1, p2 in self.res for im in (p1.fwd, p1.dg[0][2], p2.fwd,
                                                                             p2.dg[0][2])] + ud, store.device)
            self.f8a = ops.Fp8Acts(4 * n_blocks + 4, store.device)
            self.s_cat, self.s_dz3, self.s_dz2 = 4 * n_blocks, 4 * n_blocks + 1, 4 * n_blocks + 2
            self.s_x1 = 4 * n_blocks + 3   # down2's own x1 copy on the calibration step
        n_in = 5 + 2 * n_blocks
        self.norms = {k: make_norm(norm) for k in ["inc", "down1", "down2", "up1", "up2"] +
                      [f"r{b}_{i}" for b in range(n_blocks) for i in (1, 2)]}
        assert len(self.norms) == n_in
        self.bufs = Buffers(store.device)

    def pack(self):
        if self._pack_batch is None:
            self._pack_batch = ops.PackBatch(self.packs)
        self._pack_batch.run()
        if self.fp8:
            self.f8w.run()

    def _w8(self, k):
        return self.f8w.dst[k], ops.Pi(self.f8w.dq, k)

    def _res_in(self, g: Buffers, name: str, x: Feat) -> Feat:
        """A ResnetBlock conv's input as its conv reads it: x itself (reflect: folded into the
        conv's loads; zero: the conv's own padding), or the ReplicationPad2d(1) copy (kept for
        the weight gradient)."""
        if self.padding_type != "replicate":
            return x
        xp = Feat(g.get(name, (x.N, x.H + 2, x.W + 2, x.C), self.tdt))
        ops.pad(x, xp, 1, "replicate")
        return xp

    def _res_dgrad(self, g: Buffers, pc, dy: Feat, dx: Feat, accumulate, padbuf):
        """dx (+)= backward-data of a ResnetBlock conv for the padding type."""
        if self.padding_type != "replicate":
            ops.conv_dgrad(pc, dy, dx, accumulate=accumulate, pad_buf=padbuf)
            return
        dxp = Feat(g.get("res_dxp", (dx.N, dx.H + 2, dx.W + 2, dx.C), self.tdt))
        ops.conv_dgrad(pc, dy, dxp)
        ops.pad_fold(dxp, dx, 1, "replicate", accumulate=accumulate)

    def _bgrad(self, key):
        """Flat-buffer slice of parameter ``key``'s gradient, None when the layout has no
        such parameter (use_bias False: no conv biases)."""
        return self.store.krsc(key, self.store.grad) if key in self.store.shapes else None

    # -- shapes
    def _dims(self, H, W):
        H1, W1 = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        H2, W2 = (H1 - 1) // 2 + 1, (W1 - 1) // 2 + 1
        return H1, W1, H2, W2

    def fp8_layers(self, B, H, W):
        """(resblocks, down2 / up1_conv) on e4m3 for a (B, H, W) input: the fp8 conv fuses the
        InstanceNorm partials of at most IN_PARTS 16x16 output tiles per image and addresses
        fewer than 2^30 operand bytes (irgan_conv_fwd_fp8); a size beyond either runs that
        group on the bf16 kernels for this call (no EUNSUPPORTED mid-step)."""
        if not self.fp8:
            return False, False
        H1, W1, H2, W2 = self._dims(H, W)
        c1, c2 = 2 * self.ngf, 4 * self.ngf

        def ok(h, w, cin):
            return -(-h // 16) * -(-w // 16) <= ops.IN_PARTS and B * h * w * cin < (1 << 30)
        res = ok(H2, W2, c2)
        return res, res and self.fp8_ud and ok(H1, W1, c2 + c1)

    def forward(self, ir_nchw: torch.Tensor, bufs: Buffers = None, training: bool = None) -> torch.Tensor:
        """ir (B, input_nc, H, W) fp32 in [-1,1] -> fake NHWC fp32 (B, H, W, 3).
        Activations land in ``bufs`` (default: the engine's own set).  ``training``
        (default: self.training) decides nn.Dropout's mode (ir:394-395): callers outside
        the module forward / GANStep pass the module's train()/eval() state."""
        B, _, H, W = ir_nchw.shape
        g, T = bufs or self.bufs, self.tdt
        train = self.training if training is None else bool(training)
        c0, c1, c2 = self.ngf, 2 * self.ngf, 4 * self.ngf
        H1, W1, H2, W2 = self._dims(H, W)
        g.state["shape"] = (B, H, W)
        g.state.pop("dropout_seed", None)
        if self.use_dropout and train:   # a fresh mask per forward call; the backward reuses it
            self.dropout_calls += 1
            g.state["dropout_seed"] = (self.dropout_seed << 32) ^ (self.dropout_calls << 8)
        ir_buf = g.zeros("ir", (B, H, W, max(8, self.input_nc)), T)   # narrow input zero-padded to 8 ch
        ops.nchw_to_nhwc(ir_nchw.contiguous(), Feat(ir_buf, 0, self.input_nc))
        ir_t = Feat(ir_buf, 0, self.inc.cin_eff)
        cat2 = g.get("cat2", (B, H, W, c1 + c0), T)       # [up2 out | x0]
        cat1 = g.get("cat1", (B, H1, W1, c2 + c1), T)     # [up1 out | x1]
        x0 = Feat(cat2, c1, c0)
        x1 = Feat(cat1, c2, c1)
        f8, ud = self.fp8_layers(B, H, W)
        g.state["fp8"] = (f8, ud)
        A = self.f8a if f8 else None
        cat1_8 = Feat(g.get("cat1_8", (B, H1, W1, c2 + c1), torch.float8_e4m3fn)) if ud else None
        # first step (current scaling): down2 reads its own copy of x1, scaled from x1 alone,
        # for its forward AND its weight gradient; up1_conv's concat is then scaled as a whole
        calib = ud and not A.seen[self.s_cat]
        g.state["fp8_calib"] = calib
        x1_8 = Feat(g.get("x1_8c", (B, H1, W1, c1), torch.float8_e4m3fn)) if calib else \
            (cat1_8.sl(c2, c1) if ud else None)
        dq_x1 = (A.dqp(self.s_x1) if calib else A.dqp(self.s_cat)) if ud else None
        # inc: reflect-pad 3, conv7x7, IN, ReLU  (ir:458-463)
        z0 = Feat(g.get("z0", (B, H, W, c0), T))
        self.norms["inc"].conv_fwd(g, "inc", self.inc, ir_t, z0, x0, ACT_RELU)   # statistics fused where taken
        # down1 (+ blur-down)  (ir:469-474)
        if self.no_aa:
            z1 = Feat(g.get("z1", (B, H1, W1, c1), T))
            ops.conv_fwd(self.down1, x0, z1)
            self.norms["down1"].fwd(g, "down1", z1, x1, ACT_RELU)
        else:
            z1 = Feat(g.get("z1", (B, H, W, c1), T))
            self.norms["down1"].resample_fwd(g, "down1", self.down1, x0, z1, "a1", ACT_RELU, x1, ops.blur_down_in,
                                             ops.blur_down, q8=A.spec(self.s_cat, x1_8) if ud and not calib else None)
            if calib:
                A.calibrate(self.s_x1, x1, x1_8)   # down2's operand scaled from x1 alone on the first step
        # down2 (+ blur-down)  (ir:477-482)
        h = Feat(g.get("h0", (B, H2, W2, c2), T))
        if self.no_aa:
            z2 = Feat(g.get("z2", (B, H2, W2, c2), T))
            ops.conv_fwd(self.down2, x1, z2)
            self.norms["down2"].fwd(g, "down2", z2, h, ACT_RELU)
        else:
            z2 = Feat(g.get("z2", (B, H1, W1, c2), T))
            self.norms["down2"].resample_fwd(g, "down2", self.down2, x1, z2, "a2", ACT_RELU, h, ops.blur_down_in,
                                             ops.blur_down, conv8=(*self._w8(4 * self.n_blocks), x1_8,
                                                                   dq_x1) if ud else None)
        # 9 ResnetBlocks  (ir:362-418, 485-490)
        # fp8: one e4m3 operand buffer, written by the producer of each conv input (the
        # IN passes, fused; h_0 from blur-down by a quantise launch) and read by the conv
        # (one buffer per conv input slot: the fp8 weight gradients of the backward read them)
        x8s = [Feat(g.get(f"x8_{k}", (B, H2, W2, c2), torch.float8_e4m3fn)) for k in range(2 * len(self.res))] \
            if f8 else None
        if f8:
            A.quant(0, h, x8s[0])
        nres = len(self.res)
        for b, (p1, p2) in enumerate(self.res):
            r1 = Feat(g.get(f"r1_{b}", (B, H2, W2, c2), T))
            t = Feat(g.get(f"t{b}", (B, H2, W2, c2), T))
            if f8:
                self.norms[f"r{b}_1"].conv_fwd8(g, f"r{b}_1", p1, *self._w8(4 * b), x8s[2 * b], A.dqp(2 * b), r1, t,
                                                ACT_RELU, q8=A.spec(2 * b + 1, x8s[2 * b + 1]))
                A.ensure(2 * b + 1, t, x8s[2 * b + 1])
            else:
                self.norms[f"r{b}_1"].conv_fwd(g, f"r{b}_1", p1, self._res_in(g, f"xp1_{b}", h), r1, t, ACT_RELU)
            r2 = Feat(g.get(f"r2_{b}", (B, H2, W2, c2), T))
            hn = Feat(g.get(f"h{b + 1}", (B, H2, W2, c2), T))
            if f8:
                nxt = 2 * b + 2 if b + 1 < nres else None   # the next block's conv1 input
                self.norms[f"r{b}_2"].conv_fwd8(g, f"r{b}_2", p2, *self._w8(4 * b + 2), x8s[2 * b + 1],
                                                A.dqp(2 * b + 1), r2, hn, ACT_NONE, res=h,
                                                q8=A.spec(nxt, x8s[nxt]) if nxt else None)
                if nxt:
                    A.ensure(nxt, hn, x8s[nxt])
            else:
                t2 = t
                if self.use_dropout and train:   # nn.Dropout(0.5) after the ReLU (ir:394-395)
                    t2 = Feat(g.get(f"td{b}", (B, H2, W2, c2), T))
                    ops.dropout(t, t2, g.state["dropout_seed"] + 2 * b)
                self.norms[f"r{b}_2"].conv_fwd(g, f"r{b}_2", p2, self._res_in(g, f"xp2_{b}", t2), r2, hn, ACT_NONE,
                                               res=h)
            h = hn
        if f8:
            self.f8a.snapshot(0, 2 * self.n_blocks)  # the scales x8s were made with (fp8 weight gradients)
            self.f8a.update(0, 2 * self.n_blocks)    # next step's forward scales
        # up1 -> cat with x1 -> conv/IN/ReLU  (ir:554-558)
        # (odd sizes: the up-sampled map is 2*H2 x 2*W2 != H1 x W1 and is resized to the
        # skip's size, ir:555-556 -- folded into the UpsampleAA table, or a resize launch
        # after the ConvTranspose2d)
        y1 = Feat(cat1, 0, c2)
        if self.no_aa_up:
            self._convt(self.up1_up, h, y1, g, "ut1")
        else:
            ops.upsample(h, y1, q8=A.spec(self.s_cat, cat1_8.sl(0, c2)) if ud and not calib else None)
        if calib:   # up1_conv's operand scaled from the whole concat on the first step
            A.calibrate(self.s_cat, Feat(cat1), cat1_8)
        z3 = Feat(g.get("z3", (B, H1, W1, c1), T))
        # up2 -> cat with x0 -> conv/IN/ReLU  (ir:561-565)
        y2 = Feat(cat2, 0, c1)
        if self.no_aa_up:
            a3 = Feat(g.get("a3", (B, H1, W1, c1), T))   # also the ConvTranspose2d's weight-gradient input
            self.norms["up1"].conv_fwd(g, "up1", self.up1, Feat(cat1), z3, a3, ACT_RELU)
            self._convt(self.up2_up, a3, y2, g, "ut2")
        else:
            self.norms["up1"].resample_fwd(g, "up1", self.up1, Feat(cat1), z3, "a3", ACT_RELU, y2, ops.upsample_in,
                                           ops.upsample, conv8=(*self._w8(4 * self.n_blocks + 2), cat1_8,
                                                                A.dqp(self.s_cat)) if ud else None)
        if ud:
            A.snapshot(self.s_cat, 1)   # the scale cat1_8 was made with (the weight gradients)
            A.update(self.s_cat, 1)
        z4 = Feat(g.get("z4", (B, H, W, c0), T))
        a4 = Feat(g.get("a4", (B, H, W, c0), T))
        self.norms["up2"].conv_fwd(g, "up2", self.up2, Feat(cat2), z4, a4, ACT_RELU)
        # outc: reflect-pad 3, conv7x7 (+bias), tanh  (ir:527-531)
        fake = g.get("fake", (B, H, W, self.output_nc), torch.float32)
        ops.conv_fwd(self.outc, a4, Feat(fake), act=ACT_TANH)
        return fake

    def _convt(self, pc, x: Feat, y: Feat, g: Buffers, name: str):
        """ConvTranspose2d(k3, s2, p1, op1) (ir:495-500) into y, through a 2H x 2W
        temporary + bilinear resize when y's size is not 2x (ir:555-556)."""
        if (y.H, y.W) == (2 * x.H, 2 * x.W):
            ops.conv_dgrad(pc, x, y, bias=True)
            return
        t = Feat(g.get(name, (x.N, 2 * x.H, 2 * x.W, y.C), self.tdt))
        ops.conv_dgrad(pc, x, t, bias=True)
        ops.resize(t, y)

    def _convt_bwd(self, pc, key, dy: Feat, x: Feat, dx: Feat, g: Buffers, name: str):
        """Backward of _convt: bias grad, weight grad, and dx (the conv forward of the
        transposed conv); dy is the gradient at the skip-sized output."""
        S = self.store
        if (dy.H, dy.W) != (2 * x.H, 2 * x.W):
            t = Feat(g.get(name + "_d", (x.N, 2 * x.H, 2 * x.W, dy.C), self.tdt))
            ops.resize_bwd(dy, t)
            dy = t
        db = self._bgrad(key + ".bias")
        if db is not None:
            ops.channel_sum(dy, db)
        ops.conv_wgrad(pc.spec, dy, x, S.krsc(key + ".weight", S.grad), self.dtype)
        ops.conv_fwd(pc, dy, dx, bias=False)

    def backward(self, dfake: torch.Tensor, ready=None, bufs: Buffers = None):
        """dfake: dL/dfake, NHWC fp32 (B,H,W,3).  Accumulates into store.grad.
        ``bufs``: the set the matching forward wrote (default: the engine's own).

        ``ready(key)``, if given, is called each time every gradient from parameter
        ``key`` to the end of the flat buffer is final (reverse layer order), so the
        caller can start reducing that tail while the rest of the backward runs."""
        ready = ready or (lambda key: None)
        g, T, S, dt = bufs or self.bufs, self.tdt, self.store, self.dtype
        B, H, W = g.state["shape"]
        c0, c1, c2 = self.ngf, 2 * self.ngf, 4 * self.ngf
        H1, W1, H2, W2 = self._dims(H, W)
        G = S.grad
        cat1, cat2 = Feat(g.d["cat1"]), Feat(g.d["cat2"])
        x0, x1 = cat2.sl(c1, c0), cat1.sl(c2, c1)
        padbuf = g.flat("dpad", max(B * (H + 6) * (W + 6) * c0, B * (H2 + 2) * (W2 + 2) * c2))

        def wg(pc, key, x, dy):
            ops.conv_wgrad(pc.spec, x, dy, S.krsc(key + ".weight", G), dt)

        # outc: tanh' then conv backward
        fake = Feat(g.d["fake"])
        dzo_buf = g.zeros("dz_out", (B, H, W, max(8, self.output_nc)), T)   # zero-padded to 8 ch
        dzo = Feat(dzo_buf, 0, self.output_nc)
        ops.act_bwd(Feat(dfake), fake, ACT_TANH, dzo)
        a4 = Feat(g.d["a4"])
        wg(self.outc, "outc.1", a4, dzo)
        ops.channel_sum(dzo, S.krsc("outc.1.bias", G))
        da4 = Feat(g.get("da4", (B, H, W, c0), T))
        ops.conv_dgrad(self.outc, Feat(dzo_buf, 0, self.outc.cout_eff), da4, pad_buf=padbuf)
        # up2_conv
        self.norms["up2"].bwd(g, "up2", da4, Feat(g.d["z4"]), ACT_RELU, da4, db=self._bgrad("up2_conv.0.bias"))
        wg(self.up2, "up2_conv.0", cat2, da4)
        dcat2 = Feat(g.get("dcat2", (B, H, W, c1 + c0), T))
        ops.conv_dgrad(self.up2, da4, dcat2)
        # up2_up
        da3 = Feat(g.get("da3", (B, H1, W1, c1), T))
        dy2 = dcat2.sl(0, c1)
        if self.no_aa_up:
            self._convt_bwd(self.up2_up, "up2_up", dy2, Feat(g.d["a3"]), da3, g, "ut2")
        else:
            ops.upsample_bwd(dy2, da3)
        # up1_conv
        f8, ud = g.state.get("fp8", (False, False))
        A, nb4 = (self.f8a, 4 * self.n_blocks) if f8 else (None, 0)
        cat1_8 = Feat(g.d["cat1_8"]) if ud else None

        def wg8(pc, key, x8, dqx, dy8, dslot, x, dy):
            """weight gradient on the fp8 copies (x8 with the scale ``dqx`` it was made with,
            dy8); bf16 where the kernel does not take the layer"""
            if not ops.conv_wgrad_fp8(pc.spec, x8, dy8, dqx, A.dqp(dslot), S.krsc(key + ".weight", G)):
                wg(pc, key, x, dy)
        da3_8 = Feat(g.get("dz3_8", (B, H1, W1, c1), torch.float8_e4m3fn)) if ud else None
        self.norms["up1"].bwd(g, "up1", da3, Feat(g.d["z3"]), ACT_RELU, da3, db=self._bgrad("up1_conv.0.bias"),
                              q8=A.spec(self.s_dz3, da3_8) if ud else None)
        dcat1 = Feat(g.get("dcat1", (B, H1, W1, c2 + c1), T))
        if ud:
            A.ensure(self.s_dz3, da3, da3_8)
            wg8(self.up1, "up1_conv.0", cat1_8, A.dqp_used(self.s_cat), da3_8, self.s_dz3, cat1, da3)
            ops.conv_dgrad_fp8(self.up1, *self._w8(nb4 + 3), da3_8, A.dqp(self.s_dz3), da3, dcat1)
        else:
            wg(self.up1, "up1_conv.0", cat1, da3)
            ops.conv_dgrad(self.up1, da3, dcat1)
        # up1_up
        h9 = Feat(g.d[f"h{self.n_blocks}"])
        dh = Feat(g.get("dh", (B, H2, W2, c2), T))
        dy1 = dcat1.sl(0, c2)
        if self.no_aa_up:
            self._convt_bwd(self.up1_up, "up1_up", dy1, h9, dh, g, "ut1")
        else:
            ops.upsample_bwd(dy1, dh)
        ready("up1_up.weight" if self.no_aa_up else "up1_conv.0.weight")
        # resblocks, reversed: dh holds d h_{b+1}; becomes d h_b in place
        dt_ = Feat(g.get("dtmp", (B, H2, W2, c2), T))
        nb2 = 2 * self.n_blocks
        dy8 = Feat(g.get("dy8", (B, H2, W2, c2), torch.float8_e4m3fn)) if f8 else None
        k1, k2 = self.res_keys
        for b in reversed(range(self.n_blocks)):
            p1, p2 = self.res[b]
            key = f"resblocks.{b}.conv_block."
            t, hb = Feat(g.d[f"t{b}"]), Feat(g.d[f"h{b}"])
            r1, r2 = Feat(g.d[f"r1_{b}"]), Feat(g.d[f"r2_{b}"])
            drop = self.use_dropout and "dropout_seed" in g.state
            # the convs' inputs as they read them: the replicate-padded copies, the dropped-out t
            t2 = Feat(g.d[f"td{b}"]) if drop else t
            xin1 = Feat(g.d[f"xp1_{b}"]) if self.padding_type == "replicate" else hb
            xin2 = Feat(g.d[f"xp2_{b}"]) if self.padding_type == "replicate" else t2
            s2, s1 = nb2 + 2 * b, nb2 + 2 * b + 1
            self.norms[f"r{b}_2"].bwd(g, f"r{b}_2", dh, r2, ACT_NONE, dt_, db=self._bgrad(f"{key}{k2}.bias"),
                                      q8=A.spec(s2, dy8) if f8 else None)
            dr = Feat(g.get("dtmp2", (B, H2, W2, c2), T))
            if f8:
                A.ensure(s2, dt_, dy8)
                wg8(p2, f"{key}{k2}", Feat(g.d[f"x8_{2 * b + 1}"]), A.dqp_used(2 * b + 1), dy8, s2, xin2, dt_)
                ops.conv_dgrad_fp8(p2, *self._w8(4 * b + 3), dy8, A.dqp(s2), dt_, dr)
            else:
                self._res_dgrad(g, p2, dt_, dr, False, padbuf)
                wg(p2, f"{key}{k2}", xin2, dt_)
                if drop:   # backward of the dropout: the same mask and scale on the gradient
                    ops.dropout(dr, dr, g.state["dropout_seed"] + 2 * b)
            self.norms[f"r{b}_1"].bwd(g, f"r{b}_1", dr, r1, ACT_RELU, dr, db=self._bgrad(f"{key}{k1}.bias"),
                                      q8=A.spec(s1, dy8) if f8 else None)
            if f8:
                A.ensure(s1, dr, dy8)
                wg8(p1, f"{key}{k1}", Feat(g.d[f"x8_{2 * b}"]), A.dqp_used(2 * b), dy8, s1, xin1, dr)
                ops.conv_dgrad_fp8(p1, *self._w8(4 * b + 1), dy8, A.dqp(s1), dr, dh, accumulate=True)
            else:
                self._res_dgrad(g, p1, dr, dh, True, padbuf)
                wg(p1, f"{key}{k1}", xin1, dr)
            ready(f"{key}{k1}.weight")
        if f8:
            self.f8a.update(nb2, nb2)   # next step's backward-data scales
        # down2 (+ blur-down)
        z2 = Feat(g.d["z2"])
        if self.no_aa:
            self.norms["down2"].bwd(g, "down2", dh, z2, ACT_RELU, dh, db=self._bgrad("down2.0.bias"))
            dz2 = dh
        else:
            dz2 = Feat(g.get("da2", (B, H1, W1, c2), T))
            ops.blur_down_bwd(dh, dz2)
            dz2_8 = Feat(g.get("dz2_8", (B, H1, W1, c2), torch.float8_e4m3fn)) if ud else None
            self.norms["down2"].bwd(g, "down2", dz2, z2, ACT_RELU, dz2, db=self._bgrad("down2.0.bias"),
                                    q8=A.spec(self.s_dz2, dz2_8) if ud else None)
        dx1 = dcat1.sl(c2, c1)
        if ud:
            A.ensure(self.s_dz2, dz2, dz2_8)
            if g.state.get("fp8_calib"):   # the calibration step's own x1 copy (as its forward read)
                wg8(self.down2, "down2.0", Feat(g.d.pop("x1_8c")), A.dqp(self.s_x1), dz2_8, self.s_dz2, x1, dz2)
            else:
                wg8(self.down2, "down2.0", cat1_8.sl(c2, c1), A.dqp_used(self.s_cat), dz2_8, self.s_dz2, x1, dz2)
            ops.conv_dgrad_fp8(self.down2, *self._w8(nb4 + 1), dz2_8, A.dqp(self.s_dz2), dz2, dx1, accumulate=True)
            A.update(self.s_dz3, 2)   # next step's scales of the two dY slots
        else:
            wg(self.down2, "down2.0", x1, dz2)
            ops.conv_dgrad(self.down2, dz2, dx1, accumulate=True)  # x1 feeds down2 and the up1 concat
        # down1 (+ blur-down)
        z1 = Feat(g.d["z1"])
        if self.no_aa:
            dz1 = Feat(g.get("da1", (B, H1, W1, c1), T))
            self.norms["down1"].bwd(g, "down1", dx1, z1, ACT_RELU, dz1, db=self._bgrad("down1.0.bias"))
        else:
            dz1 = Feat(g.get("da1", (B, H, W, c1), T))
            ops.blur_down_bwd(dx1, dz1)
            self.norms["down1"].bwd(g, "down1", dz1, z1, ACT_RELU, dz1, db=self._bgrad("down1.0.bias"))
        wg(self.down1, "down1.0", x0, dz1)
        dx0 = dcat2.sl(c1, c0)
        ops.conv_dgrad(self.down1, dz1, dx0, accumulate=True)
        # inc
        self.norms["inc"].bwd(g, "inc", dx0, Feat(g.d["z0"]), ACT_RELU, dx0, db=self._bgrad("inc.1.bias"))
        wg(self.inc, "inc.1", Feat(g.d["ir"]), dx0)
        ready("inc.1.weight")


# ----------------------------------------------------------------------------
# discriminator  (ir:576-635)
# ----------------------------------------------------------------------------

class DiscriminatorEngine:
    _pack_batch = None  # ops.PackBatch of self.packs, built on the first pack()

    def __init__(self, store: ParamStore, dtype=BF16, input_nc=4, ndf=64, n_layers=3, norm="instance"):
        """PatchGAN with ``n_layers`` stride-2 stages (ir:585-632; train_kaist builds 3) and
        norm 'instance' or 'none' (the normalised convs then have no bias)."""
        self.store, self.dtype, self.tdt = store, dtype, ops.TORCH_DT[dtype]
        self.LAYERS = d_layers(n_layers)
        chans = d_channels(input_nc, ndf, n_layers)
        self.chans = chans
        self.packs = [_pc(store, k, ConvSpec(chans[i], chans[i + 1], 4, s, 1, PAD_ZERO), dtype)
                      for i, (k, s, _) in enumerate(self.LAYERS)]
        self.norms = [make_norm(norm) if n else None for (_, _, n) in self.LAYERS]
        self.bufs = Buffers(store.device)

    def pack(self):
        if self._pack_batch is None:
            self._pack_batch = ops.PackBatch(self.packs)
        self._pack_batch.run()

    def forward(self, din: Feat, tag="", bufs: Buffers = None) -> torch.Tensor:
        """din: NHWC (NB, H, W, 4) compute-dtype -> patch logits (NB, h, w, 1) fp32.
        The activations are kept in ``bufs`` (default: the engine's own) under ``tag``."""
        g, T = bufs or self.bufs, self.tdt
        x = din
        acts, pre = [din], {}
        g.state[tag] = (acts, pre)
        for i, pc in enumerate(self.packs):
            Ho, Wo = pc.spec.out_hw(x.H, x.W)
            last = i == len(self.packs) - 1
            y = Feat(g.get(f"{tag}e{i}", (x.N, Ho, Wo, pc.spec.cout), torch.float32 if last else T))
            if i == 0:
                ops.conv_fwd(pc, x, y, act=ACT_LRELU)
            elif last:
                if not ops.patch_head_fwd(pc, x, y.t):
                    ops.conv_fwd(pc, x, y)
            else:
                z = Feat(g.get(f"{tag}z{i}", (x.N, Ho, Wo, pc.spec.cout), T))
                self.norms[i].conv_fwd(g, f"{tag}n{i}", pc, x, z, y, ACT_LRELU)
                pre[i] = z
            acts.append(y)
            x = y
        return x.t

    def backward(self, dout: torch.Tensor, want_wgrad=True, want_dinput=False, tag="", bufs: Buffers = None,
                 ready=None):
        """dout: dL/dlogits fp32 (same shape as forward output).  Weight grads
        accumulate into store.grad; returns d input (fp32 NHWC) if asked.
        ``ready(key)`` (as GeneratorEngine.backward): called once every gradient from layer
        ``key``'s weight to the end of the flat buffer is final, so the caller's bucketed
        all-reduce starts on the tail while the earlier layers' backward still runs."""
        g, T, S = bufs or self.bufs, self.tdt, self.store
        acts, pre = g.state[tag]
        G = S.grad
        n = len(self.packs)
        def logits_grad():   # the generic kernels' bf16 copy of dL/dlogits, padded to 8 channels
            dbuf = g.zeros(f"{tag}dout_t", tuple(dout.shape[:3]) + (8,), T)
            ops.axpby(Feat(dout), 1.0, Feat(dbuf, 0, dout.shape[3]))
            return Feat(dbuf, 0, self.packs[-1].cout_eff)
        dy = None   # the PatchGAN head kernels read the fp32 dout itself
        for i in reversed(range(n)):
            pc, key = self.packs[i], self.LAYERS[i][0]
            x = acts[i]
            if dy is None and not (i == n - 1 and ops.is_patch_head(pc, x)):
                dy = logits_grad()
            bias_sum = None
            if i == n - 1:
                if want_wgrad:
                    bias_sum = Feat(dout)
            elif self.norms[i] is not None:
                self.norms[i].bwd(g, f"{tag}n{i}", dy, pre[i], ACT_LRELU, dy,
                                  db=S.krsc(key + ".bias", G) if want_wgrad and key + ".bias" in S.shapes else None)
            elif want_wgrad:  # layer 0: LReLU mask already folded into dy by the layer-1 dgrad
                bias_sum = dy
            if want_wgrad:
                if bias_sum is not None:
                    ops.channel_sum(bias_sum, S.krsc(key + ".bias", G))
                dw = S.krsc(key + ".weight", G)
                if dy is not None or not ops.patch_head_wgrad(pc, x, dout, dw):
                    dy = dy or logits_grad()
                    ops.conv_wgrad(pc.spec, x, Feat(dy.t, dy.off, pc.spec.cout), dw, self.dtype)
                if ready is not None:
                    ready(key + ".weight")
            if i == 0:
                if not want_dinput:
                    return None
                dx = Feat(g.get(f"{tag}dinput", (x.N, x.H, x.W, pc.spec.cin), torch.float32))
                ops.conv_dgrad(pc, dy or logits_grad(), dx)
                return dx
            dx = Feat(g.get(f"{tag}d{i}", (x.N, x.H, x.W, x.C), T))
            if i == 1:  # previous activation is LReLU without IN: fold its derivative in the epilogue
                ops.conv_dgrad(pc, dy, dx, mask=x, mask_act=2)
            elif not (dy is None and ops.patch_head_dgrad(pc, dout, dx)):   # the head from the fp32 dL/dlogits
                ops.conv_dgrad(pc, dy or logits_grad(), dx)
            dy = dx
        return None


# ----------------------------------------------------------------------------
# VGG-16 features[:16] perceptual extractor  (ir:642-683), frozen
# ----------------------------------------------------------------------------

NO_POOL_FUSION = bool(os.environ.get("IRGAN_NO_POOL_FUSION"))   # A/B: separate conv and maxpool launches


class VGGEngine:
    _pack_batch = None  # ops.PackBatch of self.packs, built on the first pack()

    def __init__(self, store: ParamStore, dtype=BF16):
        self.store, self.dtype, self.tdt = store, dtype, ops.TORCH_DT[dtype]
        self.packs = [_pc(store, str(i), ConvSpec(ci, co, 3, 1, 1, PAD_ZERO), dtype) for i, ci, co in VGG_CONVS]
        dev = store.device
        std = torch.tensor(IMAGENET_STD)
        mean = torch.tensor(IMAGENET_MEAN)
        # ((x+1)/2 - mean)/std  ==  x * (0.5/std) + (0.5 - mean)/std
        self.scale = (0.5 / std).float().to(dev)
        self.shift = ((0.5 - mean) / std).float().to(dev)
        self.bufs = Buffers(dev)

    def pack(self):
        if self._pack_batch is None:
            self._pack_batch = ops.PackBatch(self.packs)
        self._pack_batch.run()

    def forward(self, vin: Feat, bufs: Buffers = None, part=None, keep=True) -> Feat:
        """relu3_3 features of vin.  part = (b0, nb): compute only images [b0, b0+nb)
        into the full-batch activation buffers (the step runs the real and the fake
        half on different streams).  keep=False: no backward will read these images'
        activations (the real half), so a conv followed by MaxPool2d may write the pooled
        map alone (ops.conv_fwd_pool)."""
        g, T = bufs or self.bufs, self.tdt
        x = vin
        acts = g.state["acts"] = [vin]
        sl = (lambda f: f) if part is None else (lambda f: f.batch(*part))  # noqa: E731
        for j, pc in enumerate(self.packs):
            y = Feat(g.get(f"v{j}", (x.N, x.H, x.W, pc.spec.cout), T))
            pooled = j in (1, 3)
            if pooled:   # conv -> ReLU -> MaxPool2d(2) (ir:664), fused where a kernel takes the layer
                p = Feat(g.get(f"p{j}", (x.N, x.H // 2, x.W // 2, pc.spec.cout), T))
                if NO_POOL_FUSION or not ops.conv_fwd_pool(pc, sl(x), sl(y) if keep else None, sl(p)):
                    ops.conv_fwd(pc, sl(x), sl(y), act=ACT_RELU)
                    ops.maxpool(sl(y), sl(p))
            else:
                ops.conv_fwd(pc, sl(x), sl(y), act=ACT_RELU)
            acts.append(y)
            x = y
            if pooled:
                acts.append(p)
                x = p
        return x

    def backward_input(self, dfeat: Feat, nb: int, bufs: Buffers = None) -> Feat:
        """d(input) for the first nb images (frozen weights: backward-data only).
        dfeat = dL/d(relu3_3 output) for those images."""
        g, T = bufs or self.bufs, self.tdt
        acts = [a.batch(0, nb) for a in g.state["acts"]]
        # acts: [vin, v0, v1, p1, v2, v3, p3, v4, v5, v6]
        out_of = {0: 1, 1: 2, 2: 4, 3: 5, 4: 7, 5: 8, 6: 9}     # conv j output index in acts
        in_of = {0: 0, 1: 1, 2: 3, 3: 4, 4: 6, 5: 7, 6: 8}      # conv j input index in acts
        dz = Feat(g.get("dz6", tuple(dfeat.t.shape), T))
        ops.act_bwd(dfeat, acts[out_of[6]], ACT_RELU, dz)
        for j in reversed(range(len(self.packs))):
            pc = self.packs[j]
            xin = acts[in_of[j]]
            if j == 0:
                dvin = Feat(g.get("dvin", (nb, xin.H, xin.W, pc.spec.cin), torch.float32))
                ops.conv_dgrad(pc, dz, dvin)
                return dvin
            prev = in_of[j]
            if prev in (3, 6):  # input is a pool output: dgrad -> maxpool bwd (+relu') of the pool input
                dp = Feat(g.get(f"dp{j}", (nb, xin.H, xin.W, xin.C), T))
                ops.conv_dgrad(pc, dz, dp)
                src = acts[prev - 1]
                dzn = Feat(g.get(f"dz{j - 1}", (nb, src.H, src.W, src.C), T))
                if src.H % 2 or src.W % 2:   # floor pooling: the last odd row / column gets no gradient
                    dzn.t.zero_()
                ops.maxpool_bwd(src, dp, dzn, relu_mask=True)
            else:  # input is a ReLU output: fold relu' into the dgrad epilogue
                dzn = Feat(g.get(f"dz{j - 1}", (nb, xin.H, xin.W, xin.C), T))
                ops.conv_dgrad(pc, dz, dzn, mask=xin, mask_act=1)
            dz = dzn
        return None


# ----------------------------------------------------------------------------
# the train step
# ----------------------------------------------------------------------------

def grad_allreduce(t: torch.Tensor, group=None) -> torch.Tensor:
    """In-place mean of a flat gradient buffer over the data-parallel ranks, as
    one blocking collective.

    Every loss of the step is a mean of per-sample terms and InstanceNorm is
    per-sample, so the mean of the per-rank grads over equal shards is the
    global-batch gradient.  GANStep itself uses the overlapped
    form (BucketedAllreduce); this whole-buffer helper is the reference
    semantics the DP tests splice into the oracle step.  RCCL averages
    natively; gloo (the CPU test backend) sums and we scale.
    """
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return t
    world = dist.get_world_size(group)
    if world == 1:
        return t
    if dist.get_backend(group) == "nccl":
        dist.all_reduce(t, op=dist.ReduceOp.AVG, group=group)
    else:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        t.div_(world)
    return t


def replica_digest(tensors) -> torch.Tensor:
    """Exact int64 digest of fp32 tensors (their bit patterns): a plain and a
    position-weighted sum per tensor.  Equal digests on every rank = the data-parallel
    replicas hold bit-identical parameters (bench.py's post-run check)."""
    out = []
    for t in tensors:
        b = t.detach().reshape(-1).view(torch.int32).to(torch.int64)
        w = torch.arange(b.numel(), device=b.device, dtype=torch.int64) % 65521 + 1
        out += [b.sum(), (b * w).sum()]
    return torch.stack(out)


def replicas_identical(tensors, group=None, force=False) -> bool:
    """True when every rank of ``group`` holds bit-identical ``tensors`` (max == min of
    the digests over ranks); True without a process group (and at world size 1 unless
    ``force``: then the MAX / MIN collectives run anyway)."""
    import torch.distributed as dist
    d = replica_digest(tensors)
    if not (dist.is_available() and dist.is_initialized()) or (dist.get_world_size(group) == 1 and not force):
        return True
    if dist.get_backend(group) != "nccl":
        d = d.cpu()
    hi, lo = d.clone(), d.clone()
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    return bool(torch.equal(hi, lo))


class BucketedAllreduce:
    """Mean of a flat gradient buffer over the ranks, reduced tail-first in buckets
    while the producing backward is still running (SURVEY.md 8e overlap schedule).

    The backward calls ``ready(key)`` when every grad from ``key`` to the end of the
    flat buffer is final.  Once the not-yet-reduced tail reaches ``bucket_bytes`` it
    is handed to the collective with ``async_op=True``: RCCL runs it on its own
    stream after an event on the compute stream, so the all-reduce of layer L
    overlaps the backward of layers < L.  ``finish()`` reduces the remainder and
    makes the compute stream wait for every bucket (Adam reads the result).
    Buckets are contiguous slices of the flat buffer, so the reduction is the
    same element-wise mean as one whole-buffer all-reduce.
    """

    def __init__(self, store: ParamStore, group=None, bucket_bytes=8 << 20, force=False):
        """force: issue the collectives even at world size 1 (a process group must be
        initialised) -- the RCCL path exercised on one GPU (tests/test_gpu_dp.py)."""
        self.store, self.group, self.bucket_bytes = store, group, bucket_bytes
        self.end, self.works, self.world, self.avg = store.numel, [], 1, True
        import torch.distributed as dist
        self.force = False
        if dist.is_available() and dist.is_initialized():
            self.world = dist.get_world_size(group)
            self.avg = dist.get_backend(group) == "nccl"
            self.force = bool(force)

    @property
    def active(self):
        return self.world > 1 or self.force

    def _launch(self, start):
        import torch.distributed as dist
        if start >= self.end:
            return
        t = self.store.grad[start:self.end]
        op = dist.ReduceOp.AVG if self.avg else dist.ReduceOp.SUM
        self.works.append((dist.all_reduce(t, op=op, group=self.group, async_op=True), t, start, self.end))
        self.end = start

    def start(self):
        """Reduce the whole buffer as one asynchronous collective."""
        if self.active:
            self._launch(0)

    def ready(self, key):
        if not self.active:
            return
        start = self.store.offsets[key]
        if (self.end - start) * 4 >= self.bucket_bytes:
            self._launch(start)

    def finish(self, apply=None):
        """Reduce the remainder, then per bucket (in issue order, tail-first): make the
        compute stream wait for that bucket only and call ``apply(start, end)`` -- the
        optimizer update of the bucket is queued behind its own collective and runs
        while the later buckets are still being reduced (the G-Adam of
        bucket k overlaps the all-reduce of bucket k+1).  Each element of the flat
        buffer lies in exactly one bucket, so this is the whole-buffer mean + update."""
        if not self.active:
            if apply is not None:
                apply(0, self.store.numel)
            return
        self._launch(0)
        for w, t, a, b in self.works:
            w.wait()
            if not self.avg:
                t.div_(self.world)
            if apply is not None:
                apply(a, b)
        self.works, self.end = [], self.store.numel


# IRGAN_JOIN_TIMING=1: per step, timing events at the phase boundaries of both streams
# (diagnostics: where the D step sits on the critical path).  Keys: start, gfwd (main: G
# forward done), d0 / dend (side: the D step's first / last launch), terms (main: the G-step
# terms done), join (main: after its wait for the side stream), end.
JOIN_TIMES = [] if os.environ.get("IRGAN_JOIN_TIMING") else None


def _mark(ph, key, stream):
    if ph is not None:
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream)
        ph[key] = e


class GANStep:
    """Buffers, engines and the fused step for one rank.

    Loss slots (fp64, device): 0 loss_D, 1 lambda_gan*GAN, 2 L1*l, 3 perc*l, 4 TV*l, 5 SSIM*l.
    """

    def __init__(self, G: ParamStore, D: ParamStore, V: ParamStore, cfg, dtype=BF16, process_group=None,
                 gen: GeneratorEngine = None, dis: DiscriminatorEngine = None, vgg: VGGEngine = None,
                 force_reduce=False):
        """force_reduce: run the gradient collectives even at world size 1 (see
        BucketedAllreduce): the DP schedule on one device."""
        self.G, self.D, self.V, self.cfg, self.dtype = G, D, V, cfg, dtype
        self.tdt = ops.TORCH_DT[dtype]
        self.gen = gen or GeneratorEngine(G, dtype, ngf=cfg.ngf, input_nc=cfg.input_nc, output_nc=cfg.output_nc,
                                          no_antialias=cfg.no_antialias, no_antialias_up=cfg.no_antialias_up,
                                          fp8=getattr(cfg, "compute_dtype", "bf16") == "fp8", norm=cfg.norm)
        self.dis = dis or DiscriminatorEngine(D, dtype, input_nc=cfg.input_nc + cfg.output_nc, norm=cfg.norm)
        self.dbufs = Buffers(G.device)   # the D step's own G forward when G has dropout
        self.vgg = vgg or VGGEngine(V, dtype)
        self.bufs = Buffers(G.device)
        self.losses = torch.zeros(8, dtype=torch.float64, device=G.device)
        self.pg = process_group
        self.g_reduce = BucketedAllreduce(G, process_group, force=force_reduce)
        self.d_reduce = BucketedAllreduce(D, process_group, force=force_reduce)
        self.lr_scale = 1.0
        # the D step (D forward/backward on [real; fake] and its all-reduce) runs on a
        # side stream, concurrently with the G-step terms that do not read D (L1,
        # VGG, TV, SSIM); IRGAN_NO_D_OVERLAP=1 keeps everything on one stream
        self.side = None
        if G.device.type == "cuda" and not os.environ.get("IRGAN_NO_D_OVERLAP"):
            self.side = torch.cuda.Stream(device=G.device)
        self.G.dev_adam = self.D.dev_adam = G.device.type == "cuda"
        self.vgg.pack()
        self.gen.pack()
        self.dis.pack()

    def step(self, ir: torch.Tensor, rgb: torch.Tensor):
        """One train step on NCHW fp32 device tensors; returns the loss vector (device)."""
        cfg, b, T = self.cfg, self.bufs, self.tdt
        B, _, H, W = ir.shape
        cin, cout = cfg.input_nc, cfg.output_nc
        self.losses.zero_()
        L = self.losses
        main = torch.cuda.current_stream() if self.side is not None else None
        ph = {} if JOIN_TIMES is not None and main is not None else None
        _mark(ph, "start", main)
        side_ctx = (lambda: torch.cuda.stream(self.side)) if main is not None else _nullcontext  # noqa: E731
        rgb_h = b.get("rgb_nhwc", (B, H, W, cout), torch.float32)
        ops.nchw_to_nhwc(rgb.contiguous(), Feat(rgb_h))
        # ---- VGG features of the real images (ir:1668) need nothing from G: side stream,
        # concurrent with the G forward
        vin = Feat(b.zeros("vin", (2 * B, H, W, max(8, cout)), T), 0, self.vgg.packs[0].cin_eff)
        # D input [real; fake] as one 2B batch, cat([ir, img], 1) (ir:1639-1640) zero-padded to
        # 8 channels (narrow-input conv path): the ir channels of both halves and the real
        # images are written beside the G forward; the fake images once G has run
        dpad = max(8, cin + cout)
        din = Feat(b.zeros("din2", (2 * B, H, W, dpad), T), 0, self.dis.packs[0].cin_eff)
        vgg_side = main is not None and not os.environ.get("IRGAN_NO_VGG_OVERLAP")
        ev_in = None
        if vgg_side:
            ev_in = torch.cuda.Event()
            ev_in.record(main)                    # the real images in NHWC, the zeroed VGG input

        def vgg_real():
            with side_ctx() if vgg_side else _nullcontext():
                if ev_in is not None:
                    self.side.wait_event(ev_in)
                for h in (0, B):
                    ops.nchw_to_nhwc(ir.contiguous(), Feat(din.t[h:h + B], 0, cin))
                ops.axpby(Feat(rgb_h), 1.0, Feat(din.t[:B], cin, cout))
                ops.affine(Feat(rgb_h), self.vgg.scale, self.vgg.shift, vin.batch(B, B))
                self.vgg.forward(vin, part=(B, B), keep=False)   # no backward through the real half
            if vgg_side:
                _mark(ph, "vgg_real", self.side)
                ev = torch.cuda.Event()
                ev.record(self.side)
                return ev
            return None

        # enqueued before the G forward's launches (after them measured neutral,
        # profiles/r03_vgg_after_gfwd_ab.txt)
        ev_vgg = vgg_real()
        # ---- G forward once: ir:1638 and ir:1657 compute the same image -- unless G has
        # dropout, whose two calls draw two masks: then the D step gets its own forward
        # (ir:1638-1639, under no_grad: its activations are never read back)
        self.gen.training = True
        fake_d = self.gen.forward(ir, bufs=self.dbufs) if self.gen.use_dropout else None
        fake = self.gen.forward(ir)
        # ---- D step on [real; fake] as one 2B batch (ir:1636-1651), on the side stream
        dfake = b.get("dfake", (B, H, W, cout), torch.float32)

        def g_terms():
            # ---- G step terms that do not read D (ir:1656-1681)
            self.G.zero_grad()
            dfake.zero_()
            ops.l1(fake, rgb_h, cfg.lambda_L1, dfake, L[2:3], accumulate=True)
            # perceptual (ir:1667-1669): VGG on the fake half; the real half ran on the side stream
            ops.affine(Feat(fake), self.vgg.scale, self.vgg.shift, vin.batch(0, B))
            feat = self.vgg.forward(vin, part=(0, B))
            if ev_vgg is not None:
                main.wait_event(ev_vgg)
            dfeat = b.get("dfeat", (B, feat.H, feat.W, feat.C), T)
            ops.l1(feat.t[:B], feat.t[B:], cfg.lambda_perc, dfeat, L[3:4])
            dv = self.vgg.backward_input(Feat(dfeat), B)
            ops.affine(dv, self.vgg.scale, None, Feat(dfake), accumulate=True)
            ops.tv(Feat(fake), cfg.lambda_tv, dfake, L[4:5])
            ssim_work = b.flat("ssim_work", 10 * fake.numel())
            ops.ssim(Feat(fake), Feat(rgb_h), cfg.lambda_ssim, dfake, L[5:6], ssim_work)

        # host enqueue order: the main stream's G-step terms before the side stream's D step --
        # the dependencies are the event edges either way; enqueued first, the terms start
        # right behind the G forward instead of after ~90 D-step launches (1204 vs 1199 img/s,
        # profiles/r03_terms_first_ab.txt)
        terms_first = main is not None
        ev_fwd = None
        if main is not None:
            _mark(ph, "gfwd", main)
            ev_fwd = torch.cuda.Event()
            ev_fwd.record(main)                   # G output, the zeroed losses and D inputs
        if terms_first:
            g_terms()
        with side_ctx():
            if ev_fwd is not None:
                self.side.wait_event(ev_fwd)
                _mark(ph, "d0", self.side)
            # [real; fake] as one 2B batch.  (The real half apart, beside the G forward, measured
            # -0.8 %: the G forward slowed by what it took off the join, profiles/r05_ab1_dsplit.txt)
            self.D.zero_grad()
            ops.axpby(Feat(fake if fake_d is None else fake_d), 1.0, Feat(din.t[B:], cin, cout))
            pred = self.dis.forward(din, tag="d")
            dpred = b.get("dpred", tuple(pred.shape), torch.float32)
            ops.hinge(pred, pred[:B].numel(), 0, 1.0, dpred, L[0:1])
            # D grads reduced tail-first under the D backward (8 MB buckets: model.8 + the head
            # go out while model.5 / .2 / .0 still run), each bucket's Adam right behind it
            # (the weight gradients on the main stream instead, beside this chain: -1.4 %, the main
            # stream is still busy with the G-step terms then, profiles/r06_d_ab.txt)
            self.dis.backward(dpred, want_wgrad=True, want_dinput=False, tag="d", ready=self.d_reduce.ready)
            # D Adam, then the G-step GAN term through the updated D (ir:1651, 1659-1662),
            # still on the side stream: the main stream meanwhile runs the G-step terms
            # that do not read D (L1, VGG, TV, SSIM)
            self.d_reduce.finish(self.D.adam_begin(cfg.lr_D * self.lr_scale, cfg.beta1, cfg.beta2))
            self.dis.pack()
            # the G-step D pass reads cat([ir, fake]): the fake half of the D input (rewritten
            # when the D step saw the other dropout draw)
            if fake_d is not None:
                ops.axpby(Feat(fake), 1.0, Feat(din.t[B:], cin, cout))
            predg = self.dis.forward(din.batch(B, B), tag="g")
            dpg = b.get("dpredg", tuple(predg.shape), torch.float32)
            ops.hinge(predg, predg.numel(), 1, cfg.lambda_gan, dpg, L[1:2])
            dd = self.dis.backward(dpg, want_wgrad=False, want_dinput=True, tag="g")
            _mark(ph, "dend", self.side)
        if not terms_first:
            g_terms()
        if main is not None:
            _mark(ph, "terms", main)
            main.wait_stream(self.side)           # the GAN term's d fake
            _mark(ph, "join", main)
        ops.axpby(dd.sl(cin, cout), 1.0, Feat(dfake), 1.0)
        self.gen.backward(dfake, ready=self.g_reduce.ready)
        self.g_reduce.finish(self.G.adam_begin(cfg.lr_G * self.lr_scale, cfg.beta1, cfg.beta2))
        self.gen.pack()
        if ph is not None:
            _mark(ph, "end", main)
            JOIN_TIMES.append(ph)
        return L

    @staticmethod
    def loss_dict(L: torch.Tensor, cfg) -> dict:
        v = L.tolist()
        gan = v[1] / cfg.lambda_gan if cfg.lambda_gan else 0.0
        return dict(loss_D=v[0], loss_G=v[1] + v[2] + v[3] + v[4] + v[5], loss_G_GAN=gan, loss_G_L1=v[2],
                    loss_G_perc=v[3], loss_G_TV=v[4], loss_G_ssim=v[5])
