"""Thin typed wrappers over the C ABI (include/irgan.h) on device tensors.

Activations are NHWC ``Feat`` slices (tensor, channel offset, channel count);
torch is used for device memory and the current HIP stream only.  Every
function here launches hand-written HIP kernels from libirgan.so.
"""
from __future__ import annotations

import ctypes
import math
import os

import torch

from . import _lib
from ._lib import (ACT_LRELU, ACT_NONE, ACT_RELU, ACT_TANH, BF16, F32, FP8, IN_PARTS, PAD_REFLECT,  # noqa: F401
                   PAD_ZERO)

TORCH_DT = {F32: torch.float32, BF16: torch.bfloat16, FP8: torch.float8_e4m3fn}


def dt_code(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return F32
    if t.dtype == torch.bfloat16:
        return BF16
    if t.dtype == torch.float8_e4m3fn:
        return FP8
    raise TypeError(f"unsupported dtype {t.dtype}")


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def P(t):
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def Pi(t, i):
    """Pointer to element i of a contiguous device tensor (a scale / amax slot)."""
    return ctypes.c_void_p(t.data_ptr() + i * t.element_size())


_DET = [False]
CONV_DETERMINISTIC = _lib.header_enum("IRGAN_CONV_DETERMINISTIC")


def set_deterministic(on: bool) -> bool:
    """Deterministic mode for the launches this module makes: every split-K weight gradient
    carries IRGAN_CONV_DETERMINISTIC in its descriptor (ordered slab reduction, never fp32
    atomics), so the step is bitwise reproducible under any stream schedule.  Host-side
    state of this module (the library keeps none).  Returns the previous setting."""
    old, _DET[0] = _DET[0], bool(on)
    return old


_RING_WS = {}


def _ring_ws(dev, floats):
    """Per-(device, stream) fp32 workspace of the ring's line GEMM (irgan_reflect_dgrad_ring_ws)."""
    key = (dev, torch.cuda.current_stream(dev).cuda_stream)
    w = _RING_WS.get(key)
    if w is None or w.numel() < floats:
        w = _RING_WS[key] = torch.empty(floats, dtype=torch.float32, device=dev)
    return w


RING_LINE = [True]


def set_ring_line(on: bool) -> bool:
    """The line-GEMM ring launches (default) or the general reflect_ring_kernel for the
    ResnetBlock shapes (the A/B reference of the line form).  Returns the previous setting."""
    old, RING_LINE[0] = RING_LINE[0], bool(on)
    return old


RING_EPI = [True]


def set_ring_epi(on: bool) -> bool:
    """The ResnetBlock ring folded into the interior launch's store pass
    (irgan_conv_dgrad_reflect_line, default) or the separate fold launch after it -- the
    same dx bit for bit (tests/test_gpu_ring_epi.py).  Returns the previous setting."""
    old, RING_EPI[0] = RING_EPI[0], bool(on)
    return old


def _ring(d, dy: "Feat", buf, p, dx: "Feat"):
    """The reflect-pad ring of a bf16 backward-data onto dx (after its interior): the line
    GEMM + fold on ResnetBlock shapes, else the general ring launch (the library decides)."""
    ws = _ring_ws(dx.t.device, dx.N * 4 * 68 * dx.C)
    _lib.call("irgan_reflect_dgrad_ring_ws", ctypes.byref(d), dy.ptr, P(buf), p, dx.ptr, P(ws),
              ws.numel() if RING_LINE[0] else 0, 1 << 20, stream())


class LaunchTimer:
    """Optional HIP-event timing of tagged conv launches (bench.py's live
    roofline).  Events are recorded on the launching stream around each launch."""

    def __init__(self, tags):
        self.tags = set(tags)   # None: every tagged launch (tools/layer_times.py)
        self.pending = []
        self.enabled = False

    def wrap(self, tag, fn):
        if not self.enabled or (self.tags is not None and tag not in self.tags):
            return fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        out = fn()
        b.record()
        self.pending.append((tag, a, b))
        return out

    def summary(self):
        torch.cuda.synchronize()
        agg = {}
        for tag, a, b in self.pending:
            n, t = agg.get(tag, (0, 0.0))
            agg[tag] = (n + 1, t + a.elapsed_time(b))
        return {k: (n, t / n) for k, (n, t) in agg.items()}  # (launches, mean ms)


TIMER = LaunchTimer(())


def hbm_tag(kind, x: "Feat"):
    """Tag of an HBM-bound pass over the NHWC tensor x (bench.py's GB/s lines)."""
    return f"{kind}:b{x.N}@{x.H}x{x.W}x{x.C}"


def _timed(kind, x, fn):
    return TIMER.wrap(hbm_tag(kind, x), fn) if TIMER.enabled else fn()


def conv_tag(kind, spec, x_hw, n=None):
    pad = "r" if spec.mode == PAD_REFLECT else "z"
    nb = f"b{n}/" if n is not None else ""
    return f"{kind}:{spec.cin}x{spec.cout}k{spec.k}s{spec.stride}{pad}@{nb}{x_hw[0]}x{x_hw[1]}"


class Feat:
    """NHWC channel slice: element (p, c) at t.view(-1)[p*ld + off + c]."""
    __slots__ = ("t", "off", "C")

    def __init__(self, t: torch.Tensor, off: int = 0, C: int | None = None):
        assert t.dim() == 4 and t.is_contiguous()
        self.t, self.off = t, off
        self.C = t.shape[3] - off if C is None else C

    N = property(lambda s: s.t.shape[0])
    H = property(lambda s: s.t.shape[1])
    W = property(lambda s: s.t.shape[2])
    ld = property(lambda s: s.t.shape[3])
    dt = property(lambda s: dt_code(s.t))
    P = property(lambda s: s.t.shape[0] * s.t.shape[1] * s.t.shape[2])

    @property
    def ptr(self):
        return ctypes.c_void_p(self.t.data_ptr())

    def sl(self, off, C):
        return Feat(self.t, self.off + off, C)

    def batch(self, b0, nb):
        return Feat(self.t[b0:b0 + nb], self.off, self.C)


# ----------------------------------------------------------------------------
# convolution
# ----------------------------------------------------------------------------

class ConvSpec:
    """A conv layer's geometry.  For nn.ConvTranspose2d the spec describes the
    conv it transposes (cout = ConvT in-channels, cin = ConvT out-channels)."""

    def __init__(self, cin, cout, k, stride=1, pad=0, mode=PAD_ZERO):
        self.cin, self.cout, self.k, self.stride, self.pad, self.mode = cin, cout, k, stride, pad, mode

    def out_hw(self, H, W):
        p, k, s = self.pad, self.k, self.stride
        return (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1

    def phases(self, reflect_padded=False):
        """backward-data phase decomposition per axis: (phase, tap residue, taps, c0)."""
        k, s = self.k, self.stride
        p = 0 if reflect_padded else self.pad
        out = []
        for ph in range(s):
            tr = (ph + p) % s
            A = max(0, -(-(k - tr) // s))
            base = (ph + p - tr) // s
            out.append((ph, tr, A, base - A + 1))
        return out


def _desc(**kw):
    """irgan_conv_desc from keyword fields.  Built by the Structure's own keyword
    constructor (~2 us on the host, half the setattr loop: ~150 conv launches per step);
    values that are not plain ints (numpy / torch scalars) take the converting path."""
    try:
        return _lib.ConvDesc(**kw)
    except TypeError:
        d = _lib.ConvDesc()
        for k, v in kw.items():
            setattr(d, k, int(v))
        return d


def _rup(a, b):
    return (a + b - 1) // b * b


def weight_pack(master: torch.Tensor, dst: torch.Tensor, cout, kh, kw, cin, transpose=0, s=1, tyr=0, ay=0,
                txr=0, ax=0, cpad=0, kalign=1):
    _lib.call("irgan_weight_pack", P(master), P(dst), dt_code(dst), cout, kh, kw, cin, transpose, s, tyr, ay, txr,
              ax, cpad, kalign, stream())


def eff_channels(c, dtype):
    """Channel count a conv input is stored with: bf16 narrow inputs (1/3/4 ch)
    are zero-padded to 8 so the LDS-DMA kernel reads 16-byte chunks."""
    return 8 if (dtype == BF16 and c < 8) else c


class PackedConv:
    """Per-layer packed weights: forward (cast) and backward-data (flipped /
    per-phase) images in the compute dtype, refreshed after each optimizer step.
    bf16 rows are [taps][channels] zero-padded to a multiple of 64 (the K-tile)."""

    def __init__(self, spec: ConvSpec, master: torch.Tensor, bias: torch.Tensor | None, dtype: int,
                 need_dgrad=True, reflect_dgrad=None):
        self.spec, self.master, self.bias, self.dtype = spec, master, bias, dtype
        dev = master.device
        tdt = TORCH_DT[dtype]
        k = spec.k
        self.cin_eff = eff_channels(spec.cin, dtype)     # forward input channels as stored
        self.cout_eff = eff_channels(spec.cout, dtype)   # backward-data input (dY) channels as stored
        self.kalign = 64 if dtype == BF16 else 1
        kf = _rup(k * k * self.cin_eff, self.kalign)
        self.fwd = master if dtype == F32 else torch.empty(spec.cout * kf, dtype=tdt, device=dev)
        self.reflect = spec.mode == PAD_REFLECT if reflect_dgrad is None else reflect_dgrad
        self.dg = []
        if need_dgrad:
            for (py, tyr, ay, c0y) in spec.phases(self.reflect):
                for (px, txr, ax, c0x) in spec.phases(self.reflect):
                    kd = _rup(ay * ax * self.cout_eff, self.kalign)
                    buf = torch.empty(spec.cin * kd, dtype=tdt, device=dev)
                    self.dg.append(((py, tyr, ay, c0y), (px, txr, ax, c0x), buf))

    def jobs(self):
        """The weight_pack jobs of this layer as irgan_pack_desc records."""
        s, out = self.spec, []
        if self.dtype != F32:
            out.append(PackDesc(self.master.data_ptr(), self.fwd.data_ptr(), dt_code(self.fwd), s.cout, s.k, s.k,
                                s.cin, 0, 1, 0, 0, 0, 0, self.cin_eff, self.kalign, 0))
        for (py, tyr, ay, _), (px, txr, ax, _), buf in self.dg:
            out.append(PackDesc(self.master.data_ptr(), buf.data_ptr(), dt_code(buf), s.cout, s.k, s.k, s.cin, 1,
                                s.stride, tyr, ay, txr, ax, self.cout_eff, self.kalign, 0))
        return out

    def pack(self):
        s = self.spec
        if self.dtype != F32:
            weight_pack(self.master, self.fwd, s.cout, s.k, s.k, s.cin, cpad=self.cin_eff, kalign=self.kalign)
        for (py, tyr, ay, _), (px, txr, ax, _), buf in self.dg:
            weight_pack(self.master, buf, s.cout, s.k, s.k, s.cin, 1, s.stride, tyr, ay, txr, ax,
                        cpad=self.cout_eff, kalign=self.kalign)


class PackDesc(ctypes.Structure):
    """irgan_pack_desc (include/irgan.h)."""
    _fields_ = [("src", ctypes.c_void_p), ("dst", ctypes.c_void_p)] + [
        (n, ctypes.c_int32) for n in "dtype Cout KH KW Cin transpose s tyr Ay txr Ax cpad kalign reserved".split()]


class PackBatch:
    """All re-pack jobs of a set of layers as ONE irgan_weight_pack_batch launch.
    The descriptor table lives on the device; it is rebuilt only if a packed
    buffer moved (buffers are allocated once, so normally never)."""

    def __init__(self, packs):
        self.packs = list(packs)
        self.key, self.table, self.n = None, None, 0

    def run(self):
        jobs = [j for p in self.packs for j in p.jobs()]
        key = tuple((j.src, j.dst) for j in jobs)
        if key != self.key:
            arr = (PackDesc * len(jobs))(*jobs)
            raw = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
            self.table = raw.to(self.packs[0].master.device)
            self.key, self.n = key, len(jobs)
        if self.n:
            _lib.call("irgan_weight_pack_batch", P(self.table), self.n, stream())


def conv_fwd(pc: PackedConv, x: Feat, y: Feat, act=ACT_NONE, bias=True, accumulate=False, mask: Feat = None,
             mask_act=0):
    s = pc.spec
    Ho, Wo = s.out_hw(x.H, x.W)
    assert (y.H, y.W, y.C) == (Ho, Wo, s.cout) and x.C == pc.cin_eff and y.N == x.N, "conv_fwd shape mismatch"
    d = _desc(N=x.N, H=x.H, W=x.W, Cin=pc.cin_eff, ldx=x.ld, xoff=x.off, Ho=Ho, Wo=Wo, Cout=s.cout, ldy=y.ld,
              yoff=y.off, OH=Ho, OW=Wo, omy=1, ooy=0, omx=1, oox=0, KH=s.k, KW=s.k, sy=s.stride, sx=s.stride,
              c0y=-s.pad, c0x=-s.pad, pad_mode=s.mode, act=act, accumulate=int(accumulate), dtype=pc.dtype,
              out_dtype=y.dt, mask_act=mask_act, ldm=mask.ld if mask else 0, moff=mask.off if mask else 0,
              cin_real=s.cin if s.cin < pc.cin_eff else 0)
    assert x.dt == pc.dtype
    TIMER.wrap(conv_tag("fwd", s, (x.H, x.W), x.N), lambda: _lib.call(
        "irgan_conv_fwd", ctypes.byref(d), x.ptr, P(pc.fwd), P(pc.bias if bias else None), y.ptr,
        mask.ptr if mask else None, stream()))


IRGAN_EUNSUPPORTED = 1002   # include/irgan.h


def conv_fwd_pool(pc: PackedConv, x: Feat, y, yp: Feat, act=ACT_RELU) -> bool:
    """y = act(conv(x)) (y: a Feat, or None when only the pooled map is needed) and yp = its
    2x2 max-pool, in one launch (irgan_conv_fwd_pool: the VGG conv1_2 -> MaxPool2d(2),
    ir:664).  False when the layer has no fused kernel -- then NOTHING ran."""
    s = pc.spec
    Ho, Wo = s.out_hw(x.H, x.W)
    if pc.dtype != BF16 or yp.dt != BF16 or yp.off or yp.ld != s.cout or Ho % 2 or Wo % 2:
        return False
    assert (yp.N, yp.H, yp.W, yp.C) == (x.N, Ho // 2, Wo // 2, s.cout) and x.C == pc.cin_eff
    if y is not None:
        assert (y.H, y.W, y.C, y.N, y.dt) == (Ho, Wo, s.cout, x.N, BF16)
    d = _desc(N=x.N, H=x.H, W=x.W, Cin=pc.cin_eff, ldx=x.ld, xoff=x.off, Ho=Ho, Wo=Wo, Cout=s.cout,
              ldy=y.ld if y is not None else s.cout, yoff=y.off if y is not None else 0, OH=Ho, OW=Wo, omy=1, ooy=0,
              omx=1, oox=0, KH=s.k, KW=s.k, sy=s.stride, sx=s.stride, c0y=-s.pad, c0x=-s.pad, pad_mode=s.mode,
              act=act, accumulate=0, dtype=pc.dtype, out_dtype=BF16, mask_act=0, ldm=0, moff=0)
    fn = getattr(_lib.load(), "irgan_conv_fwd_pool")
    rc = TIMER.wrap(conv_tag("fwdpool", s, (x.H, x.W), x.N), lambda: fn(
        ctypes.byref(d), x.ptr, P(pc.fwd), P(pc.bias), y.ptr if y is not None else None, yp.ptr, stream()))
    if rc == IRGAN_EUNSUPPORTED:
        return False
    if rc != 0:
        raise _lib.IrganError(f"irgan_conv_fwd_pool failed with code {rc}")
    return True


def conv_fwd_stats(pc: PackedConv, x: Feat, y: Feat, part: torch.Tensor) -> int:
    """conv_fwd (no activation) that also writes y's InstanceNorm partials into
    ``part`` (irgan_conv_fwd_stats).  Returns the partials per image, or 0 when the
    layer has no fused kernel -- then NOTHING ran and the caller does conv_fwd +
    in_stats."""
    s = pc.spec
    if pc.dtype != BF16 or y.dt != BF16 or s.cout % 64 or s.cout == 192 or (s.stride != 1 and s.k != 4):
        return 0
    Ho, Wo = s.out_hw(x.H, x.W)
    assert (y.H, y.W, y.C) == (Ho, Wo, s.cout) and x.C == pc.cin_eff and y.N == x.N, "conv_fwd shape mismatch"
    d = _desc(N=x.N, H=x.H, W=x.W, Cin=pc.cin_eff, ldx=x.ld, xoff=x.off, Ho=Ho, Wo=Wo, Cout=s.cout, ldy=y.ld,
              yoff=y.off, OH=Ho, OW=Wo, omy=1, ooy=0, omx=1, oox=0, KH=s.k, KW=s.k, sy=s.stride, sx=s.stride,
              c0y=-s.pad, c0x=-s.pad, pad_mode=s.mode, act=ACT_NONE, accumulate=0, dtype=pc.dtype,
              out_dtype=y.dt, mask_act=0, ldm=0, moff=0, cin_real=s.cin if s.cin < pc.cin_eff else 0)
    nb = ctypes.c_int32(0)
    fn = getattr(_lib.load(), "irgan_conv_fwd_stats")
    rc = TIMER.wrap(conv_tag("fwd", s, (x.H, x.W), x.N), lambda: fn(
        ctypes.byref(d), x.ptr, P(pc.fwd), P(pc.bias), y.ptr, P(part), ctypes.byref(nb), stream()))
    if rc == IRGAN_EUNSUPPORTED:
        return 0
    if rc != 0:
        raise _lib.IrganError(f"irgan_conv_fwd_stats failed with code {rc}")
    return int(nb.value)




# D's last layer (4x4, stride 1, pad 1, one output channel) on the dedicated VALU kernels
# (csrc/head.hip); IRGAN_NO_PATCH_HEAD=1 runs it on the generic conv kernels
PATCH_HEAD = [os.environ.get("IRGAN_NO_PATCH_HEAD") != "1"]


def is_patch_head(pc: PackedConv, x: Feat) -> bool:
    s = pc.spec
    return (PATCH_HEAD[0] and pc.dtype == BF16 and x.dt == BF16 and s.cout == 1 and s.k == 4 and s.stride == 1
            and s.pad == 1 and s.mode == PAD_ZERO and s.cin == x.C == 512)


def patch_head_fwd(pc: PackedConv, x: Feat, y: torch.Tensor) -> bool:
    """y (fp32 [N][H-1][W-1][1]) = the PatchGAN head conv of x + bias (irgan_patch_head_fwd);
    False (nothing launched) where the dedicated kernel does not take the layer."""
    if not is_patch_head(pc, x):
        return False
    assert y.dtype == torch.float32 and tuple(y.shape) == (x.N, x.H - 1, x.W - 1, 1) and y.is_contiguous()

    ws = _wgrad_ws(y.device)   # the per-pixel tap products; consumed by the same stream's next launch

    def launch():
        rc = _lib.load().irgan_patch_head_fwd(x.ptr, x.N, x.H, x.W, x.C, x.ld, x.off, P(pc.fwd),
                                              P(pc.bias) if pc.bias is not None else None, P(y), P(ws),
                                              ws.numel(), stream())
        if rc not in (0, IRGAN_EUNSUPPORTED):
            raise _lib.IrganError(f"irgan_patch_head_fwd failed with code {rc}")
        return rc == 0
    return TIMER.wrap(conv_tag("fwd", pc.spec, (x.H, x.W), x.N), launch)


def patch_head_dgrad(pc: PackedConv, g: torch.Tensor, dx: Feat) -> bool:
    """dx (bf16, written) = the PatchGAN head's backward-data of g = dL/dy (fp32 [N][H-1][W-1][1])
    (irgan_patch_head_dgrad); False (nothing launched) where the kernel does not take the layer."""
    if not is_patch_head(pc, dx):
        return False
    assert g.dtype == torch.float32 and tuple(g.shape[:3]) == (dx.N, dx.H - 1, dx.W - 1) and g.is_contiguous()

    def launch():
        rc = _lib.load().irgan_patch_head_dgrad(P(g), g.shape[3], P(pc.fwd), dx.ptr, dx.N, dx.H, dx.W, dx.C, dx.ld,
                                                dx.off, stream())
        if rc not in (0, IRGAN_EUNSUPPORTED):
            raise _lib.IrganError(f"irgan_patch_head_dgrad failed with code {rc}")
        return rc == 0
    return TIMER.wrap(conv_tag("dgrad", pc.spec, (dx.H, dx.W), dx.N), launch)


def patch_head_wgrad(pc: PackedConv, x: Feat, g: torch.Tensor, dw: torch.Tensor) -> bool:
    """dw (fp32 KRSC view, accumulated) += the PatchGAN head's weight gradient from x and
    g = dL/dy (fp32 [N][H-1][W-1][1]) (irgan_patch_head_wgrad: block partials in the wgrad
    workspace, ordered reduce); False (nothing launched) where the kernel does not take it."""
    if not is_patch_head(pc, x):
        return False
    assert g.dtype == torch.float32 and tuple(g.shape[:3]) == (x.N, x.H - 1, x.W - 1) and g.is_contiguous()
    assert dw.dtype == torch.float32 and dw.is_contiguous() and dw.numel() == 16 * x.C
    ws = _wgrad_ws(dw.device)

    def launch():
        rc = _lib.load().irgan_patch_head_wgrad(x.ptr, x.N, x.H, x.W, x.C, x.ld, x.off, P(g), g.shape[3], P(dw),
                                                P(ws), ws.numel(), stream())
        if rc not in (0, IRGAN_EUNSUPPORTED):
            raise _lib.IrganError(f"irgan_patch_head_wgrad failed with code {rc}")
        return rc == 0
    return TIMER.wrap(conv_tag("wgrad", pc.spec, (x.H, x.W), x.N), launch)


def conv_dgrad(pc: PackedConv, dy: Feat, dx: Feat, accumulate=False, mask: Feat = None, mask_act=0,
               pad_buf: torch.Tensor = None, bias=False):
    """dx = d(conv)/dx^T dy.  Reflect-padded layers: interior straight into dx and the
    padded ring folded onto dx's border band -- bf16 ResnetBlock shapes: the ring's line
    GEMM, then the interior launch whose store pass adds the ring terms
    (irgan_conv_dgrad_reflect_line); other bf16 shapes: the interior launch, then the ring
    (irgan_reflect_dgrad_ring_ws); fp32: split-K ring partials in pad_buf (fp32 scratch)
    folded by irgan_reflect_ring_fold; stride-2 layers launch per phase (or all four
    phases in one irgan_conv_dgrad_s2 launch)."""
    s = pc.spec
    assert dy.C == pc.cout_eff and dx.C == s.cin and dy.dt == pc.dtype
    if pc.reflect:
        # Backward-data over the reflect-padded domain g (Hp x Wp) folded back:
        # the interior u in [p, H+p) maps 1:1 onto dx and is written there
        # directly; only the ring of width p is computed separately.
        p = s.pad
        H, W = dx.H, dx.W
        Hp, Wp = H + 2 * p, W + 2 * p
        assert mask is None
        (_, _, ay, c0y), (_, _, ax, c0x), buf = pc.dg[0]
        base = dict(N=dy.N, H=dy.H, W=dy.W, Cin=pc.cout_eff, ldx=dy.ld, xoff=dy.off, Cout=s.cin, KH=ay, KW=ax,
                    pad_mode=PAD_ZERO, act=0, dtype=pc.dtype, mask_act=0, ldm=0, moff=0,
                    cin_real=s.cout if s.cout < pc.cout_eff else 0)
        d = _desc(**base, Ho=H, Wo=W, ldy=dx.ld, yoff=dx.off, OH=H, OW=W, omy=1, ooy=0, omx=1, oox=0, sy=1, sx=1,
                  c0y=c0y + p, c0x=c0x + p, accumulate=int(accumulate), out_dtype=dx.dt)
        ring_mfma = (p > 0 and pc.dtype == BF16 and pc.cout_eff % 32 == 0 and H >= 2 * p + 2
                     and W >= 2 * p + 2 and dy.ld % 8 == 0 and dy.off % 8 == 0)

        def launch():
            if ring_mfma and RING_LINE[0] and RING_EPI[0] and dx.dt == BF16:
                # line GEMM, then the interior with the ring folded into its store pass
                ws = _ring_ws(dx.t.device, dx.N * 4 * 68 * dx.C)
                rc = _lib.load().irgan_conv_dgrad_reflect_line(ctypes.byref(d), dy.ptr, P(buf), p, dx.ptr, P(ws),
                                                              ws.numel(), stream())
                if rc == 0:
                    return
                if rc != IRGAN_EUNSUPPORTED:
                    raise _lib.IrganError(f"irgan_conv_dgrad_reflect_line failed with code {rc}")
            _lib.call("irgan_conv_fwd", ctypes.byref(d), dy.ptr, P(buf), None, dx.ptr, None, stream())
            if ring_mfma:
                _ring(d, dy, buf, p, dx)

        TIMER.wrap(conv_tag("dgrad", s, (H, W), dx.N), launch)
        if p == 0 or ring_mfma:
            return
        # ring in split-K partials: rows[ks][N][2p][Wp][C], cols[ks][N][H][2p][C]
        rsz, csz = dx.N * 2 * p * Wp * s.cin, dx.N * H * 2 * p * s.cin
        nk = -(-(ay * ax * pc.cout_eff) // 64)
        ksplit = 1 if pc.dtype == F32 else max(1, min(nk // 2, 16))
        assert pad_buf is not None
        ksplit = max(1, min(ksplit, pad_buf.numel() // (rsz + csz)))
        rows_b = pad_buf[:ksplit * rsz]
        cols_b = pad_buf[ksplit * rsz:ksplit * (rsz + csz)]
        ring = dict(base, ldy=s.cin, yoff=0, accumulate=0, out_dtype=F32)
        for k in range(p):
            # padded rows k and H+p+k (full width) -> compact rows k, p+k
            dr = _desc(**ring, Ho=2, Wo=Wp, OH=2 * p, OW=Wp, omy=p, ooy=k, omx=1, oox=0, sy=H + p, sx=1,
                       c0y=c0y + k, c0x=c0x)
            _lib.call("irgan_conv_fwd_splitk", ctypes.byref(dr), dy.ptr, P(buf), P(rows_b), ksplit, rsz, stream())
            # padded columns k and W+p+k of the interior rows -> compact columns k, p+k
            dcl = _desc(**ring, Ho=H, Wo=2, OH=H, OW=2 * p, omy=1, ooy=0, omx=p, oox=k, sy=1, sx=W + p,
                        c0y=c0y + p, c0x=c0x + k)
            _lib.call("irgan_conv_fwd_splitk", ctypes.byref(dcl), dy.ptr, P(buf), P(cols_b), ksplit, csz, stream())
        _lib.call("irgan_reflect_ring_fold", P(rows_b), P(cols_b), ksplit, dx.N, H, W, s.cin, p, dx.ptr, dx.dt,
                  dx.ld, dx.off, stream())
        return
    st = s.stride

    def phases():
        if st == 2 and len(pc.dg) == 4 and pc.dtype == BF16 and not bias and _dgrad_s2(pc, dy, dx, accumulate, mask,
                                                                                        mask_act):
            return   # all four phases in one launch (irgan_conv_dgrad_s2)
        for (py, _, ay, c0y), (px, _, ax, c0x), buf in pc.dg:
            Ho, Wo = -(-(dx.H - py) // st), -(-(dx.W - px) // st)
            if Ho <= 0 or Wo <= 0:
                continue
            assert ay > 0 and ax > 0
            d = _desc(N=dy.N, H=dy.H, W=dy.W, Cin=pc.cout_eff, ldx=dy.ld, xoff=dy.off, Ho=Ho, Wo=Wo, Cout=s.cin,
                      ldy=dx.ld, yoff=dx.off, OH=dx.H, OW=dx.W, omy=st, ooy=py, omx=st, oox=px, KH=ay, KW=ax, sy=1,
                      sx=1, c0y=c0y, c0x=c0x, pad_mode=PAD_ZERO, act=0, accumulate=int(accumulate), dtype=pc.dtype,
                      out_dtype=dx.dt, mask_act=mask_act, ldm=mask.ld if mask else 0, moff=mask.off if mask else 0,
                      cin_real=s.cout if s.cout < pc.cout_eff else 0)
            _lib.call("irgan_conv_fwd", ctypes.byref(d), dy.ptr, P(buf), P(pc.bias if bias else None), dx.ptr,
                      mask.ptr if mask else None, stream())
    TIMER.wrap(conv_tag("dgrad", s, (dx.H, dx.W), dx.N), phases)


def _dgrad_s2(pc: PackedConv, dy: Feat, dx: Feat, accumulate, mask, mask_act) -> bool:
    """The four phase launches of a 4x4 stride-2 backward-data as one irgan_conv_dgrad_s2
    launch; False (nothing ran) when the library does not take the shapes."""
    s = pc.spec
    descs, ws = (_lib.ConvDesc * 4)(), (ctypes.c_void_p * 4)()
    for k, ((py, _, ay, c0y), (px, _, ax, c0x), buf) in enumerate(pc.dg):
        Ho, Wo = -(-(dx.H - py) // 2), -(-(dx.W - px) // 2)
        descs[k] = _desc(N=dy.N, H=dy.H, W=dy.W, Cin=pc.cout_eff, ldx=dy.ld, xoff=dy.off, Ho=Ho, Wo=Wo, Cout=s.cin,
                         ldy=dx.ld, yoff=dx.off, OH=dx.H, OW=dx.W, omy=2, ooy=py, omx=2, oox=px, KH=ay, KW=ax, sy=1,
                         sx=1, c0y=c0y, c0x=c0x, pad_mode=PAD_ZERO, act=0, accumulate=int(accumulate),
                         dtype=pc.dtype, out_dtype=dx.dt, mask_act=mask_act, ldm=mask.ld if mask else 0,
                         moff=mask.off if mask else 0, cin_real=s.cout if s.cout < pc.cout_eff else 0)
        ws[k] = buf.data_ptr()
    rc = _lib.load().irgan_conv_dgrad_s2(descs, dy.ptr, ws, dx.ptr, mask.ptr if mask else None, stream())
    if rc == IRGAN_EUNSUPPORTED:
        return False
    if rc != 0:
        raise _lib.IrganError(f"irgan_conv_dgrad_s2 failed with code {rc}")
    return True


def conv_wgrad(spec: ConvSpec, x: Feat, dy: Feat, dw: torch.Tensor, dtype: int, splitk=0):
    """dw (fp32 KRSC view, accumulated) += weight gradient of conv(x) given dy."""
    Ho, Wo = spec.out_hw(x.H, x.W)
    assert (dy.H, dy.W, dy.C) == (Ho, Wo, spec.cout) and x.C >= spec.cin
    assert x.dt == dtype and dy.dt == dtype and dw.dtype == torch.float32
    d = _desc(N=x.N, H=x.H, W=x.W, Cin=spec.cin, ldx=x.ld, xoff=x.off, Ho=Ho, Wo=Wo, Cout=spec.cout, ldy=dy.ld,
              yoff=dy.off, OH=Ho, OW=Wo, omy=1, ooy=0, omx=1, oox=0, KH=spec.k, KW=spec.k, sy=spec.stride,
              sx=spec.stride, c0y=-spec.pad, c0x=-spec.pad, pad_mode=spec.mode, act=0, accumulate=1, dtype=dtype,
              out_dtype=F32, mask_act=0, ldm=0, moff=0, flags=CONV_DETERMINISTIC if _DET[0] else 0)
    ws = _wgrad_ws(dw.device) if dtype == BF16 else None
    TIMER.wrap(conv_tag("wgrad", spec, (x.H, x.W), x.N), lambda: _lib.call(
        "irgan_conv_wgrad_ws", ctypes.byref(d), x.ptr, dy.ptr, P(dw), splitk, P(ws), 0 if ws is None else ws.numel(),
        stream()))


WGRAD_WS_FLOATS = 24 << 20   # split-K slab workspace (96 MB): >= slots x tile for every layer of the step
_WGRAD_WS = {}


def _wgrad_ws(dev):
    """Per-(device, stream) fp32 workspace for the wgrad split-K partials
    (irgan_conv_wgrad_ws): plain-store slabs + an ordered reduce instead of fp32
    atomics into dw.  One per stream, so concurrent streams never share it."""
    key = (dev, torch.cuda.current_stream(dev).cuda_stream)
    w = _WGRAD_WS.get(key)
    if w is None:
        w = _WGRAD_WS[key] = torch.empty(WGRAD_WS_FLOATS, dtype=torch.float32, device=dev)
    return w


# ----------------------------------------------------------------------------
# instance norm / reductions
# ----------------------------------------------------------------------------

def in_stats(x: Feat, work: torch.Tensor, mr: torch.Tensor):
    """{mean, rstd} of x: partial-sum launch + fixed-order finalize launch."""
    _lib.call("irgan_in_stats", x.ptr, x.dt, x.N, x.H * x.W, x.C, x.ld, x.off, P(work), P(mr), stream())


def in_finalize(x: Feat, part: torch.Tensor, nb: int, mr: torch.Tensor):
    """{mean, rstd} of x from the nb per-image partials irgan_conv_fwd_stats wrote."""
    _lib.call("irgan_in_finalize", P(part), x.N, x.H * x.W, x.C, nb, P(mr), stream())


def in_apply(x: Feat, mr, y: Feat, act=ACT_NONE, res: Feat = None, xhat: torch.Tensor = None, q8=None):
    """y = act(IN(x)) [+ res].  q8 = (y8 Feat, q ptr, amax ptr): also the fp8 copy of y
    (irgan_in_apply_fp8; bf16, no xhat)."""
    assert x.dt == y.dt
    if q8 is not None:
        y8, qp, ap = q8
        assert xhat is None and x.dt == BF16 and y8.dt == FP8 and (y8.N, y8.H, y8.W, y8.C) == (y.N, y.H, y.W, y.C)
        _lib.call("irgan_in_apply_fp8", x.ptr, x.N, x.H * x.W, x.C, x.ld, x.off, P(mr), act,
                  res.ptr if res else None, res.ld if res else 0, res.off if res else 0, y.ptr, y.ld, y.off,
                  y8.ptr, y8.ld, y8.off, qp, ap, stream())
        return
    _timed("in_apply_res" if res is not None else "in_apply", x, lambda: _lib.call(
        "irgan_in_apply", x.ptr, x.dt, x.N, x.H * x.W, x.C, x.ld, x.off, P(mr), act, res.ptr if res else None,
        res.ld if res else 0, res.off if res else 0, y.ptr, y.ld, y.off, P(xhat), stream()))


def in_bwd_parts(dy: Feat, x: Feat, act: int, mr, work, red, dx: Feat, db=None, dy2: Feat = None, q8=None):
    """(reduce, apply) launch closures of in_backward (also used for per-pass timing).
    q8 = (y8 Feat, q ptr, amax ptr): the apply also writes the fp8 copy of dx."""
    N, HW, C = x.N, x.H * x.W, x.C
    d2 = (dy2.ptr, dy2.dt, dy2.ld, dy2.off) if dy2 is not None else (None, 0, 0, 0)

    def reduce():
        _lib.call("irgan_in_bwd_reduce", dy.ptr, dy.dt, dy.ld, dy.off, *d2, x.ptr, x.dt, x.ld, x.off, act, N, HW, C,
                  P(mr), P(work), P(red), stream())

    def apply():
        if q8 is not None:
            y8, qp, ap = q8
            assert db is None and y8.dt == FP8 and dx.dt == BF16 and (y8.N, y8.H, y8.W, y8.C) == (dx.N, dx.H, dx.W, C)
            _lib.call("irgan_in_bwd_apply_fp8", dy.ptr, dy.ld, dy.off, d2[0], d2[2], d2[3], x.ptr, x.ld, x.off, act,
                      N, HW, C, P(mr), P(red), dx.ptr, dx.ld, dx.off, y8.ptr, y8.ld, y8.off, qp, ap, stream())
            return
        _lib.call("irgan_in_bwd_apply", dy.ptr, dy.dt, dy.ld, dy.off, *d2, x.ptr, x.dt, x.ld, x.off, act, N, HW, C,
                  P(mr), P(red), dx.ptr, dx.dt, dx.ld, dx.off, P(db), stream())
    return reduce, apply


def in_backward(dy: Feat, x: Feat, act: int, mr, work, red, dx: Feat, db=None, dy2: Feat = None, q8=None):
    """dx = backward of act(IN(x)) applied to (dy [+ dy2]); x = PRE-norm input."""
    reduce, apply = in_bwd_parts(dy, x, act, mr, work, red, dx, db, dy2, q8)
    _timed("in_bwd_reduce", x, reduce)
    _timed("in_bwd_apply", x, apply)


_CS_WORK = {}


def channel_sum(g: Feat, db: torch.Tensor):
    key = (db.device, g.C, torch.cuda.current_stream(db.device).cuda_stream)
    w = _CS_WORK.get(key)
    if w is None:
        w = _CS_WORK[key] = torch.empty(16 * IN_PARTS * g.C, dtype=torch.float64, device=db.device)
    _lib.call("irgan_channel_sum", g.ptr, g.dt, g.P, g.C, g.ld, g.off, P(db), P(w), stream())


# ----------------------------------------------------------------------------
# resampling / elementwise
# ----------------------------------------------------------------------------

RS_DOWN, RS_UP, RS_PAD = 0, 1, 2
TMAX = 8
_TABLES = {}


def _host_table(kind, n_in, p=0, transpose=False):
    """Host (idx [rows][TMAX], w [rows][TMAX], rows) of a per-axis resampling map,
    built by the C ABI (irgan_resample_table)."""
    import numpy as np
    cap = 2 * n_in + 2 * p + 8
    idx = np.zeros(cap * TMAX, np.int32)
    w = np.zeros(cap * TMAX, np.float32)
    rows = _lib.load().irgan_resample_table(kind, n_in, p, int(transpose), idx.ctypes.data_as(ctypes.c_void_p),
                                              w.ctypes.data_as(ctypes.c_void_p), TMAX, cap)
    if rows < 0:
        raise _lib.IrganError(f"irgan_resample_table({kind}, {n_in}, {p}) failed: {rows}")
    return idx[:rows * TMAX].reshape(rows, TMAX), w[:rows * TMAX].reshape(rows, TMAX), rows


def _device_table(idx, w, rows, dev):
    """Device copy of a table; each row's taps start at slot 0, so keep only the
    widest row's tap count."""
    import numpy as np
    T = max(1, int((w != 0).sum(axis=1).max()))
    return (torch.from_numpy(np.ascontiguousarray(idx[:, :T])).to(dev),
            torch.from_numpy(np.ascontiguousarray(w[:, :T])).to(dev), rows, T)


def _dev(device):
    return torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)


def resample_table(kind, n_in, p=0, transpose=False, device=None):
    """Device (idx, w, rows, T) per-axis table of a separable resampling map, cached."""
    dev = _dev(device)
    key = (kind, n_in, p, bool(transpose), dev)
    t = _TABLES.get(key)
    if t is None:
        t = _TABLES[key] = _device_table(*_host_table(kind, n_in, p, transpose), dev)
    return t


def bilinear_matrix(n_in, n_out):
    """Dense (n_out x n_in) map of F.interpolate(mode='bilinear', align_corners=True)
    along one axis (ir:555-556, 562-563): source coordinate o*(n_in-1)/(n_out-1),
    linear weights between its two neighbours (ATen's upsample_bilinear2d)."""
    import numpy as np
    M = np.zeros((n_out, n_in), np.float64)
    scale = (n_in - 1) / (n_out - 1) if n_out > 1 else 0.0
    for o in range(n_out):
        src = np.float32(np.float32(scale) * o) if n_out > 1 else 0.0
        i0 = min(int(src), n_in - 1)
        i1 = i0 + (1 if i0 < n_in - 1 else 0)
        lam = float(src) - i0
        M[o, i0] += 1.0 - lam
        M[o, i1] += lam
    return M


def _dense(idx, w, rows, n_in):
    import numpy as np
    M = np.zeros((rows, n_in), np.float64)
    for r in range(rows):
        for t in range(idx.shape[1]):
            if w[r, t] != 0:
                M[r, idx[r, t]] += w[r, t]
    return M


def _table_from_dense(M):
    """(idx, w, rows) table of a dense map (rows x n_in), taps packed from slot 0."""
    import numpy as np
    rows = M.shape[0]
    nz = [np.nonzero(M[r])[0] for r in range(rows)]
    T = max(1, max(len(z) for z in nz))
    if T > TMAX:
        raise _lib.IrganError(f"resampling map needs {T} taps per row (> {TMAX})")
    idx = np.zeros((rows, TMAX), np.int32)
    w = np.zeros((rows, TMAX), np.float32)
    for r, z in enumerate(nz):
        idx[r, :len(z)] = z
        w[r, :len(z)] = M[r, z]
    return idx, w, rows


def resize_table(n_in, n_out, after_up=False, transpose=False, device=None):
    """Per-axis table of the odd-size decoder fallback (ir:555-556, 562-563): the
    bilinear align_corners resize from the up-sampled length to the skip's length.
    after_up=True composes it with UpsampleAA (n_in -> 2*n_in -> n_out) into ONE
    map, so the up-sample + resize is a single sep_resample launch."""
    import numpy as np
    dev = _dev(device)
    key = ("resize", n_in, n_out, bool(after_up), bool(transpose), dev)
    t = _TABLES.get(key)
    if t is None:
        if after_up:
            M = bilinear_matrix(2 * n_in, n_out) @ _dense(*_host_table(RS_UP, n_in), n_in)
        else:
            M = bilinear_matrix(n_in, n_out)
        M[np.abs(M) < 1e-12] = 0.0
        t = _TABLES[key] = _device_table(*_table_from_dense(M.T.copy() if transpose else M), dev)
    return t


def sep_resample(x: Feat, y: Feat, ytab, xtab, accumulate=False):
    (ty, wy, ry, Ty), (tx, wx, rx, Tx) = ytab, xtab
    assert (ry, rx) == (y.H, y.W) and x.C == y.C and x.N == y.N, "sep_resample shape mismatch"
    _lib.call("irgan_sep_resample", x.ptr, x.dt, x.N, x.H, x.W, x.C, x.ld, x.off, y.ptr, y.dt, y.H, y.W, y.ld, y.off,
              P(ty), P(wy), Ty, P(tx), P(wx), Tx, int(accumulate), stream())


def sep_resample_in(z: Feat, mr: torch.Tensor, act, y: Feat, ytab, xtab) -> bool:
    """y = resample(act(InstanceNorm(z))) with z's {mean, rstd} table ``mr``
    (irgan_sep_resample_in: the IN apply fused into the resample's loads).  False when
    the kernel does not take the shapes -- then NOTHING ran."""
    (ty, wy, ry, Ty), (tx, wx, rx, Tx) = ytab, xtab
    assert (ry, rx) == (y.H, y.W) and z.C == y.C and z.N == y.N, "sep_resample_in shape mismatch"
    rc = getattr(_lib.load(), "irgan_sep_resample_in")(
        z.ptr, z.dt, z.N, z.H, z.W, z.C, z.ld, z.off, P(mr), act, y.ptr, y.dt, y.H, y.W, y.ld, y.off,
        P(ty), P(wy), Ty, P(tx), P(wx), Tx, stream())
    if rc == IRGAN_EUNSUPPORTED:
        return False
    if rc != 0:
        raise _lib.IrganError(f"irgan_sep_resample_in failed with code {rc}")
    return True


def sep_resample_fp8(x: Feat, mr, act, y: Feat, ytab, xtab, q8) -> bool:
    """sep_resample (mr None) / sep_resample_in (mr: act(IN(x)) on load) into bf16 y that
    also writes y's e4m3 copy: q8 = (y8 Feat, q pointer, amax pointer) as Fp8Acts.spec()
    gives it (irgan_sep_resample_fp8).  False when the kernel does not take the shapes --
    then NOTHING ran."""
    (ty, wy, ry, Ty), (tx, wx, rx, Tx) = ytab, xtab
    y8, qp, ap = q8
    assert (ry, rx) == (y.H, y.W) and x.C == y.C and x.N == y.N, "sep_resample_fp8 shape mismatch"
    assert y8.dt == FP8 and (y8.N, y8.H, y8.W, y8.C) == (y.N, y.H, y.W, y.C)
    rc = getattr(_lib.load(), "irgan_sep_resample_fp8")(
        x.ptr, x.dt, x.N, x.H, x.W, x.C, x.ld, x.off, P(mr), act, y.ptr, y.dt, y.H, y.W, y.ld, y.off,
        P(ty), P(wy), Ty, P(tx), P(wx), Tx, y8.ptr, y8.ld, y8.off, qp, ap, stream())
    if rc == IRGAN_EUNSUPPORTED:
        return False
    if rc != 0:
        raise _lib.IrganError(f"irgan_sep_resample_fp8 failed with code {rc}")
    return True


def blur_down(x: Feat, y: Feat):
    """Downsample (ir:269-310)."""
    sep_resample(x, y, resample_table(RS_DOWN, x.H), resample_table(RS_DOWN, x.W))


def blur_down_in(z: Feat, mr: torch.Tensor, act, y: Feat, q8=None) -> bool:
    """Downsample of act(IN(z)) (ir:469-482) without storing the normalised tensor;
    q8: also y's e4m3 copy (sep_resample_fp8)."""
    if q8 is not None:
        return sep_resample_fp8(z, mr, act, y, resample_table(RS_DOWN, z.H), resample_table(RS_DOWN, z.W), q8)
    return sep_resample_in(z, mr, act, y, resample_table(RS_DOWN, z.H), resample_table(RS_DOWN, z.W))


def blur_down_bwd(dy: Feat, dx: Feat, accumulate=False):
    sep_resample(dy, dx, resample_table(RS_DOWN, dx.H, transpose=True), resample_table(RS_DOWN, dx.W, transpose=True),
                 accumulate)


def _up_axis(n_in, n_out, transpose):
    if n_out == 2 * n_in:
        return resample_table(RS_UP, n_in, transpose=transpose)
    return resize_table(n_in, n_out, after_up=True, transpose=transpose)   # odd-size fallback folded in


def upsample(x: Feat, y: Feat, q8=None):
    """UpsampleAA (ir:313-355); when y is not 2x (odd skip sizes) the reference's
    bilinear resize to the skip's size (ir:555-556, 562-563) is folded into the map.
    q8: also y's e4m3 copy (sep_resample_fp8; the plain launch + fp8_quant if the LDS
    form does not take the shapes)."""
    yt, xt = _up_axis(x.H, y.H, False), _up_axis(x.W, y.W, False)
    if q8 is not None and sep_resample_fp8(x, None, ACT_NONE, y, yt, xt, q8):
        return
    sep_resample(x, y, yt, xt)
    if q8 is not None:
        fp8_quant(y, *q8)


def upsample_in(z: Feat, mr: torch.Tensor, act, y: Feat) -> bool:
    """UpsampleAA of act(IN(z)) (ir:557-561) without storing the normalised tensor."""
    return sep_resample_in(z, mr, act, y, _up_axis(z.H, y.H, False), _up_axis(z.W, y.W, False))


def upsample_bwd(dy: Feat, dx: Feat, work=None, accumulate=False):
    sep_resample(dy, dx, _up_axis(dx.H, dy.H, True), _up_axis(dx.W, dy.W, True), accumulate)


def resize(x: Feat, y: Feat, accumulate=False):
    """F.interpolate(x, size=(y.H, y.W), mode='bilinear', align_corners=True)."""
    sep_resample(x, y, resize_table(x.H, y.H), resize_table(x.W, y.W), accumulate)


def resize_bwd(dy: Feat, dx: Feat, accumulate=False):
    sep_resample(dy, dx, resize_table(dx.H, dy.H, transpose=True), resize_table(dx.W, dy.W, transpose=True),
                 accumulate)


def pad_table(n_in, p, mode, transpose=False, device=None):
    """Per-axis (idx, w, rows, T) table of nn.ReflectionPad2d(p) (mode "reflect") or
    nn.ReplicationPad2d(p) ("replicate", ir:383, 404): padded coordinate u reads
    reflect(u - p) / clamp(u - p, 0, n_in - 1); transpose: the fold (its adjoint)."""
    if mode == "reflect":
        return resample_table(RS_PAD, n_in, p, transpose, device)
    import numpy as np
    dev = _dev(device)
    key = ("replicate", n_in, p, bool(transpose), dev)
    t = _TABLES.get(key)
    if t is None:
        M = np.zeros((n_in + 2 * p, n_in), np.float64)
        for u in range(n_in + 2 * p):
            M[u, min(max(u - p, 0), n_in - 1)] = 1.0
        t = _TABLES[key] = _device_table(*_table_from_dense(M.T.copy() if transpose else M), dev)
    return t


def pad(x: Feat, y: Feat, p: int, mode):
    """y = ReflectionPad2d(p) / ReplicationPad2d(p) of x (y is (H + 2p) x (W + 2p))."""
    sep_resample(x, y, pad_table(x.H, p, mode, device=x.t.device), pad_table(x.W, p, mode, device=x.t.device))


def pad_fold(dxp: Feat, dx: Feat, p: int, mode, accumulate=False):
    """Backward of pad(): every padded position's gradient added onto the pixel it copied."""
    sep_resample(dxp, dx, pad_table(dx.H, p, mode, True, dx.t.device), pad_table(dx.W, p, mode, True, dx.t.device),
                 accumulate)


def dropout(x: Feat, y: Feat, seed: int, p: float = 0.5):
    """nn.Dropout(p) in training mode (ir:394-395): y = x * keep / (1 - p), keep ~ Bernoulli(1 - p)
    from a counter-based hash of (seed, element index) -- the backward applies the same
    call to the gradient (same seed -> same mask, same scale)."""
    assert (x.N, x.H, x.W, x.C) == (y.N, y.H, y.W, y.C)
    _lib.call("irgan_dropout", x.ptr, x.dt, x.P, x.C, x.ld, x.off, y.ptr, y.dt, y.ld, y.off,
              ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF), ctypes.c_float(p), stream())


def reflect_fold(dxpad: Feat, dx: Feat, p: int, accumulate=False):
    """Backward of nn.ReflectionPad2d(p): dx[q] = sum over padded u with reflect(u-p) = q."""
    sep_resample(dxpad, dx, resample_table(RS_PAD, dx.H, p, transpose=True),
                 resample_table(RS_PAD, dx.W, p, transpose=True), accumulate)


def maxpool(x: Feat, y: Feat):
    assert x.off == 0 and x.C == x.ld and y.off == 0
    _lib.call("irgan_maxpool_fwd", x.ptr, x.dt, x.N, x.H, x.W, x.C, y.ptr, stream())


def maxpool_bwd(x: Feat, dy: Feat, dx: Feat, relu_mask=True):
    _lib.call("irgan_maxpool_bwd", x.ptr, dy.ptr, x.dt, x.N, x.H, x.W, x.C, dx.ptr, int(relu_mask), stream())


def nchw_to_nhwc(x: torch.Tensor, y: Feat, scale=None, shift=None):
    N, C, H, W = x.shape
    _lib.call("irgan_nchw_to_nhwc", P(x), N, C, H, W, y.ptr, y.dt, y.ld, y.off, P(scale), P(shift), stream())


def nhwc_to_nchw(x: Feat, y: torch.Tensor, scale=1.0, accumulate=False):
    _lib.call("irgan_nhwc_to_nchw", x.ptr, x.dt, x.ld, x.off, x.N, x.C, x.H, x.W, P(y), ctypes.c_float(scale),
              int(accumulate), stream())


def axpby(x: Feat, a: float, y: Feat, b: float = 0.0):
    _lib.call("irgan_axpby", x.ptr, x.dt, x.ld, x.off, ctypes.c_float(a), y.ptr, y.dt, y.ld, y.off,
              ctypes.c_float(b), x.P, x.C, stream())


def affine(x: Feat, scale, shift, y: Feat, accumulate=False):
    _lib.call("irgan_affine", x.ptr, x.dt, x.ld, x.off, P(scale), P(shift), y.ptr, y.dt, y.ld, y.off,
              int(accumulate), x.P, x.C, stream())


def act_bwd(dy: Feat, a: Feat, act: int, dx: Feat):
    _lib.call("irgan_act_bwd", dy.ptr, dy.dt, dy.ld, dy.off, a.ptr, a.dt, a.ld, a.off, act, dx.ptr, dx.dt, dx.ld,
              dx.off, dy.P, dy.C, stream())


# ----------------------------------------------------------------------------
# losses / optimizer
# ----------------------------------------------------------------------------

def hinge(pred: torch.Tensor, n_half: int, mode: int, scale: float, grad: torch.Tensor, loss: torch.Tensor):
    _lib.call("irgan_hinge", P(pred), n_half, mode, ctypes.c_float(scale), P(grad), P(loss), stream())


def l1(a: torch.Tensor, b: torch.Tensor, w: float, ga: torch.Tensor, loss: torch.Tensor, accumulate=False):
    _lib.call("irgan_l1", P(a), P(b), dt_code(a), a.numel(), ctypes.c_float(w), P(ga),
              dt_code(ga) if ga is not None else 0, int(accumulate), P(loss), stream())


def tv(x: Feat, w: float, g: torch.Tensor, loss: torch.Tensor):
    _lib.call("irgan_tv", x.ptr, x.N, x.H, x.W, x.C, ctypes.c_float(w), P(g), P(loss), stream())


def ssim(a: Feat, b: Feat, w: float, g: torch.Tensor, loss: torch.Tensor, work: torch.Tensor, window: int = 11):
    _lib.call("irgan_ssim_ws", a.ptr, b.ptr, a.N, a.H, a.W, a.C, ctypes.c_float(w), P(g), P(loss), P(work), window,
              stream())


def adam(p, g, m, v, step: int, lr: float, b1: float, b2: float, eps: float):
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    _lib.call("irgan_adam", P(p), P(g), P(m), P(v), p.numel(), ctypes.c_float(lr / bc1), ctypes.c_float(b1),
              ctypes.c_float(b2), ctypes.c_float(math.sqrt(bc2)), ctypes.c_float(eps), stream())


def adam_prep(count: torch.Tensor, lr: float, b1: float, b2: float, prm: torch.Tensor):
    """Device-side step count + bias corrections (irgan_adam_prep): count (int32[1]) += 1,
    prm (fp32[2]) = {lr / (1 - b1^t), sqrt(1 - b2^t)} -- ops.adam's host formula."""
    _lib.call("irgan_adam_prep", P(count), ctypes.c_double(lr), ctypes.c_double(b1), ctypes.c_double(b2), P(prm),
              stream())


def adam_dev(p, g, m, v, prm: torch.Tensor, b1: float, b2: float, eps: float):
    """ops.adam with step_size / bc2_sqrt read from prm on the device (irgan_adam_dev)."""
    _lib.call("irgan_adam_dev", P(p), P(g), P(m), P(v), p.numel(), P(prm), ctypes.c_float(b1), ctypes.c_float(b2),
              ctypes.c_float(eps), stream())


# ----------------------------------------------------------------------------
# fp8 (OCP e4m3) operands: BASELINE config 5
# ----------------------------------------------------------------------------

def fp8_quant(x: Feat, y: Feat = None, q=None, amax=None):
    """y = e4m3(clamp(x * q, +-448)); amax = max(amax, max|x|) (irgan_fp8_quant).
    q / amax: ctypes pointers to one float / uint32 slot (Pi), or None."""
    assert y is None or (y.dt == FP8 and (y.N, y.H, y.W, y.C) == (x.N, x.H, x.W, x.C))
    _lib.call("irgan_fp8_quant", x.ptr, x.dt, x.P, x.C, x.ld, x.off, y.ptr if y is not None else None,
              y.ld if y is not None else 0, y.off if y is not None else 0, q, amax, stream())


FP8_AMAX_PARTS = _lib.header_enum("IRGAN_FP8_AMAX_PARTS")


def amax_slots(n, device):
    """n amax slots of FP8_AMAX_PARTS partial maxima each (irgan.h)."""
    return torch.zeros(n * FP8_AMAX_PARTS, dtype=torch.int32, device=device)


def amax_ptr(amax: torch.Tensor, slot: int):
    return Pi(amax, slot * FP8_AMAX_PARTS)


def fp8_scale(amax: torch.Tensor, q: torch.Tensor, dq: torch.Tensor, reset=True, start=0, n=None):
    """Slots [start, start+n): q = 2^floor(log2(448 / amax)), dq = 1 / q (irgan_fp8_scale)."""
    n = q.numel() - start if n is None else n
    _lib.call("irgan_fp8_scale", amax_ptr(amax, start), n, Pi(q, start), Pi(dq, start), int(reset), stream())


class Fp8Job(ctypes.Structure):
    """irgan_fp8_job (include/irgan.h)."""
    _fields_ = [("src", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("n", ctypes.c_int64),
                ("slot", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class Fp8Weights:
    """fp8 copies of bf16 packed weight images, re-quantised after every re-pack with
    per-tensor current scaling: one amax launch, irgan_fp8_scale, one quantise launch
    for all of them.  ``dst[k]`` / slot k belongs to the k-th (src) image."""

    def __init__(self, srcs, device):
        self.srcs = list(srcs)
        self.dst = [torch.empty(t.numel(), dtype=torch.float8_e4m3fn, device=device) for t in self.srcs]
        n = len(self.srcs)
        self.amax = amax_slots(n, device)
        self.q = torch.ones(n, dtype=torch.float32, device=device)
        self.dq = torch.ones(n, dtype=torch.float32, device=device)
        jobs = (Fp8Job * n)(*[Fp8Job(s.data_ptr(), d.data_ptr(), s.numel(), k, 0)
                              for k, (s, d) in enumerate(zip(self.srcs, self.dst))])
        assert all(s.numel() % 8 == 0 and s.dtype == torch.bfloat16 and s.is_contiguous() for s in self.srcs)
        self.table = torch.frombuffer(bytearray(bytes(jobs)), dtype=torch.uint8).to(device)
        self.max_n = max(s.numel() for s in self.srcs)

    def run(self):
        n = len(self.srcs)
        _lib.call("irgan_fp8_quant_batch", P(self.table), n, self.max_n, None, P(self.amax), stream())
        fp8_scale(self.amax, self.q, self.dq, reset=True)
        _lib.call("irgan_fp8_quant_batch", P(self.table), n, self.max_n, P(self.q), None, stream())


class Fp8Acts:
    """Per-tensor scales of fp8 activation operands with delayed scaling: a slot's
    tensor is quantised with the q made from the amax it had at the previous step
    (its first use calibrates from its own amax).  update() turns the recorded maxima
    into the next step's q / dq."""

    def __init__(self, n, device):
        self.amax = amax_slots(n, device)
        self.q = torch.ones(n, dtype=torch.float32, device=device)
        self.dq = torch.ones(n, dtype=torch.float32, device=device)
        self.seen = [False] * n

    def quant(self, slot, x: Feat, y: Feat):
        """Standalone quantisation of x into y (irgan_fp8_quant)."""
        if not self.seen[slot]:
            fp8_quant(x, None, None, amax_ptr(self.amax, slot))
            fp8_scale(self.amax, self.q, self.dq, reset=False, start=slot, n=1)
            self.seen[slot] = True
        fp8_quant(x, y, Pi(self.q, slot), amax_ptr(self.amax, slot))

    def spec(self, slot, y: Feat):
        """The (y8, q, amax) side output for a producer that writes the fp8 copy itself
        (in_apply / in_backward q8=), or None before the slot is calibrated -- then the
        caller runs ensure() on the produced tensor."""
        return (y, Pi(self.q, slot), amax_ptr(self.amax, slot)) if self.seen[slot] else None

    def ensure(self, slot, x: Feat, y: Feat):
        if not self.seen[slot]:
            self.quant(slot, x, y)

    def calibrate(self, slot, x: Feat, y: Feat):
        """Current scaling of slot from x alone, whatever was recorded before (the slot's
        partial maxima are cleared first), then the quantisation of x into y."""
        self.amax[slot * FP8_AMAX_PARTS:(slot + 1) * FP8_AMAX_PARTS].zero_()
        self.seen[slot] = False
        self.quant(slot, x, y)

    def dqp(self, slot):
        return Pi(self.dq, slot)

    def snapshot(self, start=0, n=None):
        """Keep the dequantisation factors slots [start, start+n) were just used with (before
        update() moves them to the next step's): the weight gradients of the backward read
        the forward's e4m3 copies with them."""
        n = self.dq.numel() - start if n is None else n
        if not hasattr(self, "dq_used"):
            self.dq_used = torch.ones_like(self.dq)
        self.dq_used[start:start + n].copy_(self.dq[start:start + n])

    def dqp_used(self, slot):
        return Pi(self.dq_used, slot)

    def update(self, start=0, n=None):
        fp8_scale(self.amax, self.q, self.dq, reset=True, start=start, n=n)


def conv_fwd_fp8(pc: PackedConv, w8: torch.Tensor, dqw, x8: Feat, dqx, y: Feat, part: torch.Tensor = None,
                 act=ACT_NONE, bias=True, accumulate=False) -> int:
    """conv_fwd on fp8 operands (irgan_conv_fwd_fp8): x8 e4m3 NHWC, w8 the e4m3 copy
    of pc.fwd; dqx / dqw: pointers to the dequantisation multipliers.  With ``part``
    also the InstanceNorm partials of y; returns their count per image (else 0)."""
    s = pc.spec
    Ho, Wo = s.out_hw(x8.H, x8.W)
    assert (y.H, y.W, y.C) == (Ho, Wo, s.cout) and x8.C == s.cin and y.N == x8.N and x8.dt == FP8
    d = _desc(N=x8.N, H=x8.H, W=x8.W, Cin=s.cin, ldx=x8.ld, xoff=x8.off, Ho=Ho, Wo=Wo, Cout=s.cout, ldy=y.ld,
              yoff=y.off, OH=Ho, OW=Wo, omy=1, ooy=0, omx=1, oox=0, KH=s.k, KW=s.k, sy=s.stride, sx=s.stride,
              c0y=-s.pad, c0x=-s.pad, pad_mode=s.mode, act=act, accumulate=int(accumulate), dtype=FP8,
              out_dtype=y.dt, mask_act=0, ldm=0, moff=0)
    nb = ctypes.c_int32(0)
    TIMER.wrap(conv_tag("fwd8", s, (x8.H, x8.W), x8.N), lambda: _lib.call(
        "irgan_conv_fwd_fp8", ctypes.byref(d), x8.ptr, P(w8), dqx, dqw, P(pc.bias if bias else None), y.ptr,
        P(part), ctypes.byref(nb), stream()))
    return int(nb.value)


def conv_wgrad_fp8(spec: ConvSpec, x8: Feat, dy8: Feat, dqx, dqdy, dw: torch.Tensor) -> bool:
    """dw (fp32 KRSC view, accumulated) += weight gradient of conv(x) given dy, on the fp8
    copies x8 / dy8 with their dequantisation pointers (irgan_conv_wgrad_fp8).  False when
    the kernel does not take the layer -- then NOTHING ran (the caller runs the bf16 conv_wgrad)."""
    Ho, Wo = spec.out_hw(x8.H, x8.W)
    assert (dy8.H, dy8.W, dy8.C) == (Ho, Wo, spec.cout) and x8.C == spec.cin and x8.dt == FP8 and dy8.dt == FP8
    d = _desc(N=x8.N, H=x8.H, W=x8.W, Cin=spec.cin, ldx=x8.ld, xoff=x8.off, Ho=Ho, Wo=Wo, Cout=spec.cout, ldy=dy8.ld,
              yoff=dy8.off, OH=Ho, OW=Wo, omy=1, ooy=0, omx=1, oox=0, KH=spec.k, KW=spec.k, sy=spec.stride,
              sx=spec.stride, c0y=-spec.pad, c0x=-spec.pad, pad_mode=spec.mode, act=0, accumulate=1, dtype=FP8,
              out_dtype=F32, mask_act=0, ldm=0, moff=0, flags=CONV_DETERMINISTIC if _DET[0] else 0)
    ws = _wgrad_ws(dw.device)
    rc = [0]

    def launch():
        rc[0] = _lib.load().irgan_conv_wgrad_fp8(ctypes.byref(d), x8.ptr, dy8.ptr, dqx, dqdy, P(dw), P(ws), ws.numel(),
                                                 stream())
    TIMER.wrap(conv_tag("wgrad8", spec, (x8.H, x8.W), x8.N), launch)
    if rc[0] == IRGAN_EUNSUPPORTED:
        return False
    if rc[0] != 0:
        raise _lib.IrganError(f"irgan_conv_wgrad_fp8 failed with code {rc[0]}")
    return True


def conv_dgrad_fp8(pc: PackedConv, wd8: torch.Tensor, dqw, dy8: Feat, dqx, dy: Feat, dx: Feat, accumulate=False):
    """Backward-data of a stride-1 3x3 layer on fp8 operands (dy8 = e4m3(dy), wd8 = e4m3
    copy of the flipped image pc.dg[0]).  Reflect padding: the interior on fp8, the padded
    ring from the bf16 dy by irgan_reflect_dgrad_ring (as conv_dgrad); zero padding (down2 /
    up1_conv of config 5): the flipped conv alone (irgan_conv_fwd_fp8; dy unused)."""
    s = pc.spec
    assert s.stride == 1 and dy8.dt == FP8 and dx.C == s.cin
    if not pc.reflect:
        (py, _, ay, c0y), (px, _, ax, c0x), buf = pc.dg[0]
        assert len(pc.dg) == 1 and (dy8.H, dy8.W, dy8.C) == (dx.H, dx.W, pc.cout_eff)
        d8 = _desc(N=dy8.N, H=dy8.H, W=dy8.W, Cin=pc.cout_eff, ldx=dy8.ld, xoff=dy8.off, Ho=dx.H, Wo=dx.W,
                   Cout=s.cin, ldy=dx.ld, yoff=dx.off, OH=dx.H, OW=dx.W, omy=1, ooy=py, omx=1, oox=px, KH=ay, KW=ax,
                   sy=1, sx=1, c0y=c0y, c0x=c0x, pad_mode=PAD_ZERO, act=0, accumulate=int(accumulate), dtype=FP8,
                   out_dtype=dx.dt, mask_act=0, ldm=0, moff=0)
        nb = ctypes.c_int32(0)
        TIMER.wrap(conv_tag("dgrad8", s, (dx.H, dx.W), dx.N), lambda: _lib.call(
            "irgan_conv_fwd_fp8", ctypes.byref(d8), dy8.ptr, P(wd8), dqx, dqw, None, dx.ptr, None,
            ctypes.byref(nb), stream()))
        return
    assert pc.reflect and dy.dt == BF16
    p = s.pad
    H, W = dx.H, dx.W
    (_, _, ay, c0y), (_, _, ax, c0x), buf = pc.dg[0]
    base = dict(N=dy.N, H=dy.H, W=dy.W, Cin=pc.cout_eff, Cout=s.cin, KH=ay, KW=ax, pad_mode=PAD_ZERO, act=0,
                mask_act=0, ldm=0, moff=0, Ho=H, Wo=W, ldy=dx.ld, yoff=dx.off, OH=H, OW=W, omy=1, ooy=0, omx=1,
                oox=0, sy=1, sx=1, c0y=c0y + p, c0x=c0x + p, accumulate=int(accumulate), out_dtype=dx.dt)
    d8 = _desc(**base, ldx=dy8.ld, xoff=dy8.off, dtype=FP8)
    d = _desc(**base, ldx=dy.ld, xoff=dy.off, dtype=BF16)
    nb = ctypes.c_int32(0)

    def launch():
        if p > 0 and RING_LINE[0] and RING_EPI[0]:
            # ring line GEMM (bf16), then the fp8 interior folding it in its store pass
            ws = _ring_ws(dx.t.device, dx.N * 4 * 68 * dx.C)
            rc = _lib.load().irgan_conv_dgrad_reflect_line_fp8(ctypes.byref(d), dy.ptr, P(buf), ctypes.byref(d8),
                                                               dy8.ptr, P(wd8), dqx, dqw, p, dx.ptr, P(ws),
                                                               ws.numel(), stream())
            if rc == 0:
                return
            if rc != IRGAN_EUNSUPPORTED:
                raise _lib.IrganError(f"irgan_conv_dgrad_reflect_line_fp8 failed with code {rc}")
        _lib.call("irgan_conv_fwd_fp8", ctypes.byref(d8), dy8.ptr, P(wd8), dqx, dqw, None, dx.ptr, None,
                  ctypes.byref(nb), stream())
        if p > 0:
            _ring(d, dy, buf, p, dx)
    TIMER.wrap(conv_tag("dgrad8", s, (H, W), dx.N), launch)
