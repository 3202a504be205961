"""Microbenchmark of the separable resample kernels on the step's shapes (B=16, bf16),
with and without the fused InstanceNorm apply (irgan_sep_resample_in)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch
from conftest import pkg
ops = pkg().ops
DEV, B = "cuda", 16


def t(fn, it=20):
    fn(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e3


def feat(H, W, C, ld=None, off=0):
    ld = ld or C
    return ops.Feat(torch.randn(B, H, W, ld, device=DEV).bfloat16(), off, C)


for name, (Hi, C, Ho, kind, ldo) in {"down1": (256, 128, 128, "down", None), "down2": (128, 256, 64, "down", None),
                                     "up1": (128, 128, 256, "up", 192)}.items():
    x = feat(Hi, Hi, C)
    y = feat(Ho, Ho, C, ldo)
    mr = torch.stack([torch.zeros(B * C), torch.ones(B * C)], 1).reshape(-1).to(DEV)
    if kind == "down":
        plain = lambda: ops.blur_down(x, y)
        fused = lambda: ops.blur_down_in(x, mr, ops.ACT_RELU, y)
        bwd = lambda: ops.blur_down_bwd(y, x)
    else:
        plain = lambda: ops.upsample(x, y)
        fused = lambda: ops.upsample_in(x, mr, ops.ACT_RELU, y)
        bwd = lambda: ops.upsample_bwd(y, x)
    byt = (B * Hi * Hi * C + B * Ho * Ho * C) * 2
    for tag, fn in (("plain", plain), ("fused-IN", fused), ("bwd", bwd)):
        us = t(fn)
        print(f"{name:6s} {tag:9s} {us:8.1f} us  {byt / us / 1e3:7.0f} GB/s (in+out once)")
