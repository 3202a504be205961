"""Resblock backward-data (interior + reflect ring) timing at B=16/32 for the ring
K split IRGAN_RING_KSPLIT (read at import)."""
import importlib
import os
import sys

import torch

sys.path.insert(0, ".")
irc = importlib.import_module("infrared-colorization-with-resnet-generator-and-patchgan_amd")
ops = irc.ops
DEV = "cuda"


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


for N in (16, 32):
    C, H = 256, 64
    spec = ops.ConvSpec(C, C, 3, 1, 1, 1)
    pc = ops.PackedConv(spec, torch.randn(C * 9 * C, device=DEV) * 0.02, torch.zeros(C, device=DEV), ops.BF16)
    pc.pack()
    dy = torch.randn(N, H, H, C, device=DEV).bfloat16()
    dx = torch.empty_like(dy)
    t = timeit(lambda: ops.conv_dgrad(pc, ops.Feat(dy), ops.Feat(dx)))
    print(f"ksplit={os.environ.get('IRGAN_RING_KSPLIT', '4')} N={N}: dgrad interior+ring {t:.1f} us", flush=True)
