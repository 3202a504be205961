"""Resblock backward-data timing at B=16/32 (256 -> 256, 3x3 reflect, 64x64): the default
(ring line GEMM + interior with the ring in its store pass) and the interior launch alone
(ring skipped: the difference is the ring's cost)."""
import importlib
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
    zspec = ops.ConvSpec(C, C, 3, 1, 1, ops.PAD_ZERO)   # same interior launch, no ring
    pz = ops.PackedConv(zspec, torch.randn(C * 9 * C, device=DEV) * 0.02, torch.zeros(C, device=DEV), ops.BF16)
    pz.pack()
    ti = timeit(lambda: ops.conv_dgrad(pz, ops.Feat(dy), ops.Feat(dx)))
    print(f"N={N}: dgrad interior+ring {t:.1f} us, interior only {ti:.1f} us "
          f"(ring ~{t - ti:.1f} us)", flush=True)
