"""Kernel timing: the 8-channel-input weight gradients (G inc 7x7 at 256^2 B=16, D
model.0 4x4 s2 on the 2B = 32 D batch) through ops.conv_wgrad (dispatch included)."""
import importlib
import os
import sys

import torch

sys.path.insert(0, ".")
irc = importlib.import_module("infrared-colorization-with-resnet-generator-and-patchgan_amd")
ops = irc.ops
DEV = "cuda"


def timeit(fn, n=10):
    for _ in range(2):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


for name, (cin, k, s, p, mode, N, H) in {"inc": (1, 7, 1, 3, 1, 16, 256), "D.model0": (4, 4, 2, 1, 0, 32, 256)}.items():
    spec = ops.ConvSpec(cin, 64, k, s, p, mode)
    Ho, Wo = spec.out_hw(H, H)
    x = torch.zeros(N, H, H, 8, device=DEV, dtype=torch.bfloat16)
    x[..., :cin] = torch.randn(N, H, H, cin, device=DEV).bfloat16()
    dy = torch.randn(N, Ho, Wo, 64, device=DEV).bfloat16()
    dw = torch.zeros(64 * k * k * cin, device=DEV)
    flop = 2.0 * N * Ho * Wo * 64 * k * k * cin
    t = timeit(lambda: ops.conv_wgrad(spec, ops.Feat(x, 0, 8), ops.Feat(dy), dw, ops.BF16))
    print(f"{name}: {t:.1f} us  ({flop / t / 1e6:.1f} TF/s real-channel, {flop * 8 / cin / t / 1e6:.1f} padded)",
          flush=True)
