"""Weight-gradient timing of the narrow-output layers (G outc 64->3 7x7 reflect at 256^2 B=16;
D model.11 512->1 4x4 at 31^2 B=32); IRGAN_LIB / IRGAN_NO_ROWSPAN select the variant."""
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


for name, cin, cout, k, p, mode, H, B in (("outc_64-3k7r", 64, 3, 7, 3, ops.PAD_REFLECT, 256, 16),
                                          ("D11_512-1k4", 512, 1, 4, 1, ops.PAD_ZERO, 31, 32)):
    spec = ops.ConvSpec(cin, cout, k, 1, p, mode)
    x = torch.randn(B, H, H, cin, device=DEV).bfloat16()
    Ho, Wo = spec.out_hw(H, H)
    dy = torch.zeros(B, Ho, Wo, 8, device=DEV, dtype=torch.bfloat16)
    dy[..., :cout] = torch.randn(B, Ho, Wo, cout, device=DEV).bfloat16()
    dw = torch.zeros(cout * k * k * cin, device=DEV)
    t = timeit(lambda: ops.conv_wgrad(spec, ops.Feat(x), ops.Feat(dy, 0, cout), dw, ops.BF16))
    print(f"{name}: wgrad {t:.1f} us", flush=True)
