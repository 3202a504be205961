"""Timing of the 8-channel-input convs (conv_c8: G inc 1->64 7x7 reflect, VGG conv1_1 3->64
3x3, D model.0 4->64 4x4 s2) and G outc 64->3 7x7 at the bench shapes; IRGAN_LIB selects
an A/B build (tools/build_variant.sh)."""
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


CASES = [  # name, cin, cout, k, s, p, mode, H, B
    ("inc_1-64k7r", 1, 64, 7, 1, 3, ops.PAD_REFLECT, 256, 16),
    ("vgg11_3-64k3", 3, 64, 3, 1, 1, ops.PAD_ZERO, 256, 16),
    ("D0_4-64k4s2", 4, 64, 4, 2, 1, ops.PAD_ZERO, 256, 32),
    ("outc_64-3k7r", 64, 3, 7, 1, 3, ops.PAD_REFLECT, 256, 16),
]
for name, cin, cout, k, s, p, mode, H, B in CASES:
    spec = ops.ConvSpec(cin, cout, k, s, p, mode)
    pc = ops.PackedConv(spec, torch.randn(cout * k * k * cin, device=DEV) * 0.05, torch.zeros(cout, device=DEV),
                        ops.BF16)
    pc.pack()
    ce = pc.cin_eff
    x = torch.zeros(B, H, H, ce, device=DEV, dtype=torch.bfloat16)
    x[..., :cin] = torch.randn(B, H, H, cin, device=DEV).bfloat16()
    Ho, Wo = spec.out_hw(H, H)
    co_e = max(cout, 8)
    y = torch.empty(B, Ho, Wo, co_e, device=DEV, dtype=torch.bfloat16)
    t = timeit(lambda: ops.conv_fwd(pc, ops.Feat(x, 0, ce), ops.Feat(y, 0, cout)))
    byt = x.numel() * 2 + B * Ho * Wo * cout * 2
    print(f"{name} B={B}: fwd {t:.1f} us, {byt / t / 1e3:.0f} GB/s (in + out bytes), "
          f"{2.0 * B * Ho * Wo * cout * cin * k * k / t / 1e6:.0f} TF/s real", flush=True)
