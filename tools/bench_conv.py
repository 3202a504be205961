"""Microbenchmark of the conv kernels on the training shapes (bf16), HIP events."""
import sys, os, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch
from conftest import pkg
ops = pkg().ops
DEV = "cuda"
B = 16
CASES = [  # name, cin, cout, k, s, p, mode, H
    ("res3x3_256@64", 256, 256, 3, 1, 1, 1, 64),
    ("down1_64-128@256", 64, 128, 3, 1, 1, 0, 256),
    ("down2_128-256@128", 128, 256, 3, 1, 1, 0, 128),
    ("up2_192-64@256", 192, 64, 3, 1, 1, 0, 256),
    ("up1_384-128@128", 384, 128, 3, 1, 1, 0, 128),
    ("vgg12_64-64@256", 64, 64, 3, 1, 1, 0, 256),
    ("vgg21_64-128@128", 64, 128, 3, 1, 1, 0, 128),
    ("vgg22_128-128@128", 128, 128, 3, 1, 1, 0, 128),
    ("vgg31_128-256@64", 128, 256, 3, 1, 1, 0, 64),
    ("vgg33_256-256@64", 256, 256, 3, 1, 1, 0, 64),
    ("D2_128-256s2@64", 128, 256, 4, 2, 1, 0, 64),
    ("D3_256-512s1@32", 256, 512, 4, 1, 1, 0, 32),
    ("D1_64-128s2@128", 64, 128, 4, 2, 1, 0, 128),
    ("Dhead_512-1@31", 512, 1, 4, 1, 1, 0, 31),
    # 512 x 640 at B = 4 (BASELINE configs[3]): the ResnetBlock maps are 128 x 160
    ("res3x3_256@128x160b4", 256, 256, 3, 1, 1, 1, (128, 160, 4)),
]
def t(fn, it=20):
    fn(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / it
import argparse
ap = argparse.ArgumentParser()
ap.add_argument("--case", default=None, help="comma list of substring filters on case names")
ap.add_argument("--which", default="fwd,dgrad,wgrad")
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--batch", type=int, default=16)
ap.add_argument("--splitk", default="0", help="comma list of wgrad split-K values (0 = the kernel's choice)")
args = ap.parse_args()
B = args.batch
res = {}
for name, cin, cout, k, s, p, mode, H in CASES:
    if args.case and not any(c in name for c in args.case.split(",")):
        continue
    H, Wd, B = H if isinstance(H, tuple) else (H, H, args.batch)
    spec = ops.ConvSpec(cin, cout, k, s, p, mode)
    w = torch.randn(cout * k * k * cin, device=DEV) * 0.05
    pc = ops.PackedConv(spec, w, torch.zeros(cout, device=DEV), ops.BF16); pc.pack()
    x = torch.randn(B, H, Wd, cin, device=DEV).bfloat16()
    Ho, Wo = spec.out_hw(H, Wd)
    y = torch.empty(B, Ho, Wo, cout, device=DEV, dtype=torch.bfloat16)
    dy = torch.randn(B, Ho, Wo, pc.cout_eff, device=DEV).bfloat16()   # narrow dY: 8-padded
    dx = torch.empty(B, H, Wd, cin, device=DEV, dtype=torch.bfloat16)
    pad = torch.empty(B * (H + 2 * p) * (Wd + 2 * p) * cin, device=DEV)
    dw = torch.zeros(cout * k * k * cin, device=DEV)
    flop = 2.0 * B * Ho * Wo * cout * cin * k * k
    part = torch.empty(B * 512 * cout * 2, device=DEV)
    fns = {"fwd": lambda: ops.conv_fwd(pc, ops.Feat(x), ops.Feat(y)),
           "fwdr": lambda: ops.conv_fwd(pc, ops.Feat(x), ops.Feat(y), act=ops.ACT_RELU),
           "fwds": lambda: ops.conv_fwd_stats(pc, ops.Feat(x), ops.Feat(y), part),
           "dgrad": lambda: ops.conv_dgrad(pc, ops.Feat(dy), ops.Feat(dx), pad_buf=pad),
           # backward-data with the ReLU mask of the layer below (the VGG chain)
           "dgradm": lambda: ops.conv_dgrad(pc, ops.Feat(dy), ops.Feat(dx), mask=ops.Feat(x), mask_act=1),
           "wgrad": lambda: ops.conv_wgrad(spec, ops.Feat(x), ops.Feat(dy, 0, cout), dw, ops.BF16)}
    res[name] = {}
    for k2 in args.which.split(","):
        if k2 == "wgrad":
            for sk in (int(s) for s in args.splitk.split(",")):  # noqa: B007
                v = t(lambda: ops.conv_wgrad(spec, ops.Feat(x), ops.Feat(dy, 0, cout), dw, ops.BF16, splitk=sk),
                      args.iters)
                res[name][k2 if sk == 0 else f"wgrad@{sk}"] = (round(v, 4), round(flop / v / 1e9, 1))
            continue
        try:
            v = t(fns[k2], args.iters)
        except (AssertionError, RuntimeError) as e:   # a path this layer does not take
            res[name][k2] = f"n/a ({type(e).__name__})"
            continue
        res[name][k2] = (round(v, 4), round(flop / v / 1e9, 1))
    print(name, "ms/TFLOPs", res[name], flush=True)
print(json.dumps(res))
