"""Microbenchmark of the HBM-bound kernels (InstanceNorm passes, resampling) on the
generator's training shapes (bf16, B=16, 256x256), HIP events.  Prints, per
kernel, the mean launch time and the algorithmic bytes / time in GB/s."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402
from conftest import pkg  # noqa: E402

ops = pkg().ops
DEV = "cuda"
B = 16
IN_CASES = [("inc_64@256", 64, 256), ("down1_128@256", 128, 256), ("down2_256@128", 256, 128),
            ("res_256@64", 256, 64), ("up1_128@128", 128, 128)]
RS_CASES = [("down1_128@256", "down", 128, 256), ("down2_256@128", "down", 256, 128),
            ("up1_256@64", "up", 256, 64), ("up2_128@128", "up", 128, 128)]


def t(fn, it):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it


ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--case", default=None)
args = ap.parse_args()
res = {}


def rec(name, ms, nbytes):
    res[name] = (round(ms * 1e3, 1), round(nbytes / ms / 1e6, 0))
    print(f"{name:32s} {ms * 1e3:8.1f} us {nbytes / ms / 1e6:8.0f} GB/s", flush=True)


for name, C, H in IN_CASES:
    if args.case and args.case not in name:
        continue
    z = torch.randn(B, H, H, C, device=DEV).bfloat16()
    dy = torch.randn(B, H, H, C, device=DEV).bfloat16()
    y = torch.empty_like(z)
    dx = torch.empty_like(z)
    work = torch.empty(ops.IN_PARTS * B * C, dtype=torch.float64, device=DEV)
    mr = torch.empty(2 * B * C, device=DEV)
    red = torch.empty(2 * B * C, device=DEV)
    n = z.numel() * 2
    ops.in_stats(ops.Feat(z), work, mr)
    rec(f"in_stats:{name}", t(lambda: ops.in_stats(ops.Feat(z), work, mr), args.iters), n)
    rec(f"in_apply:{name}", t(lambda: ops.in_apply(ops.Feat(z), mr, ops.Feat(y), act=ops.ACT_RELU), args.iters), 2 * n)
    rec(f"in_bwd:{name}", t(lambda: ops.in_backward(ops.Feat(dy), ops.Feat(z), ops.ACT_RELU, mr, work, red,
                                                    ops.Feat(dx)), args.iters), 5 * n)
    red_fn, app_fn = ops.in_bwd_parts(ops.Feat(dy), ops.Feat(z), ops.ACT_RELU, mr, work, red, ops.Feat(dx))
    rec(f"in_bwd_reduce:{name}", t(red_fn, args.iters), 2 * n)
    rec(f"in_bwd_apply:{name}", t(app_fn, args.iters), 3 * n)

for name, kind, C, H in RS_CASES:
    if args.case and args.case not in name:
        continue
    Ho = H // 2 if kind == "down" else 2 * H
    x = torch.randn(B, H, H, C, device=DEV).bfloat16()
    y = torch.empty(B, Ho, Ho, C, device=DEV, dtype=torch.bfloat16)
    n = (x.numel() + y.numel()) * 2
    if kind == "down":
        rec(f"blur_down:{name}", t(lambda: ops.blur_down(ops.Feat(x), ops.Feat(y)), args.iters), n)
        rec(f"blur_down_bwd:{name}", t(lambda: ops.blur_down_bwd(ops.Feat(y), ops.Feat(x)), args.iters), n)
    else:
        rec(f"upsample:{name}", t(lambda: ops.upsample(ops.Feat(x), ops.Feat(y)), args.iters), n)
        rec(f"upsample_bwd:{name}", t(lambda: ops.upsample_bwd(ops.Feat(y), ops.Feat(x)), args.iters), n)
print(json.dumps(res))
