"""Per-layer launch times of the bench step (256^2, B=16, bf16): HIP events around every
tagged conv / InstanceNorm launch on its stream, 3 steps after 3 warm-ups.  Conv tags carry
the shape, so each line also gives TF/s against the 2.5 PF/s dense bf16 peak.  Event records
add ~5-10 us bubbles per launch, so use this for attribution, not for the step time.

    python tools/layer_times.py [--batch 16] [--size 256] [--dtype bf16|fp8]
"""
import argparse
import importlib
import re
import sys

import torch

sys.path.insert(0, ".")
irc = importlib.import_module("infrared-colorization-with-resnet-generator-and-patchgan_amd")
ops = irc.ops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"])
    a = ap.parse_args()
    cfg = irc.Config()
    cfg.device, cfg.compute_dtype, cfg.batch_size, cfg.img_size = "cuda:0", a.dtype, a.batch, a.size
    tr = irc.GANTrainer(cfg)
    tr.netG.store.load(irc.seeded_state(irc.g_param_shapes(), 0), strict=True)
    tr.netD.store.load(irc.seeded_state(irc.d_param_shapes(), 1), strict=True)
    for m in (tr.netG, tr.netD, tr.vgg):
        m.repack()
    g = torch.Generator().manual_seed(7)
    ir = (torch.rand(a.batch, 1, a.size, a.size, generator=g) * 2 - 1).cuda()
    rgb = (torch.rand(a.batch, 3, a.size, a.size, generator=g) * 2 - 1).cuda()
    for _ in range(3):
        tr.step(ir, rgb)
    torch.cuda.synchronize()
    ops.TIMER.tags = None
    ops.TIMER.enabled = True
    for _ in range(a.steps):
        tr.step(ir, rgb)
    torch.cuda.synchronize()
    ops.TIMER.enabled = False
    rows = []
    for tag, (n, ms) in ops.TIMER.summary().items():
        per_step = n / a.steps
        m = re.match(r"(\w+):(\d+)x(\d+)k(\d+)s(\d+)\w@b(\d+)/(\d+)x(\d+)", tag)
        tf = ""
        if m:
            kind, ci, co, k, s, b, h, w = m.groups()
            ci, co, k, s, b, h, w = map(int, (ci, co, k, s, b, h, w))
            ho, wo = (h, w) if kind.startswith("dgrad") else ((h + s - 1) // s, (w + s - 1) // s)
            if kind.startswith("dgrad"):   # tag carries dx size; the conv's output is the dY size
                ho, wo = (h + s - 1) // s, (w + s - 1) // s
            flop = 2.0 * b * ho * wo * co * ci * k * k
            peak = 5e15 if kind.endswith("8") else 2.5e15   # fp8 tags: the dense e4m3 peak
            tf = f"{flop / (ms * 1e-3) / 1e12:7.0f} TF/s ({flop / (ms * 1e-3) / peak:.2f})"
        rows.append((per_step * ms * 1e3, per_step, ms * 1e3, tag, tf))
    rows.sort(reverse=True)
    tot = sum(r[0] for r in rows)
    print(f"tagged launch time per step: {tot / 1e3:.3f} ms")
    print("| us/step | launches/step | avg us | tag | rate |")
    print("|---:|---:|---:|---|---|")
    for us, n, avg, tag, tf in rows:
        print(f"| {us:.0f} | {n:g} | {avg:.1f} | `{tag}` | {tf} |")


if __name__ == "__main__":
    main()
