"""Time the CPU oracle against the reference's own step on the same host cores.

Container-only (reads /root/reference through tests/golden/make_golden.py's
stubbed loader; never runs on the GPU box).  Both legs run ir:1636-1681 on
identical seeded weights and U(-1,1) data in fp32 with the same torch thread
count; the reference leg drives the reference's modules exactly as its train
loop does (two G forwards per step), the oracle leg runs oracle/step.py's
minimal step (one G forward).  Also reports both legs' first-step losses.

    python tools/oracle_speed_vs_reference.py [--size 256] [--batch 1] [--steps 3] [--threads 8]
"""
import argparse
import importlib.util
import json
import os
import sys
import time

import torch
import torch.nn as nn
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import step as O  # noqa: E402


def _make_golden():
    p = os.path.join(ROOT, "tests", "golden", "make_golden.py")
    spec = importlib.util.spec_from_file_location("make_golden", p)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    mg = _make_golden()
    R = mg.load_reference()
    H = W = a.size
    B = a.batch
    G0 = O.seeded_params(O.g_param_shapes(), 0)
    D0 = O.seeded_params(O.d_param_shapes(), 1)
    V0 = O.seeded_params(O.vgg_param_shapes(), 3, kaiming=True)
    g = torch.Generator().manual_seed(7)
    ir = torch.rand(B, 1, H, W, generator=g) * 2 - 1
    rgb = torch.rand(B, 3, H, W, generator=g) * 2 - 1

    # ---- reference leg (reference modules, the train-loop body ir:1636-1681)
    cfg = R.Config()
    cfg.device = "cpu"
    model = R.IRColorizationModel(cfg)
    model.netG.load_state_dict(G0, strict=True)
    netD = R.NLayerDiscriminator(input_nc=4, ndf=64, n_layers=3, norm_layer=R.get_norm_layer("instance"))
    netD.load_state_dict(D0, strict=True)
    vgg = R.VGGPerceptual("cpu")   # the loader's torchvision stub seeds it like V0 (seed 3)
    optG = torch.optim.Adam(model.netG.parameters(), lr=cfg.lr_G, betas=(cfg.beta1, cfg.beta2))
    optD = torch.optim.Adam(netD.parameters(), lr=cfg.lr_D, betas=(cfg.beta1, cfg.beta2))
    l1 = nn.L1Loss()

    def ref_step():
        optD.zero_grad()
        with torch.no_grad():
            fake_det = model(ir)
        pr = netD(torch.cat([ir, rgb], 1))
        pf = netD(torch.cat([ir, fake_det], 1))
        lD = 0.5 * (F.relu(1.0 - pr).mean() + F.relu(1.0 + pf).mean())
        lD.backward()
        optD.step()
        optG.zero_grad()
        fake = model(ir)
        pg = netD(torch.cat([ir, fake], 1))
        lG = (cfg.lambda_gan * -pg.mean() + l1(fake, rgb) * cfg.lambda_L1
              + F.l1_loss(vgg(fake), vgg(rgb)) * cfg.lambda_perc + R.tv_loss(fake) * cfg.lambda_tv
              + R.ssim_loss_torch((fake + 1) / 2, (rgb + 1) / 2) * cfg.lambda_ssim)
        lG.backward()
        optG.step()
        return lD.item(), lG.item()

    Go, Do = {k: v.clone() for k, v in G0.items()}, {k: v.clone() for k, v in D0.items()}
    oG, oD = O.AdamState(Go), O.AdamState(Do)

    def ora_step():
        o = O.train_step(Go, Do, V0, ir, rgb, oG, oD)
        return float(o["loss_D"]), float(o["loss_G"])

    first_ref = ref_step()
    first_ora = ora_step()

    def timed(fn):
        t0 = time.perf_counter()
        for _ in range(a.steps):
            fn()
        return (time.perf_counter() - t0) / a.steps

    t_ref = timed(ref_step)
    t_ora = timed(ora_step)
    print(json.dumps({
        "size": H, "batch": B, "threads": a.threads, "steps_timed": a.steps,
        "reference_s_per_step": round(t_ref, 3), "oracle_s_per_step": round(t_ora, 3),
        "reference_img_per_s": round(B / t_ref, 4), "oracle_img_per_s": round(B / t_ora, 4),
        "oracle_over_reference_speed": round(t_ref / t_ora, 3),
        "step1_losses_reference": first_ref, "step1_losses_oracle": first_ora,
        "note": "VGG weights: seeded (ImageNet weights unavailable offline); the reference leg "
                "runs G forward twice per step as written, the oracle once",
    }))


if __name__ == "__main__":
    main()
