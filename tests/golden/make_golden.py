"""Generate golden vectors by EXECUTING THE REFERENCE in the build container.

Run once here (the reference is not present on the GPU box):

    python tests/golden/make_golden.py

It imports ``/root/reference/Code/ir_colorization.py`` with stub ``cv2`` and
``torchvision.models`` modules (neither is installed; the hot path never calls
cv2, and ``models.vgg16`` is replaced by a VGG-16 ``features`` stack with
seeded synthetic weights because the ImageNet weights cannot be downloaded).
It then drives the reference's own modules through the train-step body of
ir:1636-1681 (two steps, same batch) and stores inputs, outputs, every loss
term, per-parameter gradient digests and post-step parameter samples in
``tests/golden/step_<variant>.npz``.  Weights come from ``oracle.seeded_params``
(a seed spec), so fixtures stay small: the tests regenerate the identical
weights from the seeds.
"""
from __future__ import annotations

import importlib.util
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import step as O  # noqa: E402

REF = "/root/reference/Code/ir_colorization.py"

SEED_G, SEED_D, SEED_V, SEED_DATA, SEED_IDX = 1, 2, 3, 7, 99
N_SAMPLES = 48
VARIANTS = {
    # name: (H, W, B, no_antialias, no_antialias_up, lambda overrides)
    "s32": (32, 32, 2, False, False, {}),
    "s64": (64, 64, 2, False, False, {}),
    "s32_noaa": (32, 32, 2, True, False, {}),
    "s32_noaaup": (32, 32, 2, False, True, {}),
    # smooth objective: drops the sign()-based terms (perceptual L1, pixel L1, TV)
    # whose discontinuities make G weight grads ill-conditioned (see make_variant)
    "s32_smooth": (32, 32, 2, False, False, {"lambda_perc": 0.0, "lambda_L1": 0.0, "lambda_tv": 0.0}),
    "s64_smooth": (64, 64, 2, False, False, {"lambda_perc": 0.0, "lambda_L1": 0.0, "lambda_tv": 0.0}),
}
LAMBDA_ORDER = ("lambda_L1", "lambda_perc", "lambda_tv", "lambda_ssim", "lambda_gan")


def _vgg_stub():
    """torchvision.models stand-in whose vgg16().features uses seeded weights."""
    tvm = types.ModuleType("torchvision.models")

    class VGG16_Weights:  # noqa: N801
        IMAGENET1K_V1 = "synthetic"

    def vgg16(weights=None, pretrained=False):
        cfg = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"]
        layers, c = [], 3
        for v in cfg:
            if v == "M":
                layers.append(nn.MaxPool2d(2, 2))
            else:
                layers += [nn.Conv2d(c, v, 3, padding=1), nn.ReLU(inplace=True)]
                c = v
        feats = nn.Sequential(*layers)
        sd = O.seeded_params(O.vgg_param_shapes(), SEED_V, kaiming=True)
        feats.load_state_dict(sd, strict=False)
        m = nn.Module()
        m.features = feats
        return m

    tvm.VGG16_Weights = VGG16_Weights
    tvm.vgg16 = vgg16
    return tvm


def load_reference():
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))
    tv = types.ModuleType("torchvision")
    tv.models = _vgg_stub()
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.models"] = tv.models
    spec = importlib.util.spec_from_file_location("ref_ir_colorization", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def digest(t, gen):
    flat = t.detach().reshape(-1).double()
    idx = torch.randint(0, flat.numel(), (min(N_SAMPLES, flat.numel()),), generator=gen)
    return idx.numpy().astype(np.int64), flat[idx].numpy(), float(flat.sum()), float(flat.abs().sum())


def run_reference(R, H, W, B, no_aa, no_aa_up, lam, dtype=torch.float32):
    """Two steps of ir:1636-1681 on the reference's own modules in `dtype`.
    Returns (record, full step-1 grads {'gG': {...}, 'gD': {...}})."""
    cfg = R.Config()
    cfg.device = "cpu"
    for k, v in lam.items():
        setattr(cfg, k, v)
    cfg.no_antialias, cfg.no_antialias_up = no_aa, no_aa_up
    model = R.IRColorizationModel(cfg)
    G0 = O.seeded_params(O.g_param_shapes(no_antialias=no_aa, no_antialias_up=no_aa_up), SEED_G, bias_std=0.02)
    model.netG.load_state_dict(G0, strict=True)
    model.netG.to(dtype)
    netD = R.NLayerDiscriminator(input_nc=4, ndf=64, n_layers=3, norm_layer=R.get_norm_layer("instance"))
    D0 = O.seeded_params(O.d_param_shapes(), SEED_D, bias_std=0.02)
    netD.load_state_dict(D0, strict=True)
    netD.to(dtype)
    optG = torch.optim.Adam(model.netG.parameters(), lr=cfg.lr_G, betas=(cfg.beta1, cfg.beta2))
    optD = torch.optim.Adam(netD.parameters(), lr=cfg.lr_D, betas=(cfg.beta1, cfg.beta2))
    vgg = R.VGGPerceptual("cpu").to(dtype)
    l1 = nn.L1Loss()

    g = torch.Generator().manual_seed(SEED_DATA)
    ir = (torch.rand(B, 1, H, W, generator=g) * 2 - 1).to(dtype)
    rgb = (torch.rand(B, 3, H, W, generator=g) * 2 - 1).to(dtype)

    rec = {"ir": ir.float().numpy(), "rgb": rgb.float().numpy(),
           "meta": np.array([H, W, B, int(no_aa), int(no_aa_up), SEED_G, SEED_D, SEED_V], np.int64),
           "lambdas": np.array([getattr(cfg, k) for k in LAMBDA_ORDER], np.float64)}
    # standalone probes of loss helpers on fixed inputs (ir:686-750)
    rec["vgg_rgb"] = vgg(rgb).detach().float().numpy()[:, :8]
    rec["tv_rgb"] = np.float64(R.tv_loss(rgb).item())
    rec["ssim_ir_rgb"] = np.float64(R.ssim_loss_torch((rgb + 1) / 2, ((ir.repeat(1, 3, 1, 1)) + 1) / 2).item())

    for step in (1, 2):
        # ---- body of ir:1636-1681, verbatim in behaviour, driving reference objects
        optD.zero_grad()
        with torch.no_grad():
            fake_det = model(ir)
        pred_real = netD(torch.cat([ir, rgb], dim=1))
        pred_fake = netD(torch.cat([ir, fake_det], dim=1))
        loss_D = 0.5 * (F.relu(1.0 - pred_real).mean() + F.relu(1.0 + pred_fake).mean())
        loss_D.backward()
        gradD = {k: p.grad.detach().clone() for k, p in netD.named_parameters()}
        optD.step()
        optG.zero_grad()
        fake = model(ir)
        pred_fake_G = netD(torch.cat([ir, fake], dim=1))
        l_gan = -pred_fake_G.mean()
        l_l1 = l1(fake, rgb) * cfg.lambda_L1
        l_perc = F.l1_loss(vgg(fake), vgg(rgb)) * cfg.lambda_perc
        l_tv = R.tv_loss(fake) * cfg.lambda_tv
        l_ssim = R.ssim_loss_torch((fake + 1.0) / 2.0, (rgb + 1.0) / 2.0) * cfg.lambda_ssim
        loss_G = cfg.lambda_gan * l_gan + l_l1 + l_perc + l_tv + l_ssim
        loss_G.backward()
        gradG = {k: p.grad.detach().clone() for k, p in model.netG.named_parameters()}
        optG.step()

        p = f"step{step}_"
        for k, v in dict(loss_D=loss_D, loss_G=loss_G, loss_G_GAN=l_gan, loss_G_L1=l_l1,
                         loss_G_perc=l_perc, loss_G_TV=l_tv, loss_G_ssim=l_ssim).items():
            rec[p + k] = np.float64(v.item())
        if step == 1:
            full = {"gG": gradG, "gD": gradD}
            rec["fake"] = fake.detach().float().numpy()
            rec["pred_real"] = pred_real.detach().float().numpy()
            rec["pred_fake"] = pred_fake.detach().float().numpy()
            rec["pred_fake_G"] = pred_fake_G.detach().float().numpy()
            gen = torch.Generator().manual_seed(SEED_IDX)
            for tag, grads, params in (("gG", gradG, dict(model.netG.named_parameters())),
                                       ("gD", gradD, dict(netD.named_parameters()))):
                for k in grads:
                    idx, samp, s, a = digest(grads[k], gen)
                    rec[f"{tag}|{k}|idx"] = idx
                    rec[f"{tag}|{k}|val"] = samp
                    rec[f"{tag}|{k}|sum"] = np.float64(s)
                    rec[f"{tag}|{k}|abs"] = np.float64(a)
                    pflat = params[k].detach().reshape(-1)
                    rec[f"{tag}|{k}|post"] = pflat[torch.from_numpy(idx)].float().numpy()
    return rec, full


def make_variant(R, name, H, W, B, no_aa, no_aa_up, lam):
    rec, g32 = run_reference(R, H, W, B, no_aa, no_aa_up, lam, torch.float32)
    rec64, g64 = run_reference(R, H, W, B, no_aa, no_aa_up, lam, torch.float64)
    # The same reference step in fp64 is the exact answer.  The perceptual L1
    # (sign of feature differences) and ReLU masks make the G weight gradient
    # discontinuous in its inputs, so the reference's OWN fp32 run differs from
    # fp64 by up to ~1e-2 (max-rel) on some G tensors; record that error per
    # tensor so parity tests can hold the HIP path to the reference's accuracy.
    for tag in ("gG", "gD"):
        for k in g32[tag]:
            a, b = g32[tag][k].double(), g64[tag][k].double()
            rec[f"{tag}|{k}|val64"] = rec64[f"{tag}|{k}|val"]
            rec[f"{tag}|{k}|err32"] = np.float64((a - b).abs().max() / b.abs().max().clamp_min(1e-30))
            rec[f"{tag}|{k}|err32l2"] = np.float64((a - b).norm() / b.norm().clamp_min(1e-30))
    for k in [k for k in rec64 if k.startswith("step")]:
        rec[k + "_64"] = rec64[k]
    rec["fake64"] = rec64["fake"]
    out = os.path.join(HERE, f"step_{name}.npz")
    np.savez_compressed(out, **rec)
    worst = max((float(rec[k]), k) for k in rec if k.endswith("|err32"))
    print("wrote", out, os.path.getsize(out), "bytes; loss_D", rec["step1_loss_D"], "loss_G", rec["step1_loss_G"],
          "worst fp32-vs-fp64 grad", worst)


def main():
    torch.set_num_threads(os.cpu_count() or 8)
    R = load_reference()
    only = sys.argv[1:]
    for name, (H, W, B, a, u, lam) in VARIANTS.items():
        if only and name not in only:
            continue
        make_variant(R, name, H, W, B, a, u, lam)


if __name__ == "__main__":
    main()
