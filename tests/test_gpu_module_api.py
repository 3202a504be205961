"""The drop-in module API run the way the reference's training loop runs it.

The reference's step body (ir:1636-1681) is reproduced below statement by
statement, but every object comes from the MI355X package: IRColorizationModel,
NLayerDiscriminator, VGGPerceptual, tv_loss, ssim_loss_torch, with two plain
torch.optim.Adam over the modules' parameters.  The call order matters: D is
called on real and then on fake before ONE loss_D.backward(), and VGG on fake
and then on rgb before loss_G.backward(), so each autograd node must keep its own
activations (the fused GANTrainer never goes through these wrappers).

Criteria are the fp32 step criteria of tests/test_gpu_step.py: losses and the G
output <= 1e-4 rel against the goldens made by executing the reference
(tests/golden/make_golden.py); weight grads in relative L2 against the fp64
reference <= max(5e-3, 5 * the reference's own fp32 error); post-step params
within 2*lr abs; step-2 losses against fp64.
"""
import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from conftest import load_golden, pkg
from oracle import step as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
LAMBDA_ORDER = ("lambda_L1", "lambda_perc", "lambda_tv", "lambda_ssim", "lambda_gan")


def _build(fx):
    irc = pkg()
    H, W, B, noaa, noaaup = [int(v) for v in fx["meta"][:5]]
    cfg = irc.Config()
    cfg.device = DEV
    cfg.compute_dtype = "fp32"
    for k, v in zip(LAMBDA_ORDER, fx["lambdas"]):
        setattr(cfg, k, float(v))
    cfg.no_antialias, cfg.no_antialias_up = bool(noaa), bool(noaaup)
    model = irc.IRColorizationModel(cfg)
    model.netG.load_state_dict(O.seeded_params(O.g_param_shapes(no_antialias=bool(noaa),
                                                                 no_antialias_up=bool(noaaup)), 1, bias_std=0.02))
    netD = irc.NLayerDiscriminator(input_nc=cfg.input_nc + cfg.output_nc, ndf=64, n_layers=3,
                                   norm_layer=irc.get_norm_layer(cfg.norm), device=DEV, compute_dtype="fp32")
    netD = irc.init_net(netD, init_type="normal", init_gain=0.02, device=DEV, initialize_weights=True)
    netD.load_state_dict(O.seeded_params(O.d_param_shapes(), 2, bias_std=0.02))
    vgg_perc = irc.VGGPerceptual(DEV, weights=O.seeded_params(O.vgg_param_shapes(), 3, kaiming=True),
                                 compute_dtype="fp32")
    return irc, cfg, model, netD, vgg_perc


def _grad_check(named, fx, tag, pre_in):
    for k, p in named:
        idx = fx[f"{tag}|{k}|idx"]
        if k in pre_in:
            continue
        g = p.grad.detach().reshape(-1).double().cpu().numpy()
        ref = fx[f"{tag}|{k}|val64"]
        err = np.linalg.norm(g[idx] - ref) / max(np.linalg.norm(ref), 1e-30)
        lim = max(5e-3, 5 * float(fx[f"{tag}|{k}|err32l2"]))
        assert err <= lim, f"{tag} grad {k}: {err} > {lim}"


def _post_check(named, fx, tag):
    for k, p in named:
        idx = fx[f"{tag}|{k}|idx"]
        post = p.detach().reshape(-1).cpu().numpy()[idx]
        assert np.max(np.abs(post - fx[f"{tag}|{k}|post"])) <= 2 * 2e-4 + 1e-6, f"{tag} post-step {k}"


@pytest.mark.parametrize("variant", ["s32", "s64", "s32_noaa", "s32_noaaup"])
def test_reference_step_body_through_module_api(variant):
    fx = load_golden(variant)
    irc, cfg, model, netD, vgg_perc = _build(fx)
    optimizerG = torch.optim.Adam(model.netG.parameters(), lr=cfg.lr_G, betas=(cfg.beta1, cfg.beta2))
    optimizerD = torch.optim.Adam(netD.parameters(), lr=cfg.lr_D, betas=(cfg.beta1, cfg.beta2))
    criterionL1 = nn.L1Loss()
    ir = torch.from_numpy(fx["ir"]).to(DEV)
    rgb = torch.from_numpy(fx["rgb"]).to(DEV)
    pre_in = set(O.pre_in_bias_keys(list(O.g_param_shapes()) + list(O.d_param_shapes())))

    for step in (1, 2):
        # ---- ir:1636-1651
        optimizerD.zero_grad()
        with torch.no_grad():
            fake_rgb_detached = model(ir)
        real_input = torch.cat([ir, rgb], dim=1)
        fake_input = torch.cat([ir, fake_rgb_detached], dim=1)
        pred_real = netD(real_input)
        pred_fake = netD(fake_input)
        loss_D_real = F.relu(1.0 - pred_real).mean()
        loss_D_fake = F.relu(1.0 + pred_fake).mean()
        loss_D = 0.5 * (loss_D_real + loss_D_fake)
        loss_D.backward()
        if step == 1:
            _grad_check(netD.named_parameters(), fx, "gD", pre_in)
        optimizerD.step()
        # ---- ir:1656-1681
        optimizerG.zero_grad()
        fake_rgb = model(ir)
        fake_input = torch.cat([ir, fake_rgb], dim=1)
        pred_fake_for_G = netD(fake_input)
        loss_G_GAN = -pred_fake_for_G.mean()
        loss_G_L1 = criterionL1(fake_rgb, rgb) * cfg.lambda_L1
        feat_fake = vgg_perc(fake_rgb)
        feat_real = vgg_perc(rgb)
        loss_G_perc = F.l1_loss(feat_fake, feat_real) * cfg.lambda_perc
        loss_G_TV = irc.tv_loss(fake_rgb) * cfg.lambda_tv
        fake_01 = (fake_rgb + 1.0) / 2.0
        real_01 = (rgb + 1.0) / 2.0
        loss_G_ssim = irc.ssim_loss_torch(fake_01, real_01) * cfg.lambda_ssim
        loss_G = cfg.lambda_gan * loss_G_GAN + loss_G_L1 + loss_G_perc + loss_G_TV + loss_G_ssim
        loss_G.backward()
        if step == 1:
            _grad_check(model.netG.named_parameters(), fx, "gG", pre_in)
        optimizerG.step()

        got = dict(loss_D=loss_D, loss_G=loss_G, loss_G_GAN=loss_G_GAN, loss_G_L1=loss_G_L1,
                   loss_G_perc=loss_G_perc, loss_G_TV=loss_G_TV, loss_G_ssim=loss_G_ssim)
        if step == 1:
            for k, v in got.items():
                ref = float(fx["step1_" + k])
                assert abs(v.item() - ref) <= 1e-4 * max(1.0, abs(ref)), (k, v.item(), ref)
            assert np.max(np.abs(fake_rgb.detach().cpu().numpy() - fx["fake"])) <= 1e-4
            scale = max(np.max(np.abs(fx["pred_real"])), 1e-6)
            assert np.max(np.abs(pred_real.detach().cpu().numpy() - fx["pred_real"])) <= 1e-4 * max(1, scale)
            assert np.max(np.abs(pred_fake.detach().cpu().numpy() - fx["pred_fake"])) <= 1e-4 * max(1, scale)
            _post_check(model.netG.named_parameters(), fx, "gG")
            _post_check(netD.named_parameters(), fx, "gD")
        else:
            for k in ("loss_D", "loss_G"):
                ref64, ref32 = float(fx["step2_" + k + "_64"]), float(fx["step2_" + k])
                assert abs(got[k].item() - ref64) <= max(1e-3 * max(1.0, abs(ref64)), 3 * abs(ref32 - ref64)), \
                    (k, got[k].item(), ref64)


def test_module_api_matches_fused_trainer():
    """The same step through the module API and through GANTrainer.step (one fused
    call) gives the same losses and the same updated weights (fp32 parity mode)."""
    fx = load_golden("s32")
    irc, cfg, model, netD, vgg_perc = _build(fx)
    tr = irc.GANTrainer(cfg)
    tr.netG.store.load(O.seeded_params(O.g_param_shapes(), 1, bias_std=0.02), strict=True)
    tr.netD.store.load(O.seeded_params(O.d_param_shapes(), 2, bias_std=0.02), strict=True)
    tr.vgg.store.load(O.seeded_params(O.vgg_param_shapes(), 3, kaiming=True), strict=True)
    for m in (tr.netG, tr.netD, tr.vgg):
        m.repack()
    ir = torch.from_numpy(fx["ir"]).to(DEV)
    rgb = torch.from_numpy(fx["rgb"]).to(DEV)
    d = tr.losses(tr.step(ir, rgb))
    optD = torch.optim.Adam(netD.parameters(), lr=cfg.lr_D, betas=(cfg.beta1, cfg.beta2))
    optD.zero_grad()
    with torch.no_grad():
        fk = model(ir)
    ld = 0.5 * (F.relu(1 - netD(torch.cat([ir, rgb], 1))).mean() + F.relu(1 + netD(torch.cat([ir, fk], 1))).mean())
    ld.backward()
    assert abs(ld.item() - d["loss_D"]) <= 1e-5 * max(1, abs(d["loss_D"]))
    # the fused step keeps its D-step gradient in the flat buffer (the G-step D pass
    # computes no weight grads): same grads up to summation order
    for k, p in netD.named_parameters():
        ref = tr.netD.store.oihw(k, tr.netD.store.grad)
        err = (p.grad - ref).abs().max().item()
        assert err <= 1e-4 * max(ref.abs().max().item(), 1e-6), (k, err)
    optD.step()


def test_ssim_size_average_false_per_image():
    """ssim_loss_torch(size_average=False) returns the per-image vector 1 - mean over
    C,H,W (ir:746-747) and its gradient, vs the CPU oracle restatement."""
    irc = pkg()
    g = torch.Generator().manual_seed(3)
    a = torch.rand(3, 3, 40, 40, generator=g)
    b = torch.rand(3, 3, 40, 40, generator=g)
    w = torch.tensor([0.3, -1.0, 2.0])
    ar = a.clone().requires_grad_(True)
    ref = torch.stack([O.ssim_loss(ar[i:i + 1], b[i:i + 1]) for i in range(3)])
    (ref * w).sum().backward()
    ad = a.to(DEV).requires_grad_(True)
    got = irc.ssim_loss_torch(ad, b.to(DEV), size_average=False)
    assert got.shape == (3,)
    (got * w.to(DEV)).sum().backward()
    torch.testing.assert_close(got.detach().cpu(), ref.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(ad.grad.cpu(), ar.grad, rtol=1e-4, atol=1e-7)
    mean = irc.ssim_loss_torch(a.to(DEV), b.to(DEV))
    assert abs(mean.item() - O.ssim_loss(a, b).item()) <= 1e-5


@pytest.mark.parametrize("noaaup", [False, True])
def test_init_net_distribution(noaaup):
    """init_net / init_weights (ir:168-209) through the module API: every conv /
    ConvTranspose weight ~ N(0, 0.02) (mean and std within 5 sigma of their
    sampling error), every bias exactly 0, blur buffers = get_filter(3) (ir:240-266);
    the same for NLayerDiscriminator built the way train_kaist builds it (ir:1591-1598)."""
    irc = pkg()
    cfg = irc.Config()
    cfg.device = DEV
    cfg.no_antialias_up = noaaup
    model = irc.IRColorizationModel(cfg)
    netD = irc.init_net(irc.NLayerDiscriminator(4, 64, 3, irc.get_norm_layer("instance"), device=DEV),
                        init_type="normal", init_gain=0.02, device=DEV, initialize_weights=True)
    for net in (model.netG, netD):
        n_w = 0
        for k, p in net.named_parameters():
            t = p.detach().double().cpu().reshape(-1)
            if k.endswith(".bias"):
                assert not t.any(), k
                continue
            n = t.numel()
            n_w += 1
            assert abs(t.mean().item()) <= 5 * 0.02 / n ** 0.5, (k, t.mean().item())
            assert abs(t.std().item() - 0.02) <= 5 * 0.02 / (2 * n) ** 0.5 + 1e-6, (k, t.std().item())
        assert n_w == sum(1 for k in net.state_dict() if k.endswith(".weight"))
    for k, v in model.netG.state_dict().items():
        if k.endswith(".filt"):
            assert torch.equal(v.cpu(), irc.get_filter(3)[None, None].expand_as(v.cpu())), k
    # the engine computes with what init wrote: a forward is finite and in tanh range
    with torch.no_grad():
        y = model(torch.rand(1, 1, 32, 32, device=DEV) * 2 - 1)
    assert torch.isfinite(y).all() and y.abs().max() <= 1
