"""The reference's NON-DEFAULT module options on the HIP engines, against goldens made by
executing the reference (tests/golden/make_module_golden.py, fp64) and the pinned oracle:

* ResnetUNetGenerator(norm_layer=get_norm_layer('none')) -- Identity norms, no conv
  biases (ir:154-165, 450-455); padding_type 'replicate' / 'zero' (ir:375-411);
  use_dropout=True (eval: the layout with the Dropout; train: nn.Dropout(0.5) masks,
  checked against the oracle run with the same masks); a ConvTranspose2d variant;
* NLayerDiscriminator(n_layers = 1, 2, 4) and norm 'none' (ir:576-635);
* ssim_loss_torch(window_size = 3, 5, 7, size_average True / False) (ir:714-750).

fp32 parity mode (1e-3 rel bar of the north star): outputs <= 1e-4 abs, input gradients
<= 1e-4 rel, parameter gradients rel-L2 <= 5e-3 on the golden's sampled entries.
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, pkg
from oracle import step as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def fx():
    return dict(np.load(os.path.join(GOLDEN, "modules.npz")))


def _grad_digest_close(fx, prefix, named, tol=5e-3):
    pre_in = set(O.pre_in_bias_keys([k for k, _ in named]))
    for k, g in named:
        if k in pre_in:
            continue
        flat = g.detach().reshape(-1).double().cpu().numpy()
        idx, ref = fx[f"{prefix}|{k}|idx"], fx[f"{prefix}|{k}|val"]
        err = np.linalg.norm(flat[idx] - ref) / max(np.linalg.norm(ref), 1e-30)
        nerr = abs(np.linalg.norm(flat) - float(fx[f"{prefix}|{k}|norm"])) / max(float(fx[f"{prefix}|{k}|norm"]), 1e-30)
        assert err <= tol and nerr <= tol, (prefix, k, err, nerr)


G_CASES = {"g_none": ("none", "reflect", False, False), "g_replicate": ("instance", "replicate", False, False),
           "g_zero": ("instance", "zero", False, False), "g_dropout_eval": ("instance", "reflect", True, False),
           "g_none_zero_up": ("none", "zero", False, True)}


@pytest.mark.parametrize("name", list(G_CASES))
def test_generator_variants_vs_reference(fx, name):
    irc = pkg()
    norm, pad, drop, noaaup = G_CASES[name]
    G = irc.ResnetUNetGenerator(1, 3, 64, norm_layer=irc.get_norm_layer(norm), use_dropout=drop, n_blocks=9,
                                padding_type=pad, no_antialias_up=noaaup, device=DEV, compute_dtype="fp32")
    shapes = O.g_param_shapes(no_antialias_up=noaaup, use_bias=norm == "instance", padding_type=pad,
                              use_dropout=drop)
    assert list(G.state_dict().keys()) == list(shapes.keys())
    G.load_state_dict(O.seeded_params(shapes, 1, bias_std=0.02))
    if drop:
        G.eval()
    x = torch.from_numpy(fx["g_x"]).float().to(DEV)
    out, _ = G(x)
    assert float(np.max(np.abs(out.detach().double().cpu().numpy() - fx[f"{name}|out"]))) <= 1e-4
    Rw = torch.randn(out.shape, generator=torch.Generator().manual_seed(11), dtype=torch.float64).float().to(DEV)
    (out * Rw).sum().backward()
    _grad_digest_close(fx, name, [(k, p.grad) for k, p in G.named_parameters()])


@pytest.mark.parametrize("name,nl,norm", [("d_n1", 1, "instance"), ("d_n2", 2, "instance"), ("d_n4", 4, "instance"),
                                          ("d_none", 3, "none")])
def test_discriminator_variants_vs_reference(fx, name, nl, norm):
    irc = pkg()
    D = irc.NLayerDiscriminator(4, 64, n_layers=nl, norm_layer=irc.get_norm_layer(norm), device=DEV,
                                compute_dtype="fp32")
    shapes = O.d_param_shapes(4, 64, nl, use_bias=norm == "instance")
    assert list(D.state_dict().keys()) == list(shapes.keys())
    D.load_state_dict(O.seeded_params(shapes, 2, bias_std=0.02))
    x = torch.from_numpy(fx["d_x"]).float().to(DEV).requires_grad_(True)
    out = D(x)
    ref = fx[f"{name}|out"]
    assert out.shape == ref.shape
    assert float(np.max(np.abs(out.detach().double().cpu().numpy() - ref))) <= 1e-4 * max(1.0, np.abs(ref).max())
    Rw = torch.randn(out.shape, generator=torch.Generator().manual_seed(12), dtype=torch.float64).float().to(DEV)
    (out * Rw).sum().backward()
    dref = fx[f"{name}|dx"]
    assert float(np.max(np.abs(x.grad.double().cpu().numpy() - dref))) <= 1e-4 * np.abs(dref).max()
    _grad_digest_close(fx, name, [(k, p.grad) for k, p in D.named_parameters()])


@pytest.mark.parametrize("ws", [3, 5, 7, 11])
@pytest.mark.parametrize("avg", [True, False])
def test_ssim_window_sizes_vs_reference(fx, ws, avg):
    irc = pkg()
    a = torch.from_numpy(fx["ssim_a"])
    b = torch.from_numpy(fx["ssim_b"])
    aa = a.float().to(DEV).requires_grad_(True)
    loss = irc.ssim_loss_torch(aa, b.float().to(DEV), window_size=ws, size_average=avg)
    w = torch.arange(1, loss.numel() + 1, dtype=torch.float32, device=DEV).reshape(loss.shape)
    (loss * w).sum().backward()
    if ws == 11:   # the default window: the oracle (pinned to the step goldens) on the same inputs
        a64 = a.clone().requires_grad_(True)
        l64 = O.ssim_loss(a64, b, 11, avg)
        (l64 * torch.arange(1, l64.numel() + 1, dtype=torch.float64).reshape(l64.shape)).sum().backward()
        rl, rg = l64.detach().numpy(), a64.grad.numpy()
    else:
        rl, rg = fx[f"ssim{ws}_{int(avg)}|loss"], fx[f"ssim{ws}_{int(avg)}|grad"]
    assert np.allclose(loss.detach().double().cpu().numpy(), rl, rtol=1e-5, atol=1e-6)
    g = aa.grad.double().cpu().numpy()
    assert np.max(np.abs(g - rg)) <= 1e-4 * np.abs(rg).max()


def test_dropout_kernel_mask_and_scale():
    """irgan_dropout: kept values are exactly x / (1 - p), the keep rate is 1 - p, the same
    seed gives the same mask (the backward), another seed an independent one."""
    ops = pkg().ops
    N, H, W, C = 4, 32, 32, 256
    x = torch.randn(N, H, W, C, device=DEV)
    y1, y2, y3 = (torch.empty_like(x) for _ in range(3))
    ops.dropout(ops.Feat(x), ops.Feat(y1), 1234)
    ops.dropout(ops.Feat(x), ops.Feat(y2), 1234)
    ops.dropout(ops.Feat(x), ops.Feat(y3), 1235)
    keep = y1 != 0
    assert torch.equal(y1, y2)
    assert torch.equal(y1[keep], x[keep] * 2.0)
    rate = keep.float().mean().item()
    assert abs(rate - 0.5) < 0.005, rate
    agree = ((y3 != 0) == keep).float().mean().item()
    assert abs(agree - 0.5) < 0.01, agree
    # bf16 in / out, in place, into a channel slice
    xb = torch.randn(N, H, W, C + 8, device=DEV).bfloat16()
    ref = xb[..., 8:].float().clone()
    ops.dropout(ops.Feat(xb, 8, C), ops.Feat(xb, 8, C), 77, 0.25)
    kb = xb[..., 8:] != 0
    assert abs(kb.float().mean().item() - 0.75) < 0.005
    assert torch.equal(xb[..., 8:][kb].float(), (ref[kb] / 0.75).bfloat16().float())


def test_generator_dropout_training_vs_oracle_with_the_same_masks():
    """use_dropout=True in training mode: nn.Dropout(0.5) after each ResnetBlock's ReLU
    (ir:394-395).  The engine's masks are recovered from its seed (the backward reuses
    them); the oracle g_forward run with exactly those masks gives the same output and
    gradients (fp32 parity mode).  Two forwards draw different masks (the reference's two
    G calls per step, ir:1638 / 1657)."""
    irc = pkg()
    ops = irc.ops
    G = irc.ResnetUNetGenerator(1, 3, 64, norm_layer=irc.get_norm_layer("instance"), use_dropout=True, n_blocks=9,
                                device=DEV, compute_dtype="fp32")
    shapes = O.g_param_shapes(use_dropout=True)
    P = O.seeded_params(shapes, 1, bias_std=0.02)
    G.load_state_dict(P)
    G.repack()
    eng = G.engine
    x = torch.rand(2, 1, 32, 32, generator=torch.Generator().manual_seed(3)) * 2 - 1
    bufs = irc.engine.Buffers(torch.device(DEV))
    fake = eng.forward(x.to(DEV), bufs=bufs).permute(0, 3, 1, 2).cpu()
    seed = bufs.state["dropout_seed"]
    B, H2, W2 = 2, 8, 8
    masks = []
    for b in range(9):
        ones = torch.ones(B, H2, W2, 256, device=DEV)
        m = torch.empty_like(ones)
        ops.dropout(ops.Feat(ones), ops.Feat(m), seed + 2 * b)
        masks.append(m.permute(0, 3, 1, 2).cpu())
    Pr = {k: v.clone().requires_grad_(not k.endswith(".filt")) for k, v in P.items()}
    ref = O.g_forward(Pr, x, dropout_masks=masks)
    assert float((fake - ref.detach()).abs().max()) < 1e-4
    dfake = torch.randn(ref.shape, generator=torch.Generator().manual_seed(4))
    (ref * dfake).sum().backward()
    G.store.zero_grad()
    eng.backward(dfake.permute(0, 2, 3, 1).contiguous().to(DEV), bufs=bufs)
    pre_in = set(O.pre_in_bias_keys(list(Pr)))
    for k, p in G.named_parameters():
        if k in pre_in:
            continue
        got = G.store.oihw(k, G.store.grad).cpu()
        err = float((got - Pr[k].grad).norm() / Pr[k].grad.norm().clamp_min(1e-30))
        assert err < 5e-3, (k, err)
    fake2 = eng.forward(x.to(DEV), bufs=irc.engine.Buffers(torch.device(DEV))).permute(0, 3, 1, 2).cpu()
    assert not torch.equal(fake, fake2), "a second training forward must draw new masks"


def test_generator_dropout_eval_mode_is_deterministic_on_every_entry():
    """use_dropout=True after model.eval(): nn.Dropout is the identity (ir:394-395, 1357), so
    the module forward, colorize_u8 (direct engine call) and validate_kaist all give the
    no-dropout output, twice in a row; validate_kaist returns the model in train mode (ir:1541)."""
    irc = pkg()
    cfg = irc.Config()
    cfg.device, cfg.compute_dtype = DEV, "fp32"
    model = irc.IRColorizationModel(cfg)
    model.netG = irc.ResnetUNetGenerator(1, 3, 64, norm_layer=irc.get_norm_layer("instance"), use_dropout=True,
                                         n_blocks=9, device=DEV, compute_dtype="fp32")
    P = O.seeded_params(O.g_param_shapes(use_dropout=True), 1, bias_std=0.02)
    model.netG.load_state_dict(P)
    x = (torch.rand(2, 1, 32, 32, generator=torch.Generator().manual_seed(5)) * 2 - 1).to(DEV)
    # eval: the Dropout layer is in the layout (conv_block.6) but multiplies by 1
    ref = O.g_forward({k: v.clone() for k, v in P.items()}, x.cpu(), dropout_masks=[torch.ones(())] * 9).detach()
    model.eval()
    with torch.no_grad():
        a, b = model(x).cpu(), model(x).cpu()
    assert torch.equal(a, b) and float((a - ref).abs().max()) < 1e-4
    u1 = irc.inference.colorize_u8(model, x)
    u2 = irc.inference.colorize_u8(model, x)
    assert torch.equal(u1, u2)
    assert torch.equal(u1, irc.inference.rgb_u8(a.to(DEV)))
    rgb = (torch.rand(2, 3, 32, 32, generator=torch.Generator().manual_seed(6)) * 2 - 1)
    loader = [{"ir": x.cpu(), "rgb": rgb}]
    model.train()
    v1 = irc.validate_kaist(model, loader, DEV)
    assert model.training and model.netG.training
    v2 = irc.validate_kaist(model, loader, DEV)
    assert v1 == v2 and abs(v1 - float((ref - rgb).abs().mean())) < 1e-5


@pytest.mark.parametrize("variant", ["norm_none", "replicate", "zero", "dropout"])
def test_train_step_variants_bf16_finite_and_close_to_fp32(variant):
    """The fused bf16 train step (GANTrainer) with a non-default generator / D: every loss,
    grad and parameter finite; losses within 5e-2 of the fp32-mode step (dropout: the two
    G forwards of ir:1638 / 1657 draw different masks, so only finiteness)."""
    irc = pkg()
    g = torch.Generator().manual_seed(61)
    ir = (torch.rand(2, 1, 64, 64, generator=g) * 2 - 1).to(DEV)
    rgb = (torch.rand(2, 3, 64, 64, generator=g) * 2 - 1).to(DEV)
    res = {}
    for dt in ("bf16", "fp32"):
        cfg = irc.Config()
        cfg.device, cfg.compute_dtype = DEV, dt
        if variant == "norm_none":
            cfg.norm = "none"
        model = irc.IRColorizationModel(cfg)
        if variant in ("replicate", "zero", "dropout"):
            model.netG = irc.ResnetUNetGenerator(1, 3, 64, norm_layer=irc.get_norm_layer(cfg.norm),
                                                 use_dropout=variant == "dropout", n_blocks=9,
                                                 padding_type="reflect" if variant == "dropout" else variant,
                                                 device=DEV, compute_dtype=dt)
        model.netG.load_state_dict(O.seeded_params(O.g_param_shapes(
            use_bias=cfg.norm == "instance", padding_type="reflect" if variant in ("dropout", "norm_none") else variant,
            use_dropout=variant == "dropout"), 1, bias_std=0.02))
        tr = irc.GANTrainer(cfg, model=model)
        tr.netD.store.load(O.seeded_params(O.d_param_shapes(use_bias=cfg.norm == "instance"), 2, bias_std=0.02),
                           strict=True)
        tr.netD.repack()
        L = tr.losses(tr.step(ir, rgb))
        for st in (tr.netG.store, tr.netD.store):
            assert torch.isfinite(st.grad).all() and torch.isfinite(st.flat).all()
        assert all(np.isfinite(v) for v in L.values()), L
        res[dt] = L
    if variant != "dropout":
        for k in ("loss_D", "loss_G", "loss_G_L1", "loss_G_perc", "loss_G_ssim"):
            assert abs(res["bf16"][k] - res["fp32"][k]) <= 5e-2 * max(1.0, abs(res["fp32"][k])), (k, res)
