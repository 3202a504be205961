"""Pin the CPU oracle against golden vectors produced by the reference itself.

CPU-only.  Tolerances are fp32-restatement level (different op order inside
ATen is allowed); post-step parameters use an absolute tolerance of 2*lr
(Adam's first step is ~lr*sign(g), so elements with tiny
gradients may flip sign), and pre-InstanceNorm biases are excluded from
gradient-value checks (their exact gradient is zero; fp32 values are noise).
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_golden
from oracle import step as O

SEEDS = dict(G=1, D=2, V=3)


def build(fx):
    H, W, B, noaa, noaaup = [int(v) for v in fx["meta"][:5]]
    G = O.seeded_params(O.g_param_shapes(no_antialias=bool(noaa), no_antialias_up=bool(noaaup)),
                        SEEDS["G"], bias_std=0.02)
    D = O.seeded_params(O.d_param_shapes(), SEEDS["D"], bias_std=0.02)
    V = O.seeded_params(O.vgg_param_shapes(), SEEDS["V"], kaiming=True)
    return G, D, V, bool(noaa), bool(noaaup)


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-12))


LAMBDA_ORDER = ("lambda_L1", "lambda_perc", "lambda_tv", "lambda_ssim", "lambda_gan")


def lambdas(fx):
    return dict(zip(LAMBDA_ORDER, (float(v) for v in fx["lambdas"])))


@pytest.mark.parametrize("variant", ["s32", "s64", "s32_noaa", "s32_noaaup", "s32_smooth"])
def test_oracle_step_matches_reference(variant):
    torch.set_num_threads(4)
    fx = load_golden(variant)
    G, D, V, noaa, noaaup = build(fx)
    ir, rgb = torch.from_numpy(fx["ir"]), torch.from_numpy(fx["rgb"])
    optG, optD = O.AdamState(G), O.AdamState(D)
    lam = lambdas(fx)
    out = O.train_step(G, D, V, ir, rgb, optG, optD, lam=lam, no_antialias=noaa, no_antialias_up=noaaup)

    assert rel(out["fake"], fx["fake"]) < 1e-5
    assert rel(out["pred_real"], fx["pred_real"]) < 1e-5
    assert rel(out["pred_fake"], fx["pred_fake"]) < 1e-5
    assert rel(out["pred_fake_G"], fx["pred_fake_G"]) < 1e-4
    for k in ("loss_D", "loss_G", "loss_G_GAN", "loss_G_L1", "loss_G_perc", "loss_G_TV", "loss_G_ssim"):
        assert abs(float(out[k]) - fx["step1_" + k]) <= 1e-5 * max(1.0, abs(fx["step1_" + k])), k

    pre_in = set(O.pre_in_bias_keys(list(G) + list(D)))
    for tag, grads, params in (("gG", out["gradG"], G), ("gD", out["gradD"], D)):
        for k, g in grads.items():
            idx = fx[f"{tag}|{k}|idx"]
            flat = g.reshape(-1).double().numpy()
            post = params[k].reshape(-1).numpy()[idx]
            assert np.max(np.abs(post - fx[f"{tag}|{k}|post"])) <= 2 * 2e-4 + 1e-6, k
            if k in pre_in:
                continue
            scale = max(fx[f"{tag}|{k}|abs"] / flat.size, 1e-12)
            assert np.max(np.abs(flat[idx] - fx[f"{tag}|{k}|val"])) <= 1e-3 * scale * 10 + 1e-6 * np.max(np.abs(flat)), k
            assert abs(flat.sum() - fx[f"{tag}|{k}|sum"]) <= 1e-4 * fx[f"{tag}|{k}|abs"] + 1e-7, k

    # second step on the same batch exercises Adam's running moments
    out2 = O.train_step(G, D, V, ir, rgb, optG, optD, lam=lam, no_antialias=noaa, no_antialias_up=noaaup)
    for k in ("loss_D", "loss_G"):
        assert abs(float(out2[k]) - fx["step2_" + k]) <= 2e-4 * max(1.0, abs(fx["step2_" + k])), k


def test_loss_probes():
    fx = load_golden("s32")
    ir, rgb = torch.from_numpy(fx["ir"]), torch.from_numpy(fx["rgb"])
    V = O.seeded_params(O.vgg_param_shapes(), SEEDS["V"], kaiming=True)
    assert rel(O.vgg_features(V, rgb)[:, :8].numpy(), fx["vgg_rgb"]) < 1e-5
    assert abs(float(O.tv_loss(rgb)) - fx["tv_rgb"]) < 1e-6
    assert abs(float(O.ssim_loss((rgb + 1) / 2, (ir.repeat(1, 3, 1, 1) + 1) / 2)) - fx["ssim_ir_rgb"]) < 1e-6


def test_lr_lambda_schedule():
    # ir:212-233: constant through epoch 40, linear to 0 at epoch 50
    assert O.lr_lambda(0) == 1.0 and O.lr_lambda(39) == 1.0
    assert abs(O.lr_lambda(40) - 0.9) < 1e-12 and abs(O.lr_lambda(44) - 0.5) < 1e-12
    assert O.lr_lambda(49) == 0.0


def test_infer_oracle_matches_reference_golden():
    """oracle/infer.py against tests/golden/infer.npz (executed reference,
    tests/golden/make_infer_golden.py): uint8 conversion bit-exact, ir_to_tensor
    exact, compute_metrics to float64 round-off."""
    import os
    from conftest import GOLDEN
    from oracle import infer as OI
    fx = dict(np.load(os.path.join(GOLDEN, "infer.npz")))
    assert np.array_equal(OI.tensor_to_rgb_image(fx["t2rgb_in"]), fx["t2rgb_out"])
    nhwc = np.transpose(fx["t2rgb_in"], (0, 2, 3, 1))
    assert np.array_equal(OI.rgb_u8_batch(nhwc)[0], fx["t2rgb_out"])
    assert np.array_equal(OI.ir_to_array(fx["ir_img"]), fx["ir_tensor"])
    for i in range(fx["met_out"].shape[0]):
        mae, mse, psnr, ssim = OI.compute_metrics(fx["met_pred_u8"][i].astype(np.float32) / 255.0,
                                                  fx["met_gt_u8"][i].astype(np.float32) / 255.0)
        assert ssim is None
        np.testing.assert_allclose([mae, mse], fx["met_out"][i, :2], rtol=1e-12)
        assert psnr == fx["met_out"][i, 2] or abs(psnr - fx["met_out"][i, 2]) < 1e-9
    # the generator's test-mode output converts to the stored uint8 images
    for i in range(fx["g_fake"].shape[0]):
        assert np.array_equal(OI.tensor_to_rgb_image(fx["g_fake"][i:i + 1]), fx["g_u8"][i])


def test_ssim_oracle_matches_skimage_golden():
    """oracle/infer.structural_similarity against scikit-image 0.18.3 itself
    (tests/golden/make_ssim_golden.py -> ssim_eval.npz): fp64 round-off."""
    import os
    from conftest import GOLDEN
    from oracle import infer as OI
    fx = dict(np.load(os.path.join(GOLDEN, "ssim_eval.npz")))
    k = 0
    while f"ssim{k}" in fx:
        for p, g, want in zip(fx[f"pred{k}"], fx[f"gt{k}"], fx[f"ssim{k}"]):
            got = OI.structural_similarity(g.astype(np.float32) / 255.0, p.astype(np.float32) / 255.0)
            assert abs(got - want) < 1e-12, (k, got, want)
        k += 1
    assert k == 3 and fx["ssim0"][1] == 1.0


def test_oracle_as_written_equals_minimal_step():
    """oracle.step.train_step(as_written=True) (bench.py's second CPU-baseline leg: the
    reference's own ir:1636-1681 order with two G forwards and D grads from loss_G) gives
    the same losses, grads and post-step parameters as the minimal step (fp64)."""
    import torch
    from oracle import step as O
    g = torch.Generator().manual_seed(2)
    ir = torch.rand(2, 1, 32, 32, generator=g, dtype=torch.float64) * 2 - 1
    rgb = torch.rand(2, 3, 32, 32, generator=g, dtype=torch.float64) * 2 - 1
    outs = []
    for aw in (False, True):
        G = {k: v.double() for k, v in O.seeded_params(O.g_param_shapes(), 1, bias_std=0.02).items()}
        D = {k: v.double() for k, v in O.seeded_params(O.d_param_shapes(), 2, bias_std=0.02).items()}
        V = {k: v.double() for k, v in O.seeded_params(O.vgg_param_shapes(), 3, kaiming=True).items()}
        o = O.train_step(G, D, V, ir, rgb, O.AdamState(G), O.AdamState(D), as_written=aw)
        outs.append((o, G, D))
    (a, Ga, Da), (b, Gb, Db) = outs
    for k in ("loss_D", "loss_G", "loss_G_GAN", "loss_G_L1", "loss_G_perc", "loss_G_TV", "loss_G_ssim"):
        assert abs(float(a[k]) - float(b[k])) <= 1e-12 * max(1.0, abs(float(a[k]))), k
    for tag in ("gradG", "gradD"):
        for k in a[tag]:
            assert torch.allclose(a[tag][k], b[tag][k], rtol=1e-10, atol=1e-14), (tag, k)
    for P, Q in ((Ga, Gb), (Da, Db)):
        for k in P:
            assert torch.equal(P[k], Q[k]) or torch.allclose(P[k], Q[k], rtol=1e-12, atol=1e-15), k


def _digest_ok(fx, prefix, named_grads, rtol=1e-9):
    """Sampled gradient entries and the norm vs the golden digest; pre-InstanceNorm biases
    are skipped (exactly-zero gradient: their fp64 values are rounding noise)."""
    import numpy as np
    skip = set(O.pre_in_bias_keys([k for k, _ in named_grads]))
    for k, g in named_grads:
        if k in skip:
            continue
        flat = g.reshape(-1).double().numpy()
        idx = fx[f"{prefix}|{k}|idx"]
        ref = fx[f"{prefix}|{k}|val"]
        scale = max(float(fx[f"{prefix}|{k}|norm"]) / max(flat.size, 1) ** 0.5, 1e-300)
        assert np.max(np.abs(flat[idx] - ref)) <= rtol * max(np.max(np.abs(ref)), scale), (prefix, k)
        assert abs(np.linalg.norm(flat) - float(fx[f"{prefix}|{k}|norm"])) <= rtol * float(fx[f"{prefix}|{k}|norm"])


def test_oracle_matches_reference_module_variants():
    """The oracle's restatement of the NON-DEFAULT module options against goldens made by
    executing the reference (tests/golden/make_module_golden.py, fp64): generator norm
    'none' / padding 'replicate' / 'zero' / the Dropout layout in eval mode / ConvTranspose2d
    without bias; PatchGAN n_layers 1, 2, 4 and norm 'none'; SSIM window sizes 3, 5, 7 with
    size_average True / False.  Outputs, input gradients and parameter-gradient digests
    agree to fp64 rounding."""
    import numpy as np
    import torch
    from oracle import step as O
    fx = dict(np.load(os.path.join(GOLDEN, "modules.npz")))
    x = torch.from_numpy(fx["g_x"])
    cases = {"g_none": ("none", "reflect", False, False), "g_replicate": ("instance", "replicate", False, False),
             "g_zero": ("instance", "zero", False, False), "g_dropout_eval": ("instance", "reflect", True, False),
             "g_none_zero_up": ("none", "zero", False, True)}
    for name, (norm, pad, drop, noaaup) in cases.items():
        shapes = O.g_param_shapes(no_antialias_up=noaaup, use_bias=norm == "instance", padding_type=pad,
                                  use_dropout=drop)
        P = {k: v.double().requires_grad_(not k.endswith(".filt"))
             for k, v in O.seeded_params(shapes, 1, bias_std=0.02).items()}
        if drop:   # eval mode: the Dropout is inactive; the conv keys follow the layout with it
            k1, k2 = O.res_conv_keys(pad, True)
            Q = {k.replace(f"conv_block.{k2}.", "conv_block.5."): v for k, v in P.items()}
            out = O.g_forward(Q, x, no_antialias_up=noaaup, norm=norm, padding_type=pad)
        else:
            out = O.g_forward(P, x, no_antialias_up=noaaup, norm=norm, padding_type=pad)
        assert np.max(np.abs(out.detach().numpy() - fx[f"{name}|out"])) <= 1e-10, name
        Rw = torch.randn(out.shape, generator=torch.Generator().manual_seed(11), dtype=torch.float64)
        (out * Rw).sum().backward()
        _digest_ok(fx, name, [(k, v.grad) for k, v in P.items() if not k.endswith(".filt")])
    xd = torch.from_numpy(fx["d_x"])
    for name, (nl, norm) in {"d_n1": (1, "instance"), "d_n2": (2, "instance"), "d_n4": (4, "instance"),
                             "d_none": (3, "none")}.items():
        shapes = O.d_param_shapes(4, 64, nl, use_bias=norm == "instance")
        P = {k: v.double().requires_grad_(True) for k, v in O.seeded_params(shapes, 2, bias_std=0.02).items()}
        xi = xd.clone().requires_grad_(True)
        out = O.d_forward(P, xi, n_layers=nl, norm=norm)
        assert np.max(np.abs(out.detach().numpy() - fx[f"{name}|out"])) <= 1e-10, name
        Rw = torch.randn(out.shape, generator=torch.Generator().manual_seed(12), dtype=torch.float64)
        (out * Rw).sum().backward()
        assert np.max(np.abs(xi.grad.numpy() - fx[f"{name}|dx"])) <= 1e-10 * max(1.0, np.abs(fx[f"{name}|dx"]).max())
        _digest_ok(fx, name, [(k, v.grad) for k, v in P.items()])
    a, b = torch.from_numpy(fx["ssim_a"]), torch.from_numpy(fx["ssim_b"])
    for ws in (3, 5, 7):
        for avg in (True, False):
            aa = a.clone().requires_grad_(True)
            loss = O.ssim_loss(aa, b, window_size=ws, size_average=avg)
            w = torch.arange(1, loss.numel() + 1, dtype=torch.float64).reshape(loss.shape)
            (loss * w).sum().backward()
            assert np.allclose(loss.detach().numpy(), fx[f"ssim{ws}_{int(avg)}|loss"], rtol=1e-12, atol=1e-14)
            assert np.allclose(aa.grad.numpy(), fx[f"ssim{ws}_{int(avg)}|grad"], rtol=1e-10, atol=1e-14)
