"""Inference path on the MI355X, through the C ABI:

* irgan_to_rgb_u8 vs the reference's tensor_to_rgb_image (ir:865-876) --
  bit-exact on the golden vectors (bucket edges, their float32 neighbours,
  out-of-range values) and on a random batch against oracle/infer.py;
* irgan_image_metrics_u8 vs the reference's compute_metrics (ir:1184-1206) --
  MAE/MSE within 1e-6 relative (the reference averages in numpy float32
  pairwise sums, the kernel in fp64), PSNR within 1e-5 dB, inf for equal images;
  the SSIM (irgan_ssim_eval_u8) within 1e-9 of the oracle's scikit-image
  restatement (test_gpu_eval.py pins it to scikit-image's own outputs);
* colorize_u8 (batched G forward + conversion) vs the reference's
  IRColorizationModel.forward + tensor_to_rgb_image at 32x32 in fp32 mode: the
  G output within 1e-4 abs, so a uint8 code may move by one where the output
  sits within 1e-4 of a bucket edge -- at most 1 LSB and on < 1 % of bytes;
* batch invariance: a batch of 4 equals four single-image calls (<= 1 LSB).
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, pkg
from oracle import infer as OI
from oracle import step as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def fx():
    return dict(np.load(os.path.join(GOLDEN, "infer.npz")))


@pytest.fixture(scope="module")
def inf():
    return pkg().inference


def test_rgb_u8_bit_exact_on_reference_golden(fx, inf):
    x = torch.from_numpy(fx["t2rgb_in"]).to(DEV)
    got = inf.tensor_to_rgb_image(x)
    assert got.dtype == np.uint8 and got.shape == fx["t2rgb_out"].shape
    assert np.array_equal(got, fx["t2rgb_out"])


@pytest.mark.parametrize("shape", [(4, 3, 37, 29), (2, 3, 256, 256), (1, 1, 5, 3)])
def test_rgb_u8_batch_matches_oracle(inf, shape):
    g = torch.Generator().manual_seed(3)
    x = torch.rand(*shape, generator=g) * 2.6 - 1.3
    got = inf.rgb_u8(x.to(DEV)).cpu().numpy()
    want = OI.rgb_u8_batch(x.permute(0, 2, 3, 1).numpy())
    assert np.array_equal(got, want)


def test_rgb_u8_from_channel_slice(inf):
    """NHWC slice input (ld > C, channel offset): the engine-output path."""
    ops = pkg().ops
    g = torch.Generator().manual_seed(4)
    buf = (torch.rand(3, 20, 24, 8, generator=g) * 2 - 1).to(DEV)
    got = inf.rgb_u8(ops.Feat(buf, 2, 3)).cpu().numpy()
    want = OI.rgb_u8_batch(buf[..., 2:5].cpu().numpy())
    assert np.array_equal(got, want)


def test_image_metrics_match_reference_golden(fx, inf):
    p = torch.from_numpy(fx["met_pred_u8"]).to(DEV)
    q = torch.from_numpy(fx["met_gt_u8"]).to(DEV)
    got = inf.image_metrics_u8(p, q)
    for i, ((mae, mse, psnr, ssim), want) in enumerate(zip(got, fx["met_out"])):
        ref_ssim = OI.structural_similarity(fx["met_gt_u8"][i] / 255.0, fx["met_pred_u8"][i] / 255.0)
        assert abs(ssim - ref_ssim) < 1e-9
        assert abs(mae - want[0]) <= 1e-6 * max(want[0], 1e-12) + 1e-12
        assert abs(mse - want[1]) <= 1e-6 * max(want[1], 1e-12) + 1e-12
        assert (np.isinf(psnr) and np.isinf(want[2])) or abs(psnr - want[2]) < 1e-5
    # the reference's host entry point (float [0,1] images) reduces on the device too
    mae, mse, psnr, _ = inf.compute_metrics(fx["met_pred_u8"][0].astype(np.float32) / 255.0,
                                            fx["met_gt_u8"][0].astype(np.float32) / 255.0)
    assert abs(mse - fx["met_out"][0, 1]) <= 1e-6 * fx["met_out"][0, 1]


def _model(dtype):
    irc = pkg()
    cfg = irc.Config()
    cfg.device = DEV
    cfg.compute_dtype = dtype
    m = irc.IRColorizationModel(cfg)
    m.netG.store.load(O.seeded_params(O.g_param_shapes(), 1, bias_std=0.02), strict=True)
    m.netG.repack()
    return m


def test_colorize_u8_matches_reference_forward(fx, inf):
    m = _model("fp32")
    ir = torch.from_numpy(fx["g_ir"]).to(DEV)
    fake = m(ir)   # IRColorizationModel.forward (ir:791-796)
    assert float((fake.cpu() - torch.from_numpy(fx["g_fake"])).abs().max()) < 1e-4
    got = inf.colorize_u8(m, ir).cpu().numpy()
    d = np.abs(got.astype(np.int32) - fx["g_u8"].astype(np.int32))
    assert d.max() <= 1 and (d > 0).mean() < 0.01


def test_colorize_u8_batch_invariant(inf):
    m = _model("bf16")
    g = torch.Generator().manual_seed(9)
    ir = (torch.rand(4, 1, 64, 64, generator=g) * 2 - 1).to(DEV)
    batch = inf.colorize_u8(m, ir).cpu().numpy().astype(np.int32)
    single = np.concatenate([inf.colorize_u8(m, ir[i:i + 1]).cpu().numpy() for i in range(4)]).astype(np.int32)
    assert np.abs(batch - single).max() <= 1
