"""Batched test-mode path: the generator call,
uint8 conversion and error metrics of run_test (ir:1379-1431), on the device.

The reference converts ONE image per call on the host (tensor_to_rgb_image,
ir:865-876: ``.cpu().numpy()``, then numpy float32 ops) and computes MAE / MSE
/ PSNR in numpy (compute_metrics, ir:1184-1206).  Here a whole batch goes
through one G forward, one ``irgan_to_rgb_u8`` launch (NHWC fp32 -> uint8
HxWx3, the reference's exact float32 pipeline) and one
``irgan_image_metrics_u8`` launch; only the uint8 images (or 2 doubles per
image) cross PCIe.  SSIM of compute_metrics (scikit-image's structural_similarity, ir:1208-1213)
runs on the device too (``irgan_ssim_eval_u8``), pinned to scikit-image 0.18.3
outputs (tests/golden/ssim_eval.npz).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import _lib, ops
from .ops import P, Feat, stream

__all__ = ["ir_to_tensor", "rgb_u8", "tensor_to_rgb_image", "colorize_u8", "image_metrics_u8", "compute_metrics"]


def ir_to_tensor(img_hw):
    """ir:855-862: HxW float32 in [0,1] -> (1,1,H,W) float32 in [-1,1] (host tensor)."""
    img = torch.from_numpy(np.ascontiguousarray(np.asarray(img_hw, np.float32)[None, None]))
    return img * 2.0 - 1.0


def rgb_u8(x, out: torch.Tensor = None) -> torch.Tensor:
    """[-1,1] images -> uint8 (B,H,W,C) on the device.

    x: an NCHW fp32 device tensor (B,C,H,W) or an NHWC ``Feat`` (the generator
    engine's own output slice)."""
    if not isinstance(x, Feat):
        if not x.is_cuda:
            raise ValueError("rgb_u8 takes a device tensor (the conversion runs on the GPU)")
        B, C, H, W = x.shape
        nhwc = torch.empty(B, H, W, C, device=x.device, dtype=torch.float32)
        ops.nchw_to_nhwc(x.float().contiguous(), Feat(nhwc))
        x = Feat(nhwc)
    if x.dt != ops.F32:
        raise TypeError("rgb_u8 converts fp32 images")
    if out is None:
        out = torch.empty(x.N, x.H, x.W, x.C, dtype=torch.uint8, device=x.t.device)
    assert out.dtype == torch.uint8 and out.is_contiguous() and tuple(out.shape) == (x.N, x.H, x.W, x.C)
    _lib.call("irgan_to_rgb_u8", x.ptr, x.N, x.H, x.W, x.C, x.ld, x.off, P(out), stream())
    return out


def tensor_to_rgb_image(tensor_bchw):
    """ir:865-876 -- the first image of a (B,3,H,W) [-1,1] device tensor as an
    HxWx3 uint8 numpy array (conversion on the device, 3 bytes/pixel copied)."""
    return rgb_u8(tensor_bchw[:1])[0].cpu().numpy()


@torch.no_grad()
def colorize_u8(model, ir_bchw: torch.Tensor) -> torch.Tensor:
    """Batched inference: IR (B,1,H,W) in [-1,1] on the device -> uint8
    (B,H,W,3) on the device.  ``model`` is an IRColorizationModel or its netG.
    One generator forward on the HIP engine (no autograd tape), then one
    conversion launch straight from the engine's NHWC fp32 output."""
    netG = getattr(model, "netG", model)
    netG._maybe_repack()
    fake = netG.engine.forward(ir_bchw.float(), training=netG.training)   # nn.Dropout follows train()/eval()
    return rgb_u8(Feat(fake))


def image_metrics_u8(pred_u8: torch.Tensor, gt_u8: torch.Tensor, with_ssim=True):
    """Per-image (mae, mse, psnr, ssim) of compute_metrics (ir:1184-1217) on uint8
    (B,H,W,C) device batches, as run_test forms them (pred_u8/255 against
    load_rgb_image's gt_u8/255, ir:1412-1415).  SSIM is scikit-image's
    structural_similarity(gt, pred, data_range=1, channel_axis=2) computed on the
    device (irgan_ssim_eval_u8); None for images smaller than its 7x7 window."""
    assert pred_u8.shape == gt_u8.shape and pred_u8.dtype == gt_u8.dtype == torch.uint8
    pred_u8, gt_u8 = pred_u8.contiguous(), gt_u8.contiguous()
    B, H, W, C = pred_u8.shape
    per = pred_u8[0].numel()
    work = torch.empty(256 * B, dtype=torch.float64, device=pred_u8.device)
    sums = torch.empty(2 * B, dtype=torch.float64, device=pred_u8.device)
    _lib.call("irgan_image_metrics_u8", P(pred_u8), P(gt_u8), B, per, P(work), work.numel(), P(sums), stream())
    ssim = [None] * B
    if with_ssim and H >= 7 and W >= 7:
        sv = torch.empty(B, dtype=torch.float64, device=pred_u8.device)
        _lib.call("irgan_ssim_eval_u8", P(pred_u8), P(gt_u8), B, H, W, C, P(work), work.numel(), P(sv), stream())
        ssim = sv.cpu().tolist()
    out = []
    for (s, q), sv_ in zip(sums.view(B, 2).cpu().tolist(), ssim):
        mae, mse = s / per, q / per
        psnr = float("inf") if mse == 0 else 20.0 * math.log10(1.0) - 10.0 * math.log10(mse + 1e-12)
        out.append((mae, mse, psnr, sv_))
    return out


def compute_metrics(pred_01, gt_01):
    """ir:1184-1206 on host HxWx3 float32 images in [0,1], as run_test calls it
    (pred_u8/255 and load_rgb_image's gt_u8/255, ir:1412-1415): the images are
    quantised back to their uint8 codes (exact for k/255 values) and reduced on
    the device.  Other inputs raise: there is no host fallback."""
    p = np.asarray(pred_01, np.float32)
    g = np.asarray(gt_01, np.float32)
    pu, gu = np.rint(p * 255.0), np.rint(g * 255.0)
    if not (np.array_equal((pu / 255.0).astype(np.float32), p) and np.array_equal((gu / 255.0).astype(np.float32), g)):
        raise ValueError("compute_metrics takes uint8-valued images (k/255), as run_test produces them")
    dev = torch.device("cuda")
    pt = torch.from_numpy(pu.astype(np.uint8)[None]).to(dev)
    gt = torch.from_numpy(gu.astype(np.uint8)[None]).to(dev)
    return image_metrics_u8(pt, gt)[0]
