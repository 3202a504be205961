"""numpy restatement of the reference's inference utilities (test oracle only).

``ir:N`` = ``/root/reference/Code/ir_colorization.py`` line N.  Only tests/
import this module; the product's device path is csrc/infer.hip.  Pinned by
``tests/golden/infer.npz`` (``tests/golden/make_infer_golden.py`` executes the
reference's own functions to produce it; ``tests/test_oracle_golden.py``).
``structural_similarity`` restates scikit-image's SSIM (the third-party
function compute_metrics calls, ir:1208-1213; scikit-image 0.18.3 is the
version in this image, outside torch's interpreter) and is pinned by
``tests/golden/ssim_eval.npz`` (``tests/golden/make_ssim_golden.py`` runs
scikit-image itself).
"""
from __future__ import annotations

import math

import numpy as np

__all__ = ["ir_to_array", "tensor_to_rgb_image", "rgb_u8_batch", "compute_metrics", "structural_similarity"]


def ir_to_array(img_hw):
    """ir:855-862 -- HxW [0,1] float32 -> (1,1,H,W) float32 in [-1,1]."""
    return (np.asarray(img_hw, np.float32)[None, None] * np.float32(2.0) - np.float32(1.0)).astype(np.float32)


def tensor_to_rgb_image(x_bchw):
    """ir:865-876 -- first image of a Bx3xHxW [-1,1] array -> HxWx3 uint8."""
    x = np.asarray(x_bchw[0], np.float32)
    x = (x + 1.0) / 2.0
    x = np.clip(x, 0.0, 1.0)
    x = (x * 255.0).astype(np.uint8)
    return np.transpose(x, (1, 2, 0))


def rgb_u8_batch(x_bhwc):
    """The same conversion for every image of an NHWC float32 batch (the
    device kernel's layout): (B,H,W,C) -> (B,H,W,C) uint8."""
    x = np.asarray(x_bhwc, np.float32)
    x = (x + 1.0) / 2.0
    x = np.clip(x, 0.0, 1.0)
    return (x * 255.0).astype(np.uint8)


def structural_similarity(im1, im2, data_range=1.0, win_size=7, K1=0.01, K2=0.03):
    """scikit-image 0.18 structural_similarity(im1, im2, data_range,
    multichannel=True) with its defaults (uniform 7x7 window, sample
    covariance): per channel, fp64 window means via scipy's uniform_filter,
    the SSIM map cropped by (win_size-1)//2 on every side and averaged; the
    channel results averaged."""
    from scipy.ndimage import uniform_filter
    im1 = np.asarray(im1, np.float64)
    im2 = np.asarray(im2, np.float64)
    if im1.ndim == 2:
        im1, im2 = im1[..., None], im2[..., None]
    if min(im1.shape[:2]) < win_size:
        raise ValueError("win_size exceeds image extent")
    NP = win_size * win_size
    cov_norm = NP / (NP - 1.0)
    C1, C2 = (K1 * data_range) ** 2, (K2 * data_range) ** 2
    pad = (win_size - 1) // 2
    vals = []
    for c in range(im1.shape[2]):
        X, Y = im1[..., c], im2[..., c]
        f = lambda a: uniform_filter(a, size=win_size)   # noqa: E731
        ux, uy = f(X), f(Y)
        vx = cov_norm * (f(X * X) - ux * ux)
        vy = cov_norm * (f(Y * Y) - uy * uy)
        vxy = cov_norm * (f(X * Y) - ux * uy)
        S = ((2 * ux * uy + C1) * (2 * vxy + C2)) / ((ux ** 2 + uy ** 2 + C1) * (vx + vy + C2))
        vals.append(S[pad:S.shape[0] - pad, pad:S.shape[1] - pad].mean())
    return float(np.mean(vals))


def compute_metrics(pred_01, gt_01, with_ssim=False):
    """ir:1184-1217.  with_ssim=False reports ssim_val None, as the reference
    does when HAVE_SKIMAGE is False (ir:1214-1215, how tests/golden/infer.npz
    was made); True adds structural_similarity(gt, pred) (ir:1210)."""
    diff = pred_01 - gt_01
    mae = float(np.mean(np.abs(diff)))
    mse = float(np.mean(diff ** 2))
    psnr = float("inf") if mse == 0 else 20.0 * math.log10(1.0) - 10.0 * math.log10(mse + 1e-12)
    ssim_val = structural_similarity(gt_01, pred_01, data_range=1.0) if with_ssim else None
    return mae, mse, psnr, ssim_val
