"""numpy restatement of the reference's inference utilities (test oracle only).

``ir:N`` = ``/root/reference/Code/ir_colorization.py`` line N.  Only tests/
import this module; the product's device path is csrc/infer.hip.  Pinned by
``tests/golden/infer.npz`` (``tests/golden/make_infer_golden.py`` executes the
reference's own functions to produce it; ``tests/test_oracle_golden.py``).
"""
from __future__ import annotations

import math

import numpy as np

__all__ = ["ir_to_array", "tensor_to_rgb_image", "rgb_u8_batch", "compute_metrics"]


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


def compute_metrics(pred_01, gt_01):
    """ir:1184-1206 without the optional skimage SSIM (skimage is not installed
    with torch here: ssim_val is None exactly as the reference reports it when
    HAVE_SKIMAGE is False, ir:1214-1215)."""
    diff = pred_01 - gt_01
    mae = float(np.mean(np.abs(diff)))
    mse = float(np.mean(diff ** 2))
    psnr = float("inf") if mse == 0 else 20.0 * math.log10(1.0) - 10.0 * math.log10(mse + 1e-12)
    return mae, mse, psnr, None
