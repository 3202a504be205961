"""Golden vectors for the eval SSIM of compute_metrics (ir:1208-1213).

The reference calls skimage.metrics.structural_similarity(gt, pred,
data_range=1.0, channel_axis=2) (falling back to multichannel=True on older
scikit-image).  scikit-image is not importable next to torch in this image;
it exists (0.18.3) only in /opt/conda's Python 3.9, so run this once there:

    /opt/conda/bin/python3.9 tests/golden/make_ssim_golden.py

(0.18.3 takes multichannel=True: the same per-channel computation, averaged.)
Inputs are uint8 images divided by 255 in float32, as run_test forms them
(ir:1412-1413); stored: the uint8 inputs and the per-image SSIM.
"""
import os

import numpy as np
from skimage.metrics import structural_similarity as ssim

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    rng = np.random.default_rng(123)
    out = {}
    cases = [(2, 64, 64), (1, 37, 50), (1, 7, 9)]
    for k, (n, h, w) in enumerate(cases):
        gt = rng.integers(0, 256, size=(n, h, w, 3), dtype=np.uint8)
        noise = rng.integers(-40, 41, size=(n, h, w, 3))
        pred = np.clip(gt.astype(np.int64) + noise, 0, 255).astype(np.uint8)
        if k == 0:
            pred[1] = gt[1]                       # identical pair: SSIM 1
        vals = []
        for i in range(n):
            p01 = pred[i].astype(np.float32) / 255.0
            g01 = gt[i].astype(np.float32) / 255.0
            try:
                v = ssim(g01, p01, data_range=1.0, channel_axis=2)
            except (TypeError, ValueError):       # scikit-image < 0.19
                v = ssim(g01, p01, data_range=1.0, multichannel=True)
            vals.append(float(v))
        out[f"pred{k}"], out[f"gt{k}"], out[f"ssim{k}"] = pred, gt, np.array(vals, np.float64)
    np.savez_compressed(os.path.join(HERE, "ssim_eval.npz"), **out)
    print({k: v for k, v in out.items() if k.startswith("ssim")})


if __name__ == "__main__":
    main()
