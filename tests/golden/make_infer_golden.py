"""Golden vectors for the inference path, made by
EXECUTING THE REFERENCE's own functions in the build container:

    python tests/golden/make_infer_golden.py

* tensor_to_rgb_image (ir:865-876) on a crafted [-1,1] tensor: out-of-range
  values, the exact k/255 bucket edges and their float32 neighbours, NaN-free
  random values;
* ir_to_tensor (ir:855-862) on a [0,1] image;
* compute_metrics (ir:1184-1217) on uint8-valued pairs (SSIM is None: the
  reference reports None without scikit-image, ir:1214-1215), including an
  identical pair (PSNR inf);
* IRColorizationModel.forward (ir:791-796) with seeded G weights at 32x32
  (the test-mode generator call of run_test, ir:1385-1389) and its uint8 image.

Stored in tests/golden/infer.npz (inputs + outputs; weights are regenerated
from the seed by oracle.step.seeded_params).
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from make_golden import load_reference  # noqa: E402
from oracle import step as O  # noqa: E402

SEED_G = 1


def edge_values():
    """[-1,1]-domain floats whose (x+1)/2*255 lands on / next to integer edges."""
    k = np.arange(256, dtype=np.float32)
    x = (k / np.float32(255.0)) * np.float32(2.0) - np.float32(1.0)
    vals = [x, np.nextafter(x, np.float32(-2)), np.nextafter(x, np.float32(2)),
            np.array([-3.0, -1.0000001, -1.0, 1.0, 1.0000001, 3.0, 0.0, -0.0], np.float32)]
    return np.concatenate(vals).astype(np.float32)


def main():
    torch.set_num_threads(os.cpu_count() or 8)
    R = load_reference()
    g = torch.Generator().manual_seed(11)
    rec = {}
    # tensor_to_rgb_image: (1, 3, H, W) with edge values + random values
    e = edge_values()
    H, W = 16, 48
    n = 3 * H * W
    x = torch.rand(n, generator=g) * 2.4 - 1.2
    x[: e.size] = torch.from_numpy(e)
    x = x.reshape(1, 3, H, W)
    rec["t2rgb_in"] = x.numpy()
    rec["t2rgb_out"] = R.tensor_to_rgb_image(x)
    # ir_to_tensor
    img = torch.rand(20, 24, generator=g).numpy().astype(np.float32)
    rec["ir_img"] = img
    rec["ir_tensor"] = R.ir_to_tensor(img).numpy()
    # compute_metrics on uint8-valued pairs (run_test's pred_u8/255 vs gt_u8/255)
    pu = torch.randint(0, 256, (3, 24, 40, 3), generator=g, dtype=torch.uint8).numpy()
    gu = torch.randint(0, 256, (3, 24, 40, 3), generator=g, dtype=torch.uint8).numpy()
    gu[2] = pu[2]  # identical pair: mse 0 -> psnr inf
    rec["met_pred_u8"], rec["met_gt_u8"] = pu, gu
    met = []
    for i in range(3):
        mae, mse, psnr, ssim = R.compute_metrics(pu[i].astype(np.float32) / 255.0, gu[i].astype(np.float32) / 255.0)
        assert ssim is None or not R.HAVE_SKIMAGE
        met.append([mae, mse, psnr])
    rec["met_out"] = np.array(met, np.float64)
    # IRColorizationModel.forward at 32x32 with seeded weights (fp32)
    cfg = R.Config()
    cfg.device = "cpu"
    model = R.IRColorizationModel(cfg)
    model.netG.load_state_dict(O.seeded_params(O.g_param_shapes(), SEED_G, bias_std=0.02), strict=True)
    model.eval()
    ir = torch.rand(2, 1, 32, 32, generator=g) * 2 - 1
    with torch.no_grad():
        fake = model(ir)
    rec["g_ir"] = ir.numpy()
    rec["g_fake"] = fake.numpy()
    rec["g_u8"] = np.stack([R.tensor_to_rgb_image(fake[i:i + 1]) for i in range(fake.shape[0])])
    out = os.path.join(HERE, "infer.npz")
    np.savez_compressed(out, **rec)
    print("wrote", out, os.path.getsize(out), "bytes; metrics", rec["met_out"].tolist())


if __name__ == "__main__":
    main()
