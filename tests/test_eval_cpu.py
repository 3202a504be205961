"""Host side of the test-mode runner (ir:945-1038, 1220-1330): Top-K ranking,
file copies and collage layout -- no GPU needed."""
import os

import numpy as np
from PIL import Image

from conftest import pkg


class _Cfg:
    topk = 2
    best50_dirname = "Best"
    comparison_dirname = "Comparisons"


def test_save_best_k_ranking_and_copies(tmp_path):
    E = pkg().evaluation
    cfg = _Cfg()
    cfg.output_dir = str(tmp_path)
    ms = [{"file": "set02/V000/I0.png", "mae": 0.1, "mse": 0.01, "psnr": 20.0, "ssim": 0.5},
          {"file": "set02/V000/I1.png", "mae": 0.2, "mse": 0.02, "psnr": 17.0, "ssim": 0.9},
          {"file": "set05/V001/I2.png", "mae": 0.0, "mse": 0.0, "psnr": float("inf"), "ssim": 0.7},
          {"file": "set05/V001/I3.png", "mae": 0.3, "mse": 0.03, "psnr": 15.0, "ssim": None}]
    for m in ms[:3]:
        p = os.path.join(cfg.output_dir, m["file"])
        os.makedirs(os.path.dirname(p), exist_ok=True)
        Image.fromarray(np.zeros((4, 4, 3), np.uint8)).save(p)
    cmp_dir = os.path.join(cfg.output_dir, "Comparisons", "set02", "V000")
    os.makedirs(cmp_dir)
    Image.fromarray(np.zeros((4, 4, 3), np.uint8)).save(os.path.join(cmp_dir, "I1_cmp.png"))
    logs = []
    E.save_best_k_outputs(cfg, ms, log=logs.append)
    best = os.path.join(cfg.output_dir, "Best")
    rank = open(os.path.join(best, "top_2_ranking.csv")).read().splitlines()
    assert rank == ["rank,file,mae,mse,psnr,ssim,metric_used",
                    "1,set02/V000/I1.png,0.20000000,0.02000000,17.000000,0.900000,ssim",
                    "2,set05/V001/I2.png,0.00000000,0.00000000,inf,0.700000,ssim"]
    assert sorted(os.listdir(os.path.join(best, "colored"))) == ["set02__V000__I1.png", "set05__V001__I2.png"]
    assert os.listdir(os.path.join(best, "collages")) == ["set02__V000__I1__cmp.png"]
    assert any("Missing collage" in line for line in logs)
    # no SSIM anywhere -> PSNR ranking, non-finite PSNR dropped
    for m in ms:
        m["ssim"] = None
    E.save_best_k_outputs(cfg, ms, log=logs.append)
    rank = open(os.path.join(best, "top_2_ranking.csv")).read().splitlines()
    assert [r.split(",")[1] for r in rank[1:]] == ["set02/V000/I0.png", "set02/V000/I1.png"]
    assert rank[1].endswith(",,psnr")
    logs.clear()
    E.save_best_k_outputs(cfg, [], log=logs.append)
    assert logs == ["[TOP-K] metrics_list empty, skipping top-K save."]


def test_collage_layout():
    E = pkg().evaluation
    ir = np.linspace(0, 1, 6 * 5, dtype=np.float32).reshape(6, 5)
    pred = np.full((6, 5, 3), 7, np.uint8)
    gt = np.full((6, 5, 3), 0.5, np.float32)
    c = E.make_comparison_collage(ir, pred, gt, add_text=False, pad=3)
    assert c.shape == (6, 5 * 3 + 6, 3) and c.dtype == np.uint8
    assert np.array_equal(c[:, :5, 0], (ir * 255.0).astype(np.uint8))
    assert (c[:, 5:8] == 0).all() and (c[:, 8:13] == 7).all() and (c[:, 16:] == 127).all()
    assert E.make_comparison_collage(ir, pred, None, add_text=True).shape == (6, 5 * 2 + 8, 3)
