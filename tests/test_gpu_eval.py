"""Test-mode evaluation on the MI355X (ir:1184-1514).

* irgan_ssim_eval_u8 (via inference.image_metrics_u8) against scikit-image
  0.18.3's structural_similarity outputs (tests/golden/ssim_eval.npz, made by
  running scikit-image itself) and against the oracle's restatement on random
  256x256 batches: within 1e-10 (both read the float32 k/255 values widened
  to fp64; the window sums round in a different order);
* run_test on a KAIST-layout tree (one sequence without visible/, one frame
  without its GT, two frame sizes, a batch boundary): every prediction PNG
  equals the batched generator output converted by the reference's
  tensor_to_rgb_image rule; metrics_test.csv has the reference's columns,
  rows, number formats and summary block, and every row matches the oracle's
  compute_metrics (with SSIM) on the saved prediction vs the host INTER_AREA
  GT; the top-K ranking / copies / collages follow save_best_k_outputs.
"""
import os

import numpy as np
import pytest
import torch
from PIL import Image

from conftest import GOLDEN, pkg
from oracle import infer as OI
from oracle import step as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_ssim_eval_matches_skimage_golden():
    inf = pkg().inference
    fx = dict(np.load(os.path.join(GOLDEN, "ssim_eval.npz")))
    for k in range(3):
        got = inf.image_metrics_u8(torch.from_numpy(fx[f"pred{k}"]).to(DEV), torch.from_numpy(fx[f"gt{k}"]).to(DEV))
        for (_, _, _, s), want in zip(got, fx[f"ssim{k}"]):
            assert abs(s - want) < 1e-10, (k, s, want)
    assert got is not None


def test_ssim_eval_random_batch_vs_oracle():
    inf = pkg().inference
    rng = np.random.default_rng(7)
    gt = rng.integers(0, 256, size=(3, 256, 256, 3), dtype=np.uint8)
    pred = np.clip(gt.astype(np.int64) + rng.integers(-60, 61, size=gt.shape), 0, 255).astype(np.uint8)
    pred[2] = rng.integers(0, 256, size=gt.shape[1:], dtype=np.uint8)    # unrelated pair: SSIM near 0
    got = inf.image_metrics_u8(torch.from_numpy(pred).to(DEV), torch.from_numpy(gt).to(DEV))
    for i, (mae, mse, psnr, s) in enumerate(got):
        rm, rs, rp, rss = OI.compute_metrics(pred[i].astype(np.float32) / 255.0, gt[i].astype(np.float32) / 255.0,
                                             with_ssim=True)
        assert abs(s - rss) < 1e-10 and abs(mse - rs) <= 1e-6 * rs
    small = inf.image_metrics_u8(torch.from_numpy(pred[:, :6, :40]).contiguous().to(DEV),
                                 torch.from_numpy(gt[:, :6, :40]).contiguous().to(DEV))
    assert all(m[3] is None for m in small)       # below skimage's 7x7 window (the reference would raise)


def _tree(root):
    """set02/V000: 3 frames 80x64 + 2 frames 96x72 (size change inside the
    sequence), frame 4's GT missing; set05/V001: no visible/ directory, so
    the scan skips it (ir:929-930)."""
    rng = np.random.default_rng(11)
    sizes = [(64, 80)] * 3 + [(72, 96)] * 2
    seq = os.path.join(root, "set02", "V000")
    os.makedirs(os.path.join(seq, "lwir"))
    os.makedirs(os.path.join(seq, "visible"))
    for i, (h, w) in enumerate(sizes):
        g = rng.integers(0, 256, size=(h, w), dtype=np.uint8)
        Image.fromarray(np.repeat(g[:, :, None], 3, 2)).save(os.path.join(seq, "lwir", f"I{i:05d}.png"))
        if i != 4:
            Image.fromarray(rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)).save(
                os.path.join(seq, "visible", f"I{i:05d}.png"))
    seq2 = os.path.join(root, "set05", "V001", "lwir")
    os.makedirs(seq2)
    Image.fromarray(rng.integers(0, 256, size=(64, 80, 3), dtype=np.uint8)).save(os.path.join(seq2, "I00000.png"))
    return [os.path.join(root, "set02"), os.path.join(root, "set05")]


def test_run_test_outputs_and_csv(tmp_path):
    irc = pkg()
    D = irc.data
    cfg = irc.Config()
    cfg.device, cfg.compute_dtype = DEV, "fp32"
    cfg.img_size, cfg.test_batch, cfg.topk = 32, 2, 3
    cfg.test_roots = _tree(str(tmp_path / "kaist"))
    cfg.output_dir = str(tmp_path / "results")
    cfg.save_comparisons, cfg.comparison_add_text = True, True
    G = O.seeded_params(O.g_param_shapes(), 1, bias_std=0.02)
    cfg.test_G_weights = str(tmp_path / "g.pth")
    torch.save(G, cfg.test_G_weights)
    logs = []
    metrics = irc.run_test(cfg, log=logs.append)
    assert len(metrics) == 4 and any("No GT RGB found for I00004.png" in line for line in logs)
    # predictions: the generator on each frame alone (fp32 mode), reference conversion rule
    m = irc.IRColorizationModel(cfg)
    m.load_weights(cfg.test_G_weights)
    m.eval()
    entries = D.collect_kaist_ir_files_from_sets(cfg.test_roots)
    assert len(entries) == 5       # set05/V001 has no visible/ sibling: not scanned (ir:929-930)
    rows = {}
    for ir_path, set_name, seq_name in entries:
        rel = os.path.join(set_name, seq_name, os.path.basename(ir_path))
        saved = np.asarray(Image.open(os.path.join(cfg.output_dir, rel)))
        ir01 = D.load_ir_image(ir_path, img_size=cfg.img_size)
        with torch.no_grad():
            fake = m(irc.ir_to_tensor(ir01).to(DEV))
        want = OI.tensor_to_rgb_image(fake.cpu().numpy())
        d = np.abs(saved.astype(int) - want.astype(int))
        assert d.max() <= 1 and (d > 0).mean() < 0.01, rel      # batch vs single-frame G: fp32 round-off
        gt_path = os.path.join(os.path.dirname(os.path.dirname(ir_path)), "visible", os.path.basename(ir_path))
        if os.path.isfile(gt_path):
            rows[rel] = OI.compute_metrics(saved.astype(np.float32) / 255.0,
                                           D.load_rgb_image(gt_path, img_size=cfg.img_size), with_ssim=True)
    assert set(rows) == {m_["file"] for m_ in metrics}
    # metrics_test.csv: columns, formats, summary
    lines = open(os.path.join(cfg.output_dir, "metrics_test.csv")).read().splitlines()
    assert lines[0] == "file,mae,mse,psnr,ssim" and lines[5] == "" and lines[6] == "# Summary"
    for line in lines[1:5]:
        f, mae, mse, psnr, ssim = line.split(",")
        r = rows[f]
        assert abs(float(mae) - r[0]) < 2e-8 and abs(float(mse) - r[1]) < 2e-8
        assert abs(float(psnr) - r[2]) < 2e-6 and abs(float(ssim) - r[3]) < 2e-6
        assert len(mae.split(".")[1]) == 8 and len(psnr.split(".")[1]) == 6 and len(ssim.split(".")[1]) == 6
    assert lines[7] == "# count,4"
    mean_ssim = np.mean([r[3] for r in rows.values()])
    assert abs(float(lines[11].split(",")[1]) - mean_ssim) < 2e-6 and lines[11].startswith("# mean_ssim,")
    # top-K: SSIM ranking, flattened copies of predictions and collages
    best = os.path.join(cfg.output_dir, cfg.best50_dirname)
    rank = open(os.path.join(best, "top_3_ranking.csv")).read().splitlines()
    assert rank[0] == "rank,file,mae,mse,psnr,ssim,metric_used" and len(rank) == 4
    order = sorted(rows, key=lambda k: rows[k][3], reverse=True)[:3]
    assert [r.split(",")[1] for r in rank[1:]] == order and all(r.endswith(",ssim") for r in rank[1:])
    for rel in order:
        flat = rel.replace(os.sep, "__")
        assert os.path.isfile(os.path.join(best, "colored", flat))
        assert os.path.isfile(os.path.join(best, "collages", os.path.splitext(flat)[0] + "__cmp.png"))
    # collages: [IR | pred | GT] with 8-pixel gutters; no GT -> two panels
    c = np.asarray(Image.open(os.path.join(cfg.output_dir, "Comparisons", "set02", "V000", "I00000_cmp.png")))
    assert c.shape == (32, 32 * 3 + 16, 3)
    # the IR panel is the reference's float01_to_uint8_rgb(load_ir_image(...)) bit for bit
    # (ir:945-958, 1374: float32 v / 255 * 255 truncated), not rebuilt from the [-1, 1] tensor
    ir_path0 = [e[0] for e in entries if e[0].endswith(os.path.join("set02", "V000", "lwir", "I00000.png"))][0]
    ir01 = D.load_ir_image(ir_path0, img_size=cfg.img_size)
    want_panel = np.repeat((np.clip(ir01, 0.0, 1.0) * 255.0).astype(np.uint8)[:, :, None], 3, axis=2)
    # (labels are drawn from x=10, y=10 on: compare the untouched left columns and top rows)
    assert np.array_equal(c[:, :10], want_panel[:, :10]) and np.array_equal(c[:10, :32], want_panel[:10])
    c4 = np.asarray(Image.open(os.path.join(cfg.output_dir, "Comparisons", "set02", "V000", "I00004_cmp.png")))
    assert c4.shape == (32, 32 * 2 + 8, 3)
    assert any(line.startswith("Mean SSIM  :") for line in logs)
