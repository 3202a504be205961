"""Test-mode runner, metrics CSV and Top-K export (SURVEY.md 8(f) rows 1 and 4;
ir:945-1038, 1184-1514), batched on the device.

The reference colorizes one IR frame per call (B = 1, ir:1379-1386), converts
and scores it on the host (tensor_to_rgb_image, compute_metrics with numpy and
scikit-image).  ``run_test`` keeps its inputs (``Config``: test_roots,
test_G_weights, output_dir, img_size, comparison / Top-K options), its outputs
(prediction PNGs mirrored under output_dir, <output_dir>/metrics_test.csv with
the same columns and summary block, <output_dir>/<best50_dirname>/ with
top_<k>_ranking.csv and the copied files, collages under comparison_dirname)
and its printed summary, but runs frames in batches of ``cfg.test_batch``:
host decode -> device INTER_AREA resize (data.DeviceResizer) -> one generator
forward -> device uint8 conversion -> device MAE / MSE / PSNR / SSIM.  Only the
uint8 predictions and four numbers per frame cross PCIe.

Collages: OpenCV's putText is not available, so the labels / metrics text are
drawn with PIL's default bitmap font at the same anchor points (visual only;
the canvas layout -- IR | pred | GT separated by ``pad`` black columns -- is the
reference's).
"""
from __future__ import annotations

import os
import shutil

import numpy as np
import torch

from . import data as D
from .inference import image_metrics_u8, rgb_u8
from .ops import Feat

__all__ = ["float01_to_uint8_rgb", "make_comparison_collage", "save_comparison_image", "save_rgb",
           "save_best_k_outputs", "run_test", "HAVE_SKIMAGE"]

HAVE_SKIMAGE = True   # the SSIM of compute_metrics runs on the device (irgan_ssim_eval_u8)


def float01_to_uint8_rgb(img01_hw_or_hwc):
    """ir:945-958."""
    x = np.clip(img01_hw_or_hwc, 0.0, 1.0)
    if x.ndim == 2:
        x = np.stack([x, x, x], axis=2)
    return (x * 255.0).astype(np.uint8)


def make_comparison_collage(ir01_hw, pred_u8_hwc, gt01_hwc=None, add_text=True, pad=8, font_scale=0.6,
                            thickness=2, metrics_text=None):
    """ir:961-1018: [IR | Pred | GT] on a black canvas, ``pad`` columns apart."""
    imgs = [float01_to_uint8_rgb(ir01_hw), pred_u8_hwc]
    if gt01_hwc is not None:
        imgs.append(float01_to_uint8_rgb(gt01_hwc))
    H = imgs[0].shape[0]
    widths = [im.shape[1] for im in imgs]
    canvas = np.zeros((H, sum(widths) + pad * (len(imgs) - 1), 3), dtype=np.uint8)
    x = 0
    for k, im in enumerate(imgs):
        canvas[:, x:x + im.shape[1], :] = im
        x += im.shape[1] + (pad if k != len(imgs) - 1 else 0)
    if add_text:
        from PIL import Image, ImageDraw
        pil = Image.fromarray(canvas)
        dr = ImageDraw.Draw(pil)
        labels = [("IR", 10), ("Pred", widths[0] + pad + 10)]
        if gt01_hwc is not None:
            labels.append(("GT", widths[0] + pad + widths[1] + pad + 10))
        for text, x0 in labels:
            dr.text((x0, 20), text, fill=(255, 255, 255))
        if metrics_text is not None:
            dr.text((10, H - 22), metrics_text, fill=(255, 255, 255))
        canvas = np.asarray(pil).copy()
    return canvas


def save_rgb(path, img_rgb):
    """ir:879-885."""
    from PIL import Image
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    Image.fromarray(img_rgb).save(path)


def save_comparison_image(cfg, out_rel, collage_u8_hwc):
    """ir:1021-1038: <output_dir>/<comparison_dirname>/<subdirs>/<stem>_cmp.png."""
    stem = os.path.splitext(os.path.basename(out_rel))[0]
    cmp_dir = os.path.join(cfg.output_dir, cfg.comparison_dirname, os.path.dirname(out_rel))
    os.makedirs(cmp_dir, exist_ok=True)
    path = os.path.join(cmp_dir, f"{stem}_cmp.png")
    save_rgb(path, collage_u8_hwc)
    return path


def save_best_k_outputs(cfg, metrics_list, log=print):
    """ir:1220-1330: rank by SSIM (when computed) else PSNR, write
    top_<k>_ranking.csv, copy the predictions and collages (flattened names)."""
    if not metrics_list:
        log("[TOP-K] metrics_list empty, skipping top-K save.")
        return
    metric_key = "ssim" if HAVE_SKIMAGE and any(m.get("ssim") is not None for m in metrics_list) else "psnr"
    valid = [m for m in metrics_list if m.get(metric_key) is not None
             and not (isinstance(m[metric_key], float) and not np.isfinite(m[metric_key]))]
    if not valid:
        log(f"[TOP-K] No valid '{metric_key}' values, skipping top-K save.")
        return
    valid.sort(key=lambda m: m[metric_key], reverse=True)   # stable: ties keep scan order
    top_k = valid[:max(1, int(cfg.topk))]
    best_dir = os.path.join(cfg.output_dir, cfg.best50_dirname)
    preds_sub = os.path.join(best_dir, getattr(cfg, "best50_preds_subdir", "colored"))
    colls_sub = os.path.join(best_dir, getattr(cfg, "best50_collages_subdir", "collages"))
    os.makedirs(preds_sub, exist_ok=True)
    os.makedirs(colls_sub, exist_ok=True)
    rank_path = os.path.join(best_dir, f"top_{len(top_k)}_ranking.csv")
    with open(rank_path, "w", encoding="utf-8") as f:
        f.write("rank,file,mae,mse,psnr,ssim,metric_used\n")
        for r, m in enumerate(top_k, start=1):
            ssim_str = "" if m.get("ssim") is None else f"{m['ssim']:.6f}"
            f.write(f"{r},{m['file']},{m['mae']:.8f},{m['mse']:.8f},{m['psnr']:.6f},{ssim_str},{metric_key}\n")
    copied_preds = copied_colls = 0
    for m in top_k:
        rel = m["file"].replace("\\", "/")
        subdir, base = os.path.dirname(rel), os.path.basename(rel)
        stem = os.path.splitext(base)[0]
        flat_base = rel.replace("/", "__")
        flat_stem = os.path.splitext(flat_base)[0]
        if getattr(cfg, "best50_copy_preds", True):
            src = os.path.join(cfg.output_dir, m["file"])
            if os.path.isfile(src):
                shutil.copy2(src, os.path.join(preds_sub, flat_base))
                copied_preds += 1
            else:
                log(f"[TOP-K][WARN] Missing prediction, cannot copy: {src}")
        if getattr(cfg, "best50_copy_collages", True):
            src = os.path.join(cfg.output_dir, cfg.comparison_dirname, subdir, f"{stem}_cmp.png")
            if not os.path.isfile(src):
                jpg = os.path.join(cfg.output_dir, cfg.comparison_dirname, subdir, f"{stem}_cmp.jpg")
                src = jpg if os.path.isfile(jpg) else src
            if os.path.isfile(src):
                shutil.copy2(src, os.path.join(colls_sub, f"{flat_stem}__cmp.png"))
                copied_colls += 1
            else:
                log(f"[TOP-K][WARN] Missing collage, cannot copy: {src}")
    log(f"[TOP-K] Saved best outputs to: {best_dir}")
    log(f"[TOP-K] Colored copied : {copied_preds}/{len(top_k)} -> {preds_sub}")
    log(f"[TOP-K] Collage copied : {copied_colls}/{len(top_k)} -> {colls_sub}")
    log(f"[TOP-K] Ranking file   : {rank_path}")


def _batches(entries, size, bs):
    """Consecutive runs of at most bs frames with one source size (one device batch)."""
    cur, key = [], None
    for e in entries:
        ir_u8 = D.imread_gray(e[0])
        k = ir_u8.shape
        if cur and (k != key or len(cur) == bs):
            yield cur
            cur = []
        cur.append((e, ir_u8))
        key = k
    if cur:
        yield cur


@torch.no_grad()
def run_test(cfg, model=None, log=print):
    """ir:1333-1514 on the device, ``cfg.test_batch`` frames per generator call."""
    from .ir_colorization import IRColorizationModel
    device = torch.device(cfg.device)
    log(f"[TEST] Device: {device}")
    if model is None:
        model = IRColorizationModel(cfg)
        if cfg.test_G_weights is not None and os.path.isfile(cfg.test_G_weights):
            log(f"Loading generator weights from: {cfg.test_G_weights}")
            model.load_weights(cfg.test_G_weights)
        else:
            log("WARNING: cfg.test_G_weights is None or does not exist; "
                "generator is randomly initialized, results will be meaningless.")
    model.eval()
    os.makedirs(cfg.output_dir, exist_ok=True)
    if not getattr(cfg, "test_roots", None):
        raise ValueError("cfg.test_roots is empty. Please set cfg.test_roots to KAIST set paths.")
    entries = D.collect_kaist_ir_files_from_sets(cfg.test_roots)
    log(f"Found {len(entries)} IR images across test sets: {cfg.test_roots}")
    resizer = D.DeviceResizer(cfg.img_size, device)
    netG = model.netG
    netG._maybe_repack()
    metrics_list = []
    sums = dict(mae=0.0, mse=0.0, psnr=0.0, ssim=0.0)
    count = 0
    best_psnr, best_psnr_sample, best_ssim, best_ssim_sample = -1.0, None, -1.0, None
    done = 0
    for chunk in _batches(entries, cfg.img_size, max(1, int(getattr(cfg, "test_batch", 16)))):
        ir8 = torch.from_numpy(np.stack([u8 for _, u8 in chunk])).to(device)
        B = ir8.shape[0]
        zero = torch.zeros(B, dtype=torch.uint8, device=device)
        ir_t, ir8r = resizer._one(ir8, 1, zero, True, keep_u8=True)   # load_ir_image + ir_to_tensor
        fake = netG.engine.forward(ir_t, training=False)              # eval mode (ir:1357); NHWC fp32
        pred8 = rgb_u8(Feat(fake))                                    # tensor_to_rgb_image, per frame
        # ground truth: <seq>/visible/<file> (ir:1401-1404), resized on the device
        gts = []
        for (ir_path, _, _), _ in chunk:
            vis = os.path.join(os.path.dirname(os.path.dirname(ir_path)), "visible")
            gp = os.path.join(vis, os.path.basename(ir_path))
            gts.append(gp if os.path.isdir(vis) and os.path.isfile(gp) else None)
        have = [i for i, g in enumerate(gts) if g is not None]
        mets = {}
        gt_u8 = {}
        if have:
            g8 = torch.from_numpy(np.stack([D.imread_rgb(gts[i]) for i in have])).to(device)
            g_res = resizer.resize_u8(g8, 3).permute(0, 2, 3, 1).contiguous()   # (h, S, S, 3)
            for i, m in zip(have, image_metrics_u8(pred8[have], g_res)):
                mets[i] = m
            for i, g in zip(have, g_res.cpu().numpy()):
                gt_u8[i] = g
        pred_np = pred8.cpu().numpy()
        # the collage's IR panel from load_ir_image's own float32 v / 255 (ir:823-827, 1374),
        # not from the [-1, 1] tensor (x + 1) / 2, which truncates some gray levels one lower
        ir_np = [D._unit_ir(u8) for u8 in ir8r[:, 0].cpu().numpy()]
        for i, ((ir_path, set_name, seq_name), _) in enumerate(chunk):
            done += 1
            base = os.path.basename(ir_path)
            out_rel = os.path.join(set_name, seq_name, base)
            out_path = os.path.join(cfg.output_dir, out_rel)
            save_rgb(out_path, pred_np[i])
            psnr_val = ssim_val = None
            if i in mets:
                mae, mse, psnr_val, ssim_val = mets[i]
                metrics_list.append({"file": out_rel, "mae": mae, "mse": mse, "psnr": psnr_val, "ssim": ssim_val})
                sums["mae"] += mae
                sums["mse"] += mse
                if np.isfinite(psnr_val):
                    sums["psnr"] += psnr_val
                if ssim_val is not None:
                    sums["ssim"] += ssim_val
                count += 1
                if np.isfinite(psnr_val) and psnr_val > best_psnr:
                    best_psnr, best_psnr_sample = psnr_val, out_rel
                if ssim_val is not None and ssim_val > best_ssim:
                    best_ssim, best_ssim_sample = ssim_val, out_rel
            elif os.path.isdir(os.path.join(os.path.dirname(os.path.dirname(ir_path)), "visible")):
                log(f"[WARN] No GT RGB found for {base}; metrics skipped for this image.")
            if getattr(cfg, "save_comparisons", False):
                text = None
                if psnr_val is not None and ssim_val is not None:
                    text = f"PSNR={psnr_val:.2f}dB  SSIM={ssim_val:.4f}"
                elif psnr_val is not None:
                    text = f"PSNR={psnr_val:.2f}dB"
                gt01 = gt_u8[i].astype(np.float32) / 255.0 if i in gt_u8 else None
                collage = make_comparison_collage(ir_np[i], pred_np[i], gt01,
                                                  add_text=getattr(cfg, "comparison_add_text", True),
                                                  pad=getattr(cfg, "comparison_pad", 8), metrics_text=text)
                save_comparison_image(cfg, out_rel, collage)
            if done % 50 == 0 or done == len(entries):
                log(f"[{done}/{len(entries)}] {ir_path} -> {out_path}")
    log("Test finished.")
    if count == 0:
        log("No metrics were computed (no matching GT RGB images found).")
        return metrics_list
    mean = {k: v / count for k, v in sums.items()}
    log("\n=== Test Metrics (on images with GT) ===")
    log(f"Count      : {count}")
    log(f"Mean MAE   : {mean['mae']:.6f}")
    log(f"Mean MSE   : {mean['mse']:.6f}")
    log(f"Mean PSNR  : {mean['psnr']:.4f} dB")
    log(f"Mean SSIM  : {mean['ssim']:.6f}")
    log(f"Best PSNR  : {best_psnr:.4f} ({best_psnr_sample})" if best_psnr_sample else "Best PSNR  : N/A")
    log(f"Best SSIM  : {best_ssim:.6f} ({best_ssim_sample})" if best_ssim_sample is not None else "Best SSIM  : N/A")
    metrics_path = os.path.join(cfg.output_dir, "metrics_test.csv")
    with open(metrics_path, "w", encoding="utf-8") as f:
        f.write("file,mae,mse,psnr,ssim\n")
        for m in metrics_list:
            ssim_str = "" if m["ssim"] is None else f"{m['ssim']:.6f}"
            f.write(f"{m['file']},{m['mae']:.8f},{m['mse']:.8f},{m['psnr']:.6f},{ssim_str}\n")
        f.write("\n# Summary\n")
        f.write(f"# count,{count}\n")
        f.write(f"# mean_mae,{mean['mae']:.8f}\n")
        f.write(f"# mean_mse,{mean['mse']:.8f}\n")
        f.write(f"# mean_psnr,{mean['psnr']:.6f}\n")
        f.write(f"# mean_ssim,{mean['ssim']:.6f}\n")
    log(f"\nMetrics saved to: {metrics_path}")
    save_best_k_outputs(cfg, metrics_list, log=log)
    return metrics_list
