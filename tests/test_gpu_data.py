"""KAIST data pipeline on the device and the train_kaist driver (SURVEY.md 8(f)
row 2; ir:1045-1177, 1521-1723).

* the device resize / flip / normalisation (csrc/data.hip) is bit-identical to
  the host path that restates the reference's per-sample code (data.py), for a
  KAIST-sized batch (640x512 -> 256x256) in both modalities;
* kaist_loader over a KAIST-layout directory yields exactly the items the
  reference-contract __getitem__ yields;
* train_kaist plumbing at 64x64, B = 5 (one step per epoch): the step-1 log
  values against the fp64 CPU oracle on the same split (ir:1563-1568), the
  val-L1 line, the LR schedule (ir:212-233, 1718-1721) and the checkpoint
  layout (ir:1706-1715); and one epoch on a KAIST tree through the device path.
"""
import os
import random
import re

import numpy as np
import pytest
import torch
from PIL import Image

from conftest import pkg
from oracle import step as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _host_item(D, ir_u8, rgb_u8, flip, size):
    ir = D.resize_area_u8(ir_u8, size).astype(np.float32)
    if ir.max() > 1.0:
        ir /= 255.0
    rgb = D.resize_area_u8(rgb_u8, size).astype(np.float32) / 255.0
    if flip:
        ir, rgb = np.fliplr(ir).copy(), np.fliplr(rgb).copy()
    return (torch.from_numpy(ir)[None] * 2.0 - 1.0,
            torch.from_numpy(np.transpose(rgb, (2, 0, 1)).copy()) * 2.0 - 1.0)


def test_device_resize_bit_identical_to_host_path():
    D = pkg().data
    rng = np.random.default_rng(0)
    B, H, W, S = 4, 512, 640, 256
    ir = rng.integers(0, 256, size=(B, H, W), dtype=np.uint8)
    ir[3] = rng.integers(0, 2, size=(H, W), dtype=np.uint8)       # max <= 1: the IR rule skips / 255 (ir:1142)
    rgb = rng.integers(0, 256, size=(B, H, W, 3), dtype=np.uint8)
    flip = torch.tensor([1, 0, 1, 0], dtype=torch.uint8)
    out = D.DeviceResizer(S, DEV)({"ir_u8": torch.from_numpy(ir), "rgb_u8": torch.from_numpy(rgb), "flip": flip})
    assert out["ir"].shape == (B, 1, S, S) and out["rgb"].shape == (B, 3, S, S)
    for b in range(B):
        hi, hr = _host_item(D, ir[b], rgb[b], bool(flip[b]), S)
        assert torch.equal(out["ir"][b].cpu(), hi), b
        assert torch.equal(out["rgb"][b].cpu(), hr), b


def _kaist_tree(root, n_seq=2, n_img=4, size=(80, 64)):
    rng = np.random.default_rng(1)
    for s in range(n_seq):
        seq = os.path.join(root, "set00", f"V{s:03d}")
        os.makedirs(os.path.join(seq, "lwir"))
        os.makedirs(os.path.join(seq, "visible"))
        for i in range(n_img):
            g = rng.integers(0, 256, size=size, dtype=np.uint8)
            Image.fromarray(np.repeat(g[:, :, None], 3, 2)).save(os.path.join(seq, "lwir", f"I{i:05d}.png"))
            Image.fromarray(rng.integers(0, 256, size=size + (3,), dtype=np.uint8)).save(
                os.path.join(seq, "visible", f"I{i:05d}.png"))
    return os.path.join(root, "set00")


def test_kaist_loader_equals_reference_items(tmp_path):
    D = pkg().data
    root = _kaist_tree(str(tmp_path))
    ds = D.KAISTPairDataset(root, img_size=32, augment=False)
    got = list(D.kaist_loader(ds, 3, DEV, shuffle=False, drop_last=False))
    assert [b["ir"].shape[0] for b in got] == [3, 3, 2]
    k = 0
    for b in got:
        for j in range(b["ir"].shape[0]):
            ref = ds[k]
            assert torch.equal(b["ir"][j].cpu(), ref["ir"]) and torch.equal(b["rgb"][j].cpu(), ref["rgb"])
            k += 1


def _floats(line, *names):
    out = []
    for n in names:
        m = re.search(re.escape(n) + r"\s*:?\s*(-?\d+\.\d+(?:e[-+]\d+)?)", line)
        out.append(float(m.group(1)))
    return out


def test_train_kaist_plumbing_vs_oracle(tmp_path):
    irc = pkg()
    cfg = irc.Config()
    cfg.device, cfg.compute_dtype = DEV, "fp32"
    cfg.epochs, cfg.lr_decay_start_epoch, cfg.save_every = 3, 1, 5
    cfg.val_ratio, cfg.batch_size = 0.3, 5          # N = 7: val 2, train 5 -> one step per epoch
    cfg.save_dir = str(tmp_path / "ckpt")
    G = O.seeded_params(O.g_param_shapes(), 1, bias_std=0.02)
    Dp = O.seeded_params(O.d_param_shapes(), 2, bias_std=0.02)
    V = O.seeded_params(O.vgg_param_shapes(), 3, kaiming=True)
    cfg.init_G_weights = str(tmp_path / "g0.pth")
    torch.save(G, cfg.init_G_weights)

    def hook(tr):
        tr.netD.store.load(Dp, strict=True)
        tr.vgg.store.load(V, strict=True)
        tr.netD.repack()
        tr.vgg.repack()

    ds = irc.SyntheticPairDataset(7, img_size=64, seed=5)
    logs = []
    hist = irc.train_kaist(cfg, dataset=ds, log=logs.append, trainer_hook=hook)
    assert len(hist) == 3
    # the split of ir:1563-1568 and the fp64 oracle step on the (one) train batch
    idxs = list(range(7))
    random.seed(42)
    random.shuffle(idxs)
    tr_i, va_i = idxs[:5], idxs[5:]
    dd = lambda P: {k: v.double().clone() for k, v in P.items()}   # noqa: E731
    G64, D64, V64 = dd(G), dd(Dp), dd(V)
    ir = torch.stack([ds[i]["ir"] for i in tr_i]).double()
    rgb = torch.stack([ds[i]["rgb"] for i in tr_i]).double()
    ref = O.train_step(G64, D64, V64, ir, rgb, O.AdamState(G64), O.AdamState(D64))
    step1 = next(line for line in logs if line.startswith("Epoch [1/3] Step [1/1]"))
    d_log, g_log = _floats(step1, "D", "G")
    assert abs(d_log - float(ref["loss_D"])) <= 2e-4 and abs(g_log - float(ref["loss_G"])) <= 2e-4, step1
    gan, l1 = _floats(step1, "GAN", "L1")
    assert abs(l1 - float(ref["loss_G_L1"])) <= 2e-4 and abs(gan - float(ref["loss_G_GAN"])) <= 2e-4
    # val L1 after epoch 1: the updated G on the val split (ir:1521-1542)
    vir = torch.stack([ds[i]["ir"] for i in va_i]).double()
    vrgb = torch.stack([ds[i]["rgb"] for i in va_i]).double()
    with torch.no_grad():
        val_ref = float((O.g_forward(G64, vir) - vrgb).abs().mean())
    done1 = next(line for line in logs if line.startswith("Epoch [1/3] DONE"))
    assert abs(_floats(done1, "val L1")[0] - val_ref) <= 1e-3, (done1, val_ref)
    # LambdaLR: 1.0 up to lr_decay_start_epoch, then linear to 0 at `epochs` (ir:212-233)
    lrs = [float(line.split(":")[1]) for line in logs if line.startswith("Current LR (G)")]
    assert lrs == [pytest.approx(1e-4), pytest.approx(0.0), pytest.approx(0.0)]
    # checkpoints: the reference's 52 OIHW keys (ir:1706-1715)
    sd = torch.load(os.path.join(cfg.save_dir, "netG_epoch_003.pth"), weights_only=True)
    assert list(sd) == list(O.g_param_shapes())
    assert all(tuple(sd[k].shape) == tuple(v) for k, v in O.g_param_shapes().items())
    assert os.path.isfile(os.path.join(cfg.save_dir, "netG_best.pth"))
    assert any(line.startswith("Training finished. Best val L1:") for line in logs)


def test_train_kaist_on_kaist_directory(tmp_path):
    """dataset=None: KAISTPairDataset over cfg.train_roots, decode in the loader,
    INTER_AREA + paired flip + normalisation on the device (bf16 step)."""
    irc = pkg()
    root = _kaist_tree(str(tmp_path))
    cfg = irc.Config()
    cfg.device = DEV
    cfg.train_roots = [root]
    cfg.img_size, cfg.batch_size, cfg.epochs, cfg.num_workers = 32, 2, 1, 0
    cfg.save_dir = str(tmp_path / "ckpt")
    logs = []
    hist = irc.train_kaist(cfg, log=logs.append)
    assert len(hist) == 1 and np.isfinite(hist[0]["loss_G"]) and np.isfinite(hist[0]["val_l1"])
    assert "Total pairs: 8, train: 7, val: 1" in logs   # val_size = max(1, int(8 * 0.1)) (ir:1565-1566)
    assert os.path.isfile(os.path.join(cfg.save_dir, "netG_epoch_001.pth"))


@pytest.mark.parametrize("H,W,S", [(200, 160, 256), (300, 200, 256), (64, 80, 100)])
def test_device_inter_area_upscale_bit_identical_to_host(H, W, S):
    """img_size above the source (an upscaling axis): irgan_linear_area_resize_u8 (OpenCV's
    linear path with area-mode coefficients, 8-bit fixed point) equals the host
    restatement data.resize_linear_area_u8 bit for bit, with the flip and the IR max rule."""
    D = pkg().data
    rng = np.random.default_rng(5)
    B = 3
    ir = rng.integers(0, 256, size=(B, H, W), dtype=np.uint8)
    ir[2] = rng.integers(0, 2, size=(H, W), dtype=np.uint8)
    rgb = rng.integers(0, 256, size=(B, H + 8, W - 8, 3), dtype=np.uint8)   # modalities of different sizes
    flip = torch.tensor([0, 1, 1], dtype=torch.uint8)
    out = D.DeviceResizer(S, DEV)({"ir_u8": torch.from_numpy(ir), "rgb_u8": torch.from_numpy(rgb), "flip": flip})
    for b in range(B):
        hi, hr = _host_item(D, ir[b], rgb[b], bool(flip[b]), S)
        assert torch.equal(out["ir"][b].cpu(), hi), b
        assert torch.equal(out["rgb"][b].cpu(), hr), b
