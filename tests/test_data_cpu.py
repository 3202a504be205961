"""KAIST data pipeline, host side (ir:803-852, 887-942,
1045-1177).  cv2 is not importable here, so INTER_AREA parity with OpenCV is
unpinned; what is pinned: the area tables against the exact area integral, the
host resize against a float64 area average (<= 1 LSB), the pairing / scanning
rules and the item contract against hand-built KAIST-layout trees, and the
cv2.imread conversions (16-bit high byte, BGR2GRAY fixed point)."""
import os
import random

import numpy as np
import pytest
import torch
from PIL import Image

from conftest import pkg


@pytest.fixture(scope="module")
def D():
    return pkg().data


def exact_area_matrix(n_in, n_out):
    """Weights of the pixel-area average: destination d covers [d*s, (d+1)*s)."""
    s = n_in / n_out
    M = np.zeros((n_out, n_in))
    for d in range(n_out):
        a, b = d * s, (d + 1) * s
        for k in range(int(np.floor(a)), int(np.ceil(b))):
            M[d, k] = (min(b, k + 1) - max(a, k)) / s
    return M


@pytest.mark.parametrize("n_in,n_out", [(640, 256), (512, 256), (500, 256), (100, 37), (64, 64), (7, 3)])
def test_area_table_is_the_area_integral(D, n_in, n_out):
    ptr, src, w = D.area_table(n_in, n_out)
    M = np.zeros((n_out, n_in))
    for d in range(n_out):
        for e in range(ptr[d], ptr[d + 1]):
            M[d, src[e]] += w[e]
    assert np.allclose(M.sum(1), 1.0, atol=1e-6)
    assert np.allclose(M, exact_area_matrix(n_in, n_out), atol=2e-6)
    assert all(np.all(np.diff(src[ptr[d]:ptr[d + 1]]) == 1) for d in range(n_out))   # ordered, contiguous


@pytest.mark.parametrize("shape,size", [((512, 640), 256), ((512, 640, 3), 256), ((97, 131, 3), 40)])
def test_host_area_resize_vs_float64(D, shape, size):
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, size=shape, dtype=np.uint8)
    got = D.resize_area_u8(img, size).astype(np.int32)
    a = img.astype(np.float64) if img.ndim == 3 else img.astype(np.float64)[:, :, None]
    My, Mx = exact_area_matrix(shape[0], size), exact_area_matrix(shape[1], size)
    ref = np.einsum("yh,hwc,xw->yxc", My, a, Mx, optimize=True)
    ref = np.clip(np.rint(ref), 0, 255)
    ref = ref[:, :, 0] if img.ndim == 2 else ref
    # the exact area means of 640 -> 256 have denominator 10, so ~10 % of them are
    # exact .5 ties that float32 accumulation (OpenCV's too) rounds either way
    d = np.abs(got - ref)
    assert d.max() <= 1 and (d > 0).mean() < 0.05


def _tree(root, n_seq=2, n_img=3, size=(40, 48), extra=True):
    """A KAIST-layout directory: setXX/Vyyy/{lwir,visible}/Izzzzz.png."""
    rng = np.random.default_rng(1)
    pairs = []
    for s in range(n_seq):
        seq = os.path.join(root, "set00", f"V{s:03d}")
        os.makedirs(os.path.join(seq, "lwir"))
        os.makedirs(os.path.join(seq, "visible"))
        for i in range(n_img):
            fn = f"I{i:05d}.png"
            ir = rng.integers(0, 256, size=size, dtype=np.uint8)
            rgb = rng.integers(0, 256, size=size + (3,), dtype=np.uint8)
            Image.fromarray(np.repeat(ir[:, :, None], 3, 2)).save(os.path.join(seq, "lwir", fn))   # KAIST lwir: 3-ch gray
            Image.fromarray(rgb).save(os.path.join(seq, "visible", fn))
            pairs.append((os.path.join(seq, "lwir", fn), os.path.join(seq, "visible", fn), ir, rgb))
        if extra:   # unmatched files on either side are skipped
            Image.fromarray(ir).save(os.path.join(seq, "lwir", "only_ir.png"))
            Image.fromarray(rgb).save(os.path.join(seq, "visible", "only_rgb.png"))
    if extra:       # an lwir folder without a sibling 'visible' contributes nothing
        os.makedirs(os.path.join(root, "set00", "V999", "lwir"))
        Image.fromarray(ir).save(os.path.join(root, "set00", "V999", "lwir", "I00000.png"))
    return pairs


def test_kaist_pairing_and_item_contract(D, tmp_path):
    pairs = _tree(str(tmp_path))
    ds = D.KAISTPairDataset(str(tmp_path / "set00"), img_size=16, augment=False)
    assert len(ds) == len(pairs)
    assert sorted(zip(ds.ir_paths, ds.rgb_paths)) == sorted((a, b) for a, b, _, _ in pairs)
    for i in range(len(ds)):   # within a sequence: sorted filename order (ir:1105)
        assert os.path.basename(ds.ir_paths[i]) == os.path.basename(ds.rgb_paths[i])
    item = ds[0]
    assert item["ir"].shape == (1, 16, 16) and item["rgb"].shape == (3, 16, 16)
    assert item["ir"].dtype == torch.float32 and item["ir"].min() >= -1 and item["ir"].max() <= 1
    k = ds.ir_paths.index(pairs[0][0])
    ir_u8, rgb_u8 = pairs[0][2], pairs[0][3]
    exp_ir = D.resize_area_u8(ir_u8, 16).astype(np.float32) / 255.0 * 2.0 - 1.0
    exp_rgb = np.transpose(D.resize_area_u8(rgb_u8, 16).astype(np.float32) / 255.0, (2, 0, 1)) * 2.0 - 1.0
    assert torch.equal(ds[k]["ir"][0], torch.from_numpy(exp_ir))
    assert torch.equal(ds[k]["rgb"], torch.from_numpy(exp_rgb))
    sub = D.KAISTPairDataset(str(tmp_path / "set00"), img_size=16, augment=False, indices=[3, 1])
    assert sub.ir_paths == [ds.ir_paths[3], ds.ir_paths[1]]
    with pytest.raises(RuntimeError, match="No IR-RGB pairs"):
        D.KAISTPairDataset(str(tmp_path / "nowhere"))


def test_kaist_paired_flip(D, tmp_path):
    _tree(str(tmp_path), n_seq=1, n_img=2, extra=False)
    ds = D.KAISTPairDataset(str(tmp_path / "set00"), img_size=16, augment=True)
    plain = D.KAISTPairDataset(str(tmp_path / "set00"), img_size=16, augment=False)
    random.seed(5)
    flips = [random.random() < 0.5 for _ in range(8)]
    random.seed(5)
    for f in flips:
        a, b = ds[0], plain[0]
        want_ir = torch.flip(b["ir"], [2]) if f else b["ir"]
        want_rgb = torch.flip(b["rgb"], [2]) if f else b["rgb"]
        assert torch.equal(a["ir"], want_ir) and torch.equal(a["rgb"], want_rgb)


def test_collect_kaist_ir_files(D, tmp_path):
    pairs = _tree(str(tmp_path))
    ent = D.collect_kaist_ir_files_from_sets([str(tmp_path / "set00"), str(tmp_path / "missing")])
    paths = [e[0] for e in ent]
    assert set(a for a, _, _, _ in pairs) <= set(paths)
    assert all(e[1] == "set00" for e in ent)
    assert {e[2] for e in ent} == {"V000", "V001"}          # V999 has no visible/


def test_imread_conversions(D, tmp_path):
    rng = np.random.default_rng(2)
    a16 = rng.integers(0, 65536, size=(5, 7), dtype=np.uint16)
    p16 = str(tmp_path / "g16.png")
    Image.fromarray(a16).save(p16)
    assert np.array_equal(D.imread_gray(p16), (a16 >> 8).astype(np.uint8))
    rgb = rng.integers(0, 256, size=(5, 7, 3), dtype=np.uint8)
    prgb = str(tmp_path / "c.png")
    Image.fromarray(rgb).save(prgb)
    r, g, b = (rgb[..., i].astype(np.int64) for i in range(3))
    assert np.array_equal(D.imread_gray(prgb), ((r * 4899 + g * 9617 + b * 1868 + 8192) >> 14).astype(np.uint8))
    assert np.array_equal(D.imread_rgb(prgb), rgb)
    ir = D.load_ir_image(prgb, 4)
    assert ir.shape == (4, 4) and ir.dtype == np.float32 and ir.max() <= 1
    assert D.load_rgb_image(prgb).shape == (5, 7, 3)


@pytest.mark.parametrize("shape,size", [((64, 80), 256), ((200, 300, 3), 256), ((512, 640), 600), ((31, 17, 3), 64)])
def test_host_inter_area_upscale_linear_area_path(D, shape, size):
    """cv2.resize(INTER_AREA) with an UPscaling axis (img_size above the source, ir:818,
    1139, 1156) is OpenCV's linear resampler with area-mode coefficients in 8-bit fixed
    point (resize_linear_area_u8, parity with cv2 itself unpinned: cv2 absent).  Pinned
    here: constant images stay constant, the fixed-point weights are the rounded float
    area-mode fractions (per destination (1 - f, f), f in [0, 1)), and the result is
    within 1 LSB of the same interpolation evaluated in float64."""
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, size=shape, dtype=np.uint8)
    got = D.resize_area_u8(img, size)
    assert got.shape == (size, size) + shape[2:] and got.dtype == np.uint8
    for c in (0, 7, 128, 255):
        assert np.all(D.resize_area_u8(np.full(shape, c, np.uint8), size) == c)
    for n, cols in zip(shape[:2], (False, True)):
        ofs, coef, lim = D.linear_area_table(n, size, cols)
        assert np.all(np.diff(ofs) >= 0) and ofs.min() >= 0 and ofs.max() <= n - 1
        assert np.all(np.abs(coef.sum(1) - 2048) <= 1) and np.all(coef >= 0)
    # float64 evaluation of the same separable interpolation (weights / 2048)
    a = img.astype(np.float64) if img.ndim == 3 else img.astype(np.float64)[:, :, None]

    def axis(n, columns):
        ofs, coef, lim = D.linear_area_table(n, size, columns)
        M = np.zeros((size, n))
        for d in range(size):
            if columns and d >= lim:
                M[d, ofs[d]] = 1.0
            else:
                M[d, ofs[d]] += coef[d, 0] / 2048
                M[d, min(ofs[d] + 1, n - 1)] += coef[d, 1] / 2048
        return M
    My, Mx = axis(shape[0], False), axis(shape[1], True)
    ref = np.einsum("yh,hwc,xw->yxc", My, a, Mx, optimize=True)
    ref = ref[:, :, 0] if img.ndim == 2 else ref
    d = np.abs(got.astype(np.float64) - ref)
    assert d.max() <= 1.0, d.max()


def test_imread_gray_jpeg_is_the_y_plane(D, tmp_path):
    """cv2.imread(IMREAD_GRAYSCALE) of a colour JPEG asks libjpeg for its
    grayscale output (the decoded Y plane), not YCbCr -> RGB -> BGR2GRAY; PIL's
    draft('L') makes the same libjpeg request."""
    rng = np.random.default_rng(4)
    rgb = rng.integers(0, 256, size=(24, 32, 3), dtype=np.uint8)
    p = str(tmp_path / "c.jpg")
    Image.fromarray(rgb).save(p, quality=90)
    with Image.open(p) as im:
        im.draft("L", im.size)
        y = np.asarray(im.convert("L"))
    with Image.open(p) as im:
        via_rgb = np.asarray(im.convert("RGB")).astype(np.int64)
    g = D.imread_gray(p)
    assert np.array_equal(g, y)
    r, gg, b = (via_rgb[..., i] for i in range(3))
    assert not np.array_equal(g, ((r * 4899 + gg * 9617 + b * 1868 + 8192) >> 14).astype(np.uint8))


def test_collate_raw_modalities_may_differ(D):
    """the IR and RGB sources of one batch may have different sizes (each is
    resized on its own, ir:1139, 1156); within one modality the size must be uniform."""
    items = [{"ir_u8": torch.zeros(64, 80, dtype=torch.uint8), "rgb_u8": torch.zeros(96, 120, 3, dtype=torch.uint8),
              "flip": i % 2} for i in range(3)]
    b = D.collate_raw(items)
    assert b["ir_u8"].shape == (3, 64, 80) and b["rgb_u8"].shape == (3, 96, 120, 3)
    items[1]["ir_u8"] = torch.zeros(65, 80, dtype=torch.uint8)
    with pytest.raises(RuntimeError):
        D.collate_raw(items)
