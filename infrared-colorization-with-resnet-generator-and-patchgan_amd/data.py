"""KAIST data pipeline: the reference's image I/O and
paired dataset (ir:803-852, 887-942, 1045-1177) with the per-sample pixel work
moved to the device.

Reference behaviour, per sample in CPU DataLoader workers: cv2.imread ->
cv2.resize(INTER_AREA) to img_size^2 -> float32 / 255 -> paired random
horizontal flip -> x * 2 - 1.  At ~1,000 img/s per GPU that is the bottleneck
(ir:107: 4 workers).  Here:

* ``KAISTPairDataset`` keeps the reference's constructor, pairing rules
  (filename intersection of sibling ``lwir`` / ``visible`` folders, os.walk
  order, ``indices`` subset) and ``__getitem__`` contract ({'ir': 1xHxW,
  'rgb': 3xHxW} float32 in [-1, 1]) -- computed on the host exactly as the
  reference does, for code that indexes the dataset directly;
* ``KAISTPairDataset.raw(i)`` returns only the DECODED uint8 images (+ the flip
  draw), and ``kaist_loader`` collates those into pinned uint8 batches that one
  ``irgan_area_resize_u8`` + one ``irgan_u8_to_unit`` launch per modality turn
  into the [-1, 1] device batch (csrc/data.hip).  ``train_kaist`` uses this path.

Decoding: OpenCV is not available in this image, so files are decoded with PIL
and converted with cv2's rules (IMREAD_GRAYSCALE: 16-bit PNG -> high byte,
colour -> BGR2GRAY fixed-point weights; IMREAD_COLOR + BGR2RGB).  INTER_AREA is
OpenCV's general area-resize recurrence (computeResizeAreaTab + resizeArea_,
float32, round half to even), restated here and in the kernel with the same
float operation order.  Parity with cv2 itself is UNPINNED (cv2 absent; the
reference ships no decoded fixtures): the host and device paths are pinned to
each other bit for bit, and the area tables to the exact area integral.
"""
from __future__ import annotations

import ctypes
import os
import random

import numpy as np
import torch

from . import _lib
from .ops import P, stream

__all__ = ["EXTS", "area_table", "linear_area_table", "resize_area_u8", "resize_linear_area_u8", "imread_gray", "imread_rgb", "load_ir_image", "load_rgb_image",
           "collect_kaist_ir_files_from_sets", "scan_kaist_pairs", "KAISTPairDataset", "DeviceResizer",
           "collate_raw", "kaist_loader"]

EXTS = ('.png', '.jpg', '.jpeg', '.bmp', '.tif', '.tiff')   # ir:901, 1072


# ----------------------------------------------------------------------------
# INTER_AREA tables (OpenCV computeResizeAreaTab) and the host resize
# ----------------------------------------------------------------------------

def area_table(ssize: int, dsize: int):
    """Per-axis INTER_AREA table as CSR arrays (ptr [dsize+1], src [k], w [k]):
    destination index d takes sum_{e in ptr[d]..ptr[d+1]-1} w[e] * S[src[e]].

    OpenCV's recurrence for scale = ssize / dsize >= 1 (cv::resize computes the
    scale as 1 / (dsize / ssize) in double): the cell [d*scale, d*scale + scale)
    clipped to the image, partial first / last source pixels weighted by their
    covered fraction, every weight divided by the cell width; entries ordered by
    source index."""
    scale = 1.0 / (dsize / ssize)
    if scale < 1.0:
        raise ValueError("area_table is the downscaling table; upscaling uses linear_area_table")
    ptr, src, w = [0], [], []
    for dx in range(dsize):
        fsx1 = dx * scale
        fsx2 = fsx1 + scale
        cell = min(scale, ssize - fsx1)
        sx1, sx2 = int(np.ceil(fsx1)), int(np.floor(fsx2))
        sx2 = min(sx2, ssize - 1)
        sx1 = min(sx1, sx2)
        if sx1 - fsx1 > 1e-3:
            src.append(sx1 - 1)
            w.append(float(np.float32((sx1 - fsx1) / cell)))
        for sx in range(sx1, sx2):
            src.append(sx)
            w.append(float(np.float32(1.0 / cell)))
        if fsx2 - sx2 > 1e-3:
            src.append(sx2)
            w.append(float(np.float32(min(min(fsx2 - sx2, 1.0), cell) / cell)))
        ptr.append(len(src))
    return np.array(ptr, np.int32), np.array(src, np.int32), np.array(w, np.float32)


INTER_RESIZE_COEF_BITS = 11
INTER_RESIZE_COEF_SCALE = 1 << INTER_RESIZE_COEF_BITS


def _cv_round(v):
    return int(np.rint(v))   # cvRound: nearest, ties to even


def linear_area_table(ssize: int, dsize: int, columns: bool = True):
    """Per-axis table of cv2.resize(INTER_AREA) when either axis UPscales: OpenCV then
    runs its linear resampler with "area mode" coefficients (resizeGeneric_ with
    area_mode): source index s = floor(d * scale), fraction
    f = (d + 1) - (s + 1) / scale (as float32), f <= 0 -> 0 else f - floor(f); left /
    right border clamps (s < 0 -> s = 0, f = 0; s >= ssize - 1 -> s = ssize - 1, f = 0);
    8-bit fixed-point weights round((1 - f) * 2048), round(f * 2048).  The border
    clamps are the column table's (columns=True); the row table keeps s and f as
    computed (OpenCV clamps the second source ROW index instead).
    Returns (ofs int32 [dsize], coef int16-valued int32 [dsize][2], lim): destinations
    d >= lim take the single tap S[ofs] * 2048 (OpenCV's xmax; rows never do)."""
    inv = dsize / ssize
    scale = 1.0 / inv
    ofs = np.zeros(dsize, np.int32)
    coef = np.zeros((dsize, 2), np.int32)
    lim = dsize
    for d in range(dsize):
        sx = int(np.floor(d * scale))
        f = float(np.float32((d + 1) - (sx + 1) * inv))
        f = 0.0 if f <= 0 else float(np.float32(f - np.floor(f)))
        if columns and sx < 0:
            f, sx = 0.0, 0
        if columns and sx + 1 >= ssize:
            lim = min(lim, d)
            if sx >= ssize - 1:
                f, sx = 0.0, ssize - 1
        ofs[d] = sx
        c0, c1 = np.float32(1.0) - np.float32(f), np.float32(f)
        coef[d] = (_cv_round(np.float32(c0 * np.float32(INTER_RESIZE_COEF_SCALE))),
                   _cv_round(np.float32(c1 * np.float32(INTER_RESIZE_COEF_SCALE))))
    return ofs, coef, lim


def resize_linear_area_u8(img: np.ndarray, width: int, height: int) -> np.ndarray:
    """cv2.resize(img, (width, height), interpolation=INTER_AREA) for uint8 when either axis
    upscales (OpenCV's generic linear path in 8-bit fixed point): horizontal
    D = S[x0] * a0 + S[x0 + C] * a1 (int32; single tap S[x0] * 2048 from the xmax border
    on), vertical dst = (((b0 * (D0 >> 4)) >> 16) + ((b1 * (D1 >> 4)) >> 16) + 2) >> 2 with
    the second row clamped to the image (VResizeLinear<uchar, int, short>)."""
    a = np.asarray(img)
    squeeze = a.ndim == 2
    if squeeze:
        a = a[:, :, None]
    H, W, C = a.shape
    xo, xc, xlim = linear_area_table(W, width)
    yo, yc, _ = linear_area_table(H, height, columns=False)
    S = a.astype(np.int64)
    x1 = np.minimum(xo + 1, W - 1)
    D = S[:, xo, :] * xc[None, :, 0, None] + S[:, x1, :] * xc[None, :, 1, None]
    D[:, xlim:, :] = S[:, xo[xlim:], :] * INTER_RESIZE_COEF_SCALE
    y1 = np.minimum(yo + 1, H - 1)
    D0, D1 = D[yo], D[y1]
    b0, b1 = yc[:, 0, None, None], yc[:, 1, None, None]
    r = (((b0 * (D0 >> 4)) >> 16) + ((b1 * (D1 >> 4)) >> 16) + 2) >> 2
    r = (r & 0xFF).astype(np.uint8)   # uchar(...) cast, no saturation (as OpenCV)
    return r[:, :, 0] if squeeze else r


def _slots(ptr, src, w):
    """Regroup a CSR table by position-within-run: slot t = the t-th entry of every
    destination that has one (so a vectorised pass adds in the table's order)."""
    n = len(ptr) - 1
    cnt = np.diff(ptr)
    out = []
    for t in range(int(cnt.max())):
        d = np.nonzero(cnt > t)[0]
        e = ptr[d] + t
        out.append((d, src[e], w[e]))
    return out


def resize_area_u8(img: np.ndarray, size: int) -> np.ndarray:
    """cv2.resize(img, (size, size), interpolation=INTER_AREA) for uint8 HxW or
    HxWxC input, host side.  Both axes downscaling (OpenCV's area path): float32 in
    OpenCV's operation order -- per destination row, each source row of its cell
    reduced horizontally (buf = 0 + a0*S0 + a1*S1 ...), then sum = b0*buf0 + b1*buf1
    ..., rounded half to even and clamped to uint8.  Otherwise (an img_size above the
    source size): resize_linear_area_u8."""
    a = np.asarray(img)
    if a.shape[0] < size or a.shape[1] < size:
        return resize_linear_area_u8(a, size, size)
    squeeze = a.ndim == 2
    if squeeze:
        a = a[:, :, None]
    H, W, C = a.shape
    yt = _slots(*area_table(H, size))
    xt = _slots(*area_table(W, size))
    S = a.astype(np.float32)
    # horizontal pass for every source row: (H, size, C)
    buf = np.zeros((H, size, C), np.float32)
    for d, s, wt in xt:
        buf[:, d, :] = buf[:, d, :] + S[:, s, :] * wt[None, :, None]
    out = np.zeros((size, size, C), np.float32)
    for t, (d, s, wt) in enumerate(yt):
        term = buf[s, :, :] * wt[:, None, None]
        out[d] = term if t == 0 else out[d] + term
    r = np.clip(np.rint(out), 0, 255).astype(np.uint8)
    return r[:, :, 0] if squeeze else r


# ----------------------------------------------------------------------------
# decoding (cv2.imread semantics through PIL) and the reference loaders
# ----------------------------------------------------------------------------

def imread_gray(path) -> np.ndarray:
    """cv2.imread(path, IMREAD_GRAYSCALE) -> HxW uint8 (ir:812, 1134).  16-bit
    sources keep their high byte (libpng strip-16, as OpenCV's PNG decoder
    without IMREAD_ANYDEPTH).  JPEG: OpenCV asks libjpeg for JCS_GRAYSCALE, i.e. the
    decoded Y plane itself -- PIL's draft('L') mode does the same (no YCbCr -> RGB ->
    gray round trip).  Other colour sources (PNG / BMP / TIFF): cvtColor's BGR2GRAY
    fixed-point weights (4899, 9617, 1868) / 2^14 with rounding."""
    from PIL import Image
    with Image.open(path) as im:
        if im.mode in ("I;16", "I;16B", "I;16L", "I"):   # 16-bit source
            return (np.asarray(im).astype(np.uint32) >> 8).astype(np.uint8)
        if im.format == "JPEG" and im.mode != "L":
            im.draft("L", im.size)                        # libjpeg's grayscale output (Y)
        if im.mode == "L":
            return np.asarray(im).copy()
        rgb = np.asarray(im.convert("RGB")).astype(np.uint32)
    g = (rgb[..., 0] * 4899 + rgb[..., 1] * 9617 + rgb[..., 2] * 1868 + (1 << 13)) >> 14
    return g.astype(np.uint8)


def imread_rgb(path) -> np.ndarray:
    """cv2.imread(path, IMREAD_COLOR) + cvtColor(BGR2RGB) -> HxWx3 uint8 (ir:842-845)."""
    from PIL import Image
    with Image.open(path) as im:
        if im.mode in ("I;16", "I;16B", "I;16L", "I"):
            g = (np.asarray(im).astype(np.uint32) >> 8).astype(np.uint8)
            return np.repeat(g[:, :, None], 3, axis=2)
        return np.asarray(im.convert("RGB")).copy()


def _unit_ir(img_u8: np.ndarray) -> np.ndarray:
    img = img_u8.astype(np.float32)
    if img.max() > 1.0:          # ir:823-827 (imread GRAYSCALE always yields uint8)
        img /= 255.0
    return np.clip(img, 0.0, 1.0)


def load_ir_image(path, img_size=None):
    """ir:803-830: HxW float32 in [0, 1], optionally INTER_AREA-resized."""
    img = imread_gray(path)
    if img_size is not None:
        img = resize_area_u8(img, img_size)
    return _unit_ir(img)


def load_rgb_image(path, img_size=None):
    """ir:833-852: HxWx3 float32 RGB in [0, 1], optionally INTER_AREA-resized."""
    img = imread_rgb(path)
    if img_size is not None:
        img = resize_area_u8(img, img_size)
    return np.clip(img.astype(np.float32) / 255.0, 0.0, 1.0)


def _list_imgs(folder):
    if not os.path.isdir(folder):
        return {}
    return {fn: os.path.join(folder, fn) for fn in os.listdir(folder) if fn.lower().endswith(EXTS)}


def collect_kaist_ir_files_from_sets(set_roots):
    """ir:887-942: [(ir_path, set_name, seq_rel)] for every image of every 'lwir'
    folder that has a sibling 'visible' folder (os.walk order, files sorted)."""
    if isinstance(set_roots, (str, bytes)):
        set_roots = [set_roots]
    entries = []
    for root in set_roots:
        if not os.path.isdir(root):
            print(f"[WARN] set root not found: {root}")
            continue
        set_name = os.path.basename(root.rstrip("\\/"))
        for dirpath, _, _ in os.walk(root):
            if os.path.basename(dirpath).lower() != "lwir":
                continue
            seq_dir = os.path.dirname(dirpath)
            if not os.path.isdir(os.path.join(seq_dir, "visible")):
                continue
            files = sorted(_list_imgs(dirpath).values())
            seq_rel = os.path.relpath(seq_dir, root)
            entries += [(p, set_name, seq_rel) for p in files]
    return entries


def scan_kaist_pairs(roots):
    """KAISTPairDataset's pairing (ir:1067-1117): per 'lwir' folder with a sibling
    'visible' folder, the sorted filename intersection; roots in order."""
    roots = list(roots) if isinstance(roots, (list, tuple)) else [roots]
    ir_paths, rgb_paths = [], []
    for one in roots:
        if not os.path.isdir(one):
            continue
        for dirpath, _, _ in os.walk(one):
            if os.path.basename(dirpath).lower() != "lwir":
                continue
            vis = os.path.join(os.path.dirname(dirpath), "visible")
            if not os.path.isdir(vis):
                continue
            irm, rgbm = _list_imgs(dirpath), _list_imgs(vis)
            for fn in sorted(set(irm) & set(rgbm)):
                ir_paths.append(irm[fn])
                rgb_paths.append(rgbm[fn])
    if not ir_paths:
        raise RuntimeError(f"No IR-RGB pairs found under roots: {roots}")
    return ir_paths, rgb_paths


class KAISTPairDataset(torch.utils.data.Dataset):
    """ir:1045-1177 with the reference's signature and item contract; see the
    module docstring for the device path (``raw`` + ``kaist_loader``)."""

    def __init__(self, root, img_size=256, augment=True, indices=None, verbose=True):
        super().__init__()
        self.img_size, self.augment = img_size, augment
        all_ir, all_rgb = scan_kaist_pairs(root)
        if indices is not None:
            self.ir_paths = [all_ir[i] for i in indices]
            self.rgb_paths = [all_rgb[i] for i in indices]
        else:
            self.ir_paths, self.rgb_paths = all_ir, all_rgb
        if verbose:
            print(f"[KAISTPairDataset] total pairs: {len(self.ir_paths)} (augment={self.augment})")

    def __len__(self):
        return len(self.ir_paths)

    def _flip(self):
        return bool(self.augment and random.random() < 0.5)   # ir:1166, python RNG in the worker

    def __getitem__(self, idx):
        ir = _unit_ir(resize_area_u8(imread_gray(self.ir_paths[idx]), self.img_size))
        rgb = np.clip(resize_area_u8(imread_rgb(self.rgb_paths[idx]), self.img_size).astype(np.float32) / 255.0,
                      0.0, 1.0)
        if self._flip():
            ir = np.fliplr(ir).copy()
            rgb = np.fliplr(rgb).copy()
        ir_t = torch.from_numpy(ir).unsqueeze(0)
        rgb_t = torch.from_numpy(np.transpose(rgb, (2, 0, 1)).copy())
        return {"ir": ir_t * 2.0 - 1.0, "rgb": rgb_t * 2.0 - 1.0}

    def raw(self, idx):
        """Decoded full-resolution uint8 images and the flip draw: the host half of
        the device path (resize / flip / normalisation run in csrc/data.hip)."""
        return {"ir_u8": torch.from_numpy(imread_gray(self.ir_paths[idx])),
                "rgb_u8": torch.from_numpy(imread_rgb(self.rgb_paths[idx])),
                "flip": int(self._flip())}


class _RawView(torch.utils.data.Dataset):
    def __init__(self, ds):
        self.ds = ds

    def __len__(self):
        return len(self.ds)

    def __getitem__(self, i):
        if isinstance(self.ds, torch.utils.data.Subset):
            return self.ds.dataset.raw(self.ds.indices[i])
        return self.ds.raw(i)


def collate_raw(items):
    """Stack decoded items into uint8 batches (pinned by the DataLoader).  Each modality
    needs one source size within the batch (one resize launch per modality); the IR and
    RGB sources may differ (the reference resizes each image on its own, ir:1139, 1156)."""
    for key in ("ir_u8", "rgb_u8"):
        shapes = {tuple(it[key].shape[:2]) for it in items}
        if len(shapes) != 1:
            raise RuntimeError(f"a device batch needs one {key[:-3]} source size, got {sorted(shapes)}")
    return {"ir_u8": torch.stack([it["ir_u8"] for it in items]),
            "rgb_u8": torch.stack([it["rgb_u8"] for it in items]),
            "flip": torch.tensor([it["flip"] for it in items], dtype=torch.uint8)}


class DeviceResizer:
    """uint8 decoded batch -> {'ir': (B,1,S,S), 'rgb': (B,3,S,S)} float32 [-1, 1] on
    the device: per modality one area-resize+flip launch and one normalisation
    launch (the IR max rule of ir:1142 included).  Tables cached per size."""

    def __init__(self, img_size, device):
        self.size, self.device = img_size, torch.device(device)
        self._tabs = {}

    def _tab(self, n):
        t = self._tabs.get(n)
        if t is None:
            t = self._tabs[n] = tuple(torch.from_numpy(a).to(self.device) for a in area_table(n, self.size))
        return t

    def _ltab(self, n, columns):
        key = ("lin", n, columns)
        t = self._tabs.get(key)
        if t is None:
            ofs, coef, lim = linear_area_table(n, self.size, columns)
            t = self._tabs[key] = (torch.from_numpy(ofs).to(self.device), torch.from_numpy(coef).to(self.device), lim)
        return t

    def resize_u8(self, u8, C, flip=None, img_max=None):
        """(B,H,W[,C]) uint8 device batch -> (B,C,S,S) uint8 (cv2.resize INTER_AREA,
        optional per-image horizontal flip)."""
        if u8.dtype != torch.uint8 or not u8.is_cuda:
            raise ValueError("resize_u8 takes a uint8 device tensor")
        u8 = u8.contiguous()
        B, H, W = u8.shape[:3]
        S = self.size
        out8 = torch.empty(B, C, S, S, dtype=torch.uint8, device=self.device)
        if H < S or W < S:   # an upscaling axis: OpenCV's linear path with area coefficients
            yo, yc, _ = self._ltab(H, False)
            xo, xc, xlim = self._ltab(W, True)
            _lib.call("irgan_linear_area_resize_u8", P(u8), B, H, W, C, ctypes.c_int64(H * W * C), P(yo), P(yc), S,
                      P(xo), P(xc), xlim, S, P(flip) if flip is not None else None, P(out8),
                      P(img_max) if img_max is not None else None, stream())
            return out8
        yp, ys, yw = self._tab(H)
        xp, xs, xw = self._tab(W)
        _lib.call("irgan_area_resize_u8", P(u8), B, H, W, C, ctypes.c_int64(H * W * C), P(yp), P(ys), P(yw), S,
                  P(xp), P(xs), P(xw), S, P(flip) if flip is not None else None, P(out8),
                  P(img_max) if img_max is not None else None, stream())
        return out8

    def _one(self, u8, C, flip, max_rule, keep_u8=False):
        """(B,C,S,S) float32 [-1, 1]; keep_u8: also the resized uint8 batch (what the
        reference's loaders hold before their float conversion)."""
        B, S = u8.shape[0], self.size
        mx = torch.zeros(B, dtype=torch.int32, device=self.device)
        out8 = self.resize_u8(u8, C, flip, mx)
        out = torch.empty(B, C, S, S, dtype=torch.float32, device=self.device)
        _lib.call("irgan_u8_to_unit", P(out8), B, ctypes.c_int64(C * S * S), P(mx), int(max_rule), P(out), stream())
        return (out, out8) if keep_u8 else out

    def __call__(self, batch):
        ir8 = batch["ir_u8"].to(self.device, non_blocking=True).contiguous()
        rgb8 = batch["rgb_u8"].to(self.device, non_blocking=True).contiguous()
        flip = batch["flip"].to(self.device, non_blocking=True)
        return {"ir": self._one(ir8, 1, flip, True), "rgb": self._one(rgb8, 3, flip, False)}


class _DeviceLoader:
    def __init__(self, loader, fn):
        self.loader, self.fn = loader, fn

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        for b in self.loader:
            yield self.fn(b)


def kaist_loader(dataset: KAISTPairDataset, batch_size, device, shuffle=False, drop_last=False, num_workers=0,
                 sampler=None):
    """DataLoader over ``dataset.raw`` (workers decode only) whose batches are
    resized / flipped / normalised on ``device`` (DeviceResizer)."""
    base = dataset.dataset if isinstance(dataset, torch.utils.data.Subset) else dataset
    dl = torch.utils.data.DataLoader(_RawView(dataset), batch_size=batch_size, shuffle=shuffle and sampler is None,
                                     sampler=sampler, num_workers=num_workers, collate_fn=collate_raw,
                                     pin_memory=torch.device(device).type == "cuda", drop_last=drop_last)
    return _DeviceLoader(dl, DeviceResizer(base.img_size, device))
