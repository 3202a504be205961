"""Where the reflect-ring launch's time goes: a RING_TS=1 build records per-block wall-clock
stamps (100 MHz) at kernel entry, after the tap list, after wave 0's K loop, after the
partial-tile reduction and after the dx read-modify-write.  Resblock dgrad shape, B=16.
usage: IRGAN_LIB=<libirgan built with -DRING_TS=1> python tools/ring_ts.py"""
import ctypes
import importlib
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
irc = importlib.import_module("infrared-colorization-with-resnet-generator-and-patchgan_amd")
ops, _lib = irc.ops, irc._lib
DEV = "cuda"
N, C, H = 16, 256, 64
spec = ops.ConvSpec(C, C, 3, 1, 1, 1)
pc = ops.PackedConv(spec, torch.randn(C * 9 * C, device=DEV) * 0.02, torch.zeros(C, device=DEV), ops.BF16)
pc.pack()
dy = torch.randn(N, H, H, C, device=DEV).bfloat16()
dx = torch.empty_like(dy)
for _ in range(5):
    ops.conv_dgrad(pc, ops.Feat(dy), ops.Feat(dx))
torch.cuda.synchronize()
import os
LINE = not os.environ.get("IRGAN_NO_RING_LINE")
nblk = 4 * (C // 64) * N if LINE else N * 2 * 2 * (C // 64)   # line GEMM: (line, tile) x image groups of 1
buf = (ctypes.c_ulonglong * (nblk * 6))()
lib = _lib.load()
assert lib.irgan_debug_ring_ts(buf, nblk) == 0
t = np.frombuffer(buf, dtype=np.uint64).reshape(nblk, 6).astype(np.int64)[:, :5]
t0 = t[:, 0].min()
us = (t - t0) / 100.0  # 100 MHz -> us
print(f"blocks {nblk}: span {us[:, 4].max():.2f} us (first start -> last end)")
print(f"start skew: median {np.median(us[:, 0]):.2f} max {us[:, 0].max():.2f} us")
for i, name in enumerate(["taplist/weights+line", "kloop(w0)/gemm", "reduce/store", "rmw/-"]):
    d = us[:, i + 1] - us[:, i]
    print(f"{name:10s} median {np.median(d):6.2f}  p90 {np.percentile(d, 90):6.2f}  max {d.max():6.2f} us")
print("end: median %.2f max %.2f us" % (np.median(us[:, 4]), us[:, 4].max()))
if LINE:
    sys.exit(0)
# row-segment vs column-segment blocks (blockIdx.x % 4 < 2: row bands, per image 2p*(segs_row+segs_col) = 4)
kind = (np.arange(nblk) % (N * 4)) % 4 < 2
for k, nm in ((True, "row seg"), (False, "col seg")):
    d = us[kind == k]
    print(f"{nm}: total median {np.median(d[:, 4] - d[:, 0]):.2f} us, kloop median {np.median(d[:, 2] - d[:, 1]):.2f}")
