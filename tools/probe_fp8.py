"""Probe the fp8 MFMA operand lane maps and the fp8 conversion (one-off; see
tools/probe_fp8.hip).  Prints which lane-map hypothesis reproduces A @ B."""
import ctypes
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "probe_fp8.so"))
dev = "cuda"
rng = np.random.default_rng(0)
codes = np.array([0x00, 0x38, 0x40, 0xB8, 0xC0, 0x30], np.uint8)   # 0, 1, 2, -1, -2, 0.5
vals = {0x00: 0.0, 0x38: 1.0, 0x40: 2.0, 0xB8: -1.0, 0xC0: -2.0, 0x30: 0.5}
dec = np.vectorize(lambda c: vals[int(c)])
P = lambda t: ctypes.c_void_p(t.data_ptr())   # noqa: E731


def run(fn, a, b):
    ta, tb = torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev)
    d = torch.zeros(64, 4, device=dev)
    assert getattr(lib, fn)(P(ta), P(tb), P(d)) == 0
    return d.cpu().numpy()


def cd(d):
    """C/D map: col = lane & 15, row = 4*(lane>>4) + r  ->  [row][col]."""
    out = np.zeros((16, 16))
    for l in range(64):
        for r in range(4):
            out[4 * (l >> 4) + r, l & 15] = d[l, r]
    return out


def mats(a, b, K, kmap):
    A, B = np.zeros((16, K)), np.zeros((K, 16))
    for l in range(64):
        for j in range(a.shape[1]):
            k = kmap(l, j)
            A[l & 15, k] = dec(a[l, j])
            B[k, l & 15] = dec(b[l, j])
    return A, B


ok = True
for fn, nb, K, hyps in [
    ("probe_plain", 8, 32, {"k=8g+j": lambda l, j: 8 * (l >> 4) + j}),
    ("probe_scaled", 32, 128, {"k=32g+j": lambda l, j: 32 * (l >> 4) + j,
                               "k=16g+j | 64+16g+j-16": lambda l, j: 16 * (l >> 4) + j if j < 16 else 64 + 16 * (l >> 4) + j - 16}),
]:
    a = rng.choice(codes, size=(64, nb))
    b = rng.choice(codes, size=(64, nb))
    D = cd(run(fn, a, b))
    for name, km in hyps.items():
        A, B = mats(a, b, K, km)
        match = np.array_equal(A @ B, D)
        print(f"{fn}: hypothesis {name}: {'MATCH' if match else 'no'}")
# fp8 conversion vs torch's float8_e4m3fn (after clamping to +-448)
x = torch.cat([torch.randn(200000) * s for s in (1e-3, 0.1, 1.0, 30.0, 300.0)] +
              [torch.tensor([448.0, 449.0, 464.0, 1e6, -1e6, 0.0, -0.0, 2 ** -9, 2 ** -10, 3 * 2 ** -10])])
y = torch.empty(x.numel(), dtype=torch.uint8, device=dev)
xd = x.to(dev)
assert lib.probe_cvt(P(xd), P(y), x.numel()) == 0
want = x.clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
diff = (y.cpu() != want).sum().item()
print(f"cvt_pk_fp8_f32 vs torch float8_e4m3fn: {diff} of {x.numel()} codes differ")
if diff:
    idx = (y.cpu() != want).nonzero()[:10, 0]
    print([(float(x[i]), int(y[i]), int(want[i])) for i in idx])
sys.exit(0)
