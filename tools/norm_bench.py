"""HBM bandwidth of the InstanceNorm elementwise passes at the resblock shape
(64x64x256 bf16 per image) -- the kernels the step runs between the convs."""
import importlib
import sys

import torch

sys.path.insert(0, ".")
irc = importlib.import_module("infrared-colorization-with-resnet-generator-and-patchgan_amd")
ops = irc.ops
DEV = "cuda"
Feat = ops.Feat


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


import os
SHAPES = [tuple(int(v) for v in s.split("x")) for s in os.environ.get("NORM_SHAPES", "64x256").split(",")]
for (H, C) in SHAPES:
  for N in (16, 32) if (H, C) == (64, 256) else (16,):
      E = N * H * H * C
      mk = lambda: torch.randn(N, H, H, C, device=DEV).bfloat16()   # noqa: E731
      z, res, y, dy, dx = mk(), mk(), mk(), mk(), mk()
      mr = torch.rand(N * C * 2, device=DEV) + 0.5
      work = torch.empty(ops.IN_PARTS * N * C, dtype=torch.float64, device=DEV)
      red = torch.empty(2 * N * C, device=DEV)
      x8 = torch.empty(N, H, H, C, device=DEV, dtype=torch.float8_e4m3fn)
      qt = torch.tensor([16.0], device=DEV)
      amax = torch.zeros(1, dtype=torch.int32, device=DEV)
      rows = []
      t = timeit(lambda: ops.in_apply(Feat(z), mr, Feat(y), act=ops.ACT_RELU)); rows.append(("apply relu", t, 4 * E))
      t = timeit(lambda: ops.in_apply(Feat(z), mr, Feat(y), res=Feat(res))); rows.append(("apply +res", t, 6 * E))
      t = timeit(lambda: ops.in_stats(Feat(z), work, mr.clone())); rows.append(("stats", t, 2 * E))
      red_fn, app_fn = ops.in_bwd_parts(Feat(dy), Feat(z), ops.ACT_RELU, mr, work, red, Feat(dx))
      t = timeit(red_fn); rows.append(("bwd reduce", t, 4 * E))
      t = timeit(app_fn); rows.append(("bwd apply", t, 6 * E))
      t = timeit(lambda: ops.fp8_quant(Feat(z), Feat(x8), ops.Pi(qt, 0), ops.Pi(amax, 0))); rows.append(("fp8 quant+amax", t, 3 * E))
      t = timeit(lambda: ops.fp8_quant(Feat(z), Feat(x8), ops.Pi(qt, 0), None)); rows.append(("fp8 quant", t, 3 * E))
      t = timeit(lambda: y.copy_(z)); rows.append(("torch copy", t, 4 * E))
      for name, t, by in rows:
          print(f"{H}x{C} N={N} {name:16s} {t:7.1f} us  {by / t / 1e3:6.0f} GB/s", flush=True)
