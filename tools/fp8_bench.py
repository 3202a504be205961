"""Kernel timing: resblock conv (256 -> 256, 3x3 reflect, 64x64) forward+stats,
backward-data and weight gradient, bf16 vs fp8 operands, at the config-5 batch (32) and the bench batch."""
import importlib
import sys

import torch

sys.path.insert(0, ".")
irc = importlib.import_module("infrared-colorization-with-resnet-generator-and-patchgan_amd")
ops = irc.ops
DEV = "cuda"


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


for N in (16, 32):
    C, H = 256, 64
    spec = ops.ConvSpec(C, C, 3, 1, 1, 1)
    w = torch.randn(C * 9 * C, device=DEV) * 0.02
    pc = ops.PackedConv(spec, w, torch.zeros(C, device=DEV), ops.BF16)
    pc.pack()
    fw = ops.Fp8Weights([pc.fwd, pc.dg[0][2]], DEV)
    fw.run()
    x = torch.randn(N, H, H, C, device=DEV).bfloat16()
    x8 = torch.empty(N, H, H, C, device=DEV, dtype=torch.float8_e4m3fn)
    qt = torch.tensor([16.0], device=DEV)
    dq = torch.tensor([1 / 16.0], device=DEV)
    ops.fp8_quant(ops.Feat(x), ops.Feat(x8), ops.Pi(qt, 0))
    y = torch.empty(N, H, H, C, device=DEV, dtype=torch.bfloat16)
    work = torch.empty(ops.IN_PARTS * N * C, dtype=torch.float64, device=DEV)
    flop = 2.0 * N * H * H * C * C * 9
    t_bf = timeit(lambda: ops.conv_fwd_stats(pc, ops.Feat(x), ops.Feat(y), work))
    t_f8 = timeit(lambda: ops.conv_fwd_fp8(pc, fw.dst[0], ops.Pi(fw.dq, 0), ops.Feat(x8), ops.Pi(dq, 0),
                                           ops.Feat(y), part=work))
    t_q = timeit(lambda: ops.fp8_quant(ops.Feat(x), ops.Feat(x8), ops.Pi(qt, 0)))
    dx = torch.empty_like(y)
    t_dbf = timeit(lambda: ops.conv_dgrad(pc, ops.Feat(x), ops.Feat(dx)))
    t_df8 = timeit(lambda: ops.conv_dgrad_fp8(pc, fw.dst[1], ops.Pi(fw.dq, 1), ops.Feat(x8), ops.Pi(dq, 0),
                                              ops.Feat(x), ops.Feat(dx)))
    dw = torch.zeros(C * 9 * C, device=DEV)
    t_wbf = timeit(lambda: ops.conv_wgrad(spec, ops.Feat(x), ops.Feat(y), dw, ops.BF16))
    t_wf8 = timeit(lambda: ops.conv_wgrad_fp8(spec, ops.Feat(x8), ops.Feat(x8), ops.Pi(dq, 0), ops.Pi(dq, 0), dw))
    print(f"N={N}: fwd+stats bf16 {t_bf:.1f} us ({flop / t_bf / 1e6:.0f} TF/s)  fp8 {t_f8:.1f} us "
          f"({flop / t_f8 / 1e6:.0f} TF/s)  quant {t_q:.1f} us | dgrad bf16 {t_dbf:.1f} us  fp8 {t_df8:.1f} us | "
          f"wgrad bf16 {t_wbf:.1f} us ({flop / t_wbf / 1e6:.0f} TF/s)  fp8 {t_wf8:.1f} us ({flop / t_wf8 / 1e6:.0f} TF/s)",
          flush=True)
