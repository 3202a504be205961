"""PatchGAN head kernels alone, for rocprofv3 --kernel-trace --stats: fwd / dgrad / wgrad at the
D step's shapes (B = 32 and 16, 31 x 31 x 512 input), 20 launches each in one HIP graph,
replayed 3 times.  IRGAN_NO_PATCH_HEAD=1
runs the same layer on the generic conv kernels instead."""
import importlib
import sys

import torch

sys.path.insert(0, ".")
ops = importlib.import_module("infrared-colorization-with-resnet-generator-and-patchgan_amd").ops
DEV = "cuda"
spec = ops.ConvSpec(512, 1, 4, 1, 1, ops.PAD_ZERO)
w = (torch.randn(16 * 512) * 0.02).bfloat16().float().to(DEV)
pc = ops.PackedConv(spec, w, torch.tensor([0.1], device=DEV), ops.BF16)
pc.pack()
for N in (32, 16):
    x = ops.Feat(torch.randn(N, 31, 31, 512).bfloat16().to(DEV))
    y = torch.empty(N, 30, 30, 1, device=DEV)
    g = torch.randn(N, 30, 30, 1, device=DEV)
    gb = torch.zeros(N, 30, 30, 8, device=DEV, dtype=torch.bfloat16)
    gb[..., 0] = g[..., 0].bfloat16()
    dx = ops.Feat(torch.empty(N, 31, 31, 512, device=DEV, dtype=torch.bfloat16))
    dw = torch.zeros(16 * 512, device=DEV)
    def body():
        if not ops.patch_head_fwd(pc, x, y):
            ops.conv_fwd(pc, x, ops.Feat(y))
        if not ops.patch_head_dgrad(pc, g, dx):
            ops.conv_dgrad(pc, ops.Feat(gb, 0, pc.cout_eff), dx)
        if not ops.patch_head_wgrad(pc, x, g, dw):
            ops.conv_wgrad(spec, x, ops.Feat(gb, 0, 1), dw, ops.BF16)
    body()
    torch.cuda.synchronize()
    # back-to-back launches (one HIP graph), as inside the step: no host gaps between kernels
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        body()
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            for _ in range(20):
                body()
    for _ in range(3):
        graph.replay()
    torch.cuda.synchronize()
print("ok")
