"""ResnetBlock backward-data with the reflect ring folded into the interior launch's store
pass (irgan_conv_dgrad_reflect_line, ir:386-411's ReflectionPad2d + Conv2d backward).

The fused path must write exactly the dx of the two-step path it replaces -- the interior
launch, then the line-ring GEMM + fold launch (irgan_reflect_dgrad_ring_ws) -- bit for bit,
with and without accumulation into an existing gradient; and both must match the fp32 torch
reference of the padded conv's backward-data to the bf16 parity bound."""
import pytest
import torch
import torch.nn.functional as F

from conftest import pkg

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("N,H,W,acc", [(2, 64, 64, False), (2, 64, 64, True), (3, 16, 16, False), (1, 20, 36, True),
                                       (2, 4, 4, False), (1, 37, 64, False)])
def test_ring_epilogue_bit_identical(N, H, W, acc):
    ops = pkg().ops
    torch.manual_seed(5)
    C = 256
    spec = ops.ConvSpec(C, C, 3, 1, 1, ops.PAD_REFLECT)
    w = (torch.randn(C * 9 * C) * (1.0 / (9 * C) ** 0.5)).bfloat16().float().to(DEV)
    pc = ops.PackedConv(spec, w, torch.zeros(C, device=DEV), ops.BF16)
    pc.pack()
    dy = ops.Feat(torch.randn(N, H, W, C, device=DEV).bfloat16())
    old = torch.randn(N, H, W, C, device=DEV).bfloat16()
    pad = torch.empty(N * (H + 2) * (W + 2) * C, device=DEV)

    def run(epi):
        dx = ops.Feat(old.clone() if acc else torch.full((N, H, W, C), 7.0, device=DEV, dtype=torch.bfloat16))
        prev = ops.set_ring_epi(epi)
        try:
            ops.conv_dgrad(pc, dy, dx, accumulate=acc, pad_buf=pad)
        finally:
            ops.set_ring_epi(prev)
        torch.cuda.synchronize()
        return dx.t

    fused, split = run(True), run(False)
    assert torch.equal(fused, split), (fused.float() - split.float()).abs().max().item()

    # fp64 reference: d/dx of conv(reflect_pad(x)) against dy, on the same bf16 operands.
    # border pixels are rounded to bf16 twice (interior, then interior + ring): bound
    # 2^-8 (|ref| + |interior|) + 2e-5 sum|terms| (test_gpu_bf16_parity.py's check(partial=))
    # (on the CPU, as test_gpu_bf16_parity.py's references)
    wt = w.view(C, 3, 3, C).permute(0, 3, 1, 2).bfloat16().double().cpu()  # [co][ci][ky][kx]
    gy = dy.t.double().permute(0, 3, 1, 2).cpu()

    def bwd(wk, g, mode):
        x = torch.zeros(N, C, H, W, dtype=torch.float64, requires_grad=True)
        (r,) = torch.autograd.grad(F.conv2d(F.pad(x, (1, 1, 1, 1), mode=mode), wk), x, g)
        return r.permute(0, 2, 3, 1)

    base = old.double().cpu() if acc else 0.0
    ref = bwd(wt, gy, "reflect") + base
    ring = ref - base - bwd(wt, gy, "constant")
    mag = bwd(wt.abs(), gy.abs(), "reflect") + (old.double().cpu().abs() if acc else 0.0)
    err = (fused.double().cpu() - ref).abs()
    partial = torch.where(ring != 0, (ref - ring).abs(), torch.zeros_like(ref))  # the first rounding's value
    ratio = err / (2 ** -8 * (ref.abs() + partial) + 2e-5 * mag)
    i = int(ratio.argmax())
    where = [int(v) for v in torch.unravel_index(torch.tensor(i), ratio.shape)]
    assert ratio.max().item() <= 1.0, (where, ratio.max().item(), err.reshape(-1)[i].item(), ref.reshape(-1)[i].item(),
                                       ring.reshape(-1)[i].item(), fused.reshape(-1)[i].item())
