"""The G inc layer's reflect-pad 7x7 conv (1 -> 64, ir:458-463) with the InstanceNorm statistics
fused into its epilogue (conv_c8r STATS through irgan_conv_fwd_stats): the conv output must be
bit-identical to the plain launch, and {mean, rstd} from its partials must match the separate
statistics pass (same bf16 values, different fp32 partial order) to fp32 summation error."""
import pytest
import torch

from conftest import pkg

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("N,H,W", [(16, 256, 256), (2, 64, 64), (3, 100, 76), (1, 20, 36)])
def test_inc_conv_fused_stats(N, H, W):
    ops = pkg().ops
    g = torch.Generator().manual_seed(N + H + W)
    spec = ops.ConvSpec(1, 64, 7, 1, 3, ops.PAD_REFLECT)
    w = (torch.randn(64 * 49, generator=g) * 0.1).to(DEV)
    pc = ops.PackedConv(spec, w, (torch.randn(64, generator=g) * 0.1).to(DEV), ops.BF16)
    pc.pack()
    x = torch.zeros(N, H, W, 8, device=DEV, dtype=torch.bfloat16)
    x[..., 0] = (torch.rand(N, H, W, generator=g) * 2 - 1).to(DEV).bfloat16()
    xf = ops.Feat(x, 0, pc.cin_eff)
    z1 = ops.Feat(torch.empty(N, H, W, 64, device=DEV, dtype=torch.bfloat16))
    z2 = ops.Feat(torch.empty(N, H, W, 64, device=DEV, dtype=torch.bfloat16))
    work = torch.empty(ops.IN_PARTS * N * 64, dtype=torch.float64, device=DEV)
    mr1 = torch.empty(2 * N * 64, device=DEV)
    mr2 = torch.empty(2 * N * 64, device=DEV)
    nb = ops.conv_fwd_stats(pc, xf, z1, work)
    assert nb == -(-H // 16) * -(-W // 16)
    ops.in_finalize(z1, work, nb, mr1)
    ops.conv_fwd(pc, xf, z2)
    ops.in_stats(z2, work, mr2)
    torch.cuda.synchronize()
    assert torch.equal(z1.t, z2.t)
    m1, m2 = mr1.view(-1, 2), mr2.view(-1, 2)
    zf = z2.t.float().view(N, -1, 64)
    scale = zf.abs().mean(1).view(-1)
    assert ((m1[:, 0] - m2[:, 0]).abs() <= 1e-5 * scale + 1e-7).all(), (m1[:, 0] - m2[:, 0]).abs().max().item()
    assert ((m1[:, 1] - m2[:, 1]).abs() <= 1e-4 * m2[:, 1].abs()).all(), ((m1[:, 1] - m2[:, 1]) / m2[:, 1]).abs().max()
