"""InstanceNorm finalize + apply in one launch (irgan_in_finalize_apply, the resblock
forward after the conv's fused statistics, ir:386-418): mr and y must be bit-identical
to irgan_in_finalize followed by irgan_in_apply."""
import pytest
import torch

from conftest import pkg

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("H,act,res", [(64, 1, False), (64, 0, True), (37, 1, True), (16, 0, False)])
def test_finalize_apply_bit_identical(H, act, res):
    ops = pkg().ops
    torch.manual_seed(5)
    N, C = 2, 256
    spec = ops.ConvSpec(C, C, 3, 1, 1, ops.PAD_REFLECT)
    pc = ops.PackedConv(spec, (torch.randn(C * 9 * C) * 0.02).to(DEV), (torch.randn(C) * 0.1).to(DEV), ops.BF16)
    pc.pack()
    x = ops.Feat(torch.randn(N, H, H, C, device=DEV).bfloat16())
    z = ops.Feat(torch.empty(N, H, H, C, device=DEV, dtype=torch.bfloat16))
    work = torch.empty(ops.IN_PARTS * N * C, dtype=torch.float64, device=DEV)
    nb = ops.conv_fwd_stats(pc, x, z, work)
    assert nb > 0
    r = ops.Feat(torch.randn(N, H, H, C + 8, device=DEV).bfloat16(), 8, C) if res else None
    mr0 = torch.empty(N * C * 2, device=DEV)
    y0 = ops.Feat(torch.empty(N, H, H, C, device=DEV, dtype=torch.bfloat16))
    ops.in_finalize(z, work, nb, mr0)
    ops.in_apply(z, mr0, y0, act=act, res=r)
    mr1 = torch.full_like(mr0, float("nan"))
    y1 = ops.Feat(torch.zeros(N, H, H, C + 8, device=DEV, dtype=torch.bfloat16), 8, C)
    assert ops.in_finalize_apply(z, work, nb, mr1, y1, act=act, res=r)
    torch.cuda.synchronize()
    assert torch.equal(mr1, mr0)
    assert torch.equal(y1.t[..., 8:], y0.t)
    assert not y1.t[..., :8].any()
