"""PatchGAN head kernels (csrc/head.hip: NLayerDiscriminator's last layer, Conv2d(512, 1, 4,
stride 1, padding 1), ir:625-627) against an fp64 torch reference on the same bf16 operands,
at the D step's shapes (B = 32 [real; fake], B = 16 GAN term, 31 x 31) and the 512 x 640
config's (62 x 78 patch map), plus odd sizes; and the same layer on the generic conv kernels
(IRGAN_NO_PATCH_HEAD's path) agrees with the dedicated one.  Forward, backward-data and the
weight gradient (irgan_patch_head_wgrad, accumulated into dw, deterministic)."""
import pytest
import torch
import torch.nn.functional as F

from conftest import pkg

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _layer(ops, seed):
    g = torch.Generator().manual_seed(seed)
    spec = ops.ConvSpec(512, 1, 4, 1, 1, ops.PAD_ZERO)
    w = (torch.randn(16 * 512, generator=g) * 0.02).bfloat16().float().to(DEV)   # KRSC [1][4][4][512]
    bias = torch.tensor([0.37], device=DEV)
    pc = ops.PackedConv(spec, w, bias, ops.BF16)
    pc.pack()
    return pc, w.view(1, 4, 4, 512).permute(0, 3, 1, 2).double().cpu()   # OIHW


@pytest.mark.parametrize("N,H,W", [(32, 32, 32), (16, 32, 32), (4, 63, 79), (3, 5, 37), (2, 2, 2)])
def test_patch_head_fwd_dgrad_vs_fp64(N, H, W):
    ops = pkg().ops
    pc, wo = _layer(ops, N + H)
    g = torch.Generator().manual_seed(H * W)
    x = torch.randn(N, H, W, 512, generator=g).bfloat16().to(DEV)
    y = torch.empty(N, H - 1, W - 1, 1, device=DEV)
    assert ops.patch_head_fwd(pc, ops.Feat(x), y)
    dy = torch.randn(N, H - 1, W - 1, 1, generator=g).to(DEV)
    dx = torch.full((N, H, W, 512), 9.0, device=DEV, dtype=torch.bfloat16)
    assert ops.patch_head_dgrad(pc, dy, ops.Feat(dx))
    torch.cuda.synchronize()
    xd = x.double().cpu().permute(0, 3, 1, 2)
    ref = F.conv2d(xd, wo, padding=1) + 0.37
    mag = F.conv2d(xd.abs(), wo.abs(), padding=1)
    err = (y.double().cpu().permute(0, 3, 1, 2) - ref).abs()
    assert (err <= 1e-5 * mag + 1e-6).all(), (err / (mag + 1e-9)).max().item()
    gd = dy.double().cpu().permute(0, 3, 1, 2)
    rdx = torch.nn.grad.conv2d_input(xd.shape, wo, gd, padding=1)
    mdx = torch.nn.grad.conv2d_input(xd.shape, wo.abs(), gd.abs(), padding=1)
    edx = (dx.double().cpu().permute(0, 3, 1, 2) - rdx).abs()
    # bf16 output rounding + the two-part (hi + lo bf16) dL/dy: 2^-16 of each |w| |dy| term
    assert (edx <= 2 ** -8 * rdx.abs() + 2 ** -15 * mdx + 1e-30).all(), (edx - 2 ** -8 * rdx.abs()).max().item()


def test_patch_head_matches_generic_conv_path():
    """The dedicated kernels against the generic conv kernels they replace, on the D step's
    shape: same forward to fp32 summation noise, same backward-data to bf16 rounding (the
    generic path reads dL/dy rounded to bf16, the head kernel the fp32 value)."""
    ops = pkg().ops
    pc, _ = _layer(ops, 7)
    g = torch.Generator().manual_seed(3)
    x = ops.Feat(torch.randn(32, 32, 32, 512, generator=g).bfloat16().to(DEV))
    y1 = torch.empty(32, 31, 31, 1, device=DEV)
    assert ops.patch_head_fwd(pc, x, y1)
    y2 = torch.empty(32, 31, 31, 1, device=DEV)
    ops.conv_fwd(pc, x, ops.Feat(y2))
    torch.cuda.synchronize()
    assert torch.allclose(y1, y2, rtol=1e-4, atol=1e-4), (y1 - y2).abs().max().item()
    dy = torch.randn(32, 31, 31, 1, generator=g).to(DEV)
    dx1 = ops.Feat(torch.empty(32, 32, 32, 512, device=DEV, dtype=torch.bfloat16))
    assert ops.patch_head_dgrad(pc, dy, dx1)
    dyb = torch.zeros(32, 31, 31, 8, device=DEV, dtype=torch.bfloat16)
    dyb[..., 0] = dy[..., 0].bfloat16()
    dx2 = ops.Feat(torch.empty(32, 32, 32, 512, device=DEV, dtype=torch.bfloat16))
    ops.conv_dgrad(pc, ops.Feat(dyb, 0, pc.cout_eff), dx2)
    torch.cuda.synchronize()
    # bound: the generic path's bf16 dL/dy (2^-9 relative per term) plus both outputs' bf16
    # rounding, scaled by sum |w| |dy| of each element
    wo = pc.master.view(1, 4, 4, 512).permute(0, 3, 1, 2).float()
    mag = torch.nn.grad.conv2d_input((32, 512, 32, 32), wo.abs(), dy.abs().permute(0, 3, 1, 2), padding=1)
    d = (dx1.t.float() - dx2.t.float()).abs().permute(0, 3, 1, 2)
    bound = 2 ** -7 * mag + 2 ** -8 * dx2.t.float().abs().permute(0, 3, 1, 2) + 1e-5
    assert (d <= bound).all(), (d - bound).max().item()


@pytest.mark.parametrize("N,H,W", [(32, 32, 32), (16, 32, 32), (4, 63, 79), (3, 5, 37), (2, 2, 2), (1, 40, 9)])
def test_patch_head_wgrad_vs_fp64(N, H, W):
    """dw += sum x * dL/dy over every pixel (fp32 g, not rounded), accumulated onto dw's
    previous contents; two runs are bit-identical (block partials, ordered reduce)."""
    ops = pkg().ops
    pc, _ = _layer(ops, N * H)
    g = torch.Generator().manual_seed(W)
    x = ops.Feat(torch.randn(N, H, W, 512, generator=g).bfloat16().to(DEV))
    dy = torch.randn(N, H - 1, W - 1, 1, generator=g).to(DEV)
    base = torch.randn(16 * 512, generator=g).to(DEV)
    dw = base.clone()
    assert ops.patch_head_wgrad(pc, x, dy, dw)
    dw2 = base.clone()
    assert ops.patch_head_wgrad(pc, x, dy, dw2)
    torch.cuda.synchronize()
    assert torch.equal(dw, dw2)
    xd = x.t.double().cpu().permute(0, 3, 1, 2)
    gd = dy.double().cpu().permute(0, 3, 1, 2)
    ref = torch.nn.grad.conv2d_weight(xd, (1, 512, 4, 4), gd, padding=1)          # [1][512][4][4]
    mag = torch.nn.grad.conv2d_weight(xd.abs(), (1, 512, 4, 4), gd.abs(), padding=1)
    ref = ref[0].permute(1, 2, 0).reshape(-1) + base.double().cpu()                # [ky][kx][c]
    mag = mag[0].permute(1, 2, 0).reshape(-1) + base.double().cpu().abs()
    err = (dw.double().cpu() - ref).abs()
    assert (err <= 2e-5 * mag + 1e-6).all(), (err / (mag + 1e-9)).max().item()


def test_patch_head_wgrad_matches_generic_conv_path():
    """Against the generic weight-gradient kernel it replaces (irgan_conv_wgrad_ws on the
    bf16-rounded dL/dy): equal to that rounding, 2^-8 of sum |x| |dy| per element."""
    ops = pkg().ops
    pc, _ = _layer(ops, 11)
    g = torch.Generator().manual_seed(5)
    x = ops.Feat(torch.randn(32, 32, 32, 512, generator=g).bfloat16().to(DEV))
    dy = torch.randn(32, 31, 31, 1, generator=g).to(DEV)
    dw1 = torch.zeros(16 * 512, device=DEV)
    assert ops.patch_head_wgrad(pc, x, dy, dw1)
    dyb = torch.zeros(32, 31, 31, 8, device=DEV, dtype=torch.bfloat16)
    dyb[..., 0] = dy[..., 0].bfloat16()
    dw2 = torch.zeros(16 * 512, device=DEV)
    ops.conv_wgrad(pc.spec, x, ops.Feat(dyb, 0, 1), dw2, ops.BF16)
    torch.cuda.synchronize()
    mag = torch.nn.grad.conv2d_weight(x.t.float().abs().permute(0, 3, 1, 2), (1, 512, 4, 4),
                                      dy.abs().permute(0, 3, 1, 2), padding=1)[0].permute(1, 2, 0).reshape(-1)
    d = (dw1 - dw2).abs()
    assert (d <= 2 ** -8 * mag + 1e-5).all(), (d - 2 ** -8 * mag).max().item()
