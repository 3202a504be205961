"""ResnetBlock backward-data that also writes the InstanceNorm backward partials of its output
(irgan_conv_dgrad_reflect_line_inred + irgan_in_bwd_finalize; ir:386-411 conv -> IN [-> ReLU]).

The fused launch must write the same dx, bit for bit, as irgan_conv_dgrad_reflect_line; and the
{mean g, mean g*xhat} it leads to must match the separate reduce pass (irgan_in_bwd_reduce over
(dx, z)) and an fp64 reference over the same bf16 dx / z to fp32 summation error (the two
paths add the same terms in different orders: not bit-identical).  Then the whole step: the
generator gradients with the fusion on and off agree to bf16 noise."""
import pytest
import torch

from conftest import pkg

pytestmark = pytest.mark.gpu
DEV = "cuda"


# the line-ring launch takes BN-256 tiles, i.e. >= 160 16x16 patches in one round (narrow_bn)
@pytest.mark.parametrize("N,H,W,acc,act", [(10, 64, 64, False, "relu"), (16, 64, 64, True, "none"),
                                           (14, 37, 64, True, "relu"), (27, 20, 36, False, "lrelu"),
                                           (160, 16, 16, False, "none")])
def test_dgrad_inred_matches_reduce_pass(N, H, W, acc, act):
    ops = pkg().ops
    A = {"none": ops.ACT_NONE, "relu": ops.ACT_RELU, "lrelu": ops.ACT_LRELU}[act]
    torch.manual_seed(11)
    C = 256
    spec = ops.ConvSpec(C, C, 3, 1, 1, ops.PAD_REFLECT)
    w = (torch.randn(C * 9 * C) * (1.0 / (9 * C) ** 0.5)).bfloat16().float().to(DEV)
    pc = ops.PackedConv(spec, w, torch.zeros(C, device=DEV), ops.BF16)
    pc.pack()
    dy = ops.Feat(torch.randn(N, H, W, C, device=DEV).bfloat16())
    old = torch.randn(N, H, W, C, device=DEV).bfloat16()
    z = ops.Feat((torch.randn(N, H, W, C, device=DEV) * 1.7 + 0.3).bfloat16())
    pad = torch.empty(N * (H + 2) * (W + 2) * C, device=DEV)
    work = torch.empty(ops.IN_PARTS * N * C, dtype=torch.float64, device=DEV)
    mr = torch.empty(2 * N * C, device=DEV)
    ops.in_stats(z, work, mr)

    def dx0():
        return ops.Feat(old.clone() if acc else torch.full((N, H, W, C), 7.0, device=DEV, dtype=torch.bfloat16))

    plain = dx0()
    assert not ops.conv_dgrad(pc, dy, plain, accumulate=acc, pad_buf=pad)
    fused = dx0()
    nb = ops.conv_dgrad(pc, dy, fused, accumulate=acc, pad_buf=pad, inred=(z, mr, A, work))
    assert nb == -(-H // 16) * -(-W // 16)
    red_f = torch.empty(2 * N * C, device=DEV)
    ops._lib.call("irgan_in_bwd_finalize", ops.P(work), N, H * W, C, nb, ops.P(red_f), ops.stream())
    torch.cuda.synchronize()
    assert torch.equal(fused.t, plain.t)

    red_r = torch.empty(2 * N * C, device=DEV)
    reduce, _ = ops.in_bwd_parts(plain, z, A, mr, work, red_r, plain)
    reduce()
    torch.cuda.synchronize()

    # fp64 reference over the same bf16 values (xhat from the fp32 {mean, rstd})
    m = mr.view(N, 1, C, 2).double().cpu()
    xh = ((z.t.double().cpu().view(N, H * W, C) - m[..., 0]) * m[..., 1])
    g = fused.t.double().cpu().view(N, H * W, C)
    if act == "relu":
        g = torch.where(xh > 0, g, torch.zeros_like(g))
    elif act == "lrelu":
        g = torch.where(xh > 0, g, 0.2 * g)
    ref = torch.stack([g.mean(1), (g * xh).mean(1)], -1)                     # [N][C][2]
    scale = torch.stack([g.abs().mean(1), (g * xh).abs().mean(1)], -1)
    for name, red in (("fused", red_f), ("reduce pass", red_r)):
        err = (red.view(N, C, 2).double().cpu() - ref).abs()
        ratio = (err / (1e-5 * scale + 1e-9)).max().item()
        assert ratio <= 1.0, (name, ratio)


def test_step_grads_with_and_without_dgrad_inred():
    """One bf16 train step at 256x256, B = 16 (the bench shape: the ResnetBlock backward-data
    takes the fused launch there) from the same weights, fusion on vs off: the generator's
    gradients agree to bf16 noise (rel-L2 < 2e-2 per tensor; the two reduce orders move
    {mean g, mean g*xhat} by fp32 rounding, which flips bf16 roundings downstream)."""
    irc = pkg()
    ops = irc.ops
    from oracle import step as O

    def run(on):
        old = ops.IN_DGRAD_REDUCE[0]
        ops.IN_DGRAD_REDUCE[0] = on
        try:
            cfg = irc.Config()
            cfg.device = DEV
            cfg.batch_size = 16
            cfg.img_size = 256
            tr = irc.GANTrainer(cfg)
            tr.netG.store.load(O.seeded_params(O.g_param_shapes(), 1), strict=True)
            tr.netD.store.load(O.seeded_params(O.d_param_shapes(), 2), strict=True)
            tr.vgg.store.load(O.seeded_params(O.vgg_param_shapes(), 3, kaiming=True), strict=True)
            for m in (tr.netG, tr.netD, tr.vgg):
                m.repack()
            g = torch.Generator().manual_seed(3)
            ir = (torch.rand(16, 1, 256, 256, generator=g) * 2 - 1).to(DEV)
            rgb = (torch.rand(16, 3, 256, 256, generator=g) * 2 - 1).to(DEV)
            tr.step(ir, rgb)
            torch.cuda.synchronize()
            st = tr.netG.store
            return {k: st.krsc(k, st.grad).float().clone() for k in st.shapes}
        finally:
            ops.IN_DGRAD_REDUCE[0] = old

    calls = []
    real = ops.in_backward
    ops.in_backward = lambda *a, **k: (calls.append(k.get("part_nb", 0)), real(*a, **k))[1]
    try:
        on = run(True)
        assert sum(1 for c in calls if c) == 17, calls   # 17 of the 18 ResnetBlock IN backwards
        calls.clear()
        off = run(False)
        assert not any(calls)
    finally:
        ops.in_backward = real
    worst = max(((on[k] - off[k]).norm() / off[k].norm().clamp_min(1e-30)).item() for k in off if off[k].norm() > 0)
    assert worst < 2e-2, worst
