"""Per-kernel numerics on the MI355X: every HIP kernel vs a plain PyTorch fp32
CPU reference of the same op (fp32 mode: ~1e-5 rel; bf16 mode: bf16-level
tolerance stated per test).  Calls go through the C ABI (libirgan.so)."""
import pytest
import torch
import torch.nn.functional as F

from conftest import pkg

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module")
def ops():
    m = pkg()
    return m.ops


def nhwc(x):  # NCHW cpu -> NHWC device
    return x.permute(0, 2, 3, 1).contiguous().to(DEV)


def nchw(x):
    return x.float().cpu().permute(0, 3, 1, 2).contiguous()


def relerr(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-12))


def ref_conv(x, w, b, k, s, p, mode):
    if mode == 1:
        x = F.pad(x, (p, p, p, p), mode="reflect")
        p = 0
    return F.conv2d(x, w, b, stride=s, padding=p)


CONV_CASES = [
    # cin, cout, k, s, p, mode, H
    (64, 128, 3, 1, 1, 0, 16),
    (256, 256, 3, 1, 1, 1, 8),
    (1, 64, 7, 1, 3, 1, 16),
    (64, 3, 7, 1, 3, 1, 16),
    (4, 64, 4, 2, 1, 0, 32),
    (64, 128, 4, 2, 1, 0, 16),
    (256, 512, 4, 1, 1, 0, 6),
    (512, 1, 4, 1, 1, 0, 5),
    (3, 64, 3, 1, 1, 0, 16),
    (64, 128, 3, 2, 1, 0, 16),
    (192, 64, 3, 1, 1, 0, 8),
    # multi-patch / ragged-edge cases for the halo kernel (16x16 output patches)
    (64, 3, 7, 1, 3, 1, 37),      # narrow-Cout kernel: G outc shape, several patches, ragged edge
    (512, 1, 4, 1, 1, 0, 31),     # narrow-Cout kernel, 8 chunks double-buffered: D's last layer
    # 8-channel-input kernel (conv_c8.hip): 2 x 18 x 18 = 648 patches > the persistent grid
    # (2 blocks x 256 CUs), ragged last patch row/column; fwd = inc / VGG conv1_1, dgrad = outc
    (1, 64, 7, 1, 3, 1, 280),
    (3, 64, 3, 1, 1, 0, 280),
    (64, 3, 7, 1, 3, 1, 280),
    (4, 64, 4, 2, 1, 0, 530),     # stride-2 c8 (D's first layer): 2 x 17 x 17 patches, ragged
    (128, 256, 3, 1, 1, 1, 37),
    (64, 64, 3, 1, 1, 0, 40),
    (128, 128, 4, 2, 1, 0, 34),
    (256, 512, 4, 1, 1, 0, 20),
    # Wo % 64 == 0: the segment (row-span) wgrad kernel
    (256, 256, 3, 1, 1, 1, 64),
    (192, 64, 3, 1, 1, 0, 64),
    (64, 3, 7, 1, 3, 1, 64),
    (64, 128, 4, 2, 1, 0, 128),
    (64, 128, 3, 2, 1, 0, 128),
    (128, 64, 4, 1, 1, 0, 67),
]


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_dgrad_wgrad(ops, case, dtype):
    cin, cout, k, s, p, mode, H = case
    torch.manual_seed(0)
    N = 2
    x = torch.randn(N, cin, H, H)
    w = torch.randn(cout, cin, k, k) * (1.0 / (cin * k * k) ** 0.5)
    b = torch.randn(cout) * 0.1
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    y_ref = ref_conv(xr, wr, b, k, s, p, mode)
    gy = torch.randn_like(y_ref)
    y_ref.backward(gy)

    code = ops.F32 if dtype == "f32" else ops.BF16
    tdt = torch.float32 if dtype == "f32" else torch.bfloat16
    tol = 2e-5 if dtype == "f32" else 3e-2
    spec = ops.ConvSpec(cin, cout, k, s, p, mode)
    master = w.permute(0, 2, 3, 1).contiguous().reshape(-1).to(DEV)
    pc = ops.PackedConv(spec, master, b.to(DEV), code)
    pc.pack()
    # forward into a channel slice of a wider tensor (exercises ld/off); narrow bf16
    # inputs are stored zero-padded to pc.cin_eff channels
    xd = torch.zeros(N, H, H, pc.cin_eff, device=DEV, dtype=tdt)
    xd[..., :cin] = nhwc(x).to(tdt)
    Ho, Wo = y_ref.shape[2:]
    ybuf = torch.zeros(N, Ho, Wo, cout + 8, device=DEV, dtype=torch.float32)
    ops.conv_fwd(pc, ops.Feat(xd), ops.Feat(ybuf, 8, cout))
    assert relerr(nchw(ybuf[..., 8:]), y_ref.detach()) < tol
    # backward-data (dY zero-padded to pc.cout_eff channels)
    gyd = torch.zeros(N, Ho, Wo, pc.cout_eff, device=DEV, dtype=tdt)
    gyd[..., :cout] = nhwc(gy).to(tdt)
    dx = torch.zeros(N, H, H, cin, device=DEV, dtype=torch.float32)
    pad = torch.empty(N * (H + 2 * p) ** 2 * cin, device=DEV) if mode == 1 else None
    ops.conv_dgrad(pc, ops.Feat(gyd), ops.Feat(dx), pad_buf=pad)
    assert relerr(nchw(dx), xr.grad) < tol
    # backward-weight
    dw = torch.zeros(cout * k * k * cin, device=DEV)
    ops.conv_wgrad(spec, ops.Feat(xd), ops.Feat(gyd, 0, cout), dw, code)
    dw = dw.view(cout, k, k, cin).permute(0, 3, 1, 2).cpu()
    assert relerr(dw, wr.grad) < (2e-5 if dtype == "f32" else 3e-2)


def test_conv_act_and_mask(ops):
    torch.manual_seed(1)
    x = torch.randn(2, 64, 8, 8)
    w = torch.randn(64, 64, 3, 3) * 0.05
    b = torch.randn(64) * 0.1
    m = torch.randn(2, 64, 8, 8)
    spec = ops.ConvSpec(64, 64, 3, 1, 1, 0)
    pc = ops.PackedConv(spec, w.permute(0, 2, 3, 1).contiguous().reshape(-1).to(DEV), b.to(DEV), ops.F32)
    pc.pack()
    for act, fn in ((ops.ACT_RELU, F.relu), (ops.ACT_LRELU, lambda t: F.leaky_relu(t, 0.2)), (ops.ACT_TANH, torch.tanh)):
        y = torch.empty(2, 8, 8, 64, device=DEV)
        ops.conv_fwd(pc, ops.Feat(nhwc(x)), ops.Feat(y), act=act)
        assert relerr(nchw(y), fn(F.conv2d(x, w, b, padding=1))) < 2e-5
    y = torch.empty(2, 8, 8, 64, device=DEV)
    ops.conv_fwd(pc, ops.Feat(nhwc(x)), ops.Feat(y), mask=ops.Feat(nhwc(m)), mask_act=2)
    ref = F.conv2d(x, w, b, padding=1) * torch.where(m > 0, 1.0, 0.2)
    assert relerr(nchw(y), ref) < 2e-5


@pytest.mark.parametrize("P,C,ld", [(100003, 3, 8), (65536, 64, 64), (777, 256, 264)])
def test_channel_sum(ops, P, C, ld):
    torch.manual_seed(5)
    g = torch.randn(P, ld, device=DEV)
    db = torch.full((C,), 0.5, device=DEV)
    ops.channel_sum(ops.Feat(g.view(1, P, 1, ld), 0, C), db)
    ref = g[:, :C].double().sum(0) + 0.5
    assert torch.allclose(db.double(), ref, rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("shape", [(2, 96, 12), (1, 64, 96), (3, 256, 40)])
@pytest.mark.parametrize("act", [0, 1, 2])
def test_instance_norm_fwd_bwd(ops, act, shape):
    torch.manual_seed(2)
    N, C, H = shape
    x = (torch.randn(N, C, H, H) * 3 + 1).requires_grad_(True)
    res = torch.randn(N, C, H, H)
    xh = F.instance_norm(x, eps=1e-5)
    y = {0: xh, 1: F.relu(xh), 2: F.leaky_relu(xh, 0.2)}[act]
    if act == 0:
        y = y + res
    gy = torch.randn_like(y)
    y.backward(gy)
    xd = nhwc(x.detach())
    work = torch.empty(ops.IN_PARTS * N * C, dtype=torch.float64, device=DEV)
    mr = torch.empty(2 * N * C, device=DEV)
    red = torch.empty(2 * N * C, device=DEV)
    ops.in_stats(ops.Feat(xd), work, mr)
    yd = torch.empty_like(xd)
    xhat = torch.empty_like(xd) if act == 0 else None
    ops.in_apply(ops.Feat(xd), mr, ops.Feat(yd), act=act, res=ops.Feat(nhwc(res)) if act == 0 else None, xhat=xhat)
    assert relerr(nchw(yd), y.detach()) < 1e-5
    dx = torch.empty_like(xd)
    db = torch.zeros(C, device=DEV)
    ops.in_backward(ops.Feat(nhwc(gy)), ops.Feat(xd), act, mr, work, red, ops.Feat(dx), db=db)
    assert relerr(nchw(dx), x.grad) < 1e-4
    assert float(db.abs().max()) < 1e-3  # sum of an IN input-grad is ~0


def test_blur_down_upsample_fold_pool(ops):
    torch.manual_seed(3)
    from oracle import step as O
    C = 16
    filt = O.binomial_filter(3)[None, None].repeat(C, 1, 1, 1)
    for H in (8, 9, 16):
        x = torch.randn(2, C, H, H, requires_grad=True)
        y = O.blur_down(x, filt)
        g = torch.randn_like(y)
        y.backward(g)
        yd = torch.empty(2, y.shape[2], y.shape[3], C, device=DEV)
        ops.blur_down(ops.Feat(nhwc(x.detach())), ops.Feat(yd))
        assert relerr(nchw(yd), y.detach()) < 1e-5
        dx = torch.empty(2, H, H, C, device=DEV)
        ops.blur_down_bwd(ops.Feat(nhwc(g)), ops.Feat(dx))
        assert relerr(nchw(dx), x.grad) < 1e-5
    for H in (4, 8, 7):
        x = torch.randn(2, C, H, H, requires_grad=True)
        y = O.up_aa(x, filt)
        g = torch.randn_like(y)
        y.backward(g)
        yd = torch.empty(2, 2 * H, 2 * H, C, device=DEV)
        ops.upsample(ops.Feat(nhwc(x.detach())), ops.Feat(yd))
        assert relerr(nchw(yd), y.detach()) < 1e-5
        dx = torch.zeros(2, H, H, C, device=DEV)
        work = torch.empty(2 * 4 * H * H * C, device=DEV)
        ops.upsample_bwd(ops.Feat(nhwc(g)), ops.Feat(dx), work)
        assert relerr(nchw(dx), x.grad) < 1e-5
    x = torch.randn(2, C, 8, 8, requires_grad=True)
    y = F.max_pool2d(F.relu(x), 2)
    g = torch.randn_like(y)
    y.backward(g)
    xr = nhwc(F.relu(x.detach()))
    yd = torch.empty(2, 4, 4, C, device=DEV)
    ops.maxpool(ops.Feat(xr), ops.Feat(yd))
    assert relerr(nchw(yd), y.detach()) < 1e-6
    dx = torch.empty_like(xr)
    ops.maxpool_bwd(ops.Feat(xr), ops.Feat(nhwc(g)), ops.Feat(dx))
    assert relerr(nchw(dx), x.grad) < 1e-6


def test_losses(ops):
    torch.manual_seed(4)
    from oracle import step as O
    N, H = 2, 24
    a = (torch.rand(N, 3, H, H) * 2 - 1).requires_grad_(True)
    b = torch.rand(N, 3, H, H) * 2 - 1
    ad, bd = nhwc(a.detach()), nhwc(b)
    loss = torch.zeros(8, dtype=torch.float64, device=DEV)
    g = torch.zeros_like(ad)
    ops.l1(ad, bd, 30.0, g, loss[0:1], accumulate=True)
    ops.tv(ops.Feat(ad), 1e-4, g, loss[1:2])
    work = torch.empty(10 * ad.numel(), device=DEV)
    ops.ssim(ops.Feat(ad), ops.Feat(bd), 2.0, g, loss[2:3], work)
    l_l1 = (a - b).abs().mean() * 30
    l_tv = O.tv_loss(a) * 1e-4
    l_ss = O.ssim_loss((a + 1) / 2, (b + 1) / 2) * 2.0
    (l_l1 + l_tv + l_ss).backward()
    lc = loss.cpu()
    assert abs(lc[0] - l_l1.item()) < 1e-5 * l_l1.item()
    assert abs(lc[1] - l_tv.item()) < 1e-5 * l_tv.item()
    assert abs(lc[2] - l_ss.item()) < 1e-5 * max(l_ss.item(), 1e-3)
    assert relerr(nchw(g), a.grad) < 1e-4
    # hinge
    p = torch.randn(2 * 50)
    pd = p.to(DEV)
    gp = torch.empty_like(pd)
    ops.hinge(pd, 50, 0, 1.0, gp, loss[3:4])
    pr = p.clone().requires_grad_(True)
    ld = 0.5 * (F.relu(1 - pr[:50]).mean() + F.relu(1 + pr[50:]).mean())
    ld.backward()
    assert abs(loss[3].item() - ld.item()) < 1e-6
    assert relerr(gp.cpu(), pr.grad) < 1e-6
    # modes other than 0 / 1 are refused (the split D-step modes were removed)
    with pytest.raises(Exception):
        ops.hinge(pd[:50].contiguous(), 50, 2, 1.0, gp[:50], loss[4:5])


@pytest.mark.parametrize("count", [1 << 20, 1001])
def test_l1_bf16_feature_maps(ops, count):
    torch.manual_seed(6)
    a = torch.randn(count).to(torch.bfloat16)
    b = torch.randn(count).to(torch.bfloat16)
    ga = torch.zeros(count, dtype=torch.bfloat16, device=DEV)
    loss = torch.zeros(1, dtype=torch.float64, device=DEV)
    ops.l1(a.to(DEV), b.to(DEV), 30.0, ga, loss)
    d = a.double() - b.double()
    ref = d.abs().mean().item() * 30
    assert abs(loss.item() - ref) < 1e-5 * ref
    want = (torch.sign(d) * 30 / count).float()
    assert torch.allclose(ga.cpu().float(), want, rtol=8e-3, atol=0)


def test_adam_matches_torch(ops):
    torch.manual_seed(5)
    p = torch.randn(1000)
    grads = [torch.randn(1000) for _ in range(3)]
    pt = p.clone().requires_grad_(True)
    opt = torch.optim.Adam([pt], lr=2e-4, betas=(0.5, 0.999))
    pd, m, v = p.to(DEV), torch.zeros(1000, device=DEV), torch.zeros(1000, device=DEV)
    for i, gr in enumerate(grads):
        pt.grad = gr.clone()
        opt.step()
        ops.adam(pd, gr.to(DEV), m, v, i + 1, 2e-4, 0.5, 0.999, 1e-8)
    assert float((pd.cpu() - pt.detach()).abs().max()) < 5e-7  # a few fp32 ulps of |p|~2


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_weight_pack_batch_matches_single_packs(ops, dtype):
    """irgan_weight_pack_batch (one launch) == one irgan_weight_pack per job:
    plain, narrow-padded, stride-2 per-phase and reflect-flipped packs."""
    code = ops.F32 if dtype == "f32" else ops.BF16
    torch.manual_seed(5)
    specs = [ops.ConvSpec(64, 128, 3, 1, 1, 0), ops.ConvSpec(1, 64, 7, 1, 3, 1), ops.ConvSpec(128, 256, 4, 2, 1, 0),
             ops.ConvSpec(256, 256, 3, 1, 1, 1), ops.ConvSpec(64, 3, 7, 1, 3, 1)]
    pcs = [ops.PackedConv(s, torch.randn(s.cout * s.k * s.k * s.cin, device=DEV), None, code) for s in specs]
    for pc in pcs:
        pc.pack()
    single = [[t.clone() for t in ([pc.fwd] if code == ops.BF16 else []) + [b for *_, b in pc.dg]] for pc in pcs]
    for pc in pcs:
        if code == ops.BF16:
            pc.fwd.zero_()
        for *_, b in pc.dg:
            b.zero_()
    ops.PackBatch(pcs).run()
    for pc, ref in zip(pcs, single):
        got = ([pc.fwd] if code == ops.BF16 else []) + [b for *_, b in pc.dg]
        for g, r in zip(got, ref):
            assert torch.equal(g, r)


@pytest.mark.parametrize("case", [(256, 256, 3, 1, 64, 2), (128, 256, 3, 0, 37, 2), (256, 512, 4, 0, 31, 2),
                                  (384, 128, 3, 0, 40, 2), (192, 64, 3, 0, 256, 1)])
def test_conv_fwd_fused_in_stats(ops, case):
    """irgan_conv_fwd_stats (conv_pp epilogue writes the IN partials of its bf16
    output) + irgan_in_finalize == irgan_conv_fwd + irgan_in_stats: same output bits,
    (mean, rstd) equal to fp32 rounding (different summation order)."""
    cin, cout, k, mode, H, N = case
    torch.manual_seed(4)
    spec = ops.ConvSpec(cin, cout, k, 1, 1, mode)
    w = torch.randn(cout * k * k * cin, device=DEV) * (1.0 / (cin * k * k) ** 0.5)
    b = torch.randn(cout, device=DEV) * 0.1
    pc = ops.PackedConv(spec, w, b, ops.BF16)
    pc.pack()
    x = ops.Feat(torch.randn(N, H, H, cin, device=DEV).bfloat16())
    Ho, Wo = spec.out_hw(H, H)
    y0 = ops.Feat(torch.empty(N, Ho, Wo, cout, device=DEV, dtype=torch.bfloat16))
    y1 = ops.Feat(torch.empty(N, Ho, Wo, cout, device=DEV, dtype=torch.bfloat16))
    work = torch.empty(ops.IN_PARTS * N * cout, dtype=torch.float64, device=DEV)
    mr0 = torch.empty(N * cout * 2, device=DEV)
    mr1 = torch.empty(N * cout * 2, device=DEV)
    ops.conv_fwd(pc, x, y0)
    ops.in_stats(y0, work, mr0)
    nb = ops.conv_fwd_stats(pc, x, y1, work)
    assert nb == ((Ho + 15) // 16) * ((Wo + 15) // 16)
    ops.in_finalize(y1, work, nb, mr1)
    torch.cuda.synchronize()
    assert torch.equal(y0.t, y1.t)
    torch.testing.assert_close(mr1, mr0, rtol=2e-5, atol=1e-6)


def test_mfma_probe_rate_is_sane():
    """irgan_mfma_probe (bench.py's measured MFMA peak): finite outputs, and a bf16 rate that is
    positive and not above the nominal 2.5 PFLOP/s dense peak (a FLOP-accounting check)."""
    import bench
    ops = pkg().ops
    tf = bench.mfma_peak_measured(ops, reps=2, iters=400)
    print("measured bf16 MFMA rate", tf, "TFLOP/s")
    assert 200.0 < tf <= bench.BF16_DENSE_PEAK_TFLOPS * 1.02, tf


@pytest.mark.parametrize("N,H,W,C,mask", [(16, 256, 256, 64, True), (16, 128, 128, 128, True), (2, 64, 48, 256, False),
                                          (3, 30, 34, 64, False), (2, 16, 16, 32, True)])
def test_maxpool_bwd_first_max_exact(N, H, W, C, mask):
    """MaxPool2d(2) backward (ir:664, VGG-16 features): dL/dy routed to the first maximum of each
    2x2 window in row-major order, times the ReLU' of the pooled value when mask -- exact against
    a torch restatement (the C = 64 / 128 / 256 bf16 layers run the row-coalesced kernel, C = 32
    the per-pixel one); ties (many zeros after a ReLU) included."""
    ops = pkg().ops
    g = torch.Generator().manual_seed(N * H + C)
    x = torch.relu(torch.randn(N, H, W, C, generator=g)).bfloat16()
    x[:, ::3, ::5] = 0.5   # exact ties
    dy = torch.randn(N, H // 2, W // 2, C, generator=g).bfloat16()
    dx = torch.full((N, H, W, C), 7.0, dtype=torch.bfloat16, device=DEV)
    ops.maxpool_bwd(ops.Feat(x.to(DEV)), ops.Feat(dy.to(DEV)), ops.Feat(dx), relu_mask=mask)
    torch.cuda.synchronize()
    xf = x.float()[:, : H // 2 * 2, : W // 2 * 2]
    win = xf.view(N, H // 2, 2, W // 2, 2, C).permute(0, 1, 3, 5, 2, 4).reshape(N, H // 2, W // 2, C, 4)
    am = win.argmax(-1)                                    # first maximum in (0,0), (0,1), (1,0), (1,1) order
    gm = dy.float() * ((win.max(-1).values > 0).float() if mask else 1.0)
    ref = torch.zeros(N, H // 2, W // 2, C, 4)
    ref.scatter_(-1, am.unsqueeze(-1), gm.unsqueeze(-1))
    ref = ref.view(N, H // 2, W // 2, C, 2, 2).permute(0, 1, 4, 2, 5, 3).reshape(N, H // 2 * 2, W // 2 * 2, C)
    got = dx.float().cpu()[:, : H // 2 * 2, : W // 2 * 2]
    assert torch.equal(got, ref.bfloat16().float())
