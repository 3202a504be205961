"""Step-level parity on the MI355X: the fused HIP train step vs the reference's
golden vectors (tests/golden, produced by executing the reference) and vs the
CPU oracle on the same seeded inputs.

Tolerances (north star: 1e-3 rel fp32):
  fp32 mode  - outputs / losses <= 1e-4 rel; post-step params within 2*lr abs
               (Adam's first step is ~lr*sign(g)); pre-IN biases excluded (their
               exact gradient is 0 -- SURVEY.md section 4).
               Weight grads are measured against the reference run in fp64 (the
               exact answer) in relative L2 norm.  They are discontinuous in the
               forward state (ReLU / LeakyReLU kinks, hinge, sign() in the L1 and
               perceptual-L1 terms): one activation that lands on the other side
               of a kink moves a whole layer's grads by ~1e-3..3e-2 (measured:
               a per-layer diagnostic in round 1 showed a single-layer jump at one resblock while all
               other layers sit at ~7e-6 = 2.5x the CPU fp32 error), and the
               reference's OWN fp32 run is off by up to ~2e-2 max-rel on some
               tensors (err32 / err32l2 per tensor in the fixtures).  Criterion:
               rel-L2 <= max(5e-3, 5*err32l2) (sampled on the golden digests,
               full tensors against the oracle).
  bf16 mode  - losses <= 3e-2 rel, G output mean |err| <= 1e-2.
"""
import numpy as np
import pytest
import torch

from conftest import load_golden, pkg
from oracle import step as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
LOSS_KEYS = ("loss_D", "loss_G", "loss_G_GAN", "loss_G_L1", "loss_G_perc", "loss_G_TV", "loss_G_ssim")


LAMBDA_ORDER = ("lambda_L1", "lambda_perc", "lambda_tv", "lambda_ssim", "lambda_gan")


def make_trainer(fx, dtype):
    irc = pkg()
    H, W, B, noaa, noaaup = [int(v) for v in fx["meta"][:5]]
    cfg = irc.Config()
    cfg.device = DEV
    cfg.compute_dtype = dtype
    for k, v in zip(LAMBDA_ORDER, fx["lambdas"]):
        setattr(cfg, k, float(v))
    cfg.no_antialias, cfg.no_antialias_up = bool(noaa), bool(noaaup)
    tr = irc.GANTrainer(cfg)
    tr.netG.store.load(O.seeded_params(O.g_param_shapes(no_antialias=bool(noaa), no_antialias_up=bool(noaaup)),
                                       1, bias_std=0.02), strict=True)
    tr.netD.store.load(O.seeded_params(O.d_param_shapes(), 2, bias_std=0.02), strict=True)
    tr.vgg.store.load(O.seeded_params(O.vgg_param_shapes(), 3, kaiming=True), strict=True)
    for m in (tr.netG, tr.netD, tr.vgg):
        m.repack()
    return tr, cfg


def digest_check(store, fx, tag, pre_in, tol, l2=False):
    """Sampled grads vs the fp64 reference: max-rel within max(tol, 3*err32[k]),
    or (l2=True) sampled relative L2 within max(tol, 5*err32l2[k])."""
    for k in store.shapes:
        g = store.oihw(k, store.grad).reshape(-1).double().cpu().numpy()
        idx = fx[f"{tag}|{k}|idx"]
        post = store.oihw(k).reshape(-1).cpu().numpy()[idx]
        assert np.max(np.abs(post - fx[f"{tag}|{k}|post"])) <= 2 * 2e-4 + 1e-6, f"post-step {k}"
        if k in pre_in:
            continue
        ref = fx[f"{tag}|{k}|val64"]
        if l2:
            err = np.linalg.norm(g[idx] - ref) / max(np.linalg.norm(ref), 1e-30)
            lim = max(tol, 5 * float(fx[f"{tag}|{k}|err32l2"]))
        else:
            err = np.max(np.abs(g[idx] - ref)) / max(np.max(np.abs(g)), 1e-12)
            lim = max(tol, 5 * float(fx[f"{tag}|{k}|err32"]))
        assert err <= lim, f"grad {k}: {err} > {lim}"


@pytest.mark.parametrize("variant", ["s32", "s64", "s32_noaa", "s32_noaaup", "s32_smooth", "s64_smooth"])
def test_step_fp32_matches_reference_golden(variant):
    fx = load_golden(variant)
    tr, cfg = make_trainer(fx, "fp32")
    ir, rgb = torch.from_numpy(fx["ir"]).to(DEV), torch.from_numpy(fx["rgb"]).to(DEV)
    L = tr.step(ir, rgb)
    d = tr.losses(L)
    for k in LOSS_KEYS:
        ref = fx["step1_" + k]
        assert abs(d[k] - ref) <= 1e-4 * max(1.0, abs(ref)), (k, d[k], ref)
    fake = tr.netG.engine.bufs.d["fake"].permute(0, 3, 1, 2).cpu().numpy()
    assert np.max(np.abs(fake - fx["fake"])) <= 1e-4
    De = tr.netD.engine   # the D step's logits on [real; fake] (tag "d")
    pred = De.bufs.d[f"de{len(De.packs) - 1}"].permute(0, 3, 1, 2).cpu().numpy()
    B = fx["ir"].shape[0]
    pred_r, pred_f = pred[:B], pred[B:]
    scale = max(np.max(np.abs(fx["pred_real"])), 1e-6)
    assert np.max(np.abs(pred_r - fx["pred_real"])) <= 1e-4 * max(1, scale)
    assert np.max(np.abs(pred_f - fx["pred_fake"])) <= 1e-4 * max(1, scale)
    pre_in = set(O.pre_in_bias_keys(list(tr.netG.store.shapes) + list(tr.netD.store.shapes)))
    digest_check(tr.netD.store, fx, "gD", pre_in, 5e-3, l2=True)
    digest_check(tr.netG.store, fx, "gG", pre_in, 5e-3, l2=True)
    L2 = tr.step(ir, rgb)
    d2 = tr.losses(L2)
    for k in ("loss_D", "loss_G"):
        # after one Adam step (~lr*sign(g) per element) the reference's own fp32 run
        # drifts from fp64 (up to 3e-3 abs on s64_smooth); hold HIP to the fp64 value
        ref64, ref32 = float(fx["step2_" + k + "_64"]), float(fx["step2_" + k])
        assert abs(d2[k] - ref64) <= max(1e-3 * max(1.0, abs(ref64)), 3 * abs(ref32 - ref64)), (k, d2[k], ref64)


def test_step_bf16_close_to_reference():
    fx = load_golden("s64")
    tr, cfg = make_trainer(fx, "bf16")
    ir, rgb = torch.from_numpy(fx["ir"]).to(DEV), torch.from_numpy(fx["rgb"]).to(DEV)
    d = tr.losses(tr.step(ir, rgb))
    for k in ("loss_D", "loss_G", "loss_G_L1", "loss_G_perc", "loss_G_ssim"):
        ref = fx["step1_" + k]
        assert abs(d[k] - ref) <= 3e-2 * max(1.0, abs(ref)), (k, d[k], ref)
    fake = tr.netG.engine.bufs.d["fake"].permute(0, 3, 1, 2).cpu().numpy()
    err = np.abs(fake - fx["fake"])
    assert err.mean() <= 1e-2 and err.max() <= 0.15, (err.mean(), err.max())


def _oracle(dtype, ir, rgb, lam):
    G = {k: v.to(dtype).clone() for k, v in O.seeded_params(O.g_param_shapes(), 1, bias_std=0.02).items()}
    D = {k: v.to(dtype).clone() for k, v in O.seeded_params(O.d_param_shapes(), 2, bias_std=0.02).items()}
    V = {k: v.to(dtype).clone() for k, v in O.seeded_params(O.vgg_param_shapes(), 3, kaiming=True).items()}
    return O.train_step(G, D, V, ir.to(dtype), rgb.to(dtype), O.AdamState(G), O.AdamState(D), lam=lam)


@pytest.mark.parametrize("seed,smooth", [(11, True), (12, True), (11, False)])
def test_step_fp32_vs_oracle_full_tensors(seed, smooth):
    """Full-tensor comparison against the CPU oracle (fp32 and fp64) on fresh seeded 64x64 batches."""
    fx = load_golden("s64_smooth" if smooth else "s64")
    lam = dict(zip(LAMBDA_ORDER, (float(v) for v in fx["lambdas"])))
    tr, cfg = make_trainer(fx, "fp32")
    g = torch.Generator().manual_seed(seed)
    ir = torch.rand(2, 1, 64, 64, generator=g) * 2 - 1
    rgb = torch.rand(2, 3, 64, 64, generator=g) * 2 - 1
    o32, o64 = _oracle(torch.float32, ir, rgb, lam), _oracle(torch.float64, ir, rgb, lam)
    d = tr.losses(tr.step(ir.to(DEV), rgb.to(DEV)))
    for k in LOSS_KEYS:
        assert abs(d[k] - float(o64[k])) <= 1e-4 * max(1.0, abs(float(o64[k]))), k
    pre_in = set(O.pre_in_bias_keys(list(o64["gradG"]) + list(o64["gradD"])))
    for store, tag in ((tr.netG.store, "gradG"), (tr.netD.store, "gradD")):
        for k, g64 in o64[tag].items():
            if k in pre_in:
                continue
            got = store.oihw(k, store.grad).cpu().double()
            den = g64.norm().clamp_min(1e-30)
            err32 = float((o32[tag][k].double() - g64).norm() / den)
            err = float((got - g64).norm() / den)
            assert err <= max(5e-3, 5 * err32), (k, err, err32)


def test_generator_module_api_and_checkpoint_layout(tmp_path):
    """nn.Module API: state_dict keys/shapes as the reference, load/save round trip,
    forward on the HIP kernels with autograd."""
    irc = pkg()
    cfg = irc.Config()
    cfg.device = DEV
    cfg.compute_dtype = "fp32"
    model = irc.IRColorizationModel(cfg)
    sd = model.netG.state_dict()
    shapes = O.g_param_shapes()
    assert list(sd.keys()) == list(shapes.keys())
    assert all(tuple(sd[k].shape) == tuple(v) for k, v in shapes.items())
    G = O.seeded_params(shapes, 1, bias_std=0.02)
    path = tmp_path / "netG.pth"
    torch.save(G, path)
    model.load_weights(str(path))
    x = torch.from_numpy(load_golden("s64")["ir"]).to(DEV)
    y = model(x)
    ref = O.g_forward(G, x.cpu())
    assert float((y.cpu() - ref).abs().max()) < 1e-4
    # autograd through the HIP backward
    xg = x.clone().requires_grad_(False)
    out, _ = model.netG(xg)
    out.square().mean().backward()
    Gr = {k: v.clone().requires_grad_(not k.endswith(".filt")) for k, v in G.items()}
    O.g_forward(Gr, x.cpu()).square().mean().backward()
    for k, p in model.netG.named_parameters():
        if k in O.PRE_IN_BIAS_G:
            continue
        err = float((p.grad.cpu() - Gr[k].grad).norm() / Gr[k].grad.norm().clamp_min(1e-12))
        assert err < 5e-3, (k, err)


def _grads_vs_oracle(tr, o, oac):
    """G / D weight grads (rel-L2 against the fp32 oracle ``o``) no further than 1.5x + 0.02
    what PyTorch's bf16 autocast of the same oracle step (``oac``) gets."""
    pre_in = set(O.pre_in_bias_keys(list(o["gradG"]) + list(o["gradD"])))
    for store, tag in ((tr.netG.store, "gradG"), (tr.netD.store, "gradD")):
        for k, gr in o[tag].items():
            if k in pre_in:
                continue
            den = gr.double().norm().clamp_min(1e-30)
            got = store.oihw(k, store.grad).cpu().double()
            e = float((got - gr.double()).norm() / den)
            e_ac = float((oac[tag][k].double() - gr.double()).norm() / den)
            print("grad rel-L2", tag, k, round(e, 4), "autocast-bf16", round(e_ac, 4))
            assert np.isfinite(e) and e <= 1.5 * e_ac + 0.02, (tag, k, e, e_ac)


def test_kaist_native_resolution_512x640():
    """BASELINE config 4 at its own resolution (512x640, KAIST native): W/4 = 160 is not
    a multiple of 64, so the wgrad row-segment kernel and several tile paths take their
    general branches.
    (a) G forward (fp32 parity mode) vs the CPU oracle.
    (b) The benchmarked bf16 step at 512x640, B=1 against the fp32 CPU oracle on the same
        seeded inputs and weights, with the bf16 rule of test_bf16_step_256_vs_oracle_...:
        losses <= 3e-2 rel, G output mean |err| <= 1e-2, G / D weight grads within 1.5x +
        0.02 of PyTorch's own bf16 autocast error on the same oracle step.
    (c) The config's per-GPU batch (B=4): one bf16 step, everything finite."""
    fx = load_golden("s32")
    lam = dict(zip(LAMBDA_ORDER, (float(v) for v in fx["lambdas"])))
    g = torch.Generator().manual_seed(21)
    ir = torch.rand(4, 1, 512, 640, generator=g) * 2 - 1
    rgb = torch.rand(4, 3, 512, 640, generator=g) * 2 - 1
    tr32, _ = make_trainer(fx, "fp32")
    fake = tr32.netG.engine.forward(ir[:1].to(DEV))          # NHWC fp32
    G = O.seeded_params(O.g_param_shapes(), 1, bias_std=0.02)
    with torch.no_grad():
        ref = O.g_forward(G, ir[:1])
    assert float((fake.cpu().permute(0, 3, 1, 2) - ref).abs().max()) < 1e-4
    del tr32
    # (b) bf16 step, B = 1, vs the oracle
    tr16, _ = make_trainer(fx, "bf16")
    d = tr16.losses(tr16.step(ir[:1].to(DEV), rgb[:1].to(DEV)))
    o = _oracle(torch.float32, ir[:1], rgb[:1], lam)
    for k in ("loss_D", "loss_G", "loss_G_L1", "loss_G_perc", "loss_G_ssim", "loss_G_GAN"):
        r = float(o[k])
        assert abs(d[k] - r) <= 3e-2 * max(1.0, abs(r)), (k, d[k], r)
    err = (tr16.netG.engine.bufs.d["fake"].permute(0, 3, 1, 2).cpu() - o["fake"]).abs()
    print("bf16 512x640 B=1: fake mean/max err", err.mean().item(), err.max().item())
    assert err.mean() <= 1e-2, err.mean()
    with torch.autocast("cpu", dtype=torch.bfloat16):
        oac = _oracle(torch.float32, ir[:1], rgb[:1], lam)
    _grads_vs_oracle(tr16, o, oac)
    del tr16
    # (c) B = 4
    t4, _ = make_trainer(fx, "bf16")
    l4 = t4.losses(t4.step(ir.to(DEV), rgb.to(DEV)))
    assert all(np.isfinite(v) for v in l4.values()), l4
    f4 = t4.netG.engine.bufs.d["fake"]
    assert torch.isfinite(f4).all() and f4.abs().max() <= 1.0
    for st in (t4.netG.store, t4.netD.store):
        assert torch.isfinite(st.grad).all() and torch.isfinite(st.flat).all()


def _seeded_trainer(irc, seed_shift=0):
    from oracle import step as O
    cfg = irc.Config()
    cfg.device = "cuda:0"
    cfg.compute_dtype = "fp32"
    tr = irc.GANTrainer(cfg)
    tr.netG.store.load(O.seeded_params(O.g_param_shapes(), 1 + seed_shift, bias_std=0.02), strict=True)
    tr.netD.store.load(O.seeded_params(O.d_param_shapes(), 2 + seed_shift, bias_std=0.02), strict=True)
    tr.vgg.store.load(O.seeded_params(O.vgg_param_shapes(), 3, kaiming=True), strict=True)
    for net in (tr.netG, tr.netD, tr.vgg):
        net.repack()
    return tr


def test_full_state_checkpoint_resume_and_torch_adam(tmp_path):
    """GANTrainer.save_checkpoint / load_checkpoint carry G, D, both
    Adams and the LR position.  (1) A fresh trainer that loads the file after 2 steps
    continues exactly as the original (same step 3, fp32 parity mode).  (2) The saved
    optimizer_G is a torch.optim.Adam state: torch's own Adam, loaded with it and fed
    step 3's gradient, reproduces the HIP Adam update (ir:1601-1609, 1681)."""
    irc = pkg()
    g = torch.Generator().manual_seed(21)
    batches = [(torch.rand(2, 1, 32, 32, generator=g) * 2 - 1, torch.rand(2, 3, 32, 32, generator=g) * 2 - 1)
               for _ in range(3)]
    a = _seeded_trainer(irc)
    for ir, rgb in batches[:2]:
        a.step(ir.cuda(), rgb.cuda())
    a.scheduler_step()
    path = tmp_path / "full.pt"
    a.save_checkpoint(path)
    sd2 = torch.load(path, map_location="cpu", weights_only=True)
    b = _seeded_trainer(irc, seed_shift=10)
    b.load_checkpoint(path)
    assert b.epoch_index == 1 and b.netG.store.step_count == 2 and b.netD.store.step_count == 2
    La = a.losses(a.step(batches[2][0].cuda(), batches[2][1].cuda()))
    Lb = b.losses(b.step(batches[2][0].cuda(), batches[2][1].cuda()))
    for k in La:
        assert abs(La[k] - Lb[k]) <= 1e-6 * max(1.0, abs(La[k])), (k, La[k], Lb[k])
    lr = a.current_lr_G
    for name in ("netG", "netD"):
        sa, sb = getattr(a, name).store, getattr(b, name).store
        for k in sa.shapes:
            d = (sa.krsc(k) - sb.krsc(k)).abs().max().item()
            assert d <= 2 * lr, (name, k, d)   # grads differ only by split-K atomics order
    # torch.optim.Adam over the step-2 state and the step-3 gradient == the HIP update
    st = a.netG.store
    params = [torch.nn.Parameter(t.double().clone()) for t in sd2["netG"].values()]
    for p, k in zip(params, st.shapes):
        p.grad = st.oihw(k, st.grad).detach().cpu().double().clone()
    opt = torch.optim.Adam(params, lr=lr, betas=(a.cfg.beta1, a.cfg.beta2))
    osd = sd2["optimizer_G"]
    osd["state"] = {i: {kk: (vv.double() if kk != "step" else vv) for kk, vv in e.items()}
                    for i, e in osd["state"].items()}
    opt.load_state_dict(osd)
    opt.param_groups[0]["lr"] = lr
    opt.step()
    for p, k in zip(params, st.shapes):
        got = st.oihw(k).detach().cpu().double()
        assert (got - p.detach()).abs().max().item() <= 1e-6 * lr + 1e-7, k


@pytest.mark.parametrize("noaa,noaaup", [(False, False), (False, True), (True, False)])
@pytest.mark.parametrize("H,W", [(45, 38), (250, 250)])
def test_odd_size_generator_forward_fallback(H, W, noaa, noaaup):
    """ir:555-556 / 562-563: when the up-sampled map is not the skip's size (H or W
    not divisible by 4), the reference resizes it (bilinear, align_corners=True)
    before the concat.  The HIP generator folds that resize into the UpsampleAA
    table (or runs it after the ConvTranspose2d); fp32 mode vs the CPU oracle."""
    irc = pkg()
    cfg = irc.Config()
    cfg.device = DEV
    cfg.compute_dtype = "fp32"
    cfg.no_antialias, cfg.no_antialias_up = noaa, noaaup
    model = irc.IRColorizationModel(cfg)
    G = O.seeded_params(O.g_param_shapes(no_antialias=noaa, no_antialias_up=noaaup), 1, bias_std=0.02)
    model.netG.load_state_dict(G)
    x = torch.rand(2, 1, H, W, generator=torch.Generator().manual_seed(5)) * 2 - 1
    with torch.no_grad():
        y = model(x.to(DEV)).cpu()
        ref = O.g_forward(G, x, no_antialias=noaa, no_antialias_up=noaaup)
    assert y.shape == ref.shape == (2, 3, H, W)
    assert float((y - ref).abs().max()) < 1e-4


@pytest.mark.parametrize("noaaup", [False, True])
def test_odd_size_step_fp32_vs_oracle(noaaup):
    """A whole fp32 train step at 45x38 (both decoder stages take the resize
    fallback, VGG pools floor odd sizes) vs the CPU oracle in fp64."""
    irc = pkg()
    fx = load_golden("s32")
    lam = dict(zip(LAMBDA_ORDER, (float(v) for v in fx["lambdas"])))
    cfg = irc.Config()
    cfg.device = DEV
    cfg.compute_dtype = "fp32"
    cfg.no_antialias_up = noaaup
    tr = irc.GANTrainer(cfg)
    shapes = O.g_param_shapes(no_antialias_up=noaaup)
    G = O.seeded_params(shapes, 1, bias_std=0.02)
    D = O.seeded_params(O.d_param_shapes(), 2, bias_std=0.02)
    V = O.seeded_params(O.vgg_param_shapes(), 3, kaiming=True)
    tr.netG.store.load(G, strict=True)
    tr.netD.store.load(D, strict=True)
    tr.vgg.store.load(V, strict=True)
    for m in (tr.netG, tr.netD, tr.vgg):
        m.repack()
    g = torch.Generator().manual_seed(9)
    ir = torch.rand(2, 1, 45, 38, generator=g) * 2 - 1
    rgb = torch.rand(2, 3, 45, 38, generator=g) * 2 - 1
    d = tr.losses(tr.step(ir.to(DEV), rgb.to(DEV)))

    def run(dt):
        c = lambda P: {k: v.to(dt).clone() for k, v in P.items()}  # noqa: E731
        Gd, Dd = c(G), c(D)
        return O.train_step(Gd, Dd, c(V), ir.to(dt), rgb.to(dt), O.AdamState(Gd), O.AdamState(Dd), lam=lam,
                            no_antialias_up=noaaup)
    o64, o32 = run(torch.float64), run(torch.float32)
    for k in LOSS_KEYS:
        assert abs(d[k] - float(o64[k])) <= 1e-4 * max(1.0, abs(float(o64[k]))), (k, d[k], float(o64[k]))
    pre_in = set(O.pre_in_bias_keys(list(o64["gradG"]) + list(o64["gradD"])))
    for store, tag in ((tr.netG.store, "gradG"), (tr.netD.store, "gradD")):
        for k, g64 in o64[tag].items():
            if k in pre_in:
                continue
            got = store.oihw(k, store.grad).cpu().double()
            den = g64.norm().clamp_min(1e-30)
            err32 = float((o32[tag][k].double() - g64).norm() / den)
            err = float((got - g64).norm() / den)
            assert err <= max(5e-3, 5 * err32), (k, err, err32)


def test_bf16_step_256_vs_oracle_and_b16_finite():
    """BASELINE config 2 at its own resolution.  (a) The benchmarked bf16 step at
    256x256, B=2 against the fp32 CPU oracle on the same seeded inputs and weights:
    losses <= 3e-2 rel, G output mean |err| <= 1e-2, and G / D weight grads no
    further from the fp32 oracle (rel-L2) than 1.5x + 0.02 what PyTorch's own bf16
    autocast of the same oracle step gets (measured: 0.2-0.35 on the early G layers
    for both -- gradients stored in bf16 lose bits to the IN-backward cancellation
    g - mean(g), whoever computes them).
    (b) The bench's 256x256, B=16 step: every loss, grad and the output finite,
    output in the tanh range, and losses within 3e-2 of the fp32-mode step."""
    fx = load_golden("s64")
    lam = dict(zip(LAMBDA_ORDER, (float(v) for v in fx["lambdas"])))
    tr, cfg = make_trainer(fx, "bf16")
    g = torch.Generator().manual_seed(31)
    ir = torch.rand(2, 1, 256, 256, generator=g) * 2 - 1
    rgb = torch.rand(2, 3, 256, 256, generator=g) * 2 - 1
    d = tr.losses(tr.step(ir.to(DEV), rgb.to(DEV)))
    o = _oracle(torch.float32, ir, rgb, lam)
    for k in ("loss_D", "loss_G", "loss_G_L1", "loss_G_perc", "loss_G_ssim", "loss_G_GAN"):
        ref = float(o[k])
        assert abs(d[k] - ref) <= 3e-2 * max(1.0, abs(ref)), (k, d[k], ref)
    fake = tr.netG.engine.bufs.d["fake"].permute(0, 3, 1, 2).cpu()
    err = (fake - o["fake"]).abs()
    print("bf16 256^2 B=2: fake mean/max err", err.mean().item(), err.max().item())
    assert err.mean() <= 1e-2, err.mean()
    with torch.autocast("cpu", dtype=torch.bfloat16):
        oac = _oracle(torch.float32, ir, rgb, lam)
    _grads_vs_oracle(tr, o, oac)
    # (b) B = 16
    g = torch.Generator().manual_seed(32)
    ir = (torch.rand(16, 1, 256, 256, generator=g) * 2 - 1).to(DEV)
    rgb = (torch.rand(16, 3, 256, 256, generator=g) * 2 - 1).to(DEV)
    t16, _ = make_trainer(fx, "bf16")
    t32, _ = make_trainer(fx, "fp32")
    l16 = t16.losses(t16.step(ir, rgb))
    l32 = t32.losses(t32.step(ir, rgb))
    f16 = t16.netG.engine.bufs.d["fake"]
    assert torch.isfinite(f16).all() and f16.abs().max() <= 1.0
    for st in (t16.netG.store, t16.netD.store):
        assert torch.isfinite(st.grad).all() and torch.isfinite(st.flat).all()
    for k in LOSS_KEYS:
        assert np.isfinite(l16[k]), k
        if k != "loss_G_TV":
            assert abs(l16[k] - l32[k]) <= 3e-2 * max(1.0, abs(l32[k])), (k, l16[k], l32[k])


@pytest.mark.parametrize("dtype", ["bf16", "fp8"])
def test_stream_overlap_schedule_bit_identical(monkeypatch, dtype):
    """The default step runs the VGG real half, the D step, D Adam and the GAN-term D pass
    on a side stream, joined to the main stream by events (GANStep.step).  In deterministic
    mode (ops.set_deterministic: every split-K weight gradient reduced through ordered
    slabs, no fp32 atomics) every kernel is run-to-run reproducible and the shared
    workspaces are per stream, so the overlapped schedule must give BIT-IDENTICAL grads,
    parameters and Adam moments to the single-stream one (IRGAN_NO_D_OVERLAP=1,
    IRGAN_NO_VGG_OVERLAP=1) over three steps: a missed wait would show up here.
    Loss values are fp64 atomic block sums (order-dependent): compared to 1e-12 rel."""
    fx = load_golden("s64")
    g = torch.Generator().manual_seed(51)
    batches = [((torch.rand(2, 1, 128, 128, generator=g) * 2 - 1).to(DEV),
                (torch.rand(2, 3, 128, 128, generator=g) * 2 - 1).to(DEV)) for _ in range(3)]
    ops = pkg().ops

    def run(overlap):
        for k in ("IRGAN_NO_D_OVERLAP", "IRGAN_NO_VGG_OVERLAP"):
            if overlap:
                monkeypatch.delenv(k, raising=False)
            else:
                monkeypatch.setenv(k, "1")
        tr, _ = make_trainer(fx, dtype)
        assert (tr.core.side is not None) == overlap
        losses = []
        for ir, rgb in batches:
            losses.append(tr.losses(tr.step(ir, rgb)))
        torch.cuda.synchronize()
        return tr, losses

    old = ops.set_deterministic(True)
    try:
        ta, la = run(True)
        tb, lb = run(False)
        tc, _ = run(True)            # the same schedule twice: reproducible at all?
    finally:
        ops.set_deterministic(old)
    for x, y in zip(la, lb):
        for k in x:
            assert abs(x[k] - y[k]) <= 1e-12 * max(1.0, abs(y[k])), (k, x[k], y[k])
    for name in ("netG", "netD"):
        sa, sb, sc = getattr(ta, name).store, getattr(tb, name).store, getattr(tc, name).store
        assert torch.equal(sa.grad, sc.grad), f"{name}: deterministic mode is not reproducible run to run"
        assert torch.equal(sa.grad, sb.grad), f"{name} grads differ between the schedules"
        assert torch.equal(sa.flat, sb.flat), f"{name} params differ between the schedules"
        assert torch.equal(sa.m, sb.m) and torch.equal(sa.v, sb.v), f"{name} Adam moments differ"
