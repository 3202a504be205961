"""Diagnostic: per-parameter gradient error of the fp32 HIP step vs the CPU oracle."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch
from conftest import pkg
from oracle import step as O

H = int(sys.argv[1]) if len(sys.argv) > 1 else 64
dt = sys.argv[2] if len(sys.argv) > 2 else "fp32"
smooth = len(sys.argv) > 3 and sys.argv[3] == "smooth"
lam = {"lambda_perc": 0.0, "lambda_L1": 0.0, "lambda_tv": 0.0} if smooth else {}
irc = pkg()
cfg = irc.Config(); cfg.device = "cuda"; cfg.compute_dtype = dt
for k, v in lam.items(): setattr(cfg, k, v)
tr = irc.GANTrainer(cfg)
G = O.seeded_params(O.g_param_shapes(), 1, bias_std=0.02)
D = O.seeded_params(O.d_param_shapes(), 2, bias_std=0.02)
V = O.seeded_params(O.vgg_param_shapes(), 3, kaiming=True)
tr.netG.store.load(G, strict=True); tr.netD.store.load(D, strict=True); tr.vgg.store.load(V, strict=True)
for m in (tr.netG, tr.netD, tr.vgg): m.repack()
g = torch.Generator().manual_seed(11)
ir = torch.rand(2, 1, H, H, generator=g) * 2 - 1
rgb = torch.rand(2, 3, H, H, generator=g) * 2 - 1
acts = {}
Gc = {k: v.clone() for k, v in G.items()}
with torch.no_grad():
    ref_fake = O.g_forward(Gc, ir, acts=acts)
out = O.train_step(G, D, V, ir, rgb, O.AdamState(G), O.AdamState(D), lam=lam)
d = tr.losses(tr.step(ir.cuda(), rgb.cuda()))
for k in d: print(f"{k:14s} hip {d[k]:.7f} ref {float(out[k]):.7f} rel {abs(d[k]-float(out[k]))/max(1e-9,abs(float(out[k]))):.2e}")
fake = tr.netG.engine.bufs.d["fake"].permute(0, 3, 1, 2).cpu()
print("fake maxabs err", float((fake - ref_fake).abs().max()))
b = tr.netG.engine.bufs.d
for name, key, off, C in (("x0", "cat2", 128, 64), ("x1", "cat1", 256, 128), ("x2", "h0", 0, 256), ("x3", "h9", 0, 256)):
    t = b[key][..., off:off + C].permute(0, 3, 1, 2).float().cpu()
    r = acts[name]
    print(f"act {name}: rel {float((t - r).abs().max() / r.abs().max()):.2e}")
for store, grads in ((tr.netG.store, out["gradG"]), (tr.netD.store, out["gradD"])):
    for k, gref in grads.items():
        gg = store.oihw(k, store.grad).cpu()
        err = float((gg - gref).abs().max() / gref.abs().max().clamp_min(1e-12))
        flag = "  <-- pre-IN bias" if k in O.PRE_IN_BIAS_G + O.PRE_IN_BIAS_D else ("  <-- BAD" if err > 1e-3 else "")
        print(f"{k:36s} {err:.2e}{flag}")

# ---- dfake check: oracle loss gradients evaluated at the HIP fake (removes forward error)
import torch.nn.functional as F
fk = fake.clone().requires_grad_(True)
terms = {
    "gan": 0.1 * (-O.d_forward(D, torch.cat([ir, fk], 1)).mean()),
    "l1": (fk - rgb).abs().mean() * (0 if smooth else 30),
    "perc": (O.vgg_features(V, fk) - O.vgg_features(V, rgb)).abs().mean() * (0 if smooth else 30),
    "tv": O.tv_loss(fk) * (0 if smooth else 1e-4),
    "ssim": O.ssim_loss((fk + 1) / 2, (rgb + 1) / 2) * 2.0,
}
tot = None
for name, l in terms.items():
    gterm, = torch.autograd.grad(l, fk, retain_graph=True)
    print(f"term {name:5s} |g|max {float(gterm.abs().max()):.3e}")
    tot = gterm if tot is None else tot + gterm
dh = tr.core.bufs.d["dfake"].permute(0, 3, 1, 2).cpu()
print("dfake rel err vs oracle-at-hip-fake:", float((dh - tot).abs().max() / tot.abs().max()))
for name in terms:
    pass
pr = tr.netD.engine.bufs.d["de4"].permute(0, 3, 1, 2).cpu().flatten()
ref = torch.cat([out["pred_real"].flatten(), out["pred_fake"].flatten()])
print("D logits hip:", [round(float(v), 6) for v in pr])
print("D logits ref:", [round(float(v), 6) for v in ref])
