import sys, os
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import torch
from conftest import pkg
m = pkg(); eng = m.engine
B, H = 2, 64
def run(fused, H=64):
    eng.INLayer.fused_in_bwd = fused
    cfg = m.Config(); cfg.device, cfg.batch_size, cfg.img_size = "cuda:0", B, H
    tr = m.GANTrainer(cfg)
    tr.netG.store.load(m.seeded_state(m.g_param_shapes(), 0), strict=True)
    tr.netD.store.load(m.seeded_state(m.d_param_shapes(), 1), strict=True)
    for mod in (tr.netG, tr.netD, tr.vgg): mod.repack()
    g = torch.Generator().manual_seed(3)
    ir = (torch.rand(B, 1, H, H, generator=g) * 2 - 1).cuda(); rgb = (torch.rand(B, 3, H, H, generator=g) * 2 - 1).cuda()
    tr.step(ir, rgb); torch.cuda.synchronize()
    return tr.netG.store.grad.clone(), tr
a, tr = run(False); b, _ = run(False); c, _ = run(True)
st = tr.netG.store
print("unfused vs unfused", ((a-b).norm()/a.norm()).item(), "fused vs unfused", ((c-a).norm()/a.norm()).item())
for k in list(st.offsets)[:60]:
    o = st.offsets[k]; n = 1
    for s_ in st.shapes[k]: n *= s_
    x, y = a[o:o+n], c[o:o+n]
    print(k, f"{((x-y).norm()/(x.norm()+1e-30)).item():.2e}", f"{x.norm().item():.3e}")
