import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch
from conftest import pkg
from oracle import step as O
irc = pkg(); E = irc.engine; ops = irc.ops
DEV = "cuda"
H = int(sys.argv[1]) if len(sys.argv) > 1 else 64
G = O.seeded_params(O.g_param_shapes(), 1, bias_std=0.02)
st = E.ParamStore(E.g_param_shapes(), torch.device(DEV)); st.load(G, strict=True)
eng = E.GeneratorEngine(st, ops.F32); eng.pack()
torch.manual_seed(0)
x = torch.rand(2, 1, H, H) * 2 - 1
fake = eng.forward(x.to(DEV))
Gr = {k: v.clone().requires_grad_(not k.endswith(".filt")) for k, v in G.items()}
for dt in (torch.float32, torch.float64):
    Gd = {k: v.detach().to(dt).clone().requires_grad_(not k.endswith(".filt")) for k, v in G.items()}
    ref = O.g_forward(Gd, x.to(dt))
    ref.square().mean().backward()
    if dt == torch.float32: G32 = Gd
    else: G64 = Gd; ref64 = ref
print("fwd err vs fp64", float((fake.permute(0, 3, 1, 2).cpu().double() - ref64.detach()).abs().max()))
dfake = (2 * fake / fake.numel()).contiguous()
st.zero_grad()
eng.backward(dfake)
for k in st.shapes:
    g = st.oihw(k, st.grad).cpu().double()
    g64 = G64[k].grad
    g32 = G32[k].grad.double()
    l2 = float((g - g64).norm() / g64.norm()); l2_32 = float((g32 - g64).norm() / g64.norm())
    mx = float((g - g64).abs().max() / g64.abs().max()); mx32 = float((g32 - g64).abs().max() / g64.abs().max())
    print(f"{k:34s} hipL2 {l2:.2e} cpu32L2 {l2_32:.2e}  hipMax {mx:.2e} cpu32Max {mx32:.2e}")
