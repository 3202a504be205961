import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch
from conftest import pkg
from oracle import step as O
irc = pkg(); E = irc.engine; ops = irc.ops
DEV = "cuda"
H = int(sys.argv[1]) if len(sys.argv) > 1 else 32
NB = int(sys.argv[2]) if len(sys.argv) > 2 else 4
D = O.seeded_params(O.d_param_shapes(), 2, bias_std=0.02)
st = E.ParamStore(E.d_param_shapes(), torch.device(DEV)); st.load(D, strict=True)
eng = E.DiscriminatorEngine(st, ops.F32); eng.pack()
torch.manual_seed(0)
x = torch.rand(NB, 4, H, H) * 2 - 1
din = x.permute(0, 2, 3, 1).contiguous().to(DEV)
out = eng.forward(ops.Feat(din), tag="t")
Dr = {k: v.clone().requires_grad_(True) for k, v in D.items()}
xr = x.clone().requires_grad_(True)
ref = O.d_forward(Dr, xr)
print("fwd err", float((out.permute(0, 3, 1, 2).cpu() - ref).abs().max() / ref.abs().max()))
gout = torch.randn_like(ref)
ref.backward(gout)
st.zero_grad()
dx = eng.backward(gout.permute(0, 2, 3, 1).contiguous().to(DEV), want_wgrad=True, want_dinput=True, tag="t")
for k in D:
    g = st.oihw(k, st.grad).cpu()
    print(f"{k:18s} {float((g - Dr[k].grad).abs().max() / Dr[k].grad.abs().max()):.2e}")
print("dinput", float((dx.t.permute(0, 3, 1, 2).cpu() - xr.grad).abs().max() / xr.grad.abs().max()))
