import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch, torch.nn.functional as F
from conftest import pkg
ops = pkg().ops
DEV = "cuda"
def nhwc(x): return x.permute(0, 2, 3, 1).contiguous().to(DEV)
def nchw(x): return x.float().cpu().permute(0, 3, 1, 2).contiguous()
torch.manual_seed(0)
for (N, C, H, ld, off, inplace, act) in [(2, 64, 32, 64, 0, False, 1), (2, 512, 3, 512, 0, True, 2), (4, 512, 3, 512, 0, True, 2), (2, 256, 4, 256, 0, True, 2), (2, 64, 16, 64, 0, True, 2), (2, 512, 3, 512, 0, True, 1)]:
    x = (torch.randn(N, C, H, H) * 2 + 0.5).requires_grad_(True)
    xh = F.instance_norm(x, eps=1e-5)
    y = F.relu(xh) if act == 1 else F.leaky_relu(xh, 0.2)
    gy = torch.randn_like(y)
    y.backward(gy)
    xd = nhwc(x.detach())
    work = torch.empty(ops.IN_PARTS * N * C, dtype=torch.float64, device=DEV); mr = torch.empty(2 * N * C, device=DEV); red = torch.empty(2 * N * C, device=DEV)
    ops.in_stats(ops.Feat(xd), work, mr)
    buf = torch.zeros(N, H, H, ld, device=DEV)
    buf[..., off:off + C] = nhwc(gy)
    dyf = ops.Feat(buf, off, C)
    dx = dyf if inplace else ops.Feat(torch.empty(N, H, H, C, device=DEV))
    db = torch.zeros(C, device=DEV)
    ops.in_backward(dyf, ops.Feat(xd), act, mr, work, red, dx, db=db)
    got = nchw(dx.t[..., dx.off:dx.off + C])
    print(N, C, H, ld, off, inplace, act, "rel err", float((got - x.grad).abs().max() / x.grad.abs().max()))
    m = mr.view(N, C, 2).cpu()
    print("  mean err", float((m[..., 0] - x.detach().mean((2, 3))).abs().max()), "rstd err", float((m[..., 1] - 1 / (x.detach().var((2, 3), unbiased=False) + 1e-5).sqrt()).abs().max()))
cs = torch.zeros(512, device=DEV)
g = torch.randn(2, 3, 3, 512)
ops.channel_sum(ops.Feat(g.to(DEV)), cs)
print("channel_sum err", float((cs.cpu() - g.sum((0, 1, 2))).abs().max()))
