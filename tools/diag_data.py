import sys, numpy as np, torch
sys.path.insert(0, "."); sys.path.insert(0, "tests")
from conftest import pkg
from test_gpu_data import _host_item
D = pkg().data
rng = np.random.default_rng(0)
B, H, W, S = 2, 512, 640, 256
ir = rng.integers(0, 256, size=(B, H, W), dtype=np.uint8)
rgb = rng.integers(0, 256, size=(B, H, W, 3), dtype=np.uint8)
for fl in ([0, 0], [1, 0]):
    flip = torch.tensor(fl, dtype=torch.uint8)
    out = D.DeviceResizer(S, "cuda")({"ir_u8": torch.from_numpy(ir), "rgb_u8": torch.from_numpy(rgb), "flip": flip})
    for b in range(B):
        hi, hr = _host_item(D, ir[b], rgb[b], bool(flip[b]), S)
        g = out["ir"][b].cpu()
        d = (g - hi).abs()
        print("flip", fl, "b", b, "ir maxdiff", d.max().item(), "count", (d > 0).sum().item(), "first", (d > 0).nonzero()[:3].tolist(), g[0, 0, :4].tolist(), hi[0, 0, :4].tolist())
        d2 = (out["rgb"][b].cpu() - hr).abs()
        print("   rgb maxdiff", d2.max().item(), "count", (d2 > 0).sum().item())
