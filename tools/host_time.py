"""Host enqueue time vs GPU time per fused train step (is the step launch-bound?)."""
import importlib, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
irc = importlib.import_module("infrared-colorization-with-resnet-generator-and-patchgan_amd")
B, H = 16, 256
cfg = irc.Config(); cfg.device = "cuda:0"; cfg.batch_size = B; cfg.img_size = H
tr = irc.GANTrainer(cfg)
tr.netG.store.load(irc.seeded_state(irc.g_param_shapes(), 0), strict=True)
tr.netD.store.load(irc.seeded_state(irc.d_param_shapes(), 1), strict=True)
for m in (tr.netG, tr.netD, tr.vgg):
    m.repack()
g = torch.Generator().manual_seed(7)
ir = (torch.rand(B, 1, H, W := H, generator=g) * 2 - 1).cuda()
rgb = (torch.rand(B, 3, H, W, generator=g) * 2 - 1).cuda()
for _ in range(5):
    tr.step(ir, rgb)
torch.cuda.synchronize()
enq = []
t0 = time.perf_counter()
for _ in range(20):
    a = time.perf_counter(); tr.step(ir, rgb); enq.append(time.perf_counter() - a)
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / 20
enq.sort()
print(f"wall/step {wall*1e3:.2f} ms, host enqueue/step median {enq[10]*1e3:.2f} ms min {enq[0]*1e3:.2f}")
# GPU-only time: queue 20 steps behind a long sleep kernel so the host is never the bottleneck
torch.cuda.synchronize()
torch.cuda._sleep(int(2e9))  # ~1 s of GPU spin: the host enqueues everything meanwhile
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    tr.step(ir, rgb)
e1.record()
torch.cuda.synchronize()
print(f"gpu-only step {e0.elapsed_time(e1)/20:.2f} ms (host queued ahead)")
