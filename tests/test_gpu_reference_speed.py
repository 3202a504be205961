"""The reference's own train step in PyTorch-ROCm eager on the same MI355X (timing only).

The reference trains in fp32 eager PyTorch, NCHW, no autocast (ir:1636-1681; no AMP anywhere
in ir_colorization.py).  This times the oracle's restatement of that step (oracle/step.py,
the same torch ops: F.conv2d / F.instance_norm / F.interpolate / autograd / Adam in torch's
single-tensor order) on `cuda`, at the bench config (256x256, batch 16), in three forms:

  * ``as_written`` fp32: the reference's own order (a no-grad G forward for the D step, a
    second G forward, D weight gradients from loss_G.backward()) -- what the reference costs
    on this GPU;
  * ``minimal`` fp32: the work the HIP step does (one G forward, no D grads in the G step);
  * ``minimal`` under torch.autocast(bf16): the fastest eager form of the same step, for
    comparison with bench.py's bf16 line.

It is a measurement, not a parity check (the parity tests live in test_gpu_step.py), and it
runs only with IRGAN_TIME_REFERENCE=1 so the default `pytest -m gpu` stays short.  Output:
one JSON line per form (profiles/r06_torch_reference_gpu.txt).
"""
import json
import os
import time

import pytest
import torch

pytestmark = pytest.mark.gpu
RUN = os.environ.get("IRGAN_TIME_REFERENCE") == "1"
B, H, W = 16, 256, 256
WARMUP, STEPS = 2, 6


def _time(as_written, bf16):
    from oracle import step as O
    dev = "cuda"
    G = {k: v.to(dev) for k, v in O.seeded_params(O.g_param_shapes(), 0).items()}
    D = {k: v.to(dev) for k, v in O.seeded_params(O.d_param_shapes(), 1).items()}
    V = {k: v.to(dev) for k, v in O.seeded_params(O.vgg_param_shapes(), 3, kaiming=True).items()}
    g = torch.Generator().manual_seed(7)
    ir = (torch.rand(B, 1, H, W, generator=g) * 2 - 1).to(dev)
    rgb = (torch.rand(B, 3, H, W, generator=g) * 2 - 1).to(dev)
    oG, oD = O.AdamState(G), O.AdamState(D)
    times = []
    for i in range(WARMUP + STEPS):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
            out = O.train_step(G, D, V, ir, rgb, oG, oD, as_written=as_written)
        torch.cuda.synchronize()
        if i >= WARMUP:
            times.append(time.perf_counter() - t0)
    assert torch.isfinite(out["loss_G"]).item() and torch.isfinite(out["loss_D"]).item()
    times.sort()
    med = times[len(times) // 2]
    return {"form": ("as_written" if as_written else "minimal") + (" bf16-autocast" if bf16 else " fp32"),
            "img_per_s": round(B / med, 2), "ms_per_step_median": round(med * 1e3, 2),
            "steps": STEPS, "batch": B, "size": f"{H}x{W}",
            "device": torch.cuda.get_device_name(0), "torch": torch.__version__,
            "peak_mem_gib": round(torch.cuda.max_memory_allocated() / 2**30, 2)}


@pytest.mark.skipif(not RUN, reason="timing only: set IRGAN_TIME_REFERENCE=1")
@pytest.mark.parametrize("as_written,bf16", [(True, False), (False, False), (False, True)])
def test_reference_step_eager_speed(as_written, bf16):
    torch.cuda.reset_peak_memory_stats()
    r = _time(as_written, bf16)
    print(json.dumps(r), flush=True)
