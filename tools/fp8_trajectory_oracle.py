"""Loss trajectories of the CPU oracle (oracle/step.py) in fp32 and in its fp8
restatement (the product's e4m3 recipe, oracle.step._Fp8ResConv / _Fp8ZeroConv), from the
same init on the same learnable synthetic pairs -- the CPU side of
tests/test_gpu_fp8.py::test_loss_trajectory_fast_dtypes (the reference's own runtime
signal is the per-epoch val-L1, ir:1521-1542, 1698-1703).

    python tools/fp8_trajectory_oracle.py [--steps 200] [--size 64] [--batch 4]

Prints per-20-step mean loss_G / L1 and the held-out val-L1 every 20 steps over the last
half, for fp32, fp8 and a chaos control: fp32 from the same init with its weights rounded
to bf16 (a perturbation at the bf16 rounding level -- how far two fp32 runs drift apart)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import step as O                     # noqa: E402
from tests.trajectory_data import learnable_pairs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    train, val = learnable_pairs(a.size, a.batch)
    res = {}
    for mode in ("fp32", "fp32-perturbed", "fp8"):
        G = O.seeded_params(O.g_param_shapes(), 1, bias_std=0.0)
        if mode == "fp32-perturbed":
            G = {k: v.bfloat16().float() for k, v in G.items()}
        D = O.seeded_params(O.d_param_shapes(), 2, bias_std=0.0)
        V = O.seeded_params(O.vgg_param_shapes(), 3, kaiming=True)
        oG, oD = O.AdamState(G), O.AdamState(D)
        lg, l1, vls = [], [], []
        f8 = mode == "fp8"
        for s in range(a.steps):
            ir, rgb = train[s % len(train)]
            o = O.train_step(G, D, V, ir, rgb, oG, oD, fp8=f8)
            lg.append(float(o["loss_G"]))
            l1.append(float(o["loss_G_L1"]) / 30.0)
            if (s + 1) % 20 == 0:
                msg = ""
                if s + 1 > a.steps // 2:
                    with torch.no_grad():
                        vls.append(sum(float((O.g_forward(G, vi, fp8=f8) - vr).abs().mean()) * vi.shape[0]
                                       for vi, vr in val) / sum(vi.shape[0] for vi, _ in val))
                    msg = f"  val-L1 {vls[-1]:.4f}"
                print(f"{mode} steps {s - 18:4d}-{s + 1:4d}: loss_G {sum(lg[-20:]) / 20:.4f}  "
                      f"L1 {sum(l1[-20:]) / 20:.4f}{msg}", flush=True)
        half = lg[a.steps // 2:]
        res[mode] = (sum(half) / len(half), sum(vls) / len(vls))
        print(f"{mode}: loss_G first {lg[0]:.4f}, mean over the last half {res[mode][0]:.4f}; "
              f"val-L1 mean of {len(vls)} evaluations {res[mode][1]:.4f}", flush=True)
    for m in ("fp32-perturbed", "fp8"):
        r = res[m][0] / res["fp32"][0] - 1, res[m][1] / res["fp32"][1] - 1
        print(f"{m} vs fp32: loss_G (last half) {r[0]:+.2%}, val-L1 (averaged) {r[1]:+.2%}")


if __name__ == "__main__":
    main()
