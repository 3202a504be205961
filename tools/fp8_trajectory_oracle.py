"""Loss trajectories of the CPU oracle (oracle/step.py) in fp32 and in its fp8
restatement (the product's e4m3 recipe, oracle.step._Fp8ResConv / _Fp8ZeroConv), from the
same init on the same learnable synthetic pairs -- the CPU side of
tests/test_gpu_fp8.py::test_loss_trajectory_fast_dtypes (the reference's own runtime
signal is the per-epoch val-L1, ir:1521-1542, 1698-1703).

    python tools/fp8_trajectory_oracle.py [--steps 200] [--size 64] [--batch 4]

Prints per-20-step mean loss_G / L1 for both and the held-out val-L1 at the end."""
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
    for mode in ("fp32", "fp8"):
        G = O.seeded_params(O.g_param_shapes(), 1, bias_std=0.0)
        D = O.seeded_params(O.d_param_shapes(), 2, bias_std=0.0)
        V = O.seeded_params(O.vgg_param_shapes(), 3, kaiming=True)
        oG, oD = O.AdamState(G), O.AdamState(D)
        lg, l1 = [], []
        for s in range(a.steps):
            ir, rgb = train[s % len(train)]
            o = O.train_step(G, D, V, ir, rgb, oG, oD, fp8=(mode == "fp8"))
            lg.append(float(o["loss_G"]))
            l1.append(float(o["loss_G_L1"]) / 30.0)
            if (s + 1) % 20 == 0:
                print(f"{mode} steps {s - 18:4d}-{s + 1:4d}: loss_G {sum(lg[-20:]) / 20:.4f}  "
                      f"L1 {sum(l1[-20:]) / 20:.4f}", flush=True)
        with torch.no_grad():
            vl = sum(float((O.g_forward(G, ir, fp8=(mode == "fp8")) - rgb).abs().mean()) * ir.shape[0]
                     for ir, rgb in val) / sum(ir.shape[0] for ir, _ in val)
        res[mode] = (sum(lg[-20:]) / 20, vl, lg[0])
        print(f"{mode}: first loss_G {lg[0]:.4f}  last-20 mean loss_G {res[mode][0]:.4f}  val-L1 {vl:.4f}",
              flush=True)
    r = res["fp8"][0] / res["fp32"][0] - 1, res["fp8"][1] / res["fp32"][1] - 1
    print(f"fp8 vs fp32: last-20 loss_G {r[0]:+.2%}, val-L1 {r[1]:+.2%}")


if __name__ == "__main__":
    main()
