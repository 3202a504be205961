"""Where the fp8 step's ResnetBlock weight-gradient drift comes from.

Runs the CPU oracle's train step (oracle/step.py, fp32) once unquantised and once per
quantisation variant of the ResnetBlock / down2 / up1_conv convs, and prints the worst and
mean rel-L2 of the 18 ResnetBlock weight gradients against the unquantised step, plus the
mean |delta| of the G output.  Variants:

  product recipe        the fp8 restatement (oracle.step._Fp8ResConv / _Fp8ZeroConv): e4m3
                        x, w (forward + backward) and dY, per-tensor power-of-two scales
  bf16 weights only     no fp8 at all: only the conv weights rounded to bf16 (the floor)
  fwd only / x / w      e4m3 on the forward operands only (dY unquantised)
  dY only (...)         e4m3 on dY only: per-tensor, per-(n, c) scales, or e5m2
  fwd block-32          x and w with one power-of-two scale per 32 K-elements (the
                        E8M0 block scales mfma_scale_f32_32x32x64_f8f6f4 takes)
  bf16 autocast         the unquantised step under torch.autocast(bf16)

    python tools/fp8_drift_diag.py [--size 64] [--data random|learnable]

No GPU, no product code: test/measurement infrastructure over the oracle only."""
import argparse
import math
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import step as O                  # noqa: E402
from tests.trajectory_data import pair        # noqa: E402

E4M3, E5M2 = (torch.float8_e4m3fn, 448.0), (torch.float8_e5m2, 57344.0)


def q_tensor(t, fmt=E4M3):
    a = float(t.detach().abs().max())
    q = 2.0 ** math.floor(math.log2(fmt[1] / a)) if a > 0 else 1.0
    return (t.detach() * q).clamp(-fmt[1], fmt[1]).to(fmt[0]).to(t.dtype) / q


def q_nc(t, fmt=E4M3):
    """one power-of-two scale per (n, c) plane (per output channel for a weight)"""
    a = t.detach().abs().amax(dim=(2, 3), keepdim=True).clamp_min(1e-30)
    q = torch.exp2(torch.floor(torch.log2(fmt[1] / a)))
    return (t.detach() * q).clamp(-fmt[1], fmt[1]).to(fmt[0]).to(t.dtype) / q


def q_block32(t, fmt=E4M3):
    """one power-of-two scale per 32 consecutive channels at each (n, y, x) / (co, ky, kx):
    the conv's K blocks (E8M0 block scales)"""
    n, c, h, w = t.shape
    if c % 32:
        return q_tensor(t, fmt)
    v = t.detach().reshape(n, c // 32, 32, h, w)
    a = v.abs().amax(dim=2, keepdim=True).clamp_min(1e-30)
    q = torch.exp2(torch.floor(torch.log2(fmt[1] / a)))
    return ((v * q).clamp(-fmt[1], fmt[1]).to(fmt[0]).to(t.dtype) / q).reshape(n, c, h, w)


def ident(t):
    return t.detach()


def variant(qx, qw, qg):
    """_Fp8ResConv / _Fp8ZeroConv with the three quantisers swapped in."""
    class R(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, w, b):
            wb = w.to(torch.bfloat16).to(w.dtype)
            ctx.save_for_backward(x, w, wb)
            return F.conv2d(O._rpad(qx(x), 1), qw(wb), b)

        @staticmethod
        def backward(ctx, gy):
            x, w, wb = ctx.saved_tensors
            gq = qg(gy)
            dw = torch.nn.grad.conv2d_weight(O._rpad(qx(x).float(), 1), w.shape, gq.float())
            H, W = x.shape[-2:]
            xp = torch.zeros(x.shape[0], x.shape[1], H + 2, W + 2, dtype=x.dtype)
            g8 = torch.nn.grad.conv2d_input(xp.shape, qw(wb), gq)
            gb = torch.nn.grad.conv2d_input(xp.shape, wb, gy)
            xf = torch.zeros_like(x, requires_grad=True)
            with torch.enable_grad():
                ring = torch.autograd.grad(O._rpad(xf, 1), xf, gb)[0] - gb[..., 1:-1, 1:-1]
            return g8[..., 1:-1, 1:-1] + ring, dw, gy.sum(dim=(0, 2, 3))

    class Z(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, w, b):
            wb = w.to(torch.bfloat16).to(w.dtype)
            ctx.save_for_backward(x, w, wb)
            return F.conv2d(qx(x), qw(wb), b, padding=1)

        @staticmethod
        def backward(ctx, gy):
            x, w, wb = ctx.saved_tensors
            gq = qg(gy)
            dw = torch.nn.grad.conv2d_weight(qx(x).float(), w.shape, gq.float(), padding=1)
            dx = torch.nn.grad.conv2d_input(x.shape, qw(wb), gq, padding=1)
            return dx, dw, gy.sum(dim=(0, 2, 3))
    return R, Z


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--data", default="random", choices=["random", "learnable"])
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    g = torch.Generator().manual_seed(41)
    if a.data == "random":   # tests/test_gpu_fp8.py::test_fp8_step_vs_fp8_oracle's inputs
        ir = torch.rand(a.batch, 1, a.size, a.size, generator=g) * 2 - 1
        rgb = torch.rand(a.batch, 3, a.size, a.size, generator=g) * 2 - 1
    else:
        ir, rgb = pair(g, a.batch, a.size)

    def run(fp8):
        G = O.seeded_params(O.g_param_shapes(), 1, bias_std=0.02)
        D = O.seeded_params(O.d_param_shapes(), 2, bias_std=0.02)
        V = O.seeded_params(O.vgg_param_shapes(), 3, kaiming=True)
        return O.train_step(G, D, V, ir, rgb, O.AdamState(G), O.AdamState(D), fp8=fp8)

    base = run(False)
    print(f"ResnetBlock dW rel-L2 vs the unquantised oracle step ({a.size}x{a.size}, B={a.batch}, {a.data} data)")

    def report(tag, o):
        errs, coss, rats = [], [], []
        for k, gr in base["gradG"].items():
            if "resblocks" in k and k.endswith(".weight"):
                d, r = o["gradG"][k].double().flatten(), gr.double().flatten()
                errs.append(float((d - r).norm() / r.norm()))
                coss.append(float(d @ r / (d.norm() * r.norm())))
                rats.append(float(d.norm() / r.norm()))
        fe = (o["fake"] - base["fake"]).abs().mean().item()
        print(f"  {tag:24s} G out mean|d| {fe:.4f}   dW rel-L2 worst {max(errs):.3f} mean "
              f"{sum(errs) / len(errs):.3f}   cosine min {min(coss):.3f}   |dW| ratio "
              f"{min(rats):.3f}-{max(rats):.3f}", flush=True)

    R0, Z0 = O._Fp8ResConv, O._Fp8ZeroConv

    def runv(tag, qx, qw, qg):
        O._Fp8ResConv, O._Fp8ZeroConv = variant(qx, qw, qg)
        try:
            report(tag, run(True))
        finally:
            O._Fp8ResConv, O._Fp8ZeroConv = R0, Z0

    report("product recipe", run(True))
    runv("bf16 weights only", ident, ident, ident)
    runv("fwd only (x, w)", q_tensor, q_tensor, ident)
    runv("x only", q_tensor, ident, ident)
    runv("w only", ident, q_tensor, ident)
    runv("dY only", ident, ident, q_tensor)
    runv("dY only, per-(n,c)", ident, ident, q_nc)
    runv("dY only, e5m2", ident, ident, lambda t: q_tensor(t, E5M2))
    runv("fwd block-32, dY", q_block32, q_block32, q_tensor)
    runv("all, dY per-(n,c)", q_tensor, q_tensor, q_nc)
    runv("all, dY e5m2", q_tensor, q_tensor, lambda t: q_tensor(t, E5M2))
    with torch.autocast("cpu", dtype=torch.bfloat16):
        report("bf16 autocast, no fp8", run(False))


if __name__ == "__main__":
    main()
