"""Golden vectors for the reference's NON-DEFAULT module options, by EXECUTING THE
REFERENCE in the build container (same loader as make_golden.py):

    python tests/golden/make_module_golden.py

* ResnetUNetGenerator with norm 'none' (get_norm_layer('none'): Identity norms and no
  conv biases, ir:154-165, 450-455), ResnetBlock padding 'replicate' / 'zero'
  (ir:375-411), use_dropout=True in eval mode (the module layout with the Dropout, which
  is then inactive), and a norm 'none' + zero-padding + ConvTranspose2d variant;
* NLayerDiscriminator with n_layers 1 / 2 / 4 and with norm 'none' (ir:576-635);
* ssim_loss_torch with window_size 3 / 5 / 7, size_average True / False (ir:714-750).

Every case runs in fp64 on seeded inputs and weights (oracle.seeded_params, so the
tests rebuild the same weights from the seeds) and stores the module output and the
gradients of the scalar objective sum(out * R) (R seeded): parameter gradients as
sampled digests (64 entries + the norm per tensor), D / SSIM input gradients in full.
Output: tests/golden/modules.npz.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, HERE)
from make_golden import load_reference  # noqa: E402
from oracle import step as O  # noqa: E402

N_SAMPLES = 64
G_CASES = {
    # name: (norm, padding_type, use_dropout, no_antialias_up)
    "g_none": ("none", "reflect", False, False),
    "g_replicate": ("instance", "replicate", False, False),
    "g_zero": ("instance", "zero", False, False),
    "g_dropout_eval": ("instance", "reflect", True, False),
    "g_none_zero_up": ("none", "zero", False, True),
}
D_CASES = {"d_n1": (1, "instance"), "d_n2": (2, "instance"), "d_n4": (4, "instance"), "d_none": (3, "none")}
SSIM_WINDOWS = (3, 5, 7)


def main():
    R = load_reference()
    rec = {}
    gen = torch.Generator().manual_seed(5)
    x = torch.rand(2, 1, 32, 32, generator=gen, dtype=torch.float64) * 2 - 1
    rec["g_x"] = x.numpy()
    for name, (norm, pad, drop, noaaup) in G_CASES.items():
        G = R.ResnetUNetGenerator(1, 3, 64, norm_layer=R.get_norm_layer(norm), use_dropout=drop, n_blocks=9,
                                  padding_type=pad, no_antialias=False, no_antialias_up=noaaup).double()
        shapes = O.g_param_shapes(no_antialias_up=noaaup, use_bias=norm == "instance", padding_type=pad,
                                  use_dropout=drop)
        sd = {k: v.double() for k, v in O.seeded_params(shapes, 1, bias_std=0.02).items()}
        assert list(G.state_dict().keys()) == list(shapes.keys()), name
        G.load_state_dict(sd, strict=True)
        G.eval() if drop else G.train()   # dropout layer present but inactive (eval); IN has no running stats
        out, _ = G(x)
        Rw = torch.randn(out.shape, generator=torch.Generator().manual_seed(11), dtype=torch.float64)
        (out * Rw).sum().backward()
        rec[f"{name}|out"] = out.detach().numpy()
        g = torch.Generator().manual_seed(99)
        for k, p in G.named_parameters():
            flat = p.grad.reshape(-1)
            idx = torch.randint(0, flat.numel(), (min(N_SAMPLES, flat.numel()),), generator=g)
            rec[f"{name}|{k}|idx"] = idx.numpy().astype(np.int64)
            rec[f"{name}|{k}|val"] = flat[idx].numpy()
            rec[f"{name}|{k}|norm"] = np.float64(flat.norm())
        print(name, "out", float(out.detach().abs().mean()))
    for name, (nl, norm) in D_CASES.items():
        D = R.NLayerDiscriminator(4, 64, n_layers=nl, norm_layer=R.get_norm_layer(norm)).double()
        shapes = O.d_param_shapes(4, 64, nl, use_bias=norm == "instance")
        assert list(D.state_dict().keys()) == list(shapes.keys()), name
        D.load_state_dict({k: v.double() for k, v in O.seeded_params(shapes, 2, bias_std=0.02).items()}, strict=True)
        xd = (torch.rand(2, 4, 64, 64, generator=torch.Generator().manual_seed(6), dtype=torch.float64) * 2 - 1)
        xd.requires_grad_(True)
        out = D(xd)
        Rw = torch.randn(out.shape, generator=torch.Generator().manual_seed(12), dtype=torch.float64)
        (out * Rw).sum().backward()
        rec["d_x"] = xd.detach().numpy()   # the same seeded input for every case
        rec[f"{name}|out"] = out.detach().numpy()
        rec[f"{name}|dx"] = xd.grad.numpy()
        g = torch.Generator().manual_seed(98)
        for k, p in D.named_parameters():
            flat = p.grad.reshape(-1)
            idx = torch.randint(0, flat.numel(), (min(N_SAMPLES, flat.numel()),), generator=g)
            rec[f"{name}|{k}|idx"] = idx.numpy().astype(np.int64)
            rec[f"{name}|{k}|val"] = flat[idx].numpy()
            rec[f"{name}|{k}|norm"] = np.float64(flat.norm())
        print(name, "out", tuple(out.shape))
    a = torch.rand(2, 3, 40, 36, generator=torch.Generator().manual_seed(7), dtype=torch.float64)
    b = torch.rand(2, 3, 40, 36, generator=torch.Generator().manual_seed(8), dtype=torch.float64)
    rec["ssim_a"], rec["ssim_b"] = a.numpy(), b.numpy()
    for ws in SSIM_WINDOWS:
        for avg in (True, False):
            aa = a.clone().requires_grad_(True)
            loss = R.ssim_loss_torch(aa, b, window_size=ws, size_average=avg)
            w = torch.arange(1, loss.numel() + 1, dtype=torch.float64).reshape(loss.shape)
            (loss * w).sum().backward()
            rec[f"ssim{ws}_{int(avg)}|loss"] = loss.detach().numpy()
            rec[f"ssim{ws}_{int(avg)}|grad"] = aa.grad.numpy()
    out = os.path.join(HERE, "modules.npz")
    np.savez_compressed(out, **rec)
    print("wrote", out, os.path.getsize(out), "bytes")


if __name__ == "__main__":
    main()
