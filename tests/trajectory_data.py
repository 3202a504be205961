"""Learnable synthetic IR/RGB pairs for the loss-trajectory checks (the reference trains
on KAIST pairs, ir:1045-1177, absent offline): IR = a smooth random field in [-1, 1]
(bicubic up-sampling of an 8x coarser uniform grid), RGB = a fixed per-channel colour map
of it, tanh(a_c * ir + b_c) -- a pair a generator can learn, unlike independent U(-1, 1)
noise.  Deterministic (seeded), CPU tensors (B, 1, H, W) / (B, 3, H, W)."""
import torch
import torch.nn.functional as F

COLOUR_A = (1.5, -0.8, 0.6)
COLOUR_B = (0.2, 0.1, -0.3)


def pair(g, batch, size):
    lo = torch.rand(batch, 1, max(2, size // 8), max(2, size // 8), generator=g) * 2 - 1
    ir = F.interpolate(lo, size=(size, size), mode="bicubic", align_corners=False).clamp(-1, 1)
    a = torch.tensor(COLOUR_A).view(1, 3, 1, 1)
    b = torch.tensor(COLOUR_B).view(1, 3, 1, 1)
    return ir.contiguous(), torch.tanh(a * ir + b).contiguous()


def learnable_pairs(size=64, batch=4, n_train=16, n_val=2, seed=2024):
    """n_train training batches (cycled by the caller) and n_val held-out batches."""
    g = torch.Generator().manual_seed(seed)
    train = [pair(g, batch, size) for _ in range(n_train)]
    val = [pair(g, batch, size) for _ in range(n_val)]
    return train, val
