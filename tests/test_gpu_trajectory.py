"""Loss trajectories of the fast dtypes against the fp32 parity mode.

The reference's only runtime correctness signal is the per-epoch validation L1
(validate_kaist, ir:1521-1542, 1698-1703) and the logged loss_G / loss_D
(ir:1683-1694).  Single-step gradient comparisons at random init cannot hold the
bf16 / fp8 paths tightly (a ReLU-mask flip per perturbed element: the fp32
reference's own weight gradients move 0.17 rel-L2 when only its weights are
rounded to bf16, tools/fp8_drift_diag.py), so this test trains: 400 steps at 64x64,
B=4 on learnable synthetic pairs (tests/trajectory_data.py: IR = a smooth field,
RGB = a fixed colour map of it) from one seeded init, in compute_dtype "fp32",
"bf16" and "fp8", scoring held-out batches with validate_kaist every 20 steps over
the second half (a single val-L1 swings +-20 % between evaluations of one run: the
GAN's oscillation; averaged over 10, two fp32 runs from inits 2^-9 apart agree to 2 %,
profiles/r06_fp8_trajectory_oracle.txt).

Pass: loss_G falls in all three (second-half mean below 0.5x the first-20 mean); the
bf16 and fp8 second-half mean loss_G within TRAJ_BAND of fp32 mode's, their averaged
val-L1 at most (1 + TRAJ_BAND) x fp32 mode's (one-sided: lower is better) and above half of it.  CPU counterpart (the oracle's fp32 and fp8 restatement on the same data):
tools/fp8_trajectory_oracle.py, profiles/r06_fp8_trajectory_oracle.txt.
"""
import pytest
import torch

from conftest import pkg
from trajectory_data import learnable_pairs

pytestmark = pytest.mark.gpu
DEV = "cuda"
STEPS, SIZE, BATCH, EVAL_EVERY = 400, 64, 4, 20
TRAJ_BAND = 0.10   # relative to fp32 mode: second-half mean loss_G and averaged val-L1


def _trainer(dtype):
    from oracle import step as O
    irc = pkg()
    cfg = irc.Config()
    cfg.device = DEV
    cfg.compute_dtype = dtype
    cfg.batch_size = BATCH
    cfg.img_size = SIZE
    tr = irc.GANTrainer(cfg)
    tr.netG.store.load(O.seeded_params(O.g_param_shapes(), 1), strict=True)
    tr.netD.store.load(O.seeded_params(O.d_param_shapes(), 2), strict=True)
    tr.vgg.store.load(O.seeded_params(O.vgg_param_shapes(), 3, kaiming=True), strict=True)
    for m in (tr.netG, tr.netD, tr.vgg):
        m.repack()
    return tr


def _train(dtype, train, val):
    irc = pkg()
    tr = _trainer(dtype)
    vbatches = [{"ir": ir, "rgb": rgb} for ir, rgb in val]
    lg, vls = [], []
    for s in range(STEPS):
        ir, rgb = train[s % len(train)]
        lg.append(tr.losses(tr.step(ir.to(DEV), rgb.to(DEV)))["loss_G"])
        if s + 1 > STEPS // 2 and (s + 1) % EVAL_EVERY == 0:
            vls.append(irc.validate_kaist(tr.model, vbatches, DEV))
    assert all(torch.isfinite(torch.tensor(lg))), dtype
    half = lg[STEPS // 2:]
    return sum(lg[:20]) / 20, sum(half) / len(half), sum(vls) / len(vls)


def test_loss_trajectory_fast_dtypes():
    train, val = learnable_pairs(SIZE, BATCH)
    res = {dt: _train(dt, train, val) for dt in ("fp32", "bf16", "fp8")}
    for dt, (first, last, vl) in res.items():
        print(f"{dt}: loss_G first-20 {first:.4f} second-half {last:.4f}  val-L1 (mean of 10) {vl:.4f}")
    for dt, (first, last, vl) in res.items():
        assert last < 0.5 * first, (dt, first, last)
    _, last32, vl32 = res["fp32"]
    for dt in ("bf16", "fp8"):
        _, last, vl = res[dt]
        print(f"{dt} vs fp32: second-half loss_G {last / last32 - 1:+.2%}, val-L1 {vl / vl32 - 1:+.2%} "
              f"(band {TRAJ_BAND:.0%})")
        assert abs(last / last32 - 1) <= TRAJ_BAND, (dt, last, last32)
        # val-L1 is one-sided: the fast dtype must not train WORSE than fp32 by more than the
        # band (the GAN's run-to-run swing reaches 10 % either way; measured fp8 -10.4 %, i.e.
        # better, on one box), and stays within a factor 2 of it (a degenerate run fails)
        assert 0.5 * vl32 <= vl <= (1 + TRAJ_BAND) * vl32, (dt, vl, vl32)
