"""Data-parallel fused step on the GPU: two ranks, one MI355X, gloo collectives; and the
RCCL branch at world size 1 with the collectives forced on.

RCCL cannot place two ranks on one device, so the ranks use gloo on device
tensors; what runs is the product's whole DP step (GANStep with the default
process group): D grads reduced asynchronously while the L1/VGG/TV/SSIM
terms run, G grads reduced tail-first in buckets during the G backward
(engine.BucketedAllreduce).  Claims checked:
  * both replicas hold bit-identical parameters after the step;
  * the reduced grads equal the single-process union-batch grads (fp32,
    summation order only: 1e-3 of each tensor's max-abs);
  * the mean of per-rank losses equals the union-batch loss.
"""
import os
import socket

import pytest
import torch

from conftest import pkg

pytestmark = pytest.mark.gpu

WORLD, PER_RANK, HW = 2, 2, 32


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _trainer(irc, dtype="fp32", force_reduce=False, deterministic=False):
    from oracle import step as O
    cfg = irc.Config()
    cfg.device = "cuda:0"
    cfg.compute_dtype = dtype
    cfg.deterministic = deterministic
    tr = irc.GANTrainer(cfg, force_reduce=force_reduce)
    tr.netG.store.load(O.seeded_params(O.g_param_shapes(), 1, bias_std=0.02), strict=True)
    tr.netD.store.load(O.seeded_params(O.d_param_shapes(), 2, bias_std=0.02), strict=True)
    tr.vgg.store.load(O.seeded_params(O.vgg_param_shapes(), 3, kaiming=True), strict=True)
    for net in (tr.netG, tr.netD, tr.vgg):
        net.repack()
    return tr


def _data():
    g = torch.Generator().manual_seed(11)
    ir = torch.rand(WORLD * PER_RANK, 1, HW, HW, generator=g) * 2 - 1
    rgb = torch.rand(WORLD * PER_RANK, 3, HW, HW, generator=g) * 2 - 1
    return ir, rgb


def _worker(rank, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    irc = pkg()
    tr = _trainer(irc)
    ir, rgb = _data()
    sl = slice(rank * PER_RANK, (rank + 1) * PER_RANK)
    L = tr.losses(tr.step(ir[sl].cuda(), rgb[sl].cuda()))
    torch.cuda.synchronize()
    s = tr.core
    torch.save({"G": s.G.flat.cpu(), "D": s.D.flat.cpu(), "gG": s.G.grad.cpu(), "gD": s.D.grad.cpu(),
                "L": L}, os.path.join(out, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _close(a, b, name):
    tol = 1e-3 * max(b.abs().max().item(), 1e-12)
    d = (a - b).abs().max().item()
    assert d <= tol, (name, d, tol)


def test_dp_step_two_ranks_matches_union_batch(tmp_path):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    r = [torch.load(tmp_path / f"r{k}.pt", weights_only=True) for k in range(WORLD)]
    assert torch.equal(r[0]["G"], r[1]["G"]) and torch.equal(r[0]["D"], r[1]["D"])
    tr = _trainer(pkg())
    ir, rgb = _data()
    L = tr.losses(tr.step(ir.cuda(), rgb.cuda()))
    s = tr.core
    for name, ref, got in (("G", s.G, r[0]["gG"]), ("D", s.D, r[0]["gD"])):
        for k in ref.shapes:
            _close(ref.krsc(k, got), ref.krsc(k, ref.grad).cpu(), (name, k))
    for k in ("loss_D", "loss_G", "loss_G_L1", "loss_G_perc", "loss_G_ssim"):
        m = sum(x["L"][k] for x in r) / WORLD
        assert abs(m - L[k]) <= 1e-4 * max(1.0, abs(L[k])), (k, m, L[k])


def _rccl_worker(rank, store, out, dtype):
    """World size 1 over RCCL ("nccl"), the gradient collectives forced on: the step issues
    real ReduceOp.AVG async all-reduces (the D grads on the side stream, the G grads in
    8 MB tail-first buckets under the G backward, each bucket's Adam right after it), and
    the post-run replica digest runs its MAX / MIN all-reduces on the device."""
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"file://{store}", rank=0, world_size=1,
                           device_id=torch.device("cuda", 0))
    irc = pkg()
    res = {}
    for force in (True, False):
        tr = _trainer(irc, dtype, force_reduce=force, deterministic=True)
        core = tr.core
        assert core.g_reduce.active == force and core.d_reduce.active == force
        assert core.g_reduce.avg, "RCCL averages natively (ReduceOp.AVG)"
        g = torch.Generator().manual_seed(5)
        for _ in range(2):
            ir = (torch.rand(2, 1, 64, 64, generator=g) * 2 - 1).cuda()
            rgb = (torch.rand(2, 3, 64, 64, generator=g) * 2 - 1).cuda()
            L = tr.losses(tr.step(ir, rgb))
        torch.cuda.synchronize()
        assert irc.engine.replicas_identical([core.G.flat, core.D.flat], force=True)
        res[force] = {"G": core.G.flat.cpu(), "D": core.D.flat.cpu(), "gG": core.G.grad.cpu(),
                      "gD": core.D.grad.cpu(), "L": L}
    torch.save(res, os.path.join(out, "rccl.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_rccl_world1_forced_collectives_bit_identical(tmp_path, dtype):
    """The RCCL branch of the DP step (ReduceOp.AVG on the side stream and under the G
    backward, per-bucket Adam, the device-side replica check) on one MI355X: at world size
    1 the mean over ranks is the identity, so two steps with the collectives forced on
    equal two steps without them bit for bit (deterministic mode: ordered weight-gradient
    reductions, so the stream schedule cannot move a bit)."""
    import torch.multiprocessing as mp
    mp.spawn(_rccl_worker, args=(str(tmp_path / "store"), str(tmp_path), dtype), nprocs=1, join=True)
    r = torch.load(tmp_path / "rccl.pt", weights_only=True)
    for k in ("G", "D", "gG", "gD"):
        assert torch.equal(r[True][k], r[False][k]), k
    for k, v in r[False]["L"].items():   # loss VALUES are fp64 atomic block sums (they feed no gradient)
        assert abs(r[True]["L"][k] - v) <= 1e-12 * max(1.0, abs(v)), (k, r[True]["L"][k], v)
