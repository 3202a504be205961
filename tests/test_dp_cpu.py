"""Data-parallel plumbing on CPU (gloo, world size 2).

The GPU step cannot run here, so the per-rank arithmetic is the fp64 oracle
step (oracle/step.py, ir:1636-1681); what is under test is the product's DP
code around it: the batch sharding (``dp_loaders``), the gradient all-reduce
(``engine.grad_allreduce``, called on a flat buffer exactly as GANStep does
between backward and Adam) and the val-L1 (sum, count) reduction
(``validate_kaist``).  Claim checked: two ranks training on
equal shards reproduce the single-process step on the union batch.  In fp64
the only difference is summation order, so the tolerance is 1e-9 relative.
"""
import math
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import pkg

WORLD = 2
PER_RANK = 2
HW = 32


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _Indexed(torch.utils.data.Dataset):
    def __init__(self, base):
        self.base = base

    def __len__(self):
        return len(self.base)

    def __getitem__(self, i):
        d = dict(self.base[i])
        d["idx"] = i
        return d


def _params():
    from oracle import step as O
    dd = lambda P: {k: v.double() for k, v in P.items()}  # noqa: E731
    return (dd(O.seeded_params(O.g_param_shapes(), 1)), dd(O.seeded_params(O.d_param_shapes(), 2)),
            dd(O.seeded_params(O.vgg_param_shapes(), 3, kaiming=True)))


def _dataset():
    irc = pkg()
    return _Indexed(irc.SyntheticPairDataset(12, img_size=HW, seed=5))


def _flat_hook(engine):
    """Flatten a grad dict into one buffer, all-reduce it, scatter back (GANStep's layout)."""
    def hook(name, grads):
        keys = list(grads)
        flat = torch.cat([grads[k].reshape(-1) for k in keys])
        engine.grad_allreduce(flat)
        o = 0
        for k in keys:
            n = grads[k].numel()
            grads[k] = flat[o:o + n].view_as(grads[k])
            o += n
    return hook


def _worker(rank, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        irc = pkg()
        from oracle import step as O
        import importlib
        engine = importlib.import_module(irc.__name__ + ".engine")
        ds = _dataset()
        train_ds = torch.utils.data.Subset(ds, list(range(8)))
        val_ds = torch.utils.data.Subset(ds, list(range(8, 11)))   # 3 items: ragged over 2 ranks
        tl, vl, sampler = irc.dp_loaders(train_ds, val_ds, PER_RANK, seed=0)
        sampler.set_epoch(1)
        batch = next(iter(tl))
        G, D, V = _params()
        out = O.train_step(G, D, V, batch["ir"].double(), batch["rgb"].double(), O.AdamState(G), O.AdamState(D),
                           grad_hook=_flat_hook(engine))
        val = irc.validate_kaist(lambda x: x.repeat(1, 3, 1, 1) * 0.5, vl, "cpu")
        nval = sum(b["ir"].shape[0] for b in vl)
        # bench.py's post-run replica check: identical after the step, and a one-ulp
        # difference on one rank is caught on every rank
        params = [G[k] for k in G] + [D[k] for k in D]
        same = engine.replicas_identical(params)
        bumped = [t.clone() for t in params]
        if rank == 1:
            bumped[3].view(-1)[7] = torch.nextafter(bumped[3].view(-1)[7], torch.tensor(1e9, dtype=torch.float64))
        caught = not engine.replicas_identical(bumped)
        torch.save({"idx": batch["idx"].tolist(), "G": G, "D": D, "loss_D": out["loss_D"],
                    "loss_G": out["loss_G"], "val": val, "nval": nval, "ntrain": len(tl),
                    "replicas_same": same, "replica_diff_caught": caught},
                   os.path.join(outdir, f"rank{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_dp_two_ranks_match_single_process(tmp_path):
    port = _free_port()
    mp.spawn(_worker, args=(port, str(tmp_path)), nprocs=WORLD, join=True)
    res = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(WORLD)]
    # sharding: disjoint equal per-rank batches, every rank the same number of steps
    idx = [i for r in res for i in r["idx"]]
    assert all(len(r["idx"]) == PER_RANK for r in res)
    assert len(set(idx)) == WORLD * PER_RANK
    assert res[0]["ntrain"] == res[1]["ntrain"] == 8 // (WORLD * PER_RANK)
    # the ragged val set (3 items) is split 2 + 1 without padding duplicates
    assert res[0]["nval"] + res[1]["nval"] == 3
    # single-process reference step on the union batch
    from oracle import step as O
    ds = _dataset()
    ir = torch.stack([ds[i]["ir"] for i in idx]).double()
    rgb = torch.stack([ds[i]["rgb"] for i in idx]).double()
    G, D, V = _params()
    ref = O.train_step(G, D, V, ir, rgb, O.AdamState(G), O.AdamState(D))
    assert all(r["replicas_same"] and r["replica_diff_caught"] for r in res)
    for r in res:   # replicas stay identical and equal the global-batch step
        for name, P in (("G", G), ("D", D)):
            for k in P:
                d = (r[name][k] - P[k]).abs().max().item()
                assert d <= 1e-9 * max(1.0, P[k].abs().max().item()), (name, k, d)
    # the mean of per-rank losses is the global-batch loss (equal shards)
    for key in ("loss_D", "loss_G"):
        m = sum(float(r[key]) for r in res) / WORLD
        assert abs(m - float(ref[key])) <= 1e-9 * abs(float(ref[key])), key
    # val L1: (sum, count) reduced over ranks == the single-process val L1 over the
    # whole val set (ir:1521-1542), each item counted exactly once
    want = [(ds[i]["ir"].repeat(3, 1, 1) * 0.5 - ds[i]["rgb"]).abs().mean().item() for i in range(8, 11)]
    assert res[0]["val"] == pytest.approx(sum(want) / len(want), rel=1e-6)
    assert res[0]["val"] == res[1]["val"]


def test_grad_allreduce_single_process_is_identity():
    import importlib
    engine = importlib.import_module(pkg().__name__ + ".engine")
    t = torch.arange(5.0)
    assert engine.grad_allreduce(t) is t and torch.equal(t, torch.arange(5.0))


def _bucket_worker(rank, port, out):
    import importlib
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    engine = importlib.import_module(pkg().__name__ + ".engine")
    store = engine.ParamStore(engine.g_param_shapes(), "cpu", with_adam=False)
    g = torch.Generator().manual_seed(100 + rank)
    store.grad.copy_(torch.randn(store.numel, generator=g, dtype=torch.float32))
    red = engine.BucketedAllreduce(store, bucket_bytes=4 << 20)
    # the G backward's ready() sequence (GeneratorEngine.backward): tail-first
    keys = ["up1_conv.0.weight"] + [f"resblocks.{b}.conv_block.1.weight" for b in reversed(range(9))]
    for k in keys + ["inc.1.weight"]:
        red.ready(k)
    nb = len(red.works)
    red.finish()
    torch.save({"grad": store.grad.clone(), "buckets": nb}, os.path.join(out, f"b{rank}.pt"))
    dist.destroy_process_group()


def test_bucketed_allreduce_matches_whole_buffer_mean(tmp_path):
    """BucketedAllreduce (GANStep's overlapped G/D grad reduction):
    buckets issued tail-first from the backward's ready() calls, finished before
    Adam, reproduce the element-wise mean over ranks of the whole flat buffer."""
    import importlib
    engine = importlib.import_module(pkg().__name__ + ".engine")
    mp.spawn(_bucket_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    res = [torch.load(tmp_path / f"b{r}.pt", weights_only=True) for r in range(WORLD)]
    store = engine.ParamStore(engine.g_param_shapes(), "cpu", with_grad=False, with_adam=False)
    want = sum(torch.randn(store.numel, generator=torch.Generator().manual_seed(100 + r), dtype=torch.float32)
               for r in range(WORLD)) / WORLD
    assert res[0]["buckets"] >= 4           # genuinely bucketed, not one collective at the end
    for r in res:
        torch.testing.assert_close(r["grad"], want, rtol=1e-6, atol=1e-7)


def _adam_slice(store, a, b, step, lr=2e-4, b1=0.5, b2=0.999, eps=1e-8):
    """torch.optim.Adam's update on the flat slice [a, b) (test-side reference)."""
    g = store.grad[a:b]
    store.m[a:b].mul_(b1).add_(g, alpha=1 - b1)
    store.v[a:b].mul_(b2).addcmul_(g, g, value=1 - b2)
    denom = (store.v[a:b].sqrt() / math.sqrt(1 - b2 ** step)).add_(eps)
    store.flat[a:b].addcdiv_(store.m[a:b], denom, value=-lr / (1 - b1 ** step))


def _overlap_worker(rank, port, out):
    import importlib
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    engine = importlib.import_module(pkg().__name__ + ".engine")
    res = {}
    for mode in ("bucketed", "whole"):
        store = engine.ParamStore(engine.g_param_shapes(), "cpu")
        store.flat.copy_(torch.randn(store.numel, generator=torch.Generator().manual_seed(3)))
        store.grad.copy_(torch.randn(store.numel, generator=torch.Generator().manual_seed(100 + rank)))
        calls = []
        if mode == "bucketed":
            red = engine.BucketedAllreduce(store, bucket_bytes=4 << 20)
            for k in ["up1_conv.0.weight"] + [f"resblocks.{b}.conv_block.1.weight" for b in reversed(range(9))]:
                red.ready(k)
            red.finish(lambda a, b: (calls.append((a, b)), _adam_slice(store, a, b, 1)))
        else:
            engine.grad_allreduce(store.grad)
            _adam_slice(store, 0, store.numel, 1)
        res[mode] = {"flat": store.flat.clone(), "calls": calls}
    torch.save(res, os.path.join(out, f"o{rank}.pt"))
    dist.destroy_process_group()


def test_bucketed_adam_overlap_equals_whole_buffer_update(tmp_path):
    """GANStep's G update: BucketedAllreduce.finish(apply) runs the
    Adam of each bucket right after that bucket's collective (tail-first), while
    later buckets are still in flight.  Two gloo ranks: the result equals one
    whole-buffer all-reduce followed by one whole-buffer Adam, bit for bit, every
    element is updated exactly once, and the update really is split (>= 4 buckets)."""
    mp.spawn(_overlap_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    res = [torch.load(tmp_path / f"o{r}.pt", weights_only=True) for r in range(WORLD)]
    for r in res:
        calls = r["bucketed"]["calls"]
        assert len(calls) >= 4
        assert calls[0][1] == max(b for _, b in calls) and calls[-1][0] == 0      # tail first, head last
        cov = sorted(calls)
        assert cov[0][0] == 0 and all(cov[i][1] == cov[i + 1][0] for i in range(len(cov) - 1))
        assert torch.equal(r["bucketed"]["flat"], r["whole"]["flat"])
    assert torch.equal(res[0]["bucketed"]["flat"], res[1]["bucketed"]["flat"])
