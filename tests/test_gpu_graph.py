"""The train step captured as one HIP graph (GANStep._graph_step) against the eager step.

With the whole step in a graph, the host no longer feeds the two streams launch by
launch; what differs from eager is only WHEN kernels are issued.  In deterministic mode
(ops.set_deterministic) every kernel is run-to-run reproducible, so graph replays must
give bit-identical losses-to-1e-12, grads, parameters and Adam moments to eager steps
(the default; IRGAN_GRAPH=1 turns the graph on) -- including across a learning-rate
change (re-capture) and across a checkpoint save / load in the middle of a run (the Adam
step count lives on the device and is resynced from the loaded state)."""
import pytest
import torch

from conftest import load_golden, pkg
from test_gpu_step import make_trainer

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _batches(n, size=128, seed=61):
    g = torch.Generator().manual_seed(seed)
    return [((torch.rand(2, 1, size, size, generator=g) * 2 - 1).to(DEV),
             (torch.rand(2, 3, size, size, generator=g) * 2 - 1).to(DEV)) for _ in range(n)]


def _same(ta, tb, what):
    for name in ("netG", "netD"):
        sa, sb = getattr(ta, name).store, getattr(tb, name).store
        assert torch.equal(sa.grad, sb.grad), f"{what}: {name} grads differ"
        assert torch.equal(sa.flat, sb.flat), f"{what}: {name} params differ"
        assert torch.equal(sa.m, sb.m) and torch.equal(sa.v, sb.v), f"{what}: {name} Adam moments differ"
        assert sa.step_count == sb.step_count, what


def _run(monkeypatch, graph, batches, lr_change_after=None):
    if graph:
        monkeypatch.setenv("IRGAN_GRAPH", "1")
    else:
        monkeypatch.delenv("IRGAN_GRAPH", raising=False)
    tr, _ = make_trainer(load_golden("s64"), "bf16")
    losses, captures, last = [], 0, None
    for i, (ir, rgb) in enumerate(batches):
        losses.append(tr.losses(tr.step(ir, rgb)))
        if tr.core._graph is not None and tr.core._graph is not last:
            captures += 1
            last = tr.core._graph
        if lr_change_after is not None and i == lr_change_after:
            tr.scheduler_step()
            tr.core.lr_scale = 0.5   # a visible change (the default schedule keeps 1.0 early)
    torch.cuda.synchronize()
    return tr, losses, captures


def test_graph_replay_bit_identical_to_eager(monkeypatch):
    ops = pkg().ops
    batches = _batches(5)
    old = ops.set_deterministic(True)
    try:
        tg, lg, caps = _run(monkeypatch, True, batches, lr_change_after=2)
        te, le, caps_e = _run(monkeypatch, False, batches, lr_change_after=2)
    finally:
        ops.set_deterministic(old)
    assert caps_e == 0 and caps == 2, (caps, caps_e)   # steps 2-3 in one graph, 4-5 in the re-capture
    for x, y in zip(lg, le):
        for k in x:
            assert abs(x[k] - y[k]) <= 1e-12 * max(1.0, abs(y[k])), (k, x[k], y[k])
    _same(tg, te, "graph vs eager")


def test_graph_resume_from_checkpoint(monkeypatch, tmp_path):
    """4 graph steps in one run == 2 graph steps, checkpoint, a fresh trainer that loads it
    and runs 2 more graph steps: the device step count follows the loaded Adam state."""
    ops = pkg().ops
    monkeypatch.setenv("IRGAN_GRAPH", "1")
    batches = _batches(4, seed=62)
    old = ops.set_deterministic(True)
    try:
        ta, _, caps = _run(monkeypatch, True, batches)
        assert caps == 1
        tb, _, _ = _run(monkeypatch, True, batches[:2])
        path = tmp_path / "ck.pt"
        tb.save_checkpoint(str(path))
        tc, _ = make_trainer(load_golden("s64"), "bf16")
        tc.load_checkpoint(str(path))
        for ir, rgb in batches[2:]:
            tc.step(ir, rgb)
        torch.cuda.synchronize()
    finally:
        ops.set_deterministic(old)
    _same(ta, tc, "resumed graph run")
