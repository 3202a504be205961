"""GAN train-step throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--size 256] [--batch 16]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

A step = the fused HIP train step (G forward, D fwd/bwd on [real; fake], D
Adam, D fwd/bwd on fake, VGG/L1/TV/SSIM losses, G backward, G Adam) on one
synthetic 256x256 batch of 16 IR/RGB pairs per GPU, bf16 operands with fp32
accumulation, random-init weights of the reference architecture.  Weak scaling:
every rank trains on its own 16-pair shard and all-reduces grads (RCCL).

Prints ONE JSON line (rank 0) with the metric, a live roofline for the dominant
conv kernel (HIP events around its launches) and the CPU-oracle baseline.
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
PKG = "infrared-colorization-with-resnet-generator-and-patchgan_amd"

METRIC = "GAN train-step img/s (G+D fwd/bwd) at 256×256, 1/2/4/8 MI355X"
MIN_GFLOP_PER_IMG_256 = 534.85   # minimal-step algorithmic FLOPs per image at 256^2
BF16_DENSE_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
FP8_DENSE_PEAK_TFLOPS = 5000.0   # MI355X dense fp8 (block-scaled f8f6f4 MFMA, MI355X_MICROARCH.md)
FP32_MFMA_PEAK_TFLOPS = 157.3


# minimal-step GFLOP per image measured on the reference modules (FlopCounterMode)
MIN_GFLOP_MEASURED = {(64, 64): 33.05, (256, 256): MIN_GFLOP_PER_IMG_256, (512, 640): 2680.06}


def min_gflop_per_img(H, W):
    # the measured figure where SURVEY has one; otherwise scaled with the pixel count (the
    # architecture is fully convolutional; the PatchGAN's valid-padded tail makes it ~0.2 % off)
    return MIN_GFLOP_MEASURED.get((H, W), MIN_GFLOP_PER_IMG_256 * (H * W) / (256 * 256))


def pmc_file():
    """The newest committed PMC summary (profiles/rNN_pmc_traffic.json, highest round)."""
    import glob
    fs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_pmc_traffic.json")))
    return fs[-1] if fs else None


def pmc_traffic(family):
    """HBM bytes per launch of the resblock conv `family` (fwd / dgrad / wgrad),
    from the newest committed rocprofv3 --pmc passes of tools/gpu_traffic.sh (FETCH_SIZE
    doubled per the gfx950 correction, plus WRITE_SIZE).  PMC counters cannot be
    collected inside this process, so the measured figure is read, not recomputed."""
    p = pmc_file()
    try:
        with open(p) as f:
            return json.load(f)[family]["hbm_bytes"]
    except (OSError, KeyError, ValueError, TypeError):
        return None


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_share():
    """CPUs this process may actually run on: the affinity mask, capped by the
    cgroup CPU quota (a GPU box shows every host CPU in os.cpu_count() but grants
    a share of them; oversubscribing the share makes torch's CPU threads crawl)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                n = min(n, max(1, int(q) // int(per)))
        except (OSError, ValueError):
            pass
    return max(1, n)


def mfma_peak_measured(ops, reps=3, iters=1500):
    """bf16 MFMA rate this box sustains on random operands (irgan_mfma_probe: every wave issues
    back-to-back v_mfma_f32_16x16x32_bf16, no memory traffic), best of `reps` timed launches after
    one warm-up, in TFLOP/s -- SURVEY.md 8d asks for the roofline's peak measured on the box; the
    chip holds a lower clock under dense MFMA load than the 2.4 GHz the nominal 2.5 PF assumes."""
    import torch
    cus = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
    blocks = 4 * cus   # 4 waves per block: 4 waves per SIMD
    g = torch.Generator().manual_seed(11)
    src = torch.randn(4096 * 8, generator=g).bfloat16().cuda()
    out = torch.empty(blocks * 256, device="cuda")
    flop = blocks * 4 * iters * 8 * 16384
    best = 0.0
    for r in range(reps + 1):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        ops._lib.call("irgan_mfma_probe", ops.P(src), ops.P(out), blocks, iters, ops.stream())
        b.record()
        torch.cuda.synchronize()
        if r:
            best = max(best, flop / (a.elapsed_time(b) * 1e-3) / 1e12)
    assert bool(torch.isfinite(out).all())
    return round(best, 1)


def _time_oracle(O, G, D, V, ir, rgb, threads, budget_s, min_steps, max_steps, warmup=1, as_written=False):
    """Median seconds per oracle step on `threads` torch CPU threads."""
    import torch
    torch.set_num_threads(threads)
    oG, oD = O.AdamState(G), O.AdamState(D)
    tag = "as-written" if as_written else "minimal"
    for _ in range(warmup):   # allocator, oneDNN primitives for these shapes
        t0 = time.perf_counter()
        O.train_step(G, D, V, ir, rgb, oG, oD, as_written=as_written)
        print(f"[cpu_baseline] {tag} warm-up step {time.perf_counter() - t0:.1f}s on {threads} threads",
              file=sys.stderr, flush=True)
    times, t_start = [], time.perf_counter()
    while len(times) < max_steps:
        t0 = time.perf_counter()
        O.train_step(G, D, V, ir, rgb, oG, oD, as_written=as_written)
        times.append(time.perf_counter() - t0)
        print(f"[cpu_baseline] {tag} step {len(times)}: {times[-1]:.1f}s", file=sys.stderr, flush=True)
        if len(times) >= min_steps and time.perf_counter() - t_start >= budget_s:
            break
    times.sort()
    return times[len(times) // 2], len(times)


def cpu_baseline(H, W, batch=16, budget_s=12.0, min_steps=3):
    """The CPU oracle (fp32 PyTorch-CPU restatement of ir:1636-1681, oracle/step.py)
    at the bench's own config (batch, H x W), on every CPU the process is granted
    (cpu_share(): affinity mask and cgroup quota -- os.cpu_count() reports the
    whole host); median of >= min_steps timed steps after one warm-up step.

    Two legs: ``value`` is the oracle's MINIMAL step (one G forward reused, no D
    weight gradients in the G backward -- the same work the HIP step does, 534.85
    GFLOP/img); ``as_written`` runs the reference's own order (a no-grad G forward for
    the D step, a second G forward, D grads from loss_G.backward(): 678.40 GFLOP/img,
    SURVEY.md 8d) on the same operands, which is what the reference itself costs."""
    import torch
    from oracle import step as O
    G = O.seeded_params(O.g_param_shapes(), 0)
    D = O.seeded_params(O.d_param_shapes(), 1)
    V = O.seeded_params(O.vgg_param_shapes(), 3, kaiming=True)
    g = torch.Generator().manual_seed(7)
    ir = torch.rand(batch, 1, H, W, generator=g) * 2 - 1
    rgb = torch.rand(batch, 3, H, W, generator=g) * 2 - 1
    ncpu = os.cpu_count() or 1
    share = cpu_share()
    med, n = _time_oracle(O, G, D, V, ir, rgb, share, budget_s, min_steps, 10)
    # as written: the minimal leg's warm-up already built the oneDNN primitives of these shapes
    med_w, n_w = _time_oracle(O, G, D, V, ir, rgb, share, 0.0, min_steps, min_steps, warmup=0, as_written=True)
    return {"value": round(batch / med, 4), "unit": "img/s", "cores": share, "kind": "port",
            "cpu_model": _cpu_model(), "nproc": ncpu, "cpu_share": share, "torch_threads": share,
            "steps": n, "s_per_step_median": round(med, 3),
            "as_written": {"value": round(batch / med_w, 4), "unit": "img/s", "steps": n_w,
                           "s_per_step_median": round(med_w, 3),
                           "minimal_over_as_written": round(med_w / med, 3)},
            "sample": f"oracle/step.py train_step at batch {batch}, {H}x{W}, fp32 (the bench config), minimal "
                      f"step (one G forward reused; the reference as written does 678.40 vs 534.85 GFLOP/img: "
                      f"see as_written): median of {n} steps after 1 warm-up, {share} torch threads = the CPUs "
                      f"granted to the process ({ncpu} host CPUs, {_cpu_model()})"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--size", type=int, default=256, help="square image side (default for --height/--width)")
    ap.add_argument("--height", type=int, default=None, help="image height (BASELINE configs[3]: 512)")
    ap.add_argument("--width", type=int, default=None, help="image width (BASELINE configs[3]: 640)")
    ap.add_argument("--batch", type=int, default=16, help="per-GPU batch")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32", "fp8"],
                    help="fp8: BASELINE configs[4] -- the ResnetBlock convs on e4m3 operands (use --batch 32)")
    ap.add_argument("--kernel-steps", type=int, default=5,
                    help="steps after the timed region with per-kernel HIP events (roofline lines)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds per CPU thread-count run")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    irc = importlib.import_module(PKG)
    ops = irc.ops

    H = args.height or args.size
    W = args.width or args.size
    B = args.batch
    cfg = irc.Config()
    cfg.device = f"cuda:{local}"
    cfg.compute_dtype = args.dtype
    cfg.batch_size = B
    cfg.img_size = H
    tr = irc.GANTrainer(cfg)
    # random-init weights of the reference architecture (seeded; identical on every rank)
    tr.netG.store.load(irc.seeded_state(irc.g_param_shapes(), 0), strict=True)
    tr.netD.store.load(irc.seeded_state(irc.d_param_shapes(), 1), strict=True)
    for m in (tr.netG, tr.netD, tr.vgg):
        m.repack()
    g = torch.Generator().manual_seed(7 + rank)
    ir = (torch.rand(B, 1, H, W, generator=g) * 2 - 1).cuda()
    rgb = (torch.rand(B, 3, H, W, generator=g) * 2 - 1).cuda()

    # dominant kernel for the live roofline: the resblock 3x3 conv (256->256 @ H/4)
    res_tags = [ops.conv_tag(k, ops.ConvSpec(256, 256, 3, 1, 1, ops.PAD_REFLECT), (H // 4, W // 4), B)
                for k in (("fwd8", "dgrad8", "wgrad8") if args.dtype == "fp8" else ("fwd", "dgrad", "wgrad"))]
    for _ in range(args.warmup):
        tr.step(ir, rgb)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # HBM-bound passes at the resblock shape (reported separately as GB/s)
    rb = ops.Feat(torch.empty(B, H // 4, W // 4, 256, device="meta"))
    hbm_bytes = {ops.hbm_tag("in_bwd_reduce", rb): 4, ops.hbm_tag("in_bwd_apply", rb): 6,
                 ops.hbm_tag("in_apply", rb): 4, ops.hbm_tag("in_apply_res", rb): 6}   # bytes per element
    # the ResnetBlock reflect ring when it runs on the side stream beside the weight gradient
    ring_tag = ops.conv_tag("ring", ops.ConvSpec(256, 256, 3, 1, 1, ops.PAD_REFLECT), (H // 4, W // 4), B)
    ops.TIMER.tags = set(res_tags) | set(hbm_bytes) | {ring_tag}
    # per-step HIP events (no host sync inside the timed region) for the median; the
    # per-kernel events of the roofline are recorded in the --kernel-steps steps right
    # after it (an event record between two launches is a ~5-10 us bubble on the stream:
    # around every tagged launch it would inflate the timed step by ~0.5 ms)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    evs[0].record()
    for i in range(args.steps):
        L = tr.step(ir, rgb)
        evs[i + 1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    # per-kernel HIP events on the launching streams, same inputs, right after the timed region
    ops.TIMER.enabled = True
    for _ in range(args.kernel_steps):
        tr.step(ir, rgb)
    torch.cuda.synchronize()
    ops.TIMER.enabled = False
    el_min = el
    replicas_ok = True
    if world > 1:
        t = torch.tensor([el], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        tmin = torch.tensor([el], device="cuda")
        dist.all_reduce(tmin, op=dist.ReduceOp.MIN)
        el, el_min = float(t), float(tmin)
        # every rank must still hold bit-identical G and D after the timed steps
        replicas_ok = irc.engine.replicas_identical([tr.netG.store.flat, tr.netD.store.flat])
    timing = ops.TIMER.summary()
    step_ms = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps))
    median_ms = step_ms[len(step_ms) // 2]
    losses = tr.losses(L)

    if rank == 0:
        imgs = B * world * args.steps
        value = imgs / el
        ms = el / args.steps * 1e3
        # roofline of the dominant kernel family: algorithmic FLOPs per launch / mean launch time
        res_flop = 2.0 * B * (H // 4) * (W // 4) * 256 * 256 * 9
        def peak_of(tag):
            if args.dtype == "fp32":
                return FP32_MFMA_PEAK_TFLOPS
            return FP8_DENSE_PEAK_TFLOPS if tag.split(":")[0].endswith("8") else BF16_DENSE_PEAK_TFLOPS
        kern = {}
        for tg in res_tags:
            if tg in timing:
                n, mean_ms = timing[tg]
                kern[tg] = {"launches": n, "mean_ms": round(mean_ms, 4),
                            "tflops": round(res_flop / (mean_ms * 1e-3) / 1e12, 2), "peak": peak_of(tg)}
        dom = max(kern, key=lambda k: kern[k]["launches"] * kern[k]["mean_ms"]) if kern else None
        ring = None
        if ring_tag in timing:   # off the critical path: beside the wgrad on the side stream
            n, mean_ms = timing[ring_tag]
            ring = {"launches": n, "mean_ms": round(mean_ms, 4), "stream": "side (under the weight gradient)"}
            dg = [t for t in kern if t.startswith("dgrad:")]
            if dg:
                tot = kern[dg[0]]["mean_ms"] + mean_ms
                ring["dgrad_plus_ring_ms"] = round(tot, 4)
                ring["dgrad_plus_ring_tflops"] = round(res_flop / (tot * 1e-3) / 1e12, 2)
        hbm = {}
        nel = B * (H // 4) * (W // 4) * 256
        for tg, bpe in hbm_bytes.items():
            if tg in timing:
                n, mean_ms = timing[tg]
                hbm[tg] = {"launches": n, "mean_ms": round(mean_ms, 4), "alg_bytes": bpe * nel,
                           "gbps": round(bpe * nel / (mean_ms * 1e-3) / 1e9, 1),
                           "frac_of_8tbs": round(bpe * nel / (mean_ms * 1e-3) / 8e12, 4)}
        achieved = kern[dom]["tflops"] if dom else None
        peak = peak_of(dom) if dom else BF16_DENSE_PEAK_TFLOPS
        traffic = pmc_traffic(dom.split(":")[0]) if (dom and H == 256 and B == 16 and args.dtype == "bf16") else None
        mp = mfma_peak_measured(ops) if args.dtype != "fp32" else None
        # fp8 (block-scaled f8f6f4, 32x32x64): the cycles of the bf16 32x32x16 at 4x the K, i.e. 2x
        # the bf16 rate per clock (MI355X_MICROARCH.md), so its measured peak is 2x the bf16 probe
        mpeak = (2 * mp if (dom or "").split(":")[0].endswith("8") else mp) if mp else None
        step_tflops = value * min_gflop_per_img(H, W) / 1e3 / world
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "img/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3),
            "ms_per_step_median": round(median_ms, 3), "img_per_s_median_step": round(B * world / median_ms * 1e3, 3),
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": args.dtype, "data": "synthetic (U(-1,1) IR/RGB pairs, seeded; random-init weights)",
            "config": {"workload": workload_label(H, W, B, args.dtype, world), "global_batch": B * world,
                       "img_size": H, "height": H, "width": W, "parallelism": f"dp{world}",
                       "min_gflop_per_img": round(min_gflop_per_img(H, W), 2),
                       "step_tflops_per_gpu": round(step_tflops, 2),
                       "step_frac_of_bf16_peak": round(step_tflops / BF16_DENSE_PEAK_TFLOPS, 4)},
            "roofline": {"bound": "mfma", "kernel": dom, "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                         "frac": round(achieved / peak, 4) if achieved else None, "traffic": traffic,
                         "peak_measured": mpeak, "frac_of_measured_peak": round(achieved / mpeak, 4)
                         if (achieved and mpeak) else None,
                         "peak_measured_note": "irgan_mfma_probe: back-to-back bf16 16x16x32 MFMAs on random "
                                               "operands, every SIMD 4 waves deep, no memory traffic (the rate the "
                                               "box sustains under MFMA load); fp8: 2x that (f8f6f4 cycles per "
                                               "FLOP); `peak` stays the nominal dense figure",
                         "traffic_unit": "HBM bytes per launch (rocprofv3 PMC: 2*FETCH_SIZE + WRITE_SIZE, "
                                         f"{os.path.relpath(pmc_file(), ROOT) if pmc_file() else 'none'})",
                         "flop_per_launch": res_flop, "per_kernel": kern,
                         "kernel_timing": f"HIP events around each tagged launch on its stream, {args.kernel_steps} "
                                          "steps right after the timed region (same process, inputs and "
                                          "buffers); the timed region itself carries no per-kernel events",
                         "reflect_ring": ring,
                         "ring_note": "dgrad = the backward-data launch on the main stream; with reflect_ring "
                                      "set, the reflect-pad ring of each ResnetBlock dgrad (the fold of the padded "
                                      "border, 6% of the FLOPs) runs as its own launches on the side stream, "
                                      "concurrently with that conv's weight gradient (which leaves 16 CUs idle)",
                         "hbm_kernels": hbm,
                         "hbm_note": "InstanceNorm passes at the resblock shape, HIP events on the launching "
                                     "stream; alg_bytes = bf16 bytes read + written once (in_bwd_reduce: dy, z; "
                                     "_apply: dy, z, dx; in_apply: z, y; _res: + residual); in_bwd_reduce "
                                     "includes its finalize launch"},
            "dp": {"rccl_world": world, "backend": dist.get_backend() if world > 1 else None,
                   "rank_time_s": {"max": round(el, 4), "min": round(el_min, 4)},
                   "replicas_bit_identical": replicas_ok},
            "losses": {k: round(v, 5) for k, v in losses.items()},
            **(step_phases(irc.engine.JOIN_TIMES[-args.steps:]) if irc.engine.JOIN_TIMES else {}),
        }
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(H, W, B, args.cpu_budget)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def workload_label(H, W, B, dtype, world):
    """Names the workload from the actual (H, W, B, dtype); a BASELINE config is named only
    when the per-GPU shape is exactly that config's (BASELINE.json configs: [1] 256^2 B=16
    bf16 1 GPU, [2] the same at DP8, [3] 512x640 B=4/GPU, [4] 256^2 fp8 B=32/GPU)."""
    base = f"GAN train step {H}x{W}, batch {B}/GPU, {dtype}"
    if dtype == "fp8":
        base += " (conv operands on e4m3 where the fp8 path covers the layer)"
    tag = None
    if (H, W, B, dtype) == (256, 256, 16, "bf16"):
        tag = "BASELINE configs[2]" if world > 1 else "BASELINE configs[1]"
    elif (H, W, B) == (512, 640, 4) and dtype != "fp8":
        tag = "BASELINE configs[3] per-GPU shape"
    elif (H, W, B, dtype) == (256, 256, 32, "fp8"):
        tag = "BASELINE configs[4] per-GPU shape"
    return f"{base} ({tag})" if tag else base


def step_phases(steps):
    """IRGAN_JOIN_TIMING=1 diagnostics: the main stream's wait for the side stream's D step
    (join_wait_ms) and each phase mark's median offset from the step start (ms)."""
    import statistics
    keys = [k for k in steps[0] if k != "start"]
    off = {k: round(statistics.median(p["start"].elapsed_time(p[k]) for p in steps), 4) for k in keys}
    wait = statistics.mean(p["terms"].elapsed_time(p["join"]) for p in steps)
    return {"join_wait_ms": round(wait, 4), "step_phase_ms": off}


if __name__ == "__main__":
    main()
