"""Build libirgan.so (gfx950) in-tree with hipcc.  No JIT cache, no torch extension:
the C ABI in include/irgan.h is the boundary, bound with ctypes by _lib.py."""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(ROOT, "include")
LIB = os.path.join(HERE, "libirgan.so")
SOURCES = ["conv.hip", "conv_glds.hip", "conv_halo.hip", "conv_pp.hip", "conv_res64.hip", "conv_wgrad_halo.hip", "conv_wgrad_pc.hip", "conv_wgrad_f8.hip", "conv_wgrad_narrow.hip", "conv_ring.hip", "conv_c8.hip", "conv_rowspan.hip", "conv_dgrad_s2.hip", "fp8.hip", "infer.hip", "data.hip", "norm.hip", "resample.hip", "loss.hip"]
ARCH = os.environ.get("IRGAN_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", INCLUDE, "-I", CSRC,
         "-Wno-unused-result", "-fvisibility=hidden"]


def _hipcc():
    for c in ("/opt/rocm/bin/hipcc", "hipcc"):
        if os.path.exists(c) or c == "hipcc":
            return c
    raise RuntimeError("hipcc not found")


def _stale(obj, src):
    if not os.path.exists(obj):
        return True
    deps = [src] + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")] + \
        [os.path.join(INCLUDE, "irgan.h")]
    return any(os.path.getmtime(d) > os.path.getmtime(obj) for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    hipcc = _hipcc()
    objdir = os.path.join(HERE, "build")
    os.makedirs(objdir, exist_ok=True)
    jobs = []
    for s in SOURCES:
        src = os.path.join(CSRC, s)
        obj = os.path.join(objdir, s.replace(".hip", ".o"))
        if force or _stale(obj, src):
            jobs.append([hipcc, *FLAGS, "-c", src, "-o", obj])

    def run(cmd):
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose:
            print(" ".join(cmd), file=sys.stderr)

    with ThreadPoolExecutor(max_workers=min(4, max(1, len(jobs)))) as ex:
        list(ex.map(run, jobs))
    objs = [os.path.join(objdir, s.replace(".hip", ".o")) for s in SOURCES]
    if force or jobs or not os.path.exists(LIB) or any(os.path.getmtime(o) > os.path.getmtime(LIB) for o in objs):
        run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs])
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
