"""Build libirgan.so (gfx950) in-tree with hipcc.  No JIT cache, no torch extension:
the C ABI in include/irgan.h is the boundary, bound with ctypes by _lib.py.

Provenance: `source_id()` hashes every csrc/*.hip, csrc/*.h and include/irgan.h; the id is
compiled into the library (`irgan_build_id`, csrc/build_id.hip) and `_lib.load()` refuses a
library whose id differs from the tree.  Objects are rebuilt when the hash of their inputs
(source, every header, flags) changes -- never on mtimes, so a stale object cannot mask an
edited source."""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(ROOT, "include")
HEADER = os.path.join(INCLUDE, "irgan.h")
LIB = os.path.join(HERE, "libirgan.so")
OBJDIR = os.path.join(HERE, "build")
SOURCES = ["conv.hip", "conv_glds.hip", "conv_halo.hip", "conv_pp.hip", "conv_res64.hip", "conv_wgrad_halo.hip",
           "conv_wgrad_pc.hip", "conv_wgrad_f8.hip", "conv_wgrad_narrow.hip", "conv_ring.hip", "conv_c8.hip",
           "conv_rowspan.hip", "conv_dgrad_s2.hip", "fp8.hip", "infer.hip", "data.hip", "norm.hip",
           "resample.hip", "loss.hip", "head.hip", "probe.hip", "build_id.hip"]
ARCH = os.environ.get("IRGAN_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", INCLUDE, "-I", CSRC,
         "-Wno-unused-result", "-fvisibility=hidden"]


def _hipcc():
    for c in ("/opt/rocm/bin/hipcc", "hipcc"):
        if os.path.exists(c) or c == "hipcc":
            return c
    raise RuntimeError("hipcc not found")


def _read(path):
    with open(path, "rb") as f:
        return f.read()


def _headers():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")) + [HEADER]


def source_id() -> str:
    """16 hex digits over the names and bytes of every source and header of the library."""
    files = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".h"))) + [HEADER]
    h = hashlib.sha256()
    for p in files:
        h.update(os.path.basename(p).encode() + b"\0" + _read(p) + b"\0")
    return h.hexdigest()[:16]


def _sig(parts) -> str:
    h = hashlib.sha256()
    for p in parts:
        h.update(p if isinstance(p, bytes) else str(p).encode())
        h.update(b"\0")
    return h.hexdigest()


def _sig_path(obj):
    return obj + ".sig"


def _current(path, sig):
    return os.path.exists(path) and os.path.exists(_sig_path(path)) and _read(_sig_path(path)).decode() == sig


def build(force: bool = False, verbose: bool = False, extra_flags=(), lib: str = LIB, objdir: str = OBJDIR,
          only=None) -> str:
    """Compile the sources whose inputs changed and link `lib`.  extra_flags (A/B variant
    builds, tools/build_variant.sh) apply to every object -- or, with ``only`` (a list of
    source names), to those alone, the others linked from the default objects -- and land
    in the objects' signatures, so variant objects never stand in for the default build's."""
    hipcc = _hipcc()
    os.makedirs(objdir, exist_ok=True)
    sid = source_id()
    hdr = [_read(h) for h in _headers()]
    jobs, objs = [], []
    for s in SOURCES:
        src = os.path.join(CSRC, s)
        var = only is None or s in only
        obj = os.path.join(objdir if var else OBJDIR, s.replace(".hip", ".o"))
        flags = list(FLAGS) + (list(extra_flags) if var else [])
        if s == "build_id.hip":
            flags.append(f'-DIRGAN_SOURCE_ID="{sid}"')
        sig = _sig([hipcc, *flags, _read(src), *hdr])
        objs.append(obj)
        if force or not _current(obj, sig):
            jobs.append(([hipcc, *flags, "-c", src, "-o", obj], obj, sig))

    def run(cmd):
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose:
            print(" ".join(cmd), file=sys.stderr)

    def compile_one(job):
        cmd, obj, sig = job
        if os.path.exists(_sig_path(obj)):
            os.remove(_sig_path(obj))
        run(cmd)
        with open(_sig_path(obj), "w") as f:
            f.write(sig)

    with ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as ex:
        list(ex.map(compile_one, jobs))
    lsig = _sig([_read(_sig_path(o)) for o in objs])
    # the link signature also covers the library's own bytes, so a library copied over the
    # linked one (another tree's build) is relinked rather than trusted
    if force or jobs or not (os.path.exists(lib) and _current(lib, _sig([lsig, _read(lib)]))):
        if os.path.exists(_sig_path(lib)):
            os.remove(_sig_path(lib))
        run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib, *objs])
        with open(_sig_path(lib), "w") as f:
            f.write(_sig([lsig, _read(lib)]))
    return lib


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
