"""ctypes binding of the C ABI declared in include/irgan.h.

Signatures are generated from the header itself, so the Python side cannot
drift from the ABI.  There is NO fallback: if libirgan.so is missing or does
not export a declared symbol, loading raises.  (The CPU oracle under oracle/ is
test infrastructure and is never imported by the product package.)
"""
from __future__ import annotations

import ctypes
import os
import re
import warnings

HERE = os.path.dirname(os.path.abspath(__file__))
HEADER = os.path.join(os.path.dirname(HERE), "include", "irgan.h")
# IRGAN_LIB: an alternative build of the same ABI (kernel A/B experiments, tools/)
LIB_PATH = os.environ.get("IRGAN_LIB") or os.path.join(HERE, "libirgan.so")

F32, BF16, FP8 = 0, 1, 2
PAD_ZERO, PAD_REFLECT = 0, 1
ACT_NONE, ACT_RELU, ACT_LRELU, ACT_TANH = 0, 1, 2, 3


class IrganError(RuntimeError):
    pass


def _header_text() -> str:
    """include/irgan.h: the ctypes signatures are generated from it, so a deployment ships it
    next to libirgan.so (the csrc/ sources are optional, see load())."""
    try:
        with open(HEADER) as f:
            return f.read()
    except OSError as e:
        raise IrganError(f"{HEADER} is missing ({e}): the binding reads the ABI from the header") from None


def header_enum(name: str) -> int:
    return int(re.search(name + r"\s*=\s*(\d+)", _header_text()).group(1))


IN_PARTS = header_enum("IRGAN_IN_PARTS")


def _desc_fields():
    src = _header_text()
    body = re.search(r"typedef struct irgan_conv_desc \{(.*?)\} irgan_conv_desc;", src, re.S).group(1)
    names = []
    for line in body.splitlines():
        line = line.split("/*")[0].strip()
        if not line.startswith("int32_t"):
            continue
        names += [n.strip() for n in line[len("int32_t"):].rstrip(";").split(",")]
    return names


class ConvDesc(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in _desc_fields()]


_CTYPES = {
    "int32_t": ctypes.c_int32, "int64_t": ctypes.c_int64, "float": ctypes.c_float, "double": ctypes.c_double,
    "uint32_t": ctypes.c_uint32,
    "uint64_t": ctypes.c_uint64,
    "irgan_stream_t": ctypes.c_void_p, "void": None,
}


def _ctype(decl: str):
    decl = decl.strip().replace("const ", "")
    if "*" in decl:
        base = decl.split("*")[0].strip()
        if base == "irgan_conv_desc":
            return ctypes.POINTER(ConvDesc)
        return ctypes.c_void_p
    toks = decl.split()
    return _CTYPES[toks[0]]


def parse_header():
    """[(name, restype, [argtypes])] for every prototype in irgan.h."""
    src = re.sub(r"/\*.*?\*/", "", _header_text(), flags=re.S)
    out = []
    for m in re.finditer(r"\b(int)\s+(irgan_\w+)\s*\(([^)]*)\)\s*;", src):
        args = [a for a in (x.strip() for x in m.group(3).split(",")) if a and a != "void"]
        out.append((m.group(2), ctypes.c_int, [_ctype(a) for a in args]))
    return out


PROTOS = parse_header()
_lib = None


def load(path: str = LIB_PATH):
    """Load libirgan.so (after torch, so the process shares one HIP runtime)."""
    global _lib
    if _lib is not None:
        return _lib
    import torch  # noqa: F401  -- torch's libamdhip64 must be the one in the process
    if not os.path.exists(path):
        raise IrganError(f"{path} is missing: build it with __graft_entry__.build() "
                         "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    for name, res, args in PROTOS:
        fn = getattr(lib, name)  # AttributeError == symbol missing -> loud failure
        fn.restype = res
        fn.argtypes = args
    got, want = build_id(lib), tree_id()
    if want is None:
        # a deployment with the library, the Python files and the header but no csrc/:
        # nothing to compare the compiled-in id with
        warnings.warn(f"no kernel sources next to {path}: build id {got} not checked against a tree",
                      RuntimeWarning)
    elif got != want:
        raise IrganError(f"{path} was built from sources {got}, but this tree is {want}: the library is "
                         "stale -- rebuild it with __graft_entry__.build()")
    _lib = lib
    return lib


def tree_id():
    """Source id of the csrc/ + include/ tree next to this file (_build.source_id), or None
    when the csrc/ directory is absent (a library-only deployment).  A tree that exists
    but cannot be read raises IrganError."""
    from . import _build
    if not os.path.isdir(_build.CSRC):
        return None
    try:
        return _build.source_id()
    except OSError as e:
        raise IrganError(f"cannot hash the kernel sources for the build-id check: {e}") from None


def build_id(lib=None) -> str:
    """The source id compiled into a loaded library (irgan_build_id)."""
    lib = lib if lib is not None else load()
    buf = ctypes.create_string_buffer(64)
    if lib.irgan_build_id(buf, len(buf)) != 0:
        raise IrganError("irgan_build_id failed")
    return buf.value.decode()


def call(name, *args):
    rc = getattr(load(), name)(*args)
    if rc != 0:
        raise IrganError(f"{name} failed with code {rc}")
    return rc
