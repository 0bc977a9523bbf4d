"""Build libdct_amd.so (all HIP sources, gfx950 only) in-tree.

    python -m dct_amd.build            # or dct_amd.build.build()

Explicit hipcc lines (one object per source, compiled in parallel, then one
link) -- no torch extension machinery: the library is a plain
C-ABI shared object that a C host links with -ldct_amd and Python loads with
ctypes.  -ffp-contract=off is load-bearing (DESIGN.md "Exactness"): the exact
tie path must not fuse multiply-add, and the fast path asks for every FMA it
wants explicitly.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libdct_amd.so")
SOURCES = ["api.hip", "legacy.hip", "fdct8.hip", "fdct8_aux.hip", "f64_pair.hip", "rle.hip", "roundtrip.hip", "encode.hip", "huffman.hip"]
HEADERS = ["dctq_internal.h", "fdct8_bound.h", "host_tables.h", "aan_f64.h", "fdct8_core.h", "pair_core.h", "scan_core.h", "zigzag.h"]
ARCH = "gfx950"


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps += [os.path.join(ROOT, "include", f) for f in os.listdir(os.path.join(ROOT, "include"))]
    return any(os.path.getmtime(d) > t for d in deps)


def _flags():
    return ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
            "-fno-slp-vectorize", "-Wall", "-Wno-unused-command-line-argument",
            "-I" + os.path.join(ROOT, "include"), "-I" + CSRC]


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile each source to an object in parallel (dct_amd/_obj/), then link the .so."""
    if not force and not _stale():
        return LIB
    from concurrent.futures import ThreadPoolExecutor
    objdir = os.path.join(HERE, "_obj")
    os.makedirs(objdir, exist_ok=True)
    objs = [os.path.join(objdir, os.path.splitext(src)[0] + ".o") for src in SOURCES]

    def compile_one(src_obj):
        src, obj = src_obj
        cmd = _flags() + ["-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd))
        return subprocess.run(cmd, capture_output=True, text=True)

    jobs = min(len(SOURCES), max(1, min(16, os.cpu_count() or 1)))
    with ThreadPoolExecutor(jobs) as ex:
        results = list(ex.map(compile_one, zip(SOURCES, objs)))
    for src, out in zip(SOURCES, results):
        if out.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n" + out.stdout + out.stderr)
    cmd = _flags() + ["-shared", *objs, "-o", LIB + ".tmp"]
    if verbose:
        print(" ".join(cmd))
    out = subprocess.run(cmd, capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("hipcc link failed:\n" + out.stdout + out.stderr)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
