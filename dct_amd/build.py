"""Build libdct_amd.so (all HIP sources, gfx950 only) in-tree.

    python -m dct_amd.build            # or dct_amd.build.build()

One explicit hipcc line -- no torch extension machinery: the library is a plain
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


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-ffp-contract=off", "-fno-slp-vectorize", "-Wall", "-Wno-unused-command-line-argument",
           "-I" + os.path.join(ROOT, "include"), "-I" + CSRC,
           *[os.path.join(CSRC, s) for s in SOURCES], "-o", LIB + ".tmp"]
    if verbose:
        print(" ".join(cmd))
    out = subprocess.run(cmd, capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("hipcc failed:\n" + out.stdout + out.stderr)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
