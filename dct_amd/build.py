"""Build libdct_amd.so (all HIP sources, gfx950 only) in-tree.

    python -m dct_amd.build            # or dct_amd.build.build()

Explicit hipcc lines (one object per source, compiled in parallel, then two
links) -- no torch extension machinery: the library is a plain
C-ABI shared object that a C host links with -ldct_amd and Python loads with
ctypes.  Two libraries come out of the same objects:
  libdct_amd.so       the product: exports exactly the functions declared in
                      include/*.h (a version script generated from them);
  libdct_amd_diag.so  + diag.hip: the diagnostic entry points of
                      csrc/dctq_diag.h (kernel selection for tests, movement and
                      hardware ceilings for bench.py, host table introspection).  -ffp-contract=off is load-bearing (DESIGN.md "Exactness"): the exact
tie path must not fuse multiply-add, and the fast path asks for every FMA it
wants explicitly.
"""
from __future__ import annotations

import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libdct_amd.so")
DIAG_LIB = os.path.join(HERE, "libdct_amd_diag.so")
DIAG_SOURCES = ["diag.hip", "fdct8_diag.hip"]
SOURCES = ["api.hip", "legacy.hip", "fdct8.hip", "fdct8_aux.hip", "f64_pair.hip", "rle.hip", "roundtrip.hip", "encode.hip", "huffman.hip"]
HEADERS = ["dctq_internal.h", "plan.h", "dctq_diag.h", "fdct8_bound.h", "idct8_bound.h", "host_tables.h", "aan_f64.h", "fdct8_core.h", "pair_core.h", "scan_core.h", "zigzag.h"]
ARCH = "gfx950"


INFO = os.path.join(HERE, "build_info.json")


def _sha256(path: str) -> str:
    import hashlib
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def _inputs() -> dict:
    """Every file the libraries are built from (sources, headers, public headers, this script) -> sha256."""
    deps = [os.path.join(CSRC, f) for f in SOURCES + DIAG_SOURCES + HEADERS] + [os.path.abspath(__file__)]
    deps += [os.path.join(ROOT, "include", f) for f in sorted(os.listdir(os.path.join(ROOT, "include")))]
    return {os.path.relpath(d, ROOT): _sha256(d) for d in deps}


def build_info() -> dict:
    """The manifest the last build wrote (dct_amd/build_info.json), or {}."""
    import json
    try:
        with open(INFO) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def _stale() -> bool:
    """Content-gated: rebuild unless both libraries exist and the manifest of the
    last build names exactly these inputs and these library bytes."""
    if not os.path.exists(LIB) or not os.path.exists(DIAG_LIB):
        return True
    info = build_info()
    return (info.get("inputs") != _inputs() or info.get("lib_sha256") != _sha256(LIB)
            or info.get("diag_sha256") != _sha256(DIAG_LIB) or info.get("flags") != _portable_flags())


def _portable_flags() -> list:
    """_flags() with the checkout's path replaced, so a manifest stays valid in a copy of the tree."""
    return [f.replace(ROOT, "$ROOT") for f in _flags()]


def _flags():
    return ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
            "-fno-slp-vectorize", "-Wall", "-Wno-unused-command-line-argument",
            "-I" + os.path.join(ROOT, "include"), "-I" + CSRC]


def declared_functions(headers) -> list:
    """C function names declared in the given headers (comments stripped)."""
    names = set()
    for h in headers:
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w \*]*?\b([a-z_][a-z0-9_]*)\s*\(", src, flags=re.M):
            if m.group(1) not in ("if", "while", "for", "return", "sizeof", "defined"):
                names.add(m.group(1))
    return sorted(names)


def public_headers() -> list:
    inc = os.path.join(ROOT, "include")
    return [os.path.join(inc, f) for f in sorted(os.listdir(inc)) if f.endswith(".h")]


def _version_script(path: str, names) -> str:
    with open(path, "w") as f:
        f.write("{\n  global:\n" + "".join(f"    {n};\n" for n in names) + "  local: *;\n};\n")
    return path


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile each source to an object in parallel (dct_amd/_obj/), then link both libraries."""
    if not force and not _stale():
        return LIB
    from concurrent.futures import ThreadPoolExecutor
    objdir = os.path.join(HERE, "_obj")
    os.makedirs(objdir, exist_ok=True)
    srcs = SOURCES + DIAG_SOURCES
    objs = {src: os.path.join(objdir, os.path.splitext(src)[0] + ".o") for src in srcs}

    def compile_one(src):
        # a compilation-unit id from the file name, not hipcc's default hash of the
        # path: the same sources give the same library bytes in any checkout
        cuid = "dctamd_" + os.path.splitext(src)[0]
        cmd = _flags() + [f"-cuid={cuid}", "-c", os.path.join(CSRC, src), "-o", objs[src]]
        if verbose:
            print(" ".join(cmd))
        return subprocess.run(cmd, capture_output=True, text=True)

    jobs = min(len(srcs), max(1, min(16, os.cpu_count() or 1)))
    with ThreadPoolExecutor(jobs) as ex:
        results = list(ex.map(compile_one, srcs))
    for src, out in zip(srcs, results):
        if out.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n" + out.stdout + out.stderr)
    pub = declared_functions(public_headers())
    diag = declared_functions(public_headers() + [os.path.join(CSRC, "dctq_diag.h")])
    for lib, names, parts in ((LIB, pub, SOURCES), (DIAG_LIB, diag, srcs)):
        vs = _version_script(os.path.join(objdir, os.path.basename(lib) + ".map"), names)
        cmd = _flags() + ["-shared", *[objs[s_] for s_ in parts], f"-Wl,--version-script={vs}", "-o", lib + ".tmp"]
        if verbose:
            print(" ".join(cmd))
        out = subprocess.run(cmd, capture_output=True, text=True)
        if out.returncode != 0:
            raise RuntimeError("hipcc link failed:\n" + out.stdout + out.stderr)
        os.replace(lib + ".tmp", lib)
    import json
    import time
    ver = subprocess.run(["hipcc", "--version"], capture_output=True, text=True).stdout.strip().splitlines()
    info = {"lib_sha256": _sha256(LIB), "diag_sha256": _sha256(DIAG_LIB), "inputs": _inputs(), "flags": _portable_flags(),
            "hipcc": ver[:2], "arch": ARCH, "built_utc": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())}
    with open(INFO + ".tmp", "w") as f:
        json.dump(info, f, indent=1, sort_keys=True)
    os.replace(INFO + ".tmp", INFO)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
