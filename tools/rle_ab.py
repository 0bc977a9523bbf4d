"""A/B of dctq_rle_count / dctq_rle_emit / dctq_rle_decode between the default libdct_amd.so and
diagnostic builds (tools/ubench/libvar_*.so, tools/ubench/variant.sh), same inputs,
interleaved, HIP events; outputs must match the default build.

    python tools/rle_ab.py [frames]
"""
import ctypes as C
import glob
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import dct_amd  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 64
W, H = 3840, 2160
nblk = F * (W // 8) * (H // 8)
libs = {"default": dct_amd.lib()}
for p in sorted(glob.glob(os.path.join(ROOT, "tools", "ubench", "libvar_*.so"))):
    L = C.CDLL(p)
    L.dctq_rle_emit.argtypes = [C.c_void_p, C.c_longlong, C.c_void_p, C.c_void_p, C.c_void_p]
    L.dctq_rle_decode.argtypes = [C.c_void_p, C.c_void_p, C.c_longlong, C.c_void_p, C.c_void_p]
    L.dctq_rle_count.argtypes = [C.c_void_p, C.c_longlong, C.c_void_p, C.c_void_p, C.c_void_p]
    libs[os.path.basename(p)[7:-3]] = L
s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
vp = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
for kind, q in (("uniform", 50), ("smooth", 50), ("smooth", 90), ("const", 50), ("extreme", 50)):
    coef = dct_amd.Plan(q, 0).forward_quant(dct_amd.synth(9, kind, W, H, F))
    kind = f"{kind}/q{q}"
    off, sym = dct_amd.rle_encode(coef)
    ref_sym = sym.clone()
    # ONE output buffer per operation, shared by every build: separate buffers put
    # the variants' stores on different physical pages (seen: +-12 % on identical code)
    out_sym = torch.empty_like(sym)
    back = torch.empty_like(coef)
    out_off = torch.empty_like(off)
    ws = torch.empty(int(dct_amd.lib().dctq_rle_workspace_bytes(nblk)) // 4 + 1, dtype=torch.int32, device="cuda")
    jobs = {}
    for k, L in libs.items():
        jobs[f"count {k}"] = (lambda L=L: L.dctq_rle_count(vp(coef), nblk, vp(out_off), vp(ws), s), k, "count")
        jobs[f"emit {k}"] = (lambda L=L: L.dctq_rle_emit(vp(coef), nblk, vp(off), vp(out_sym), s), k, "emit")
        jobs[f"decode {k}"] = (lambda L=L: L.dctq_rle_decode(vp(sym), vp(off), nblk, vp(back), s), k, "decode")
    times = {j: [] for j in jobs}
    for r in range(9):
        for j, (fn, k, op) in jobs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            assert fn() == 0
            e1.record()
            torch.cuda.synchronize()
            if r:
                times[j].append(e0.elapsed_time(e1) * 1e-3)
            if r == 0:
                if op == "count":
                    assert torch.equal(out_off, off), f"{k}: count output differs"
                elif op == "emit":
                    assert torch.equal(out_sym, ref_sym), f"{k}: emit output differs"
                else:
                    assert torch.equal(back, coef), f"{k}: decode output differs"
    for j, ts in times.items():
        print(f"{kind:12s} {j:24s} median {statistics.median(ts) * 1e6:7.1f} us")
