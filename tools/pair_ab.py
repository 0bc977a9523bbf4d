"""Same-box A/B of the paired-lane fp64 kernels (f64_pair.hip: dctq_inverse and
dctq_forward_float) between the product library and diagnostic builds
(tools/ubench/libvar_*.so), 64 4K luma frames, q50, interleaved rounds, each sample
3 launches back to back after one untimed launch; outputs compared with the product's.

    python tools/pair_ab.py [--rounds 10] [--kind uniform] [--adaptive 0]
"""
import argparse
import ctypes as C
import glob
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import dct_amd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=10)
ap.add_argument("--frames", type=int, default=64)
ap.add_argument("--kind", default="uniform")
ap.add_argument("--adaptive", type=int, default=0)
args = ap.parse_args()

px = dct_amd.synth(777, args.kind, 3840, 2160, args.frames)
nb = args.frames * 480 * 270
vn = torch.empty(nb, dtype=torch.int32, device="cuda")
coef = dct_amd.Plan(50, args.adaptive).forward_quant(px, var_num=vn)
desc = dct_amd.plane_desc(px)
rec = torch.empty((nb, 64), dtype=torch.float32, device="cuda")
stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
libs = {"default": dct_amd.LIB_PATH}
for p in sorted(glob.glob(os.path.join(ROOT, "tools", "ubench", "libvar_*.so"))):
    libs[os.path.basename(p)[7:-3]] = p
runs = {}
for k, path in libs.items():
    L = C.CDLL(path)
    L.dctq_plan_create.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_void_p)]
    L.dctq_inverse.argtypes = [C.c_void_p] * 3 + [C.c_longlong] + [C.c_void_p] * 2
    L.dctq_forward_float.argtypes = [C.c_void_p, C.POINTER(dct_amd._Plane), C.c_void_p, C.c_void_p]
    h = C.c_void_p()
    assert L.dctq_plan_create(50, args.adaptive, C.byref(h)) == 0
    runs[(k, "inverse")] = lambda L=L, h=h: L.dctq_inverse(h, coef.data_ptr(), vn.data_ptr(), nb, rec.data_ptr(), stream)
    runs[(k, "forward_float")] = lambda L=L, h=h: L.dctq_forward_float(h, C.byref(desc), rec.data_ptr(), stream)
times = {k: [] for k in runs}
for r in range(args.rounds + 1):
    for k, fn in runs.items():
        assert fn() == 0, k
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            fn()
        e1.record()
        torch.cuda.synchronize()
        if r:
            times[k].append(e0.elapsed_time(e1) / 3 * 1e-3)
ref = {}
for k, fn in runs.items():
    assert fn() == 0, k
    torch.cuda.synchronize()
    if k[1] not in ref:
        ref[k[1]] = rec.clone()
    same = torch.equal(rec, ref[k[1]])
    print(f"{k[0]:12s} {k[1]:14s} identical to default: {same}")
    assert same or k[0].startswith("no"), k
bpb = {"inverse": 128 + 4 + 256, "forward_float": 64 + 256}
for k, v in times.items():
    m = statistics.median(v)
    base = statistics.median(times[("default", k[1])])
    print(f"{k[0]:12s} {k[1]:14s} median {m * 1e6:8.1f} us  {nb * bpb[k[1]] / m / 8e12:6.3f} of 8 TB/s  "
          f"x{m / base:5.3f} of default")
