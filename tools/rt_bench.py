#!/usr/bin/env python3
"""Fused round trip (dctq_round_trip_planes) vs the unfused pair (forward_quant_planes
with var_num, then dctq_inverse per plane) on the bench workload: F 4K 4:2:0 frames
(Y planes + Cb/Cr planes, two planes per launch).  Also times diagnostic builds
tools/ubench/libvar_*.so (tools/ubench/variant.sh) of the fused kernel, interleaved.

    python tools/rt_bench.py [F] [--adaptive] [--kind=uniform] [--q=50]
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

args = [a for a in sys.argv[1:] if not a.startswith("--")]
F = int(args[0]) if args else 64
AD = int("--adaptive" in sys.argv)
KIND = next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--kind=")), "uniform")
Q = int(next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--q=")), "50"))
ROUNDS = 10
luma = dct_amd.synth(7, KIND, 3840, 2160, F)
chroma = dct_amd.synth(8, KIND, 1920, 1080, 2 * F)
planes = [luma, chroma]
nbs = [F * 480 * 270, 2 * F * 240 * 135]
nblk = sum(nbs)
coef = [torch.empty((n, 64), dtype=torch.int16, device="cuda") for n in nbs]
var = [torch.empty(n, dtype=torch.int32, device="cuda") for n in nbs]
rec = [torch.empty((n, 64), dtype=torch.float32, device="cuda") for n in nbs]
coef2 = [torch.empty_like(c) for c in coef]
rec2 = [torch.empty_like(r) for r in rec]
stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
descs = (dct_amd._Plane * 2)(*[dct_amd.plane_desc(p) for p in planes])


def arr(ts):
    return C.cast((C.c_void_p * len(ts))(*[t.data_ptr() for t in ts]), C.c_void_p)


libs = {"fused": dct_amd.LIB_PATH}
for p in sorted(glob.glob(os.path.join(ROOT, "tools", "ubench", "libvar_*.so"))):
    libs["fused-" + os.path.basename(p)[len("libvar_"):-3]] = p
runs = {}
for name, path in libs.items():
    L = C.CDLL(path)
    L.dctq_plan_create.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_void_p)]
    L.dctq_round_trip_planes.argtypes = [C.c_void_p, C.POINTER(dct_amd._Plane), C.c_int] + [C.c_void_p] * 4
    h = C.c_void_p()
    assert L.dctq_plan_create(Q, AD, C.byref(h)) == 0
    runs[name] = (lambda L=L, h=h: L.dctq_round_trip_planes(h, descs, 2, arr(coef2), None, arr(rec2), stream))
plan = dct_amd.Plan(Q, AD)


def unfused():
    plan.forward_quant_planes(planes, outs=coef, var_nums=var)
    for c, v, r in zip(coef, var, rec):
        plan.inverse(c, var_num=v, out=r)
    return 0


runs["unfused"] = unfused
times = {k: [] for k in runs}
for r in range(ROUNDS + 2):
    for name, fn in runs.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        assert fn() == 0
        e1.record()
        torch.cuda.synchronize()
        if r >= 2:
            times[name].append(e0.elapsed_time(e1) * 1e-3)
        if name != "unfused" and r == 0:
            ok = all(torch.equal(a, b) for a, b in zip(coef, coef2))
            err = max(float((a - b).abs().max()) for a, b in zip(rec, rec2))
            if "unfused" in times and times["unfused"]:
                print(f"{name}: coef equal {ok}, recon max |diff| {err:.2e}")
for name, ts in times.items():
    med = statistics.median(ts)
    bpb = 584 if name == "unfused" else 448
    print(f"{name:22s} {KIND} q{Q} adaptive={AD} median {med*1e6:8.1f} us  {nblk/med/1e9:6.2f} G blocks/s  "
          f"{nblk*bpb/med/1e9:6.0f} GB/s ({bpb} B/block)")
# correctness of the default library against the unfused pair (after all rounds)
runs["fused"]()
unfused()
torch.cuda.synchronize()
ok = all(torch.equal(a, b) for a, b in zip(coef, coef2))
err = max(float((a - b).abs().max()) for a, b in zip(rec, rec2))
print(f"check fused vs unfused: coef equal {ok}, recon max |diff| {err:.2e}")
