"""Steady-state A/B of diagnostic builds (tools/ubench/libvar_*.so) against the
default library for the fused round trip (dctq_round_trip_planes) on the bench workload (F 4K 4:2:0 frames, Y + Cb/Cr
planes in one launch): clock pre-warm, then per sample one untimed launch of the
variant followed by 3 timed back to back, interleaved rounds; outputs compared.

    python tools/grid_ab.py [F] [--adaptive]"""
import ctypes as C
import glob
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import dct_amd  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
F = int(args[0]) if args else 64
AD = int("--adaptive" in sys.argv)
ROUNDS, B2B = 10, 3
luma = dct_amd.synth(7, "uniform", 3840, 2160, F)
chroma = dct_amd.synth(8, "uniform", 1920, 1080, 2 * F)
planes = [luma, chroma]
nbs = [F * 480 * 270, 2 * F * 240 * 135]
nblk = sum(nbs)
coef = [torch.empty((n, 64), dtype=torch.int16, device="cuda") for n in nbs]
rec = [torch.empty((n, 64), dtype=torch.float32, device="cuda") for n in nbs]
stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
descs = (dct_amd._Plane * 2)(*[dct_amd.plane_desc(p) for p in planes])
arr = lambda ts: C.cast((C.c_void_p * len(ts))(*[t.data_ptr() for t in ts]), C.c_void_p)  # noqa: E731
libs = {"default": dct_amd.LIB_PATH}
for p in sorted(glob.glob(os.path.join(ROOT, "tools", "ubench", "libvar_*.so"))):
    libs[os.path.basename(p)[len("libvar_"):-3]] = p
jobs = {}
for name, path in libs.items():
    L = C.CDLL(path)
    L.dctq_plan_create.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_void_p)]
    L.dctq_round_trip_planes.argtypes = [C.c_void_p, C.POINTER(dct_amd._Plane), C.c_int] + [C.c_void_p] * 4
    h = C.c_void_p()
    assert L.dctq_plan_create(50, AD, C.byref(h)) == 0
    jobs[("round_trip", name)] = (lambda L=L, h=h: L.dctq_round_trip_planes(h, descs, 2, arr(coef), None, arr(rec),
                                                                         stream))
t_end = time.perf_counter() + 0.3
while time.perf_counter() < t_end:
    for _ in range(4):
        jobs[("round_trip", "default")]()
    torch.cuda.synchronize()
ref = None
times = {k: [] for k in jobs}
for r in range(ROUNDS + 1):
    for key, fn in jobs.items():
        assert fn() == 0
        torch.cuda.synchronize()
        if r == 0:
            got = [c.clone() for c in coef] + [x.clone() for x in rec]
            if ref is None:
                ref = got
            else:
                assert all(torch.equal(a, b) for a, b in zip(ref, got)), f"{key} differs"
            continue
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(B2B):
            fn()
        e1.record()
        torch.cuda.synchronize()
        times[key].append(e0.elapsed_time(e1) * 1e-3 / B2B)
for (op, name), ts in times.items():
    med = statistics.median(ts)
    print(f"{op:10s} {name:10s} adaptive={AD} median {med * 1e6:8.1f} us  {nblk / med / 1e9:6.2f} G blocks/s  "
          f"{nblk * 448 / med / 8e12 * 100:5.1f} % of 8 TB/s (448 B/block)", flush=True)
