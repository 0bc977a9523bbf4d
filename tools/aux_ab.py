"""Steady-state A/B of diagnostic builds (tools/ubench/libvar_*.so) against the
default library for the paired fp64 kernels (forward_float, inverse) and the
encoder (dctq_encode_planes) on 64 4K luma planes (encoder: the bench's 4:2:0
step): clock pre-warm, then per sample one untimed call followed by 3 timed back
to back, interleaved rounds; outputs compared with the default build's.

    python tools/aux_ab.py [F]"""
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

F = int(sys.argv[1]) if len(sys.argv) > 1 else 64
ROUNDS, B2B = 8, 3
px = dct_amd.synth(7, "uniform", 3840, 2160, F)
chroma = dct_amd.synth(8, "uniform", 1920, 1080, 2 * F)
nblk = F * 480 * 270

plans = {"default": dct_amd.Plan(50, 0)}
for p in sorted(glob.glob(os.path.join(ROOT, "tools", "ubench", "libvar_*.so"))):
    name = os.path.basename(p)[len("libvar_"):-3]
    pl = dct_amd.Plan(50, 0)
    L = dct_amd._bind(C.CDLL(p), False)
    h = C.c_void_p()
    assert L.dctq_plan_create(50, 0, C.byref(h)) == 0
    pl._L, pl._h = L, h  # the variant library's own plan (the default one is freed with pl's old handle leaked)
    plans[name] = pl
coef = plans["default"].forward_quant(px)
ff = torch.empty((nblk, 64), dtype=torch.float32, device="cuda")
rec = torch.empty((nblk, 64), dtype=torch.float32, device="cuda")
jobs = {}
for name, pl in plans.items():
    jobs[("forward_float", name)] = (lambda pl=pl: pl.forward_float(px, out=ff), lambda: ff)
    jobs[("inverse", name)] = (lambda pl=pl: pl.inverse(coef, out=rec), lambda: rec)
    jobs[("encode", name)] = (lambda pl=pl: pl.encode_planes([px, chroma]), None)
t_end = time.perf_counter() + 0.3
while time.perf_counter() < t_end:
    for _ in range(4):
        jobs[("inverse", "default")][0]()
    torch.cuda.synchronize()
refs, times = {}, {k: [] for k in jobs}
for r in range(ROUNDS + 1):
    for key, (fn, out) in jobs.items():
        res = fn()
        torch.cuda.synchronize()
        if r == 0:
            got = (out().clone(),) if out else (res[1].clone(), res[2].clone())  # offsets, symbols (int32 or int16)
            if key[0] not in refs:
                refs[key[0]] = got
            else:
                assert all(torch.equal(a, b) for a, b in zip(refs[key[0]], got)), f"{key} differs"
            continue
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(B2B):
            fn()
        e1.record()
        torch.cuda.synchronize()
        times[key].append(e0.elapsed_time(e1) * 1e-3 / B2B)
for (op, name), ts in times.items():
    print(f"{op:14s} {name:10s} median {statistics.median(ts) * 1e6:8.1f} us", flush=True)
