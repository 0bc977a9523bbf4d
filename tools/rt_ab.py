"""Same-box A/B of the fused round trip (BASELINE configs[4]) on the bench step:
64 4K 4:2:0 frames (Y stack + Cb/Cr stack), q50, interleaved rounds, each sample
3 launches back to back after one untimed launch (steady state, HISTORY.md 3.1b).

    python tools/rt_ab.py [--rounds 10] [--kind uniform] [--quality 50] [--adaptive 0] [ENTRY...]

ENTRY: "fused" (the product library), "fused64" (the diagnostic library with the
paired fp64 inverse forced), "flat" (dctq_diag_stream kind 5: the same bytes as a
flat 1:2:4 stream over a constant source), "flatpx" (the same over the workload's own pixel
bytes: HBM moves constant data faster), "flat2" (the same bytes, pixel source, in the round trip's
two-array output layout: coefficients and recon in separate regions), "flat2g" (flat2 with the round
trip's three store groups and their drains), "rows8" (flat2g with the round trip's load shape: 8-byte row
loads per lane, the batch contiguous), "rows2d" (rows8 over a 3840-px-wide plane: the luma row pitch), "rows2d_wg" / "rows2d_wave" (rows2d
with workgroup- / wave-contiguous runs of batches), "rows2d16" (rows2d with 16-byte loads, two rows per
instruction), "flat2g32" / "rows2d32" (flat2g / rows2d on 32 x the resident grid), "mv" (the diagnostic library's movement twin), or "mv:PATH" /
"fused:PATH" (those of a build at PATH, tools/ubench/variant.sh, DIAG=1 for mv).
Default: fused fused64 flat mv.
"""
import argparse
import ctypes as C
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import dct_amd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("entries", nargs="*", default=["fused", "fused64", "flat", "mv"])
ap.add_argument("--rounds", type=int, default=10)
ap.add_argument("--frames", type=int, default=64)
ap.add_argument("--kind", default="uniform")
ap.add_argument("--quality", type=int, default=50)
ap.add_argument("--adaptive", type=int, default=0)
args = ap.parse_args()

F = args.frames
luma = dct_amd.synth(12345, args.kind, 3840, 2160, F)
chroma = dct_amd.synth(12345 + 50000, args.kind, 1920, 1080, 2 * F)
planes = [luma, chroma]
nbs = [F * 480 * 270, 2 * F * 240 * 135]
nblk = sum(nbs)
co = [torch.empty((n, 64), dtype=torch.int16, device="cuda") for n in nbs]
rec = [torch.empty((n, 64), dtype=torch.float32, device="cuda") for n in nbs]
descs = (dct_amd._Plane * 2)(*[dct_amd.plane_desc(p) for p in planes])
stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
cp = C.cast((C.c_void_p * 2)(*[t.data_ptr() for t in co]), C.c_void_p)
rp = C.cast((C.c_void_p * 2)(*[t.data_ptr() for t in rec]), C.c_void_p)
nflat = nblk // 64 * 64
src = torch.full((nflat * 64,), 7, dtype=torch.uint8, device="cuda")  # "flat": a constant source (rounds 3-5)
srcpx = torch.cat([p.reshape(-1) for p in planes])[:nflat * 64].contiguous()  # "flatpx": the workload's pixels
dst = torch.empty(nflat * 384, dtype=torch.uint8, device="cuda")


def lib_plan(path, inverse=None):
    L = C.CDLL(path)
    L.dctq_plan_create.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_void_p)]
    h = C.c_void_p()
    assert L.dctq_plan_create(args.quality, args.adaptive, C.byref(h)) == 0
    if inverse is not None:
        L.dctq_diag_plan_set_inverse.argtypes = [C.c_void_p, C.c_int]
        assert L.dctq_diag_plan_set_inverse(h, inverse) == 0
    return L, h


runs = {}
for e in args.entries:
    kind, _, path = e.partition(":")
    if kind in ("flat", "flatpx", "flat2", "flat2g", "rows8", "rows2d", "rows2d_wg", "rows2d_wave", "rows2d16", "flat2g32", "rows2d32"):
        D = dct_amd.diag()
        buf = src if kind == "flat" else srcpx
        sk = {"flat": 5, "flatpx": 5, "flat2": 8, "flat2g": 9, "rows8": 10, "rows2d": 11, "rows2d_wg": 12, "rows2d_wave": 13, "rows2d16": 15, "flat2g32": 16, "rows2d32": 17}[kind]
        runs[e] = lambda D=D, buf=buf, sk=sk: D.dctq_diag_stream(sk, buf.data_ptr(), dst.data_ptr(), nflat, stream)
        continue
    if kind in ("fused", "fused64"):
        L, h = lib_plan(path or (dct_amd.LIB_PATH if kind == "fused" else dct_amd.DIAG_PATH),
                        0 if kind == "fused64" else None)
        L.dctq_round_trip_planes.argtypes = [C.c_void_p, C.POINTER(dct_amd._Plane), C.c_int] + [C.c_void_p] * 4
        runs[e] = lambda L=L, h=h: L.dctq_round_trip_planes(h, descs, 2, cp, None, rp, stream)
    elif kind == "mv":
        L, h = lib_plan(path or dct_amd.DIAG_PATH)
        L.dctq_diag_rt_movement_planes.argtypes = [C.c_void_p, C.POINTER(dct_amd._Plane), C.c_int] + [C.c_void_p] * 3
        runs[e] = lambda L=L, h=h: L.dctq_diag_rt_movement_planes(h, descs, 2, cp, rp, stream)
    else:
        raise SystemExit(f"unknown entry {e}")

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
# every entry's outputs against the first entry's (coefficients; recon -- the fp64 inverse
# differs from the fp32 one within its bound)
first = None
for k, fn in runs.items():
    if k.startswith(("flat", "rows")):
        continue
    assert fn() == 0, k
    torch.cuda.synchronize()
    snap = ([t.clone() for t in co], [t.clone() for t in rec])
    if first is None:
        first = snap
    same_c = all(torch.equal(a, b) for a, b in zip(snap[0], first[0]))
    same_r = all(torch.equal(a, b) for a, b in zip(snap[1], first[1]))
    dr = max(float((a - b).abs().max()) for a, b in zip(snap[1], first[1]))
    print(f"{k:40s} coef identical {same_c}  recon identical {same_r}  max |d recon| {dr:.3g}")
base = statistics.median(times[args.entries[0]])
for k, v in times.items():
    m = statistics.median(v)
    b = nblk * 448 if k != "flat" else nflat * 448
    print(f"{k:40s} median {m * 1e6:8.1f} us  min {min(v) * 1e6:8.1f}  {b / m / 8e12:6.3f} of 8 TB/s  "
          f"x{m / base:5.3f} of {args.entries[0]}")
