"""A/B of diagnostic builds of libdct_amd.so on the bench step: the one
multi-plane forward launch over 64 4K 4:2:0 frames (Y stack + Cb/Cr stack),
interleaved rounds, HIP events, medians; every build's output compared with
the first build's (bit-exact builds must agree).

    python tools/lib_ab.py [--rounds 12] [--kind uniform] [--quality 50] [--adaptive 0] LIB...

LIB = path of a .so (tools/ubench/variant.sh / policy.sh output), "default", or
"movement" (the diagnostic build's dctq_diag_movement_planes: the same bytes, no math),
or "movement:PATH" (the movement kernel of a diagnostic build at PATH, e.g. one
built by policy.sh with DIAG=1).
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
ap.add_argument("libs", nargs="+")
ap.add_argument("--rounds", type=int, default=12)
ap.add_argument("--frames", type=int, default=64)
ap.add_argument("--kind", default="uniform")
ap.add_argument("--quality", type=int, default=50)
ap.add_argument("--adaptive", type=int, default=0)
ap.add_argument("--luma-only", action="store_true")
ap.add_argument("--chroma-only", action="store_true")
ap.add_argument("--b2b", type=int, default=1,
                help="launches back to back per timed sample (steady state: each launch pays for the write-back "
                     "its predecessor left in the caches; with 1, a variant's deferred write-back is charged to "
                     "the next variant in the rotation)")
args = ap.parse_args()

F = args.frames
y = dct_amd.synth(12345, args.kind, 3840, 2160, F)
c = dct_amd.synth(12345 + 50000, args.kind, 1920, 1080, 2 * F)
planes = [y] if args.luma_only else [c] if args.chroma_only else [y, c]
descs = (dct_amd._Plane * len(planes))(*[dct_amd.plane_desc(p) for p in planes])
nbs = [p.shape[0] * (p.shape[1] // 8) * (p.shape[2] // 8) for p in planes]
nblk = sum(nbs)
outs = [torch.empty((n, 64), dtype=torch.int16, device="cuda") for n in nbs]
optr = (C.c_void_p * len(planes))(*[o.data_ptr() for o in outs])
stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)

builds = {}
for path in args.libs:
    mv8 = path == "movement8"  # the movement diagnostic on the x8 grid (dctq_diag_movement_grid_planes)
    mv = mv8 or path == "movement" or path.startswith("movement:")
    p = {"default": dct_amd.LIB_PATH, "movement": dct_amd.DIAG_PATH, "movement8": dct_amd.DIAG_PATH}.get(path) or \
        os.path.abspath(path.split(":", 1)[-1])
    L = C.CDLL(p)
    L.dctq_plan_create.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_void_p)]
    L.dctq_forward_quant_planes.argtypes = [C.c_void_p, C.POINTER(dct_amd._Plane), C.c_int, C.c_void_p, C.c_void_p,
                                            C.c_void_p]
    h = C.c_void_p()
    assert L.dctq_plan_create(args.quality, args.adaptive, C.byref(h)) == 0
    if mv:
        L.dctq_diag_movement_planes.argtypes = [C.c_void_p, C.POINTER(dct_amd._Plane), C.c_int, C.c_void_p,
                                                C.c_void_p]
    if mv8:
        L.dctq_diag_movement_grid_planes.argtypes = [C.c_void_p, C.POINTER(dct_amd._Plane), C.c_int, C.c_void_p,
                                                     C.c_int, C.c_void_p]
    builds[("movement8:" if mv8 else "movement:" if mv else "") + os.path.basename(p)] = (L, h)


def launch(L, h, name=""):
    if name.startswith("movement8:"):
        rc = L.dctq_diag_movement_grid_planes(h, descs, len(planes), C.cast(optr, C.c_void_p), 8, stream)
    elif name.startswith("movement:"):
        rc = L.dctq_diag_movement_planes(h, descs, len(planes), C.cast(optr, C.c_void_p), stream)
    else:
        rc = L.dctq_forward_quant_planes(h, descs, len(planes), C.cast(optr, C.c_void_p), None, stream)
    assert rc == 0, rc


ref = None
for name, (L, h) in builds.items():
    if name.startswith("movement"):
        continue
    for o in outs:
        o.zero_()
    launch(L, h, name)
    torch.cuda.synchronize()
    got = [o.clone() for o in outs]
    if ref is None:
        ref = got
    elif not all(torch.equal(a, b) for a, b in zip(got, ref)):
        print(f"{name}: OUTPUT DIFFERS from {next(iter(builds))}")
times = {k: [] for k in builds}
for r in range(args.rounds + 2):
    for name, (L, h) in builds.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        launch(L, h, name)  # the variant's own predecessor in the timed window
        e0.record()
        for _ in range(args.b2b):
            launch(L, h, name)
        e1.record()
        torch.cuda.synchronize()
        if r >= 2:
            times[name].append(e0.elapsed_time(e1) * 1e-3 / args.b2b)
for name, ts in times.items():
    med = statistics.median(ts)
    print(f"{name:28s} median {med*1e6:7.1f} us  min {min(ts)*1e6:7.1f}  {nblk*192/med/8e12*100:5.1f} % of 8 TB/s  "
          f"[{args.kind} q{args.quality} a{args.adaptive}{' luma' if args.luma_only else ' chroma' if args.chroma_only else ''}]")
