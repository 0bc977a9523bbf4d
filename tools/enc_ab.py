"""Same-box A/B of the encoder (dctq_encode_planes16 / dctq_encode_planes) between the
product library and diagnostic builds (tools/ubench/libvar_*.so) on the bench's encode
step: 64 4K 4:2:0 frames (Y stack + Cb/Cr stack), q50, interleaved rounds, each sample
3 launches back to back after one untimed launch; every build's coefficients, offsets
and symbols compared with the product's.

    python tools/enc_ab.py [--rounds 10] [--kind uniform] [--symbol-bytes 2]
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
ap.add_argument("--symbol-bytes", type=int, default=2, choices=(2, 4))
args = ap.parse_args()

F = args.frames
planes = [dct_amd.synth(12345, args.kind, 3840, 2160, F), dct_amd.synth(12345 + 50000, args.kind, 1920, 1080, 2 * F)]
nbs = [F * 480 * 270, 2 * F * 240 * 135]
nb = sum(nbs)
descs = (dct_amd._Plane * 2)(*[dct_amd.plane_desc(p) for p in planes])
co = [torch.empty((n, 64), dtype=torch.int16, device="cuda") for n in nbs]
cp = C.cast((C.c_void_p * 2)(*[t.data_ptr() for t in co]), C.c_void_p)
off = torch.empty(nb + 1, dtype=torch.int32, device="cuda")
cap = 64 * nb
sym = torch.empty(cap, dtype=torch.int16 if args.symbol_bytes == 2 else torch.int32, device="cuda")
stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)

libs = {"default": dct_amd.LIB_PATH}
for p in sorted(glob.glob(os.path.join(ROOT, "tools", "ubench", "libvar_*.so"))):
    libs[os.path.basename(p)[7:-3]] = p
runs = {}
for k, path in libs.items():
    L = C.CDLL(path)
    L.dctq_plan_create.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_void_p)]
    L.dctq_encode_workspace_bytes.argtypes = [C.c_longlong]
    L.dctq_encode_workspace_bytes.restype = C.c_size_t
    fn = L.dctq_encode_planes16 if args.symbol_bytes == 2 else L.dctq_encode_planes
    fn.argtypes = [C.c_void_p, C.POINTER(dct_amd._Plane), C.c_int] + [C.c_void_p] * 3 + [C.c_longlong] + [C.c_void_p] * 2
    h = C.c_void_p()
    assert L.dctq_plan_create(50, 0, C.byref(h)) == 0
    ws = torch.empty(int(L.dctq_encode_workspace_bytes(nb)) // 4 + 1, dtype=torch.int32, device="cuda")
    runs[k] = (lambda fn=fn, h=h, ws=ws: fn(h, descs, 2, cp, off.data_ptr(), sym.data_ptr(), cap, ws.data_ptr(), stream),
               ws)

times = {k: [] for k in runs}
for r in range(args.rounds + 1):
    for k, (fn, _) in runs.items():
        assert fn() == 0, k
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            fn()
        e1.record()
        torch.cuda.synchronize()
        if r:
            times[k].append(e0.elapsed_time(e1) / 3 * 1e-3)
ref = None
for k, (fn, _) in runs.items():
    assert fn() == 0, k
    torch.cuda.synchronize()
    total = int(off[nb].item()) & 0xFFFFFFFF
    snap = ([t.clone() for t in co], off.clone(), sym[:total].clone())
    if ref is None:
        ref = snap
    same = all(torch.equal(a, b) for a, b in zip(snap[0], ref[0])) and torch.equal(snap[1], ref[1]) and \
        torch.equal(snap[2], ref[2])
    print(f"{k:12s} outputs identical to default: {same}  ({total / nb:.2f} symbols/block)")
    assert same or k.startswith("no"), k  # libvar_no*.so: timing ablations, outputs knowingly wrong
base = statistics.median(times["default"])
for k, v in times.items():
    m = statistics.median(v)
    print(f"{k:12s} median {m * 1e6:8.1f} us  min {min(v) * 1e6:8.1f}  {nb / m / 1e9:6.2f} Gblk/s  x{m / base:5.3f} of default")
