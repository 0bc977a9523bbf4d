"""Probe of the q99-q100 measurement artifact: the tie-heavy forward
(fdct8_quant_v2, the stash kernel) measured 5-8 % slower through a second library
than through libdct_amd.so in the same process.  One scenario per process:

    python tools/lib_order_probe.py product     # libdct_amd.so only
    python tools/lib_order_probe.py diag        # libdct_amd_diag.so only (its own synth)
    python tools/lib_order_probe.py both        # product first, then the diagnostic library, then product again
    python tools/lib_order_probe.py streams     # product only, on the default stream, then a second stream
                                                # (each stream has its own tie stash), then the first again

Prints the median launch time of the bench step (64 4K 4:2:0 frames, q100) per phase.
"""
import ctypes as C
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import dct_amd  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "both"
Q = int(sys.argv[2]) if len(sys.argv) > 2 else 100
F = 64


def bind(path):
    L = dct_amd._bind(C.CDLL(path), False)
    return L


def synth_with(L, seed, w, h, f):
    t = torch.empty((f, h, w), dtype=torch.uint8, device="cuda")
    d = dct_amd.plane_desc(t)
    assert L.dctq_synth(seed, 0, C.byref(d), C.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
    return t


def run(L, planes, outs, stream, reps=10, b2b=3):
    h = C.c_void_p()
    assert L.dctq_plan_create(Q, 0, C.byref(h)) == 0
    descs = (dct_amd._Plane * 2)(*[dct_amd.plane_desc(p) for p in planes])
    optr = (C.c_void_p * 2)(*[o.data_ptr() for o in outs])
    s = C.c_void_p(stream.cuda_stream)

    def launch():
        assert L.dctq_forward_quant_planes(h, descs, 2, C.cast(optr, C.c_void_p), None, s) == 0

    ts = []
    with torch.cuda.stream(stream):
        for r in range(reps + 2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            launch()
            e0.record(stream)
            for _ in range(b2b):
                launch()
            e1.record(stream)
            stream.synchronize()
            if r >= 2:
                ts.append(e0.elapsed_time(e1) * 1e3 / b2b)
    L.dctq_plan_destroy(h)
    return statistics.median(ts), min(ts)


P = bind(dct_amd.LIB_PATH) if mode != "diag" else None
D = bind(dct_amd.DIAG_PATH) if mode in ("diag", "both") else None
first = D if mode == "diag" else P
y = synth_with(first, 12345, 3840, 2160, F)
c = synth_with(first, 62345, 1920, 1080, 2 * F)
outs = [torch.empty((F * 480 * 270, 64), dtype=torch.int16, device="cuda"),
        torch.empty((2 * F * 240 * 135, 64), dtype=torch.int16, device="cuda")]
s0 = torch.cuda.current_stream()
phases = {"product": [("product", P, s0)], "diag": [("diag", D, s0)],
          "both": [("product", P, s0), ("diag", D, s0), ("product again", P, s0)],
          "streams": [("product, stream 0", P, s0), ("product, stream 1", P, torch.cuda.Stream()),
                      ("product, stream 0 again", P, s0)]}[mode]
for name, L, st in phases:
    med, mn = run(L, [y, c], outs, st)
    print(f"{mode:8s} q{Q} {name:26s} median {med:7.1f} us  min {mn:7.1f}", flush=True)
