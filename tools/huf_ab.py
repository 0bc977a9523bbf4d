"""A/B of dctq_huffman_bits between the default libdct_amd.so and diagnostic
builds (tools/ubench/libvar_*.so; libvar_no*.so are ablations whose output is not
checked), same quantized planes (64 4K luma frames of
each input kind, q50), interleaved, HIP events; outputs must match.

    python tools/huf_ab.py [frames] [--pixels]

--pixels: dctq_huffman_bits_planes (forward + quantization + sizes in one launch,
huffman_from_pixels_kernel) over the same luma frames instead.
"""
import ctypes as C
import glob
import os
import statistics
import time
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import dct_amd  # noqa: E402

PIXELS = "--pixels" in sys.argv
argv = [a for a in sys.argv[1:] if a != "--pixels"]
F = int(argv[0]) if argv else 64
nblk = F * 480 * 270
libs = {"default": dct_amd.lib()}
for p in sorted(glob.glob(os.path.join(ROOT, "tools", "ubench", "libvar_*.so"))):
    L = C.CDLL(p)
    L.dctq_huffman_bits.argtypes = [C.c_void_p, C.c_longlong, C.c_void_p, C.c_void_p]
    libs[os.path.basename(p)[7:-3]] = L
plans = {}
for k, L in libs.items():
    L.dctq_plan_create.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_void_p)]
    h = C.c_void_p()
    assert L.dctq_plan_create(50, 0, C.byref(h)) == 0
    L.dctq_huffman_bits_planes.argtypes = [C.c_void_p, C.POINTER(dct_amd._Plane), C.c_int, C.c_void_p, C.c_void_p]
    plans[k] = h
s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
for kind in ("uniform", "smooth", "const", "extreme"):
    px = dct_amd.synth(9, kind, 3840, 2160, F)
    desc = dct_amd.plane_desc(px)
    coef = dct_amd.Plan(50, 0).forward_quant(px)
    out = torch.zeros(nblk, dtype=torch.int32, device="cuda")  # shared by every build (see tools/rle_ab.py)
    ref = None
    times = {k: [] for k in libs}
    t_pre = time.perf_counter()  # ~30 ms of launches back to back first: an idle box drops its clocks
    while time.perf_counter() - t_pre < 0.03:
        for _ in range(4):
            assert libs["default"].dctq_huffman_bits(C.c_void_p(coef.data_ptr()), nblk, C.c_void_p(out.data_ptr()), s) == 0
        torch.cuda.synchronize()
    for r in range(9):
        for k, L in libs.items():
            # steady state: one untimed launch, then 3 back to back (the bench's method)
            if PIXELS:
                launch = lambda: L.dctq_huffman_bits_planes(plans[k], C.byref(desc), 1, C.c_void_p(out.data_ptr()), s)
            else:
                launch = lambda: L.dctq_huffman_bits(C.c_void_p(coef.data_ptr()), nblk, C.c_void_p(out.data_ptr()), s)
            assert launch() == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                assert launch() == 0
            e1.record()
            torch.cuda.synchronize()
            if r:
                times[k].append(e0.elapsed_time(e1) * 1e-3 / 3)
            elif ref is None:
                ref = out.clone()
            elif not k.startswith("no"):  # libvar_no*.so: timing ablations, outputs knowingly wrong
                assert torch.equal(out, ref), f"{k} differs on {kind}"
    for k in libs:
        med = statistics.median(times[k])
        print(f"{kind:8s} {k:12s} median {med * 1e6:7.1f} us  {nblk / med / 1e9:6.2f} Gblk/s", flush=True)
