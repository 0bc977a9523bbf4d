"""Time the v2 forward kernel against diagnostic builds with parts removed
(tools/ubench/ablate.sh), interleaved in one process.  Outputs of the ablated
builds are wrong by construction; only their time matters."""
import ctypes as C
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import dct_amd  # noqa: E402

libs = {"full": dct_amd.LIB_PATH}
NAMES = {1: "no-tie-flags", 2: "no-butterfly", 8: "flags-no-queue", 16: "append-no-drain", 32: "queue-code-idle",
         64: "no-pixel-loads", 128: "no-coef-stores", 192: "no-loads-no-stores", 194: "no-mem-no-butterfly",
         256: "const-tables", 448: "const-tables-no-mem",
         1024: "no-stash-stores", 1040: "no-stash-no-drain", 2048: "no-final-drain"}
for m, name in sorted(NAMES.items()):
    p = os.path.join(ROOT, "tools", "ubench", f"libablate_{m}.so")
    if os.path.exists(p):
        libs[name] = p
import glob  # noqa: E402
for p in sorted(glob.glob(os.path.join(ROOT, "tools", "ubench", "libpolicy_*.so"))):  # tools/ubench/policy.sh
    libs["policy-" + os.path.basename(p)[len("libpolicy_"):-3]] = p
for p in sorted(glob.glob(os.path.join(ROOT, "tools", "ubench", "libvar_*.so"))):  # tools/ubench/variant.sh
    libs["var-" + os.path.basename(p)[len("libvar_"):-3]] = p
F = int(sys.argv[1]) if len(sys.argv) > 1 else 64
px = dct_amd.synth(7, "uniform", 3840, 2160, F)
d = dct_amd.plane_desc(px)
nblk = F * 480 * 270
out = torch.empty((nblk, 64), dtype=torch.int16, device="cuda")
plans = {}
for name, path in libs.items():
    L = C.CDLL(path)
    L.dctq_plan_create.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_void_p)]
    L.dctq_forward_quant.argtypes = [C.c_void_p, C.POINTER(dct_amd._Plane), C.c_void_p, C.c_void_p, C.c_void_p]
    h = C.c_void_p()
    assert L.dctq_plan_create(50, 0, C.byref(h)) == 0
    plans[name] = (L, h)
stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
times = {k: [] for k in plans}
for r in range(12):
    for name, (L, h) in plans.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        assert L.dctq_forward_quant(h, C.byref(d), C.c_void_p(out.data_ptr()), None, stream) == 0
        e1.record()
        torch.cuda.synchronize()
        if r >= 2:
            times[name].append(e0.elapsed_time(e1) * 1e-3)
# variants that must be correct: compare with the default build
ref = None
for name, (L, h) in plans.items():
    if name == "full" or name.startswith("policy-") or name.startswith("var-"):
        o = torch.zeros_like(out)
        assert L.dctq_forward_quant(h, C.byref(d), C.c_void_p(o.data_ptr()), None, stream) == 0
        torch.cuda.synchronize()
        if ref is None:
            ref = o
        elif not torch.equal(o, ref):
            print(f"{name}: OUTPUT DIFFERS from the default build ({int((o != ref).sum())} coefficients)")
for name, ts in times.items():
    med = statistics.median(ts)
    print(f"{name:24s} median {med*1e6:7.1f} us  {nblk*192/med/1e9:6.0f} GB/s")
