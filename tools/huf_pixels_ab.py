"""A/B of dctq_huffman_bits_planes across builds (default + tools/ubench/libvar_*.so) on the
bench's 64-frame 4K 4:2:0 stack, interleaved, 3 calls back to back per sample; outputs compared.

    python tools/huf_pixels_ab.py [kind] [quality]"""
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

kind = sys.argv[1] if len(sys.argv) > 1 else "uniform"
Q = int(sys.argv[2]) if len(sys.argv) > 2 else 50
planes = [dct_amd.synth(1, kind, 3840, 2160, 64), dct_amd.synth(2, kind, 1920, 1080, 128)]
descs = (dct_amd._Plane * 2)(*[dct_amd.plane_desc(p) for p in planes])
nblk = 64 * 480 * 270 + 128 * 240 * 135
s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
builds = {}
for name, path in [("default", dct_amd.LIB_PATH)] + [
        (os.path.basename(p)[7:-3], p) for p in sorted(glob.glob(os.path.join(ROOT, "tools", "ubench", "libvar_*.so")))]:
    L = dct_amd._bind(C.CDLL(path), False)
    h = C.c_void_p()
    assert L.dctq_plan_create(Q, 0, C.byref(h)) == 0
    builds[name] = (L, h, torch.empty(nblk, dtype=torch.int32, device="cuda"))


def run(name):
    L, h, out = builds[name]
    assert L.dctq_huffman_bits_planes(h, descs, 2, C.c_void_p(out.data_ptr()), s) == 0


t_end = time.perf_counter() + 0.3
while time.perf_counter() < t_end:
    run("default")
    torch.cuda.synchronize()
for name in builds:
    run(name)
torch.cuda.synchronize()
for name, (_, _, out) in builds.items():  # libvar_no*.so are timing ablations: output not checked
    if not name.startswith("no"):
        assert torch.equal(out, builds["default"][2]), f"{name} differs"
times = {k: [] for k in builds}
for r in range(10):
    for name in builds:
        run(name)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            run(name)
        e1.record()
        torch.cuda.synchronize()
        times[name].append(e0.elapsed_time(e1) * 1e-3 / 3)
for name, ts in times.items():
    m = statistics.median(ts)
    print(f"{kind:8s} q{Q:<3d} {name:10s} median {m * 1e6:8.1f} us  {nblk / m / 1e9:6.2f} G blocks/s", flush=True)
