"""Same-box timing of the forward DCT+quant launch per plane geometry: the 64
luma planes alone, the 128 chroma planes alone, and the bench's one
multi-plane launch over both (HIP events, interleaved rounds, median).

    python tools/plane_bench.py [--frames 64] [--rounds 15] [--kind uniform]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dct_amd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=64)
ap.add_argument("--rounds", type=int, default=15)
ap.add_argument("--kind", default="uniform")
ap.add_argument("--quality", type=int, default=50)
ap.add_argument("--adaptive", type=int, default=0)
args = ap.parse_args()

F = args.frames
y = dct_amd.synth(1, args.kind, 3840, 2160, F)
c = dct_amd.synth(2, args.kind, 1920, 1080, 2 * F)
plan = dct_amd.Plan(args.quality, args.adaptive)
dplan = dct_amd.Plan(args.quality, args.adaptive, diagnostic=True)  # movement diagnostic (libdct_amd_diag.so)
ny, nc = F * 480 * 270, 2 * F * 240 * 135
oy = torch.empty((ny, 64), dtype=torch.int16, device="cuda")
oc = torch.empty((nc, 64), dtype=torch.int16, device="cuda")
cases = {
    "luma": (ny, lambda: plan.forward_quant(y, out=oy)),
    "chroma": (nc, lambda: plan.forward_quant(c, out=oc)),
    "luma+chroma (one launch)": (ny + nc, lambda: plan.forward_quant_planes([y, c], outs=[oy, oc])),
    "movement luma": (ny, lambda: dplan.diag_movement_planes([y], [oy])),
    "movement chroma": (nc, lambda: dplan.diag_movement_planes([c], [oc])),
    "movement luma+chroma": (ny + nc, lambda: dplan.diag_movement_planes([y, c], [oy, oc])),
}
for _, fn in cases.values():
    fn()
torch.cuda.synchronize()
times = {k: [] for k in cases}
for _ in range(args.rounds):
    for k, (_, fn) in cases.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        times[k].append(e0.elapsed_time(e1) * 1e-3)
for k, (n, _) in cases.items():
    med = statistics.median(times[k])
    print(f"{k:26s} {n:9d} blocks  median {med*1e6:7.1f} us  min {min(times[k])*1e6:7.1f} us  "
          f"{n/med/1e9:6.2f} Gblk/s  {n*192/med/8e12*100:5.1f} % of 8 TB/s  [{args.kind} q{args.quality} a{args.adaptive}]")
