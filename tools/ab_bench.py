"""Interleaved A/B timing of fdct8_quant variants in ONE process (rule 24 of the
HIP guide): same inputs, rounds alternate variants, report median/min per variant.

    python tools/ab_bench.py [--frames 64] [--rounds 10] [--variants 1,2] [--kind uniform] [--quality 50]
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
ap.add_argument("--rounds", type=int, default=10)
ap.add_argument("--variants", default="1,2")
ap.add_argument("--kind", default="uniform")
ap.add_argument("--quality", type=int, default=50)
ap.add_argument("--adaptive", type=int, default=0)
ap.add_argument("--no-check", action="store_true", help="timing only (diagnostic variants may differ)")
ap.add_argument("--b2b", type=int, default=0, help="also time N back-to-back launches per variant (no host sync)")
args = ap.parse_args()

W, H = 3840, 2160
px = dct_amd.synth(7, args.kind, W, H, args.frames)
nblk = args.frames * (W // 8) * (H // 8)
plans = {}
for v in args.variants.split(","):
    plans[v] = dct_amd.Plan(args.quality, args.adaptive, variant=int(v))
# ONE output buffer shared by the variants (separate buffers put their stores on
# different physical pages: +-12 % seen on identical code, tools/rle_ab.py)
out = torch.empty((nblk, 64), dtype=torch.int16, device="cuda")
ref = None
for v, p in plans.items():
    p.forward_quant(px, out=out)
    torch.cuda.synchronize()
    if ref is None:
        ref = out.clone()
    elif not args.no_check:
        assert torch.equal(ref, out), f"variant {v} differs"
times = {v: [] for v in plans}
for r in range(args.rounds):
    for v, p in plans.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        p.forward_quant(px, out=out)
        e1.record()
        torch.cuda.synchronize()
        times[v].append(e0.elapsed_time(e1) * 1e-3)
for v, ts in times.items():
    med = statistics.median(ts)
    print(f"variant {v}: median {med*1e6:.1f} us  min {min(ts)*1e6:.1f} us  -> {nblk/med/1e9:.2f} Gblk/s, "
          f"{nblk*192/med/1e9:.0f} GB/s ({nblk*192/med/8e12*100:.1f}% of 8 TB/s)  [{args.kind} q{args.quality} a{args.adaptive}]")

if args.b2b:
    for v, p in plans.items():
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.b2b + 1)]
        torch.cuda.synchronize()
        evs[0].record()
        for k in range(args.b2b):
            p.forward_quant(px, out=out)
            evs[k + 1].record()
        torch.cuda.synchronize()
        ts = [evs[k].elapsed_time(evs[k + 1]) * 1e-3 for k in range(args.b2b)]
        med = statistics.median(ts)
        print(f"variant {v} back-to-back x{args.b2b}: median {med*1e6:.1f} us  min {min(ts)*1e6:.1f} us  "
              f"({nblk*192/med/8e12*100:.1f}% of 8 TB/s)")
