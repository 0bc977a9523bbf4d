"""Per-launch time series of the bench step's forward launch from a cold start:
does the box need a clock/power ramp before launches reach steady state?

    python tools/ramp.py [--launches 2000] [--every 25] [--sleep-ms 0]

Prints the mean launch time of consecutive groups of `every` launches (HIP
events around each launch), from the first launch of the process on."""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import dct_amd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--launches", type=int, default=2000)
ap.add_argument("--every", type=int, default=25)
ap.add_argument("--sleep-ms", type=float, default=0.0, help="host sleep before the series (GPU idle)")
args = ap.parse_args()

y = dct_amd.synth(12345, "uniform", 3840, 2160, 64)
c = dct_amd.synth(12345 + 50000, "uniform", 1920, 1080, 128)
oy = torch.empty((y.numel() // 64, 64), dtype=torch.int16, device="cuda")
oc = torch.empty((c.numel() // 64, 64), dtype=torch.int16, device="cuda")
plan = dct_amd.Plan(50, 0)
torch.cuda.synchronize()
if args.sleep_ms:
    time.sleep(args.sleep_ms / 1e3)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.launches + 1)]
ev[0].record()
for i in range(args.launches):
    plan.forward_quant_planes([y, c], outs=[oy, oc])
    ev[i + 1].record()
torch.cuda.synchronize()
t = [ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(args.launches)]
nb = oy.shape[0] + oc.shape[0]
cum = 0.0
for g in range(0, args.launches, args.every):
    seg = t[g:g + args.every]
    m = sum(seg) / len(seg)
    print(f"launches {g:5d}-{g + len(seg) - 1:5d}  t0 {cum / 1e3:8.2f} ms  mean {m:7.1f} us  "
          f"{nb * 192 / m / 8e6 * 100:5.1f} % of 8 TB/s  min {min(seg):7.1f}  max {max(seg):7.1f}")
    cum += sum(seg)
