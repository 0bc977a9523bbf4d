"""How much of bench.py's per-step time is a fixed cost of the timed region
(the host latency of the first launch after the synchronize, the last launch's
drain) rather than the kernel: the timed region of bench.py (sync, ev0, K
steps, ev1, sync) for several K, plus the host time of one step() call.

    python tools/step_overhead.py [--reps 5]
"""
import argparse
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import dct_amd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--frames", type=int, default=64)
args = ap.parse_args()

F = args.frames
luma = dct_amd.synth(12345, "uniform", 3840, 2160, F)
chroma = dct_amd.synth(12345 + 50000, "uniform", 1920, 1080, 2 * F)
coef_y = torch.empty((luma.numel() // 64, 64), dtype=torch.int16, device="cuda")
coef_c = torch.empty((chroma.numel() // 64, 64), dtype=torch.int16, device="cuda")
plan = dct_amd.Plan(50, 0)


def step():
    plan.forward_quant_planes([luma, chroma], outs=[coef_y, coef_c])


t = time.perf_counter()
while time.perf_counter() - t < 0.3:
    for _ in range(8):
        step()
    torch.cuda.synchronize()

# host cost of one call while the GPU is busy (the queue is not empty)
for _ in range(4):
    step()
h = []
for _ in range(200):
    t = time.perf_counter()
    step()
    h.append(time.perf_counter() - t)
torch.cuda.synchronize()
print(f"host time per step() call: median {statistics.median(h) * 1e6:.1f} us, min {min(h) * 1e6:.1f} us")

for K in (5, 10, 20, 50, 100):
    wall, ev = [], []
    for _ in range(args.reps):
        for _ in range(5):
            step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        for _ in range(K):
            step()
        e1.record()
        torch.cuda.synchronize()
        wall.append((time.perf_counter() - t0) / K)
        ev.append(e0.elapsed_time(e1) * 1e-3 / K)
    print(f"K={K:4d}  wall {statistics.median(wall) * 1e6:7.1f} us/step   events {statistics.median(ev) * 1e6:7.1f} us/step")

# steady state without a synchronize in front: ev0 queued behind running work
for K in (10, 20):
    ev = []
    for _ in range(args.reps):
        for _ in range(5):
            step()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(K):
            step()
        e1.record()
        torch.cuda.synchronize()
        ev.append(e0.elapsed_time(e1) * 1e-3 / K)
    print(f"K={K:4d}  queued-behind-work events {statistics.median(ev) * 1e6:7.1f} us/step")
