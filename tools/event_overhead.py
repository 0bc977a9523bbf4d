"""Cost of HIP event records inside bench.py's timed loop: K back-to-back
bench steps (one multi-plane forward launch each, 64 4K 4:2:0 frames) timed
by the host bracket with 0, 1 or 2 event records per step, interleaved rounds.

    python tools/event_overhead.py [steps] [rounds]"""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dct_amd  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
R = int(sys.argv[2]) if len(sys.argv) > 2 else 12
F = 64
luma = dct_amd.synth(7, "uniform", 3840, 2160, F)
chroma = dct_amd.synth(50007, "uniform", 1920, 1080, 2 * F)
cy = torch.empty((F * 480 * 270, 64), dtype=torch.int16, device="cuda")
cc = torch.empty((2 * F * 240 * 135, 64), dtype=torch.int16, device="cuda")
plan = dct_amd.Plan(50, 0)
nblk = cy.shape[0] + cc.shape[0]


def step():
    plan.forward_quant_planes([luma, chroma], outs=[cy, cc])


t_end = time.perf_counter() + 0.3
while time.perf_counter() < t_end:  # clock ramp
    for _ in range(8):
        step()
    torch.cuda.synchronize()
res = {0: [], 1: [], 2: []}
for r in range(R):
    for ne in (0, 1, 2):
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(K + 1)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(K):
            if ne >= 1:
                evs[k][0].record()
            step()
            if ne == 2:
                evs[k][1].record()
        if ne == 1:
            evs[K][0].record()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if r:
            res[ne].append(el / K)
for ne, v in res.items():
    m = statistics.median(v)
    print(f"{ne} event records per step: {m * 1e6:7.1f} us per step  {nblk / m / 1e9:6.2f} G blocks/s "
          f"= {nblk * 192 / m / 8e12 * 100:5.1f} % of 8 TB/s", flush=True)
