"""Launch tails between back-to-back bench steps: K steps (one multi-plane forward
launch each, 64 4K 4:2:0 frames) on one stream, against the same K steps
alternating over two streams with one output set each (the next launch fills
the CUs the previous one's last waves leave).  Interleaved rounds, host bracket.

    python tools/stream_overlap.py [steps] [rounds]"""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dct_amd  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
R = int(sys.argv[2]) if len(sys.argv) > 2 else 10
F = 64
luma = dct_amd.synth(7, "uniform", 3840, 2160, F)
chroma = dct_amd.synth(50007, "uniform", 1920, 1080, 2 * F)
outs = [[torch.empty((F * 480 * 270, 64), dtype=torch.int16, device="cuda"),
         torch.empty((2 * F * 240 * 135, 64), dtype=torch.int16, device="cuda")] for _ in range(2)]
plan = dct_amd.Plan(50, 0)
nblk = outs[0][0].shape[0] + outs[0][1].shape[0]
streams = [torch.cuda.current_stream(), torch.cuda.Stream()]


def run(nstreams):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        s = streams[k % nstreams]
        with torch.cuda.stream(s):
            plan.forward_quant_planes([luma, chroma], outs=outs[k % nstreams])
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / K


t_end = time.perf_counter() + 0.3
while time.perf_counter() < t_end:
    run(1)
res = {1: [], 2: []}
for r in range(R):
    for n in (1, 2):
        res[n].append(run(n))
for n, v in res.items():
    m = statistics.median(v[1:])
    print(f"{n} stream(s): {m * 1e6:7.1f} us per step  {nblk / m / 1e9:6.2f} G blocks/s = "
          f"{nblk * 192 / m / 8e12 * 100:5.1f} % of 8 TB/s", flush=True)
