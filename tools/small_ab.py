"""Single-frame launches (BASELINE configs[1] 512x512, one 4K 4:2:0 frame) with
the queue kernel forced (Plan(variant=4), diagnostic library) against the default dispatch
(variant 2: in-place ties when every wave has at most one batch), same inputs,
back-to-back launches timed with HIP events, outputs compared.

    python tools/small_ab.py
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dct_amd  # noqa: E402

plans = {}
for v in ("4", "2"):
    plans[v] = dct_amd.Plan(50, 0, variant=int(v))
cases = {"512x512": [dct_amd.synth(3, "uniform", 512, 512)],
         "4K 4:2:0 frame": [dct_amd.synth(4, "uniform", 3840, 2160), dct_amd.synth(5, "uniform", 1920, 1080, 2)]}
for name, planes in cases.items():
    outs = {v: p.forward_quant_planes(planes) for v, p in plans.items()}
    torch.cuda.synchronize()
    for a, b in zip(outs["4"], outs["2"]):
        assert torch.equal(a, b), name
    times = {v: [] for v in plans}
    for r in range(6):
        for v, p in plans.items():
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            evs[0].record()
            for _ in range(100):
                p.forward_quant_planes(planes, outs=outs[v])
            evs[1].record()
            torch.cuda.synchronize()
            if r:
                times[v].append(evs[0].elapsed_time(evs[1]) * 1e-3 / 100)
    for v in plans:
        med = statistics.median(times[v])
        label = "queue kernel (v2)" if v == "4" else "default dispatch"
        print(f"{name:15s} {label:18s} {med * 1e6:7.2f} us per launch", flush=True)
