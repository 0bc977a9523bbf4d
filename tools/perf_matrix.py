"""Forward DCT+quant over the bench's step (64 4K luma + 128 1080p chroma planes, one
multi-plane launch) for every input kind x plan, each next to the no-arithmetic
movement of the same planes (dctq_diag_movement_planes) on the same box.  The
forward runs through the product library (libdct_amd.so), the movement through
the diagnostic one (round 4: through the diagnostic library the tie-heavy rows
read 5-8 % slower, HISTORY.md 8.5):
HIP events, medians of samples of 3 launches back to back after one untimed
launch of the same kind (steady state: profiles/r02/policy_b2b.md).  Prints one
line per configuration.

    python tools/perf_matrix.py [frames]
"""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dct_amd  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 64
ny, nc = F * 480 * 270, 2 * F * 240 * 135
n = ny + nc
oy = torch.empty((ny, 64), dtype=torch.int16, device="cuda")
oc = torch.empty((nc, 64), dtype=torch.int16, device="cuda")
fb = torch.zeros(1, dtype=torch.int64, device="cuda")


def timed(fn, reps=8, b2b=3):
    ts = []
    for r in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        e0.record()
        for _ in range(b2b):
            fn()
        e1.record()
        torch.cuda.synchronize()
        if r:
            ts.append(e0.elapsed_time(e1) * 1e-3 / b2b)
    return statistics.median(ts)


# clock ramp (profiles/r02/clock_ramp.md): an idle box needs ~25 ms of load to leave its low clocks,
# which the first configuration's samples would otherwise absorb
_y = dct_amd.synth(1, "uniform", 3840, 2160, F)
_c = dct_amd.synth(2, "uniform", 1920, 1080, 2 * F)
_p = dct_amd.Plan(50, 0)
_t = time.perf_counter()
while time.perf_counter() - _t < 0.3:
    for _ in range(8):
        _p.forward_quant_planes([_y, _c], outs=[oy, oc])
    torch.cuda.synchronize()
del _y, _c, _p

print(f"{'kind':8s} {'plan':8s} {'forward us':>10s} {'% 8TB/s':>8s} {'ceiling us':>10s} {'% 8TB/s':>8s} "
      f"{'fwd/ceil':>8s} {'ties/blk':>8s}")
for kind in ("uniform", "smooth", "const", "extreme"):
    y = dct_amd.synth(12345, kind, 3840, 2160, F)
    c = dct_amd.synth(62345, kind, 1920, 1080, 2 * F)
    for q, ad in ((50, 0), (90, 0), (50, 1), (10, 0), (100, 0)):
        plan = dct_amd.Plan(q, ad)
        dplan = dct_amd.Plan(q, ad, diagnostic=True)
        fb.zero_()
        plan.set_fallback_counter(fb)
        plan.forward_quant_planes([y, c], outs=[oy, oc])
        torch.cuda.synchronize()
        ties = int(fb.item()) / n
        plan.set_fallback_counter(None)
        tf = timed(lambda: plan.forward_quant_planes([y, c], outs=[oy, oc]))
        tm = timed(lambda: dplan.diag_movement_planes([y, c], [oy, oc]))
        gf, gm = n * 192 / tf / 8e12 * 100, n * 192 / tm / 8e12 * 100
        print(f"{kind:8s} q{q}a{ad:<5d} {tf * 1e6:10.1f} {gf:8.1f} {tm * 1e6:10.1f} {gm:8.1f} {tm / tf:8.3f} "
              f"{ties:8.4f}", flush=True)
