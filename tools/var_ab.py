"""Same-box timing of the forward launch with and without the var_num output
(profiles/r01: the luma stack WITH var_num measured 283.9 us against 473.5 us
for the bench's 2-plane launch without it -- is the extra store faster?)."""
import statistics
import sys
import os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dct_amd  # noqa: E402

F = 64
y = dct_amd.synth(12345, "uniform", 3840, 2160, F)
c = dct_amd.synth(12345 + 50000, "uniform", 1920, 1080, 2 * F)
y7 = dct_amd.synth(7, "uniform", 3840, 2160, F)
plan = dct_amd.Plan(50, 0)
ny, nc = F * 480 * 270, 2 * F * 240 * 135
oy = torch.empty((ny, 64), dtype=torch.int16, device="cuda")
oc = torch.empty((nc, 64), dtype=torch.int16, device="cuda")
vy = torch.empty(ny, dtype=torch.int32, device="cuda")
vc = torch.empty(nc, dtype=torch.int32, device="cuda")
cases = {
    "luma": (ny, lambda: plan.forward_quant(y, out=oy)),
    "luma +var": (ny, lambda: plan.forward_quant(y, out=oy, var_num=vy)),
    "luma seed7": (ny, lambda: plan.forward_quant(y7, out=oy)),
    "luma seed7 +var": (ny, lambda: plan.forward_quant(y7, out=oy, var_num=vy)),
    "2-plane": (ny + nc, lambda: plan.forward_quant_planes([y, c], outs=[oy, oc])),
    "2-plane +var": (ny + nc, lambda: plan.forward_quant_planes([y, c], outs=[oy, oc], var_nums=[vy, vc])),
}
for _, fn in cases.values():
    fn()
torch.cuda.synchronize()
times = {k: [] for k in cases}
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 12):
    for k, (_, fn) in cases.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        times[k].append(e0.elapsed_time(e1) * 1e-3)
for k, (n, _) in cases.items():
    med = statistics.median(times[k])
    print(f"{k:18s} {n:9d} blocks  median {med*1e6:7.1f} us  {n*192/med/8e12*100:5.1f} % of 8 TB/s (192 B/blk)")
