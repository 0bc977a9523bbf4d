"""dctq_round_trip_planes on the bench step (F 4K 4:2:0 frames, Y stack + Cb/Cr
stack, one fused launch), 6 launches back to back: a target for rocprofv3 --pmc
passes over roundtrip8 (tools/pmc_rt.sh).

    python tools/rt_one.py [kind] [F] [--adaptive] [--q=50] [--movement]

--movement launches the diagnostic's no-arithmetic twin (roundtrip_movement)
instead, over the same planes.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dct_amd  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
kind = args[0] if args else "uniform"
F = int(args[1]) if len(args) > 1 else 64
AD = int("--adaptive" in sys.argv)
Q = int(next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--q=")), "50"))
luma = dct_amd.synth(12345, kind, 3840, 2160, F)
chroma = dct_amd.synth(12345 + 50000, kind, 1920, 1080, 2 * F)
planes = [luma, chroma]
nbs = [F * 480 * 270, 2 * F * 240 * 135]
coef = [torch.empty((n, 64), dtype=torch.int16, device="cuda") for n in nbs]
rec = [torch.empty((n, 64), dtype=torch.float32, device="cuda") for n in nbs]
if "--movement" in sys.argv:
    plan = dct_amd.Plan(Q, AD, diagnostic=True)
    run = lambda: plan.diag_rt_movement_planes(planes, coef, rec)  # noqa: E731
else:
    plan = dct_amd.Plan(Q, AD)
    run = lambda: plan.round_trip_planes(planes, outs=coef, recons=rec)  # noqa: E731
for _ in range(6):
    run()
torch.cuda.synchronize()
print("ok", sum(nbs), "blocks")
