"""Exact-path recomputations (tie-queue entries) per block and per 64-block
batch of the forward kernel, by input kind and quality (fallback counter).

    python tools/tie_counts.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dct_amd  # noqa: E402

for kind in ("uniform", "smooth", "const", "extreme"):
    px = dct_amd.synth(777, kind, 3840, 2160, 8)
    nblk = 8 * 480 * 270
    for q, a in ((10, 0), (50, 0), (90, 0), (90, 1), (100, 0)):
        plan = dct_amd.Plan(q, a)
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        plan.set_fallback_counter(cnt)
        plan.forward_quant(px)
        torch.cuda.synchronize()
        n = int(cnt.item())
        print(f"{kind:8s} q{q:<3d} a{a}  entries {n:9d}  per block {n / nblk:.4f}  per batch {64 * n / nblk:6.2f}")
