"""Structure of the exact ties of an input kind (CPU, oracle synth + numpy fp64
DCT): entries per flagged block, coefficient positions, flagged lanes per
64-block batch.  Decides whether per-block queue entries (block, 64-bit mask)
would save exact-path work over per-coefficient ones.

    python tools/tie_structure.py [kind] [q ...]"""
import os
import sys
from collections import Counter

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402  (test infrastructure: an analysis tool, not a product path)

kind = sys.argv[1] if len(sys.argv) > 1 else "extreme"
qs = [int(a) for a in sys.argv[2:]] or [10, 100]
px = oracle.synth_plane(777, oracle.KINDS[kind], 3840, 2160).astype(np.float64) - 128.0
D = oracle.dct_matrix(8)
b = px.reshape(270, 8, 480, 8).transpose(0, 2, 1, 3).reshape(-1, 8, 8)
for q in qs:
    Y = np.einsum("ik,bkl,jl->bij", D, b, D) / oracle.quant_matrix(8, q)
    tie = np.abs(np.abs(Y) - np.floor(np.abs(Y)) - 0.5) < 1e-7  # exact ties up to fp64 noise
    per = tie.reshape(len(b), -1).sum(1)
    print(f"{kind} q{q}: exact ties per block {per.mean():.4f}, flagged blocks per block {np.mean(per > 0):.4f}")
    print("  entries per flagged block:", sorted(Counter(per[per > 0].tolist()).items()))
    pos = tie.reshape(len(b), 64).sum(0)
    print("  top coefficients (count, index 8i+j):", sorted([(int(c), i) for i, c in enumerate(pos)], reverse=True)[:6])
    lanes = (per > 0).reshape(-1, 64).sum(1)
    print(f"  flagged lanes per 64-block batch: mean {lanes.mean():.2f}, p10/p50/p90 {np.percentile(lanes, [10, 50, 90])}")
