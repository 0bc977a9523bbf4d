"""Compare two forward-kernel variants on one input and describe where they differ."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dct_amd  # noqa: E402
import oracle as O  # noqa: E402

va, vb = sys.argv[1], sys.argv[2]
F = int(sys.argv[3]) if len(sys.argv) > 3 else 1
px = dct_amd.synth(7, "uniform", 3840, 2160, F)
outs = {}
for v in (va, vb):
    plan = dct_amd.Plan(50, 0, variant=int(v))
    outs[v] = plan.forward_quant(px).cpu().numpy()
want = O.forward_plane(px[0].cpu().numpy(), 50, 0, 8)
n0 = want.shape[0]
for v, o in outs.items():
    bad = np.nonzero((o[:n0] != want).any(1))[0]
    print(f"variant {v}: {len(bad)} of {n0} blocks differ from the oracle")
    if len(bad):
        print("  first blocks:", bad[:20].tolist())
        print("  batch ids:", np.unique(bad // 64)[:20].tolist(), "count", len(np.unique(bad // 64)))
        b = bad[0]
        print("  coef diff positions of first bad block:", np.nonzero(o[b] != want[b])[0].tolist())
        print("  got :", o[b][:16].tolist())
        print("  want:", want[b][:16].tolist())
        allzero = (o[bad] == 0).all(1).sum()
        print("  bad blocks all-zero:", int(allzero))
