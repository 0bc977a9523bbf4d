"""Probe the float forward / inverse kernels with simple inputs (diagnostic)."""
import os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dct_amd, oracle as O
np.set_printoptions(linewidth=200, precision=4, suppress=True)
plan = dct_amd.Plan(50, 0)
for name, px in [("const129", np.full((8, 64), 129, np.uint8)),
                 ("impulse", np.pad(np.full((8, 8), 128, np.uint8), ((0, 0), (0, 56)), constant_values=128))]:
    if name == "impulse":
        px = px.copy(); px[0, 0] = 129
    got = plan.forward_float(torch.from_numpy(np.ascontiguousarray(px)).cuda()).cpu().numpy()
    _, want = O.forward_plane(px, 50, 0, want_float=True)
    print(name, "got block0\n", got[0].reshape(8, 8), "\nwant\n", want.reshape(-1, 64)[0].reshape(8, 8))
