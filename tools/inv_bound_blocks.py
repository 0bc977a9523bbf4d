"""Which blocks a PER-BLOCK bound would admit to the fp32 inverse (CPU only).

    python tools/inv_bound_blocks.py [--width 1920 --height 1080]

The fused round trip runs its inverse in fp32 only for plans whose worst-case
block is proven within kInvTol = 5e-5 (tools/inv_bound.py: non-adaptive q <= 71,
where the reference's bug-compatible 1/Q dequantization keeps the inverse's inputs
tiny).  Every other plan runs the paired fp64 inverse.  A per-block bound would
use each block's own quantized magnitudes and its own dequantization scale instead
of the plan's maximum.  This script measures what that would buy:

  * exact: max over output pixels p of G[p].B (1 + u) + u (128 + A[p].B) with
    B_k = |q_k| * scale_k * S_u S_v of the block (G, A from tools/inv_bound.py);
  * cheap: the one a kernel could afford per block (64 multiply-adds):
    (max_p G[p]) . B (1 + u) + u (128 + (max_p A[p]) . B);

and reports, per plan and input kind, the fraction of blocks admitted and the
fraction of 64-block batches (one wave of the round trip) admitted whole -- the
only granularity at which a wave can pick its inverse without running both.
Scales: non-adaptive 1/Q (src/quantization.c:139,144); adaptive Q (2 - nv) with the
DC keeping Q (src/quantization.c:136-144,171-211).  Pixels: the oracle's generator
(the bench's synthetic kinds).
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import oracle  # noqa: E402
from aan_model import scales  # noqa: E402
from inv_bound import U, bound, quant_table  # noqa: E402

TOL = 5e-5

ap = argparse.ArgumentParser()
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
args = ap.parse_args()

G, L = bound()
A = np.abs(L)
gmax, amax = G.max(axis=0), A.max(axis=0)
S = np.array(scales())
SS = np.outer(S, S).ravel()

print(f"{'plan':16s} {'kind':8s} {'blocks admitted':>16s} {'(cheap)':>8s} {'batches admitted':>17s} "
      f"{'(cheap)':>8s} {'median bound':>13s}")
for quality, adaptive in [(50, 1), (25, 1), (75, 1), (90, 1), (80, 0), (90, 0), (100, 0)]:
    Q = quant_table(quality).ravel()
    for kind in ("uniform", "smooth", "const", "extreme"):
        px = oracle.synth_plane(7, oracle.KINDS[kind], args.width, args.height)
        q = oracle.forward_plane(px, quality, adaptive).astype(np.float64)
        if adaptive:
            var = oracle.plane_variance(px)
            nv = np.clip(var / 1000.0, 0.1, 1.0)
            scale = Q[None, :] * (2.0 - nv)[:, None]
            scale[:, 0] = Q[0]
        else:
            scale = np.broadcast_to(1.0 / Q, q.shape)
        B = np.abs(q) * scale * SS
        exact = ((B @ G.T) * (1 + U) + U * (128.0 + B @ A.T)).max(axis=1) + 1e-9
        cheap = (B @ gmax) * (1 + U) + U * (128.0 + B @ amax) + 1e-9
        nb = len(exact) // 64 * 64
        ok_e, ok_c = exact <= TOL, cheap <= TOL
        be = ok_e[:nb].reshape(-1, 64).all(axis=1).mean()
        bc = ok_c[:nb].reshape(-1, 64).all(axis=1).mean()
        name = f"q{quality} {'adaptive' if adaptive else 'fixed'}"
        print(f"{name:16s} {kind:8s} {ok_e.mean():16.3f} {ok_c.mean():8.3f} {be:17.3f} {bc:8.3f} "
              f"{np.median(exact):13.3g}")
