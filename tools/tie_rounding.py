"""Which way does the reference round an exact .5 tie of a rational coefficient at q100?
For (u, v) in {0, 4}^2 the exact coefficient of an integer block is a multiple of 1/8, so
1 block in 8 is an exact half-integer; the reference's fp64 sum (src/dct.c:57-74, D from
dct_init's expression, src/dct.c:19-30) lands slightly above, below or exactly on it.
Counts over random blocks show the direction is ~evenly split, i.e. there is no cheaper
rule than the reference-order evaluation itself (HISTORY.md 3.2, round 4 session 3).

    python tools/tie_rounding.py [blocks_per_coefficient]"""
import math
import sys
from collections import Counter

import numpy as np

N = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
PI = 3.14159265358979323846  # include/dct.h
D = np.zeros((8, 8))
for i in range(8):
    a = 1.0 / math.sqrt(8) if i == 0 else math.sqrt(2.0 / 8)
    for j in range(8):
        D[i][j] = a * math.cos((PI * (2 * j + 1) * i) / (2.0 * 8))
DT = D.T.copy()


def reference_order(x, u, v):
    t = []
    for k in range(8):
        s = 0.0
        for l in range(8):
            s += float(x[k][l]) * DT[l][v]
        t.append(s)
    o = 0.0
    for k in range(8):
        o += D[u][k] * t[k]
    return o


rng = np.random.default_rng(1)
for u, v in [(0, 0), (0, 4), (4, 0), (4, 4)]:
    c, n = Counter(), 0
    while n < N:
        x = rng.integers(0, 256, (8, 8)).astype(np.int64) - 128
        exact8 = int(np.rint(8 * (D[u][:, None] * x * D[v][None, :]).sum()))  # 8 * coefficient, an integer
        if exact8 % 8 != 4 and exact8 % 8 != -4:
            continue
        n += 1
        e = reference_order(x, u, v) - exact8 / 8
        c["up" if e > 0 else "down" if e < 0 else "exact"] += 1
    print(f"({u},{v}): {dict(c)}")
