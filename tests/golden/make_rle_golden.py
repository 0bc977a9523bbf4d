#!/usr/bin/env python3
"""RLE / zigzag golden vectors from the REFERENCE (src/entropy.c compiled into
oracle/_ref/libref.so): tests/golden/rle.json.

Blocks: edge cases (all zero, DC only, last element only, first and last,
a full block), the textbook example block's q50 coefficients
(tests/test_entropy.c:290-299) and seeded random sparse / dense blocks."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle as O  # noqa: E402
from golden.make_golden import EXAMPLE  # noqa: E402


def ref_encode(block):
    c = np.ascontiguousarray(block, np.int32).ravel()
    n = int(round(len(c) ** 0.5))
    v = np.zeros(n * n, np.int32)
    r = np.zeros(n * n, np.int32)
    cnt = O.ref().ref_rle_encode(n, c, v, r)
    return v[:cnt].tolist(), r[:cnt].tolist()


def ref_decode(values, runs, n=8):
    out = np.zeros(n * n, np.int32)
    O.ref().ref_rle_decode(n, np.array(values, np.int32), np.array(runs, np.int32), len(values), out)
    return out.tolist()


if __name__ == "__main__":
    rng = np.random.default_rng(2025)
    blocks = {"zero": np.zeros(64, int), "dc": np.eye(1, 64, 0, dtype=int)[0] * -26,
              "last": np.eye(1, 64, 63, dtype=int)[0] * 5, "first_last": np.eye(1, 64, 0, dtype=int)[0] * 3
              + np.eye(1, 64, 63, dtype=int)[0] * -1, "full": rng.integers(1, 9, 64) * rng.choice([-1, 1], 64)}
    x = EXAMPLE.reshape(8, 8).astype(np.float64) - 128.0
    blocks["example_q50"] = O.quantize(O.forward(x), 50).ravel()
    for k in range(40):
        dens = [0.03, 0.1, 0.3, 0.7][k % 4]
        b = rng.integers(-300, 300, 64) * (rng.random(64) < dens)
        blocks[f"random_{k}"] = b
    out = {"zigzag": {}, "blocks": {}}
    for n in (4, 8, 16):
        zz = np.zeros(n * n, np.int32)
        O.ref().ref_zigzag(n, np.arange(n * n, dtype=np.int32), zz)
        out["zigzag"][str(n)] = zz.tolist()
    for name, b in blocks.items():
        v, r = ref_encode(b)
        out["blocks"][name] = {"coeffs": [int(t) for t in b], "values": v, "runs": r, "decoded": ref_decode(v, r)}
    json.dump(out, open(os.path.join(ROOT, "tests", "golden", "rle.json"), "w"))
    print(len(out["blocks"]), "blocks")
