#!/usr/bin/env python3
"""Per-block Huffman size golden vectors from the REFERENCE (src/entropy.c
compiled into oracle/_ref/libref.so, driven by oracle/ref_driver.c
ref_huffman_bits = run_length_encode -> build_huffman_codes -> get_encoded_size,
as tests/test_entropy.c:329-341 calls them): tests/golden/huffman.json.

Blocks: edge cases (all zero, one value repeated, last element only, 64
distinct values, extreme magnitudes, frequency ties of every shape), the
textbook example block's q50/q90 coefficients (tests/test_entropy.c:290-299)
and seeded random blocks of several densities and amplitudes.  Run where
/root/reference exists:  make -C oracle && python tests/golden/make_huffman_golden.py"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle as O  # noqa: E402
from golden.make_golden import EXAMPLE  # noqa: E402


def ref_bits(block):
    c = np.ascontiguousarray(block, np.int32).ravel()
    ns, nc = C.c_int(), C.c_int()
    bits = O.ref().ref_huffman_bits(8, c, C.byref(ns), C.byref(nc))
    return bits, ns.value, nc.value


def blocks():
    rng = np.random.default_rng(4242)
    e = lambda i, v: np.eye(1, 64, i, dtype=int)[0] * v  # noqa: E731
    out = {"zero": np.zeros(64, int), "dc": e(0, -26), "last": e(63, 5), "last_neg": e(63, -1024),
           "all_same": np.full(64, 3), "all_same_last_zero": np.r_[np.full(63, -7), 0],
           "distinct64": np.arange(1, 65) * np.where(np.arange(64) % 2, 1, -1),
           "extremes": np.where(np.arange(64) % 2, 1024, -1024), "two_values": np.where(np.arange(64) < 32, 1, 2),
           "pow2_freqs": np.repeat([1, 2, 3, 4, 5, 6, 7], [32, 16, 8, 4, 2, 1, 1]),
           "fib_freqs": np.r_[np.repeat([9, 8, 7, 6, 5, 4, 3, 2, 1], [21, 13, 8, 5, 3, 2, 1, 1, 1]), np.zeros(9, int)],
           "ties_equal": np.r_[np.repeat(np.arange(1, 17), 2), np.zeros(32, int)],
           "int16_range": np.r_[np.full(32, 32767), np.full(32, -32768)]}
    x = EXAMPLE.reshape(8, 8).astype(np.float64) - 128.0
    for q in (10, 50, 90):
        out[f"example_q{q}"] = O.quantize(O.forward(x), q).ravel()
    for k in range(120):
        dens = [0.02, 0.1, 0.3, 0.6, 0.9, 1.0][k % 6]
        amp = [1, 2, 4, 30, 300, 1024][(k // 6) % 6]
        out[f"random_{k}"] = rng.integers(-amp, amp + 1, 64) * (rng.random(64) < dens)
    return out


if __name__ == "__main__":
    res = {}
    for name, b in blocks().items():
        bits, ns, nc = ref_bits(b)
        res[name] = {"coeffs": [int(t) for t in b], "bits": bits, "symbols": ns, "codes": nc}
    json.dump({"blocks": res}, open(os.path.join(ROOT, "tests", "golden", "huffman.json"), "w"))
    print(len(res), "blocks")
