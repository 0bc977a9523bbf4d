"""Generate the golden fixtures in tests/golden/ from the REFERENCE itself.

Every expected value below is produced by the reference's own functions
(/root/reference/src/{dct,quantization,utils}.c compiled by oracle/Makefile into
oracle/_ref/libref.so and driven through oracle/ref_driver.c).  Inputs are
synthetic (the counter-based generator shared by oracle/ and the device) or the
reference tests' own example block (tests/test_dct.c:33-42 ==
tests/test_entropy.c:290-299).  Run in the container where /root/reference
exists:

    make -C oracle && python tests/golden/make_golden.py
"""
from __future__ import annotations

import ctypes as C
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import oracle as O  # noqa: E402

EXAMPLE = np.array([52, 55, 61, 66, 70, 61, 64, 73, 63, 59, 55, 90, 109, 85, 69, 72,
                    62, 59, 68, 113, 144, 104, 66, 73, 63, 58, 71, 122, 154, 106, 70, 69,
                    67, 61, 68, 104, 126, 88, 68, 70, 79, 65, 60, 70, 77, 68, 58, 75,
                    85, 71, 64, 59, 55, 61, 65, 83, 87, 79, 69, 68, 65, 76, 78, 94], np.uint8)

QUALITIES = [1, 10, 25, 50, 75, 90, 100]
TILE = 128          # 128x128 tiles = 256 blocks
SEED = 12345


def bits(a):
    return [int(x) for x in np.asarray(a, np.float64).ravel().view(np.uint64)]


def ref_forward(x):
    out = np.zeros(x.size)
    O.ref().ref_forward(int(round(x.size ** 0.5)), np.ascontiguousarray(x, np.float64).ravel(), out)
    return out


def ref_inverse(c):
    out = np.zeros(c.size)
    O.ref().ref_inverse(int(round(c.size ** 0.5)), np.ascontiguousarray(c, np.float64).ravel(), out)
    return out


def ref_quant(c, q, ad, var):
    out = np.zeros(c.size, np.int32)
    O.ref().ref_quantize(8, q, ad, var, np.ascontiguousarray(c, np.float64).ravel(), out)
    return out


def ref_dequant(qi, q, ad, var):
    out = np.zeros(qi.size)
    O.ref().ref_dequantize(8, q, ad, var, np.ascontiguousarray(qi, np.int32).ravel(), out)
    return out


def ref_plane(px, q, ad):
    h, w = px.shape
    out = np.zeros(((h // 8) * (w // 8), 64), np.int16)
    O.ref().ref_forward_plane(np.ascontiguousarray(px).ravel(), w, h, q, ad, out.ravel(), 8, 0)
    return out


def main():
    O.build()
    r = O.ref()
    fx = {}
    # --- tables (src/dct.c:17-30, src/quantization.c:51-111)
    for n in (4, 8, 16):
        d = np.zeros(n * n)
        r.ref_dct_matrix(n, d)
        fx[f"dct{n}"] = bits(d)
        for q in [0, 1, 10, 25, 49, 50, 51, 75, 90, 99, 100, 101]:
            qq, dq, cq = np.zeros(n * n), np.zeros(n * n), C.c_int()
            r.ref_quant_tables(n, q, 0, qq, dq, C.byref(cq))
            fx[f"q{n}_{q}"] = bits(qq)
            fx[f"dq{n}_{q}"] = bits(dq)
            fx[f"clamped_{q}"] = cq.value
    # --- the reference tests' example block (tests/test_entropy.c:290-373 pipeline)
    x = EXAMPLE.astype(np.float64) - 128.0
    c = ref_forward(x)
    fx["example_forward"] = bits(c)
    var = r.ref_variance(8, x.copy())
    fx["example_variance"] = var
    for q in QUALITIES:
        for ad in (0, 1):
            qi = ref_quant(c, q, ad, var)
            dq = ref_dequant(qi, q, ad, var)
            rec = ref_inverse(dq)
            fx[f"example_q{q}_a{ad}"] = [int(v) for v in qi]
            fx[f"example_dq{q}_a{ad}"] = bits(dq)
            fx[f"example_recon{q}_a{ad}"] = bits(rec)
    fx["example_inverse_of_forward"] = bits(ref_inverse(c))
    ci = np.zeros(64, np.int32)
    r.ref_copy_to_coefficients(8, c.copy(), ci)
    fx["example_round"] = [int(v) for v in ci]
    for vv in (0.0, 8.02, 99.5, 500.0, 864.2, 1000.0, 5000.0):
        for isq in (0, 1):
            m = np.zeros(64)
            r.ref_adjust(8, 50, vv, isq, m)
            fx[f"adjust_50_{vv}_{isq}"] = bits(m)
    # non-8 block sizes through the per-block API
    rng = np.random.default_rng(SEED)
    for n in (4, 16):
        xb = rng.integers(-128, 128, (n, n)).astype(np.float64)
        fx[f"blk{n}_in"] = [int(v) for v in xb.ravel()]
        fx[f"blk{n}_forward"] = bits(ref_forward(xb))
        fx[f"blk{n}_inverse"] = bits(ref_inverse(xb))
    with open(os.path.join(HERE, "reference_blocks.json"), "w") as f:
        json.dump(fx, f, indent=0, sort_keys=True)

    # --- 128x128 tiles of every synthetic kind, quantized by the reference
    arrays = {}
    for kind, k in O.KINDS.items():
        px = O.synth_plane(SEED, k, TILE, TILE)
        arrays[f"{kind}_px"] = px
        for q in QUALITIES:
            for ad in (0, 1):
                arrays[f"{kind}_q{q}_a{ad}"] = ref_plane(px, q, ad)
        # raw double coefficients of the first 32 blocks (float-path tolerance check)
        fl = np.zeros((32, 64))
        for b in range(32):
            by, bx = divmod(b, TILE // 8)
            blk = px[by * 8:by * 8 + 8, bx * 8:bx * 8 + 8].astype(np.float64) - 128.0
            fl[b] = ref_forward(blk)
        arrays[f"{kind}_forward32"] = fl
    np.savez_compressed(os.path.join(HERE, "tiles.npz"), **arrays)

    # --- full-size digests (GPU parity at BASELINE sizes): sha256 of int16 planes
    dig = {"seed": SEED, "entries": []}
    planes = [("4k_luma", 3840, 2160), ("4k_chroma", 1920, 1080), ("512", 512, 512)]
    for name, w, h in planes:
        for kind, k in O.KINDS.items():
            px = O.synth_plane(SEED, k, w, h)
            for q, ad in [(50, 0), (50, 1), (90, 0), (75, 0), (100, 0), (10, 1)]:
                if name == "4k_luma" or (q, ad) in [(50, 0), (90, 0)]:
                    co = ref_plane(px, q, ad)
                    dig["entries"].append({"plane": name, "width": w, "height": h, "kind": kind, "quality": q,
                                           "adaptive": ad, "sha256": hashlib.sha256(co.tobytes()).hexdigest()})
    with open(os.path.join(HERE, "digests.json"), "w") as f:
        json.dump(dig, f, indent=1)
    print("fixtures written:", sorted(os.listdir(HERE)))


if __name__ == "__main__":
    main()
