"""CPU: pin the oracle (oracle/dct_oracle.c) to the reference's golden vectors.

The fixtures in tests/golden/ were produced by the reference itself
(tests/golden/make_golden.py over oracle/_ref/libref.so); these tests show the
clean-room restatement reproduces them bit for bit, so the GPU tests can use it
as the checker at sizes the fixtures do not cover."""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle as O
from conftest import ROOT, f64

QUALITIES = [1, 10, 25, 50, 75, 90, 100]


def test_tables_bit_exact(blocks):
    for n in (4, 8, 16):
        assert (O.dct_matrix(n).ravel().view(np.uint64) == np.array(blocks[f"dct{n}"], np.uint64)).all()
        for q in [0, 1, 10, 25, 49, 50, 51, 75, 90, 99, 100, 101]:
            cq = O.orc().orc_clamp_quality(q)
            assert cq == blocks[f"clamped_{q}"]
            qm = O.quant_matrix(n, cq)
            assert (qm.ravel().view(np.uint64) == np.array(blocks[f"q{n}_{q}"], np.uint64)).all(), (n, q)
            dq = O.dequant_matrix(qm)
            assert (dq.ravel().view(np.uint64) == np.array(blocks[f"dq{n}_{q}"], np.uint64)).all(), (n, q)


def test_example_block(blocks):
    from golden.make_golden import EXAMPLE
    x = EXAMPLE.reshape(8, 8).astype(np.float64) - 128.0
    c = O.forward(x)
    assert (c.ravel().view(np.uint64) == np.array(blocks["example_forward"], np.uint64)).all()
    assert c[0, 0] == -415.37499999999994  # SURVEY 4 known answer
    var = O.variance(x)
    assert var == blocks["example_variance"]
    for q in QUALITIES:
        for ad in (0, 1):
            qi = O.quantize(c, q, ad, var)
            assert qi.ravel().tolist() == blocks[f"example_q{q}_a{ad}"], (q, ad)
            dq = O.dequantize(qi, q, ad, var)
            assert (dq.ravel().view(np.uint64) == np.array(blocks[f"example_dq{q}_a{ad}"], np.uint64)).all()
            rec = O.inverse(dq)
            assert (rec.ravel().view(np.uint64) == np.array(blocks[f"example_recon{q}_a{ad}"], np.uint64)).all()
    # textbook JPEG q50 result (tests/test_entropy.c output)
    assert blocks["example_q50_a0"][:8] == [-26, -3, -6, 2, 2, -1, 0, 0]
    assert blocks["example_q90_a0"][:8] == [-130, -14, -31, 9, 12, -3, 0, 0]
    assert (O.inverse(c).ravel().view(np.uint64) == np.array(blocks["example_inverse_of_forward"], np.uint64)).all()


def test_example_block_psnr(blocks):
    """Bug-compatible round trip PSNR of the example block (tests/test_entropy.c:376-393)."""
    from golden.make_golden import EXAMPLE
    rec = f64(blocks["example_recon50_a0"]) + 128.0
    rec = np.clip(rec, 0, 255)
    mse = np.mean((EXAMPLE.astype(np.float64) - rec) ** 2)
    assert round(10 * np.log10(255 * 255 / mse), 2) == 13.21


def test_adjust(blocks):
    q = O.quant_matrix(8, 50)
    dq = O.dequant_matrix(q)
    for vv in (0.0, 8.02, 99.5, 500.0, 864.2, 1000.0, 5000.0):
        for isq in (0, 1):
            m = O.adjust(q if isq else dq, vv, isq)
            assert (m.ravel().view(np.uint64) == np.array(blocks[f"adjust_50_{vv}_{isq}"], np.uint64)).all()


def test_other_block_sizes(blocks):
    for n in (4, 16):
        x = np.array(blocks[f"blk{n}_in"], np.float64).reshape(n, n)
        assert (O.forward(x).ravel().view(np.uint64) == np.array(blocks[f"blk{n}_forward"], np.uint64)).all()
        assert (O.inverse(x).ravel().view(np.uint64) == np.array(blocks[f"blk{n}_inverse"], np.uint64)).all()


@pytest.mark.parametrize("kind", ["uniform", "smooth", "const", "extreme"])
def test_tiles(tiles, kind):
    px = tiles[f"{kind}_px"]
    assert np.array_equal(px, O.synth_plane(12345, O.KINDS[kind], 128, 128))
    for q in QUALITIES:
        for ad in (0, 1):
            assert np.array_equal(O.forward_plane(px, q, ad), tiles[f"{kind}_q{q}_a{ad}"]), (kind, q, ad)
    _, fl = O.forward_plane(px, 50, 0, want_float=True)
    assert (fl[:32].view(np.uint64) == tiles[f"{kind}_forward32"].view(np.uint64)).all()


def test_full_size_digests(digests):
    """BASELINE sizes: sha256 of the oracle's int16 planes == the reference's."""
    for e in digests["entries"]:
        px = O.synth_plane(digests["seed"], O.KINDS[e["kind"]], e["width"], e["height"])
        co = O.forward_plane(px, e["quality"], e["adaptive"], 8)
        assert hashlib.sha256(co.tobytes()).hexdigest() == e["sha256"], e


def test_oracle_vs_compiled_reference_random():
    """Where the compiled reference is present (this container), cross-check random blocks."""
    if not O.ref_available():
        pytest.skip("oracle/_ref/libref.so not built here")
    r = O.ref()
    rng = np.random.default_rng(99)
    for _ in range(300):
        x = rng.integers(-128, 128, (8, 8)).astype(np.float64)
        a = np.zeros(64)
        r.ref_forward(8, x.ravel().copy(), a)
        assert (a.view(np.uint64) == O.forward(x).ravel().view(np.uint64)).all()
        var = O.variance(x)
        for q in (int(rng.integers(1, 101)),):
            for ad in (0, 1):
                qi = np.zeros(64, np.int32)
                r.ref_quantize(8, q, ad, var, a, qi)
                assert (qi == O.quantize(a.reshape(8, 8), q, ad, var).ravel()).all()


def test_synth_kinds_are_distinct():
    a = [O.synth_plane(1, k, 64, 64) for k in range(4)]
    assert len({x.tobytes() for x in a}) == 4
    assert set(np.unique(a[3])) <= {0, 255}
    c = a[2].reshape(8, 8, 8, 8).transpose(0, 2, 1, 3).reshape(64, 64)
    assert (c == c[:, :1]).all()  # constant 8x8 blocks


def test_reference_programs_golden():
    """The committed expected output of the reference's own test programs is what
    they print here, linked against the reference (oracle/_ref/test_*_cpu)."""
    import json
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    want = json.load(open(os.path.join(root, "tests", "golden", "ref_programs.json")))
    for prog, w in want.items():
        exe = os.path.join(root, "oracle", "_ref", f"test_{prog}_cpu")
        if not os.path.exists(exe):
            pytest.skip("oracle/_ref/test_*_cpu not built (needs /root/reference)")
        r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
        assert (r.returncode, r.stdout) == (w["rc"], w["stdout"]), prog


def test_rle_oracle_vs_reference_golden():
    """Zigzag order and run-length symbols (src/entropy.c:158-256,327-351):
    the oracle reproduces the reference's own outputs (tests/golden/rle.json)."""
    import json
    import os
    g = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rle.json")))
    for n, zz in g["zigzag"].items():
        assert O.zigzag_order(int(n)).tolist() == zz, n
    for name, b in g["blocks"].items():
        v, r = O.rle_encode(np.array(b["coeffs"]).reshape(8, 8))
        assert v.tolist() == b["values"] and r.tolist() == b["runs"], name
        assert O.rle_decode(v, r).ravel().tolist() == b["decoded"] == b["coeffs"], name
    # the symbol count is 1 + nnz(all but the last zigzag element) -- what the GPU encoder relies on
    for name, b in g["blocks"].items():
        zz = np.array(b["coeffs"])[O.zigzag_order(8)]
        assert len(b["values"]) == 1 + int(np.count_nonzero(zz[:63])), name


def test_rle_plane_format():
    """Batched device format: offsets + packed (uint16 value | run << 16) symbols."""
    rng = np.random.default_rng(3)
    coef = (rng.integers(-50, 50, (300, 64)) * (rng.random((300, 64)) < 0.2)).astype(np.int16)
    off, sym = O.rle_encode_plane(coef)
    assert off[0] == 0 and off[-1] == len(sym)
    for b in range(coef.shape[0]):
        s = sym[off[b]:off[b + 1]]
        v = (s & 0xFFFF).astype(np.uint16).view(np.int16)
        r = s >> 16
        v2, r2 = O.rle_encode(coef[b].reshape(8, 8))
        assert v.tolist() == v2.tolist() and r.tolist() == r2.tolist()


def test_two_byte_symbols():
    """The 2-byte symbol format (include/dct_amd.h): pack16/unpack16 round-trip every symbol
    of blocks with |q| <= 511 -- runs 0..63, and the all-zero block's (0, 64) as 0x0000, a
    code no other symbol takes -- and refuse what does not fit."""
    rng = np.random.default_rng(5)
    coef = (rng.integers(-511, 512, (400, 64)) * (rng.random((400, 64)) < 0.1)).astype(np.int16)
    coef[:7] = 0                       # all-zero blocks: one symbol (0, 64)
    coef[7, 63] = -511                 # a lone last element: run 63
    coef[8, 62] = 511                  # run 62, then (0, 1)
    off, sym = O.rle_encode_plane(coef)
    s16 = O.pack16(sym)
    assert np.array_equal(O.unpack16(s16), sym)
    zero_blocks = [b for b in range(coef.shape[0]) if not coef[b].any()]
    assert (s16 == 0).sum() == len(zero_blocks) >= 7
    assert all(s16[off[b]] == 0 and off[b + 1] - off[b] == 1 for b in zero_blocks)
    for bad in ([512, 0], [-512, 0]):
        c = np.zeros((1, 64), np.int16)
        c[0, 0] = bad[0]
        with pytest.raises(ValueError):
            O.pack16(O.rle_encode_plane(c)[1])


def _huffman_golden():
    import json
    import os
    return json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "huffman.json")))


def bucket_merge_bits(block):
    """Python model of the GPU's per-block Huffman size (dct_amd/csrc/huffman.hip):
    frequencies of the symbol values (every nonzero coefficient, plus one 0 if
    c[63] == 0), then the bucket merge: cnt[w] nodes of weight w, scanned upward,
    pairs within a bucket, an odd node left pending for the next bucket.
    bits = 8 * symbols + sum of internal node weights."""
    c = np.asarray(block).ravel()
    vals = [int(v) for v in c if v != 0] + ([0] if c[63] == 0 else [])
    freq = {}
    for v in vals:
        freq[v] = freq.get(v, 0) + 1
    cnt = [0] * 65
    for f in freq.values():
        cnt[f] += 1
    nodes, wpl, pending = len(freq), 0, 0
    for w in range(1, 65):
        if nodes <= 1:
            break
        c_w = cnt[w]
        if pending and c_w:
            wpl += pending + w
            cnt[pending + w] += 1
            c_w -= 1
            nodes -= 1
            pending = 0
        pairs = c_w // 2
        if pairs:
            wpl += pairs * 2 * w
            nodes -= pairs
            cnt[2 * w] += pairs
        if c_w & 1:
            pending = w
    return 8 * len(vals) + wpl


def test_huffman_oracle_vs_reference_golden():
    """Per-block Huffman size (src/entropy.c:261-328 + 363-399 as tests/test_entropy.c:329-341
    calls them): the oracle's literal restatement of the reference heap reproduces the
    reference's own numbers (tests/golden/huffman.json)."""
    g = _huffman_golden()
    for name, b in g["blocks"].items():
        assert O.huffman_bits(np.array(b["coeffs"])) == b["bits"], name
    plane = np.array([b["coeffs"] for b in g["blocks"].values()], np.int16)
    assert O.huffman_bits_plane(plane).tolist() == [b["bits"] for b in g["blocks"].values()]


def test_huffman_bucket_model_is_exact():
    """The GPU's bucket merge (tie-order free: a Huffman tree's weighted path length is the
    optimum for every tie order) gives the reference's size on the golden blocks and on
    random blocks of every density/amplitude against the oracle."""
    g = _huffman_golden()
    for name, b in g["blocks"].items():
        assert bucket_merge_bits(b["coeffs"]) == b["bits"], name
    rng = np.random.default_rng(99)
    for k in range(3000):
        dens = rng.random()
        amp = int(rng.choice([1, 2, 3, 8, 100, 1024]))
        blk = rng.integers(-amp, amp + 1, 64) * (rng.random(64) < dens)
        assert bucket_merge_bits(blk) == O.huffman_bits(blk), blk.tolist()


def register_merge_wpl(freqs):
    """Python model of the narrow path's register merge (dct_amd/csrc/huffman.hip,
    narrow_merge), operation for operation:
      * leaf weights <= 16 counted in 16 buckets; the bucket merge scans w = 1..16
        (a pending node merges with one node of the next non-empty bucket, the rest
        pair up);
      * a pending merge makes ONE node of weight p + w in (w, 2w), and successive
        ones are strictly heavier, so they are bits of a mask (bit p + w), never
        two in one bucket;
      * every node heavier than 16 -- leaves, pairs of w >= 9 (at most 3 per w, kept
        as 2-bit fields), pending merges -- waits aside.  All node weights add up to
        the symbol count (<= 65), so there are at most 3 of them, and their count,
        sum, min and max give them sorted;
      * the pending node (<= 16, the lightest) and those finish in closed form;
      * the WPL (sum of internal node weights) is the sum of EVERY node's weight but
        the root's (each non-root node is a child of exactly one internal node): the
        nodes of each light bucket (acc), the heavy nodes (hs), the internal nodes of
        the closed-form finish (fin), minus the root (the symbol count).
    Returns the weighted path length."""
    cnt = [0] * 17
    hn, hs, hmn, hmx = 0, 0, 0xFF, 0  # heavy nodes: count, sum, min, max
    for f in freqs:
        if f > 16:
            hn, hs, hmn, hmx = hn + 1, hs + f, min(hmn, f), max(hmx, f)
        else:
            cnt[f] += 1
    p = pm = acc = qp = qs = 0
    for w in range(1, 17):
        c = cnt[w] + (((pm >> w) & 1) if w >= 3 else 0)
        acc += c * w  # bucket w's nodes
        mp = min(p, c) != 0  # the pending node merges with one node of bucket w
        c -= 1 if mp else 0
        pm |= (1 << w) << p if mp else 0
        p = (0 if mp else p) + (c & 1) * w
        pairs = c >> 1
        if 2 * w <= 16:
            cnt[2 * w] += pairs
        else:
            assert pairs <= 3
            qp |= pairs << (2 * (w - 9))
            qs += pairs * 2 * w
    pc = lambda x: bin(x).count("1")  # noqa: E731
    qn = pc(qp & 0x5555) + 2 * pc(qp & 0xAAAA)
    qmn = 18 + 2 * (((qp & -qp).bit_length() - 1) >> 1) if qp else 0xFF
    qmx = 18 + 2 * ((qp.bit_length() - 1) >> 1) if qp else 0
    b = pm & ~0x1FFFF  # pending merges above 16: <= 3 bits
    n = pc(b)
    lo = (b & -b).bit_length() - 1 if b else 0xFF
    hi = b.bit_length() - 1 if b else 0
    mid = ((b & (b - 1)) & -(b & (b - 1))).bit_length() - 1 if n == 3 else 0
    hn += n + qn
    hs += (lo if n else 0) + (mid if n == 3 else 0) + (hi if n >= 2 else 0) + qs
    hmn, hmx = min(hmn, qmn, lo), max(hmx, qmx, hi)
    assert hn <= 3, hn
    h1, h3 = hmn, hmx
    h2 = hs - h1 - h3 if hn == 3 else h3
    if p:  # p < 17 <= h1: nodes p, h1, h2, h3
        s = p + h1
        fin = 2 * s + 2 * h2 + h3 + min(s, h3) if hn == 3 else 2 * s + h2 if hn == 2 else s if hn == 1 else 0
    else:
        fin = 2 * (h1 + h2) + h3 if hn == 3 else h1 + h3 if hn == 2 else 0
    return acc + hs + fin - sum(freqs)


def test_huffman_register_merge_model_is_exact():
    """The narrow path's register merge (16 weight buckets + <= 3 heavy nodes + a final
    merge of <= 4 nodes) gives the reference heap's size on every golden block and on
    random frequency multisets of every shape a block can hold (<= 65 symbols): many
    light leaves, heavy leaves (17..64), and mixes whose pending merges reach every bucket."""
    g = _huffman_golden()

    def bits(block):
        c = np.asarray(block).ravel()
        vals = [int(v) for v in c if v != 0] + ([0] if c[63] == 0 else [])
        _, f = np.unique(vals, return_counts=True)
        return 8 * len(vals) + register_merge_wpl([int(x) for x in f])

    for name, b in g["blocks"].items():
        assert bits(b["coeffs"]) == b["bits"], name
    rng = np.random.default_rng(1234)
    for k in range(4000):
        dens = rng.random()
        amp = int(rng.choice([1, 2, 3, 5, 8, 16, 31, 100]))
        blk = rng.integers(-amp, amp + 1, 64) * (rng.random(64) < dens)
        assert bits(blk) == O.huffman_bits(blk), blk.tolist()
    # frequency multisets straight from a partition of up to 64 symbols (distinct nonzero values;
    # c[63] nonzero, so no extra zero symbol): heavy leaves (17..64) and light ones in every mix
    for k in range(4000):
        left, f = int(rng.integers(1, 65)), []
        while left:
            x = int(min(left, rng.choice([1, 1, 2, 3, 4, int(rng.integers(1, 65))])))
            f.append(x)
            left -= x
        blk = np.array([v + 1 for v, x in enumerate(f) for _ in range(x)] + [0] * 64)[:64]
        blk = np.roll(blk, 64 - sum(f))  # nonzeros last: c[63] != 0
        assert 8 * sum(f) + register_merge_wpl(f) == O.huffman_bits(blk), f


def test_legacy_tables_golden():
    """The oracle's explicit-table transforms reproduce the reference's outputs for
    block sizes above 64 and for caller-edited public tables (tests/golden/
    make_legacy_golden.py, generated from the compiled reference)."""
    import hashlib
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from make_legacy_golden import case_inputs
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "legacy_tables.json")))
    for c in g["cases"]:
        x, d, t = case_inputs(c["n"], c["seed"], c["edit"])
        fw = O.forward_tables(x, d, t)
        assert hashlib.sha256(fw.tobytes()).hexdigest() == c["forward_sha256"], c["name"]
        inv = O.inverse_tables(fw, d, t)
        assert hashlib.sha256(inv.tobytes()).hexdigest() == c["inverse_of_forward_sha256"], c["name"]
        if c["edit"] is None:
            assert np.array_equal(O.forward(x).view(np.uint64), fw.view(np.uint64))
