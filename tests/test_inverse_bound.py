"""CPU: the rigorous error bound that admits a plan to the fused round trip's
fp32 inverse (roundtrip8_f32).

tools/inv_bound.py tracks the kernel's inverse (fp32 scale, the transposed AAN
graph over columns then rows, + 128) as linear forms with rounding bounds that
are linear in the per-coefficient input magnitudes, and generates
dct_amd/csrc/idct8_bound.h; api.hip evaluates it per plan.  Here:
  * the committed header is exactly the generator's output;
  * the library's per-plan bound (host-only diag entry point) equals the
    generator's for every standard quality, and admits exactly q <= 71;
  * an fp32 simulation of the kernel's operation sequence on blocks that maximise
    each coefficient (and on noise) stays within the bound against the oracle's
    fp64 reference inverse (src/dct.c:80-105, src/quantization.c:133-151).
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import inv_bound as IB  # noqa: E402
from aan_model import aan8t, scales, C4, C6, C2mC6, C2pC6  # noqa: E402,F401


@pytest.fixture(scope="module")
def GL():
    G, L = IB.bound()
    IB.check_linear(L)
    return G, L


def test_header_is_generated(GL):
    with open(os.path.join(ROOT, "dct_amd", "csrc", "idct8_bound.h")) as f:
        assert f.read() == IB.header(*GL)


def test_library_bound_equals_generator(GL):
    import dct_amd
    admitted = []
    for q in range(1, 101):
        b, a = dct_amd.inverse_bound(q, 0)
        want = IB.plan_error(q, *GL)[0]
        assert abs(b - want) <= 1e-9 * want, (q, b, want)
        assert a == (b <= 5e-5)
        assert dct_amd.inverse_bound(q, 1)[1] is False
        if a:
            admitted.append(q)
    assert admitted == list(range(1, 72)), admitted


class F32:
    """The kernel's fp32 arithmetic on numpy arrays: every op rounded to fp32
    (fma: the exact product plus the addend in fp64, then one rounding)."""
    f = staticmethod(np.float32)

    def add(self, a, b): return (a + b).astype(np.float32)
    def sub(self, a, b): return (a - b).astype(np.float32)
    def neg(self, a): return -a
    def mul(self, a, k): return (a * np.float32(k)).astype(np.float32)
    def fma(self, k, a, b):
        return (np.float64(np.float32(k)) * a.astype(np.float64) + b.astype(np.float64)).astype(np.float32)


def _kernel_inverse(q, iscale32):
    """recon of int coefficient blocks q [n, 64] as roundtrip.hip inverse_block_f32 computes it."""
    A = F32()
    x = (q.astype(np.float32) * iscale32[None, :]).astype(np.float32)
    x = [x[:, k] for k in range(64)]
    for v in range(8):
        col = aan8t([x[u * 8 + v] for u in range(8)], A)
        for i in range(8):
            x[i * 8 + v] = col[i]
    for i in range(8):
        row = aan8t(x[i * 8:i * 8 + 8], A)
        x[i * 8:i * 8 + 8] = row
    return np.stack([(xx + np.float32(128.0)).astype(np.float32) for xx in x], axis=1)


def _basis_sign_blocks():
    import oracle as O
    D = O.dct_matrix(8)
    out = []
    for u in range(8):
        for v in range(8):
            sg = np.where(np.outer(D[u], D[v]) >= 0, 1, -1)
            out += [128 + 127 * sg, 128 - 128 * sg]
    return np.clip(np.array(out), 0, 255).astype(np.uint8)


@pytest.mark.parametrize("q", [1, 10, 25, 50, 71])
def test_fp32_inverse_simulation_within_bound(GL, q):
    import oracle as O
    rng = np.random.default_rng(q)
    blocks = np.concatenate([_basis_sign_blocks(), rng.integers(0, 256, (4000, 8, 8)).astype(np.uint8),
                             rng.choice([0, 255], (2000, 8, 8)).astype(np.uint8)])
    plane = np.ascontiguousarray(blocks.transpose(1, 0, 2).reshape(8, -1))
    coef = O.forward_plane(plane, q, 0)
    want = O.inverse_plane(coef, q, 0) + 128.0
    S = np.array(scales())
    iscale32 = (O.dequant_matrix(O.quant_matrix(8, q)).ravel() * np.outer(S, S).ravel()).astype(np.float32)
    got = _kernel_inverse(coef, iscale32).astype(np.float64)
    err = float(np.abs(got - want).max())
    bound = IB.plan_error(q, *GL)[0]
    assert err <= bound, (q, err, bound)
    assert bound <= 5e-5


def test_symbol_format_bound():
    """dctq_plan_symbol_bytes: 2-byte symbols exactly when the plan bounds every |quantized
    coefficient| by 511 (128 * L1(D[u]) * L1(D[v]) / Q_uv rounded, Q from
    src/quantization.c:51-77) -- standard tables q <= 90; and the bound holds on the
    oracle's forward of blocks built to hit it (each coefficient's sign pattern at +-128/127)."""
    import dct_amd
    import oracle as O
    got = [dct_amd.symbol_bytes(q) for q in range(1, 101)]
    want = [2 if np.floor(IB.coef_max() / IB.quant_table(q) + 0.5).max() <= 511 else 4 for q in range(1, 101)]
    assert got == want
    assert got == [2] * 90 + [4] * 10
    assert all(dct_amd.symbol_bytes(q, True) == got[q - 1] for q in (1, 50, 90, 91, 100))
    D = O.dct_matrix(8)
    blocks = []
    for u in range(8):
        for v in range(8):
            s = np.sign(np.outer(D[u], D[v]))
            blocks += [np.where(s >= 0, 127, -128) + 128, np.where(s >= 0, -128, 127) + 128]
    px = np.concatenate([np.concatenate(blocks[i:i + 8], axis=1) for i in range(0, 128, 8)], axis=0).astype(np.uint8)
    for q in (50, 90, 91, 100):
        m = int(np.abs(O.forward_plane(px, q, 0).astype(np.int32)).max())
        assert m <= np.floor(IB.coef_max() / IB.quant_table(q) + 0.5).max()
        if q <= 90:
            assert m <= 511
