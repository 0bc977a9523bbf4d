"""Model of the fp32 fast path's butterfly (AAN factorisation of the 8-point DCT-II).

The same flow graph as dct_amd/csrc/fdct8_fast.h, written once over an abstract
"arith" object so it can be (a) evaluated numerically and (b) evaluated over
linear forms with a rigorous rounding-error bound (tools/guard_bound.py).
"""
import math

C4 = math.cos(math.pi / 4)            # cos(4pi/16)
C6 = math.cos(6 * math.pi / 16)       # cos(6pi/16)
C2mC6 = math.cos(2 * math.pi / 16) - C6
C2pC6 = math.cos(2 * math.pi / 16) + C6


def aan8(v, A):
    """v: list of 8 values; A: arith with add(a,b), sub(a,b), mul(a,K), fma(K,a,b)=K*a+b."""
    a0, b0 = A.add(v[0], v[7]), A.sub(v[0], v[7])
    a1, b1 = A.add(v[1], v[6]), A.sub(v[1], v[6])
    a2, b2 = A.add(v[2], v[5]), A.sub(v[2], v[5])
    a3, b3 = A.add(v[3], v[4]), A.sub(v[3], v[4])
    # even half
    e0, e3 = A.add(a0, a3), A.sub(a0, a3)
    e1, e2 = A.add(a1, a2), A.sub(a1, a2)
    y0, y4 = A.add(e0, e1), A.sub(e0, e1)
    m = A.mul(A.add(e2, e3), C4)
    y2, y6 = A.add(e3, m), A.sub(e3, m)
    # odd half
    o0 = A.add(b3, b2)
    o1 = A.add(b2, b1)
    o2 = A.add(b1, b0)
    z5 = A.mul(A.sub(o0, o2), C6)
    z2 = A.fma(C2mC6, o0, z5)
    z4 = A.fma(C2pC6, o2, z5)
    z3 = A.mul(o1, C4)
    z11, z13 = A.add(b0, z3), A.sub(b0, z3)
    y5, y3 = A.add(z13, z2), A.sub(z13, z2)
    y1, y7 = A.add(z11, z4), A.sub(z11, z4)
    return [y0, y1, y2, y3, y4, y5, y6, y7]


class Exact:
    def add(self, a, b): return a + b
    def sub(self, a, b): return a - b
    def mul(self, a, k): return a * k
    def fma(self, k, a, b): return k * a + b
    def neg(self, a): return -a


def scales():
    """S[k] with X_k = S[k] * y_k for the orthonormal DCT-II of src/dct.c:17-30."""
    import numpy as np
    n = 8
    D = np.array([[ (1/math.sqrt(n) if i == 0 else math.sqrt(2/n)) * math.cos(math.pi*(2*j+1)*i/(2*n))
                    for j in range(n)] for i in range(n)])
    Y = np.array([aan8(list(np.eye(8)[c]), Exact()) for c in range(8)]).T   # Y[k][c]
    S = []
    for k in range(8):
        ratio = D[k] / Y[k]
        assert np.allclose(ratio, ratio[0], rtol=1e-12), (k, ratio)
        S.append(ratio[0])
    return S

if __name__ == "__main__":
    print(scales())


def aan8t(v, A):
    """The transposed flow graph A^T (dct_amd/csrc/aan_f64.h aan8t_d and the fp32
    inverse of roundtrip.hip, operation for operation): with D = diag(S) A
    orthonormal, D^T X = A^T (S .* X).  fma(K, a, b) = K*a + b."""
    gz13, gz2 = A.add(v[5], v[3]), A.sub(v[5], v[3])
    gz11, gz4 = A.add(v[1], v[7]), A.sub(v[1], v[7])
    gb0, gz3 = A.add(gz11, gz13), A.sub(gz11, gz13)
    go1 = A.mul(gz3, C4)
    gz5 = A.mul(A.add(gz2, gz4), C6)
    go0 = A.fma(C2mC6, gz2, gz5)
    go2 = A.fma(C2pC6, gz4, A.neg(gz5))
    gb3, gb2, gb1 = go0, A.add(go0, go1), A.add(go1, go2)
    gb0 = A.add(gb0, go2)
    ge3, gm = A.add(v[2], v[6]), A.sub(v[2], v[6])
    gs = A.mul(gm, C4)
    ge2 = gs
    ge3 = A.add(ge3, gs)
    ge0, ge1 = A.add(v[0], v[4]), A.sub(v[0], v[4])
    ga0, ga3, ga1, ga2 = A.add(ge0, ge3), A.sub(ge0, ge3), A.add(ge1, ge2), A.sub(ge1, ge2)
    return [A.add(ga0, gb0), A.add(ga1, gb1), A.add(ga2, gb2), A.add(ga3, gb3),
            A.sub(ga3, gb3), A.sub(ga2, gb2), A.sub(ga1, gb1), A.sub(ga0, gb0)]
