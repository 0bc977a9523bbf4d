// dct_amd/csrc/aan_f64.h -- the 8-point AAN flow graph and its transpose in
// fp64 (the float-output forward DCT and the inverse path; ~1e-13 error, so no
// bound table is needed).  Shared by fdct8_aux.hip and f64_pair.hip.
#pragma once
#include "dctq_internal.h"

namespace dctq {

__device__ __forceinline__ double fma_d(double a, double b, double c) { return __builtin_fma(a, b, c); }

// Exact-math AAN constants in fp64 (the fp64 paths carry ~1e-13 error; no bound table needed).
constexpr double kC4 = 0.70710678118654752440;
constexpr double kC6 = 0.38268343236508977173;
constexpr double kC2mC6 = 0.54119610014619698440;
constexpr double kC2pC6 = 1.30656296487637652786;

__device__ __forceinline__ void aan8_d(double &v0, double &v1, double &v2, double &v3, double &v4, double &v5,
                                       double &v6, double &v7) {
    double a0 = v0 + v7, b0 = v0 - v7, a1 = v1 + v6, b1 = v1 - v6;
    double a2 = v2 + v5, b2 = v2 - v5, a3 = v3 + v4, b3 = v3 - v4;
    double e0 = a0 + a3, e3 = a0 - a3, e1 = a1 + a2, e2 = a1 - a2;
    double m = (e2 + e3) * kC4;
    double o0 = b3 + b2, o1 = b2 + b1, o2 = b1 + b0;
    double z5 = (o0 - o2) * kC6;
    double z2 = fma_d(kC2mC6, o0, z5), z4 = fma_d(kC2pC6, o2, z5);
    double z3 = o1 * kC4;
    double z11 = b0 + z3, z13 = b0 - z3;
    v0 = e0 + e1;
    v4 = e0 - e1;
    v2 = e3 + m;
    v6 = e3 - m;
    v1 = z11 + z4;
    v7 = z11 - z4;
    v5 = z13 + z2;
    v3 = z13 - z2;
}

// Transposed AAN flow graph (A^T): with D = diag(S) A orthonormal, D^T X = A^T (S .* X).
__device__ __forceinline__ void aan8t_d(double &v0, double &v1, double &v2, double &v3, double &v4, double &v5,
                                        double &v6, double &v7) {
    // odd half (inputs y1,y3,y5,y7)
    double gz13 = v5 + v3, gz2 = v5 - v3, gz11 = v1 + v7, gz4 = v1 - v7;
    double gb0 = gz11 + gz13, gz3 = gz11 - gz13;
    double go1 = gz3 * kC4;
    double gz5 = (gz2 + gz4) * kC6;
    double go0 = fma_d(kC2mC6, gz2, gz5);
    double go2 = fma_d(kC2pC6, gz4, -gz5);
    double gb3 = go0, gb2 = go0 + go1, gb1 = go1 + go2;
    gb0 = gb0 + go2;
    // even half (inputs y0,y2,y4,y6)
    double ge3 = v2 + v6, gm = v2 - v6;
    double gs = gm * kC4;
    double ge2 = gs;
    ge3 = ge3 + gs;
    double ge0 = v0 + v4, ge1 = v0 - v4;
    double ga0 = ge0 + ge3, ga3 = ge0 - ge3, ga1 = ge1 + ge2, ga2 = ge1 - ge2;
    v0 = ga0 + gb0;
    v7 = ga0 - gb0;
    v1 = ga1 + gb1;
    v6 = ga1 - gb1;
    v2 = ga2 + gb2;
    v5 = ga2 - gb2;
    v3 = ga3 + gb3;
    v4 = ga3 - gb3;
}

}  // namespace dctq
