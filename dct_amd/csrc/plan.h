// dct_amd/csrc/plan.h -- the plan object and the argument helpers shared by the
// product C-ABI (api.hip) and the diagnostic library's entry points (diag.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "dct_amd.h"
#include "dctq_internal.h"

struct dctq_plan {
    int quality, adaptive, device, num_cus;
    int variant;                 // 2: the product kernels; 1 / 4 only through the dctq_diag_* entry points
    dctq::FastTables fast;       // thresholds for the mode in `adaptive`
    dctq::DevTables host;        // host copy of the device tables
    dctq::DevTables *dev;        // device copy
    unsigned long long *fallbacks;
    int inv_f32;                 // round trip: fp32 inverse admitted (|recon err| <= inv_bound <= kInvTol)
    double inv_bound;            // the fp32 inverse's rigorous error bound for this plan (idct8_bound.h)
    int symbol_bytes;            // the encoder's symbol format: 2 when every |quantized coefficient| <= 511, else 4
};

namespace dctq {
// records `what` (+ the HIP error string) for dctq_error_string and returns `code`
int fail(int code, const char *what, hipError_t e = hipSuccess);
int check_plan(const dctq_plan *plan);
int plane_args(const dctq_plane *s, PlaneArgs *a);
// validates the pixel planes and fills ps (batch prefixes); no outputs
int plane_inputs(const dctq_plane *planes, int nplanes, PlaneSet *ps);
// plane_inputs plus the per-plane coefficient (and optional var_num) outputs
int plane_set(const dctq_plane *planes, int nplanes, int16_t *const *coef, int32_t *const *var_num, PlaneSet *ps);
void fill_fast_tables(const double *q, int adaptive, FastTables *t);
// quantized DC of every constant block, in the reference's operation order (api.hip)
void dc_const_table(const double *d, const double *q, int16_t *tab);
// rigorous bound of |recon - reference| of the fused round trip's fp32 inverse for the
// plan's tables (non-adaptive dequantisation; tools/inv_bound.py, idct8_bound.h)
double inverse_f32_bound(const DevTables &t);
// the largest |quantized coefficient| a plan's table admits for u8 input: |c_uv| <=
// 128 L1(D_u) L1(D_v) (centred pixels), |q| <= round(c_max / M) with M >= Q (adaptive
// divisors Q (2 - nv) >= Q; the DC keeps Q)
int max_abs_quantized(const DevTables &t);
}  // namespace dctq
// the admission tolerance of that bound (== idct8_bound.h kInvTol; api.hip checks they agree)
constexpr double kInvTolDiag = 5e-5;
namespace dctq {
}  // namespace dctq

#define HIPCHK(call, what)                                               \
    do {                                                                 \
        hipError_t e_ = (call);                                          \
        if (e_ != hipSuccess) return ::dctq::fail(DCTQ_EHIP, what, e_); \
    } while (0)
