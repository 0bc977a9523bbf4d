// dct_amd/csrc/host_tables.h -- host-side constant generation.
//
// The tables are computed on the host with the reference's own expressions and
// glibc libm (the same image on the GPU box), then uploaded bit-identical; the
// device never evaluates cos/sqrt.  Compiled with -ffp-contract=off.
#pragma once
#include <math.h>

namespace dctq_host {

// src/quantization.c:8-17 (JPEG Annex K luminance table)
static const int kLuma[64] = {16, 11, 10,  16,  24,  40,  51,  61,  12, 12, 14, 19,  26,  58,  60,  55,
                              14, 13, 16,  24,  40,  57,  69,  56,  14, 17, 22, 29,  51,  87,  80,  62,
                              18, 22, 37,  56,  68,  109, 103, 77,  24, 35, 55, 64,  81,  104, 113, 92,
                              49, 64, 78,  87,  103, 121, 120, 101, 72, 92, 95, 98,  112, 100, 103, 99};

// src/dct.c:17-30: alpha_i * cos((PI * (2j+1) * i) / (2.0 * N)), PI of include/dct.h:15.
inline void dct_matrix(int n, double *d) {
    const double pi = 3.14159265358979323846;
    for (int i = 0; i < n; ++i) {
        const double alpha = (i == 0) ? 1.0 / sqrt((double)n) : sqrt(2.0 / n);
        for (int j = 0; j < n; ++j) d[i * n + j] = alpha * cos((pi * (2 * j + 1) * i) / (2.0 * n));
    }
}

// src/quantization.c:26-31
inline int clamp_quality(int q) { return q < 1 ? 1 : q > 100 ? 100 : q; }

// src/quantization.c:51-99 (no clamping of `quality` here, as in the reference)
inline void quant_matrix(int n, int quality, double *q) {
    double scale = quality < 50 ? 5000.0 / quality : 200.0 - 2 * quality;
    scale /= 100.0;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            double v = (n == 8) ? kLuma[i * 8 + j] * scale : (1.0 + sqrt((double)(i * i + j * j))) * scale * 8.0;
            v = v < 1.0 ? 1.0 : v;
            v = v > 255.0 ? 255.0 : v;
            q[i * n + j] = v;
        }
}

}  // namespace dctq_host
