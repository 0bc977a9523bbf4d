/*
 * quantization.h -- per-block quantization API, drop-in for the reference's
 * include/quantization.h:18-98 (same prototypes, same public QuantContext
 * layout).  Implemented by libdct_amd.so (dct_amd/csrc/legacy.hip); the
 * per-element arithmetic runs on the GPU with the reference's fp64 semantics
 * (IEEE division, round half away from zero), bit-identical to
 * src/quantization.c -- including the non-adaptive dequantize that multiplies
 * by 1/Q (src/quantization.c:139,144; see DESIGN.md "Bug compatibility").
 */
#ifndef DCT_AMD_QUANTIZATION_H
#define DCT_AMD_QUANTIZATION_H

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "utils.h"

#ifdef __cplusplus
extern "C" {
#endif

/* include/quantization.h:18-24 -- layout kept identical (public fields). */
typedef struct {
    int block_size;
    int quality; /* clamped to 1..100 by quant_init */
    double **quant_matrix;
    double **dequant_matrix; /* 1 / quant_matrix */
    int adaptive;
} QuantContext;

/* replaces include/quantization.h:34 (src/quantization.c:19-41) */
QuantContext *quant_init(int block_size, int quality, int adaptive);
/* replaces include/quantization.h:41 (src/quantization.c:43-49) */
void quant_free(QuantContext *ctx);
/* replaces include/quantization.h:50 (src/quantization.c:51-99) */
double **generate_quant_matrix(int block_size, int quality);
/* replaces include/quantization.h:59 (src/quantization.c:101-111) */
double **generate_dequant_matrix(double **quant_matrix, int block_size);
/* replaces include/quantization.h:69 (src/quantization.c:113-131) */
void quantize(QuantContext *ctx, double **dct_coeffs, int **quant_coeffs, double block_variance);
/* replaces include/quantization.h:79 (src/quantization.c:133-151) */
void dequantize(QuantContext *ctx, int **quant_coeffs, double **dct_coeffs, double block_variance);
/* replaces include/quantization.h:88 (src/quantization.c:153-169) */
double calculate_block_variance(double **block, int block_size);
/* replaces include/quantization.h:98 (src/quantization.c:171-211) */
double **adjust_matrix_for_block(QuantContext *ctx, double variance, int is_quantize);

#ifdef __cplusplus
}
#endif
#endif
