/*
 * dct.h -- per-block DCT API, drop-in for the reference's include/dct.h:21-82.
 *
 * Same prototypes and the same PUBLIC struct layout (DCTContext,
 * include/dct.h:21-25): callers may read dct_matrix / transposed_dct.
 * Implemented by libdct_amd.so (dct_amd/csrc/legacy.hip): the transforms run on
 * the GPU in the reference's exact fp64 operation order, so results are
 * bit-identical to src/dct.c.  Frame-level callers should use the batched API
 * in dct_amd.h instead (one launch per plane rather than per block).
 */
#ifndef DCT_AMD_DCT_H
#define DCT_AMD_DCT_H

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "utils.h"

/* include/dct.h:15 */
#define PI 3.14159265358979323846

#ifdef __cplusplus
extern "C" {
#endif

/* include/dct.h:21-25 -- layout kept identical (public fields). */
typedef struct {
    int block_size;
    double **dct_matrix;     /* D[i][j] = alpha_i cos(PI (2j+1) i / 2N) */
    double **transposed_dct; /* D^T */
} DCTContext;

/* replaces include/dct.h:34 (src/dct.c:7-40) */
DCTContext *dct_init(int block_size);
/* replaces include/dct.h:41 (src/dct.c:43-49) */
void dct_free(DCTContext *ctx);
/* replaces include/dct.h:51 (src/dct.c:52-77): output = D * input * D^T */
void dct_forward(DCTContext *ctx, double **input, double **output);
/* replaces include/dct.h:61 (src/dct.c:80-105): output = D^T * input * D */
void dct_inverse(DCTContext *ctx, double **input, double **output);
/* replaces include/dct.h:73 (src/dct.c:109-120): block[i][j] = px[(r+i)*w + c+j] - 128 */
double **create_block_from_pixels(unsigned char *pixels, int width, int row_start, int col_start, int block_size);
/* replaces include/dct.h:82 (src/dct.c:123-129): coefficients = (int) round(block) */
void copy_block_to_coefficients(double **block, int **coefficients, int block_size);

#ifdef __cplusplus
}
#endif
#endif
