/*
 * utils.h -- 2-D row-pointer arrays of the per-block API (drop-in for the
 * reference's include/utils.h:21-46; implemented in dct_amd/csrc/legacy.hip).
 *
 * Same layout and ownership as the reference (src/utils.c:8-61): `rows` row
 * pointers, each to `cols` zero-initialised elements; allocation failure prints
 * to stderr and exits with EXIT_FAILURE.
 */
#ifndef DCT_AMD_UTILS_H
#define DCT_AMD_UTILS_H

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#ifdef __cplusplus
extern "C" {
#endif

/* replaces include/utils.h:28  (src/utils.c:8-25) */
double **alloc_array(int rows, int cols);
/* replaces include/utils.h:34  (src/utils.c:28-33) */
void free_array(double **array, int rows);
/* replaces include/utils.h:41  (src/utils.c:36-53) */
int **alloc_int_array(int rows, int cols);
/* replaces include/utils.h:46  (src/utils.c:56-61) */
void free_int_array(int **array, int rows);

#ifdef __cplusplus
}
#endif
#endif
