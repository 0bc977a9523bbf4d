/*
 * host/legacy_latency.c -- per-call latency of the reference's per-block API
 * (include/dct.h, include/quantization.h) served by libdct_amd.so: the loop a
 * relinked reference host runs (tests/test_entropy.c:300-373 per block).
 * Prints microseconds per call for each function, then for the whole per-block
 * pipeline.  Output values are not checked here (tests/test_gpu_parity.py does).
 */
#define _POSIX_C_SOURCE 199309L
#include <stdio.h>
#include <time.h>

#include "dct.h"
#include "quantization.h"

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

int main(void) {
    const int reps = 2000;
    unsigned char px[64];
    for (int i = 0; i < 64; ++i) px[i] = (unsigned char)(37 * i + 11);
    DCTContext *dct = dct_init(8);
    QuantContext *qc = quant_init(8, 50, 0);
    double **x = create_block_from_pixels(px, 8, 0, 0, 8);
    double **c = alloc_array(8, 8), **dq = alloc_array(8, 8), **rec = alloc_array(8, 8);
    int **q = alloc_int_array(8, 8);
    double var = 0.0;
    for (int w = 0; w < 50; ++w) dct_forward(dct, x, c);  /* warm up */
    double t0 = now();
    for (int r = 0; r < reps; ++r) dct_forward(dct, x, c);
    double t1 = now();
    for (int r = 0; r < reps; ++r) var = calculate_block_variance(x, 8);
    double t2 = now();
    for (int r = 0; r < reps; ++r) quantize(qc, c, q, var);
    double t3 = now();
    for (int r = 0; r < reps; ++r) {
        dct_forward(dct, x, c);
        var = calculate_block_variance(x, 8);
        quantize(qc, c, q, var);
        dequantize(qc, q, dq, var);
        dct_inverse(dct, dq, rec);
    }
    double t4 = now();
    printf("dct_forward_us %.2f\n", (t1 - t0) / reps * 1e6);
    printf("calculate_block_variance_us %.2f\n", (t2 - t1) / reps * 1e6);
    printf("quantize_us %.2f\n", (t3 - t2) / reps * 1e6);
    printf("pipeline_us %.2f (forward, variance, quantize, dequantize, inverse)\n", (t4 - t3) / reps * 1e6);
    printf("q00 %d\n", q[0][0]);
    free_array(x, 8);
    free_array(c, 8);
    free_array(dq, 8);
    free_array(rec, 8);
    free_int_array(q, 8);
    dct_free(dct);
    quant_free(qc);
    return 0;
}
