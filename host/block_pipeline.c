/*
 * host/block_pipeline.c -- a plain C99 host of the reference's per-block API
 * (include/dct.h, include/quantization.h), linked against libdct_amd.so instead
 * of src/dct.c + src/quantization.c.  It drives the same per-block pipeline as
 * the reference's tests/test_entropy.c:278-393 (pixels-128 -> dct_forward ->
 * calculate_block_variance -> quantize -> dequantize -> dct_inverse -> PSNR),
 * with no source change other than the link line.
 */
#include <stdint.h>
#include <string.h>

#include "dct.h"
#include "quantization.h"

static const unsigned char kBlock[64] = {52, 55, 61, 66, 70, 61, 64, 73, 63, 59, 55, 90, 109, 85, 69, 72,
                                         62, 59, 68, 113, 144, 104, 66, 73, 63, 58, 71, 122, 154, 106, 70, 69,
                                         67, 61, 68, 104, 126, 88, 68, 70, 79, 65, 60, 70, 77, 68, 58, 75,
                                         85, 71, 64, 59, 55, 61, 65, 83, 87, 79, 69, 68, 65, 76, 78, 94};

static void run(int quality, const char *tag) {
    DCTContext *dct = dct_init(8);
    QuantContext *qc = quant_init(8, quality, 0);
    double **x = create_block_from_pixels((unsigned char *)kBlock, 8, 0, 0, 8);
    double **c = alloc_array(8, 8);
    int **q = alloc_int_array(8, 8);
    dct_forward(dct, x, c);
    double var = calculate_block_variance(x, 8);
    quantize(qc, c, q, var);
    printf("%s:", tag);
    for (int i = 0; i < 8; ++i)
        for (int j = 0; j < 8; ++j) printf(" %d", q[i][j]);
    printf("\n");
    if (quality == 50) {
        uint64_t b;
        memcpy(&b, &c[0][0], sizeof b);
        printf("forward_bits0:%016llx\n", (unsigned long long)b);
        double **dq = alloc_array(8, 8), **rec = alloc_array(8, 8);
        dequantize(qc, q, dq, var);
        dct_inverse(dct, dq, rec);
        double mse = 0.0;
        for (int i = 0; i < 8; ++i)
            for (int j = 0; j < 8; ++j) {
                double r = rec[i][j] + 128.0;
                r = r < 0 ? 0 : r > 255 ? 255 : r;
                double e = kBlock[i * 8 + j] - r;
                mse += e * e;
            }
        mse /= 64.0;
        printf("psnr:%.2f\n", 10 * log10(255 * 255 / mse));
        free_array(dq, 8);
        free_array(rec, 8);
    }
    free_array(x, 8);
    free_array(c, 8);
    free_int_array(q, 8);
    dct_free(dct);
    quant_free(qc);
}

int main(void) {
    run(50, "q50");
    run(90, "q90");
    return 0;
}
