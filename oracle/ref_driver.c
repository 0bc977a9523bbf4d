/*
 * oracle/ref_driver.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Flat-array entry points over the REFERENCE's own functions (include/dct.h,
 * include/quantization.h, include/utils.h of /root/reference), compiled
 * together with the reference sources by oracle/Makefile into
 * oracle/_ref/libref.so.  Used (1) to generate the golden fixtures in
 * tests/golden/ and (2) as the "reference" CPU baseline in bench.py.
 * Nothing here re-implements the reference: every number comes from
 * dct_forward / quantize / dequantize / dct_inverse / ... as shipped.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <dct.h>
#include <quantization.h>
#include <utils.h>

static void to2d(const double *src, double **dst, int n) {
    for (int i = 0; i < n; ++i) memcpy(dst[i], src + i * n, sizeof(double) * n);
}
static void from2d(double **src, double *dst, int n) {
    for (int i = 0; i < n; ++i) memcpy(dst + i * n, src[i], sizeof(double) * n);
}

void ref_dct_matrix(int n, double *d) {
    DCTContext *c = dct_init(n);
    from2d(c->dct_matrix, d, n);
    dct_free(c);
}

void ref_quant_tables(int n, int quality, int adaptive, double *q, double *dq, int *clamped_quality) {
    QuantContext *c = quant_init(n, quality, adaptive);
    from2d(c->quant_matrix, q, n);
    from2d(c->dequant_matrix, dq, n);
    if (clamped_quality) *clamped_quality = c->quality;
    quant_free(c);
}

void ref_forward(int n, const double *x, double *out) {
    DCTContext *c = dct_init(n);
    double **a = alloc_array(n, n), **b = alloc_array(n, n);
    to2d(x, a, n);
    dct_forward(c, a, b);
    from2d(b, out, n);
    free_array(a, n);
    free_array(b, n);
    dct_free(c);
}

void ref_inverse(int n, const double *x, double *out) {
    DCTContext *c = dct_init(n);
    double **a = alloc_array(n, n), **b = alloc_array(n, n);
    to2d(x, a, n);
    dct_inverse(c, a, b);
    from2d(b, out, n);
    free_array(a, n);
    free_array(b, n);
    dct_free(c);
}

/* dct_forward / dct_inverse on a context whose PUBLIC tables the caller set:
 * dct_init(n), then ctx->dct_matrix := d and ctx->transposed_dct := t. */
static void ref_tables_call(int n, const double *d, const double *t, const double *x, double *out, int fwd) {
    DCTContext *c = dct_init(n);
    to2d(d, c->dct_matrix, n);
    to2d(t, c->transposed_dct, n);
    double **a = alloc_array(n, n), **b = alloc_array(n, n);
    to2d(x, a, n);
    if (fwd)
        dct_forward(c, a, b);
    else
        dct_inverse(c, a, b);
    from2d(b, out, n);
    free_array(a, n);
    free_array(b, n);
    dct_free(c);
}

void ref_forward_tables(int n, const double *d, const double *t, const double *x, double *out) {
    ref_tables_call(n, d, t, x, out, 1);
}

void ref_inverse_tables(int n, const double *d, const double *t, const double *x, double *out) {
    ref_tables_call(n, d, t, x, out, 0);
}

double ref_variance(int n, const double *x) {
    double **a = alloc_array(n, n);
    to2d(x, a, n);
    double v = calculate_block_variance(a, n);
    free_array(a, n);
    return v;
}

void ref_quantize(int n, int quality, int adaptive, double var, const double *c, int *q) {
    QuantContext *ctx = quant_init(n, quality, adaptive);
    double **a = alloc_array(n, n);
    int **o = alloc_int_array(n, n);
    to2d(c, a, n);
    quantize(ctx, a, o, var);
    for (int i = 0; i < n; ++i) memcpy(q + i * n, o[i], sizeof(int) * n);
    free_array(a, n);
    free_int_array(o, n);
    quant_free(ctx);
}

void ref_dequantize(int n, int quality, int adaptive, double var, const int *q, double *c) {
    QuantContext *ctx = quant_init(n, quality, adaptive);
    int **a = alloc_int_array(n, n);
    double **o = alloc_array(n, n);
    for (int i = 0; i < n; ++i) memcpy(a[i], q + i * n, sizeof(int) * n);
    dequantize(ctx, a, o, var);
    from2d(o, c, n);
    free_int_array(a, n);
    free_array(o, n);
    quant_free(ctx);
}

void ref_adjust(int n, int quality, double var, int is_quantize, double *m) {
    QuantContext *ctx = quant_init(n, quality, 1);
    double **r = adjust_matrix_for_block(ctx, var, is_quantize);
    from2d(r, m, n);
    free_array(r, n);
    quant_free(ctx);
}

void ref_copy_to_coefficients(int n, const double *x, int *out) {
    double **a = alloc_array(n, n);
    int **o = alloc_int_array(n, n);
    to2d(x, a, n);
    copy_block_to_coefficients(a, o, n);
    for (int i = 0; i < n; ++i) memcpy(out + i * n, o[i], sizeof(int) * n);
    free_array(a, n);
    free_int_array(o, n);
}

/* The per-block pipeline of tests/test_entropy.c:300-316 over a whole plane,
 * driven exactly as a frame-level caller of the reference API would:
 * create_block_from_pixels -> dct_forward -> calculate_block_variance ->
 * quantize, one shared read-only DCTContext/QuantContext, pthreads over block
 * rows (the reference API is reentrant: SURVEY.md section 8(b)). */
typedef struct {
    DCTContext *dct;
    QuantContext *qc;
    unsigned char *px;
    int width, bw, row_lo, row_hi;
    int16_t *out;
} ref_job;

static void ref_rows(ref_job *j) {
    int **qi = alloc_int_array(8, 8);
    double **c = alloc_array(8, 8);
    for (int by = j->row_lo; by < j->row_hi; ++by)
        for (int bx = 0; bx < j->bw; ++bx) {
            double **x = create_block_from_pixels(j->px, j->width, by * 8, bx * 8, 8);
            dct_forward(j->dct, x, c);
            double var = calculate_block_variance(x, 8);
            quantize(j->qc, c, qi, var);
            int16_t *o = j->out + ((long)by * j->bw + bx) * 64;
            for (int r = 0; r < 8; ++r)
                for (int k = 0; k < 8; ++k) o[r * 8 + k] = (int16_t)qi[r][k];
            free_array(x, 8);
        }
    free_array(c, 8);
    free_int_array(qi, 8);
}

static void *ref_thread(void *a) {
    ref_rows((ref_job *)a);
    return NULL;
}

/* rows: only block rows [0, rows) are processed (bounded CPU-baseline sample);
 * rows <= 0 means the whole plane.  Returns the number of blocks done. */
long ref_forward_plane(unsigned char *px, int width, int height, int quality, int adaptive, int16_t *out,
                       int nthreads, int rows) {
    int bw = width / 8, bh = height / 8;
    if (rows > 0 && rows < bh) bh = rows;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > bh) nthreads = bh;
    DCTContext *dct = dct_init(8);
    QuantContext *qc = quant_init(8, quality, adaptive);
    ref_job *jobs = calloc((size_t)nthreads, sizeof *jobs);
    pthread_t *th = calloc((size_t)nthreads, sizeof *th);
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].dct = dct;
        jobs[t].qc = qc;
        jobs[t].px = px;
        jobs[t].width = width;
        jobs[t].bw = bw;
        jobs[t].row_lo = (int)((long)bh * t / nthreads);
        jobs[t].row_hi = (int)((long)bh * (t + 1) / nthreads);
        jobs[t].out = out;
    }
    for (int t = 1; t < nthreads; ++t) pthread_create(&th[t], NULL, ref_thread, &jobs[t]);
    ref_rows(&jobs[0]);
    for (int t = 1; t < nthreads; ++t) pthread_join(th[t], NULL);
    free(jobs);
    free(th);
    dct_free(dct);
    quant_free(qc);
    return (long)bh * bw;
}

/* ---- the reference's run-length coder (src/entropy.c), one block -------- */
#include <entropy.h>

int ref_rle_encode(int n, const int *coeffs, int *values, int *runs) {
    int **b = alloc_int_array(n, n);
    for (int i = 0; i < n; ++i) memcpy(b[i], coeffs + i * n, sizeof(int) * n);
    EntropyContext *e = entropy_init(0);
    int cnt = run_length_encode(e, b, n);
    for (int k = 0; k < cnt; ++k) {
        values[k] = e->symbols[k].value;
        runs[k] = e->symbols[k].run_length;
    }
    entropy_free(e);
    free_int_array(b, n);
    return cnt;
}

void ref_rle_decode(int n, const int *values, const int *runs, int count, int *coeffs) {
    EntropyContext *e = entropy_init(0);
    if (count > e->capacity) {
        e->symbols = (RLESymbol *)realloc(e->symbols, sizeof(RLESymbol) * count);
        e->capacity = count;
    }
    for (int k = 0; k < count; ++k) {
        e->symbols[k].value = values[k];
        e->symbols[k].run_length = runs[k];
    }
    e->count = count;
    int **b = alloc_int_array(n, n);
    run_length_decode(e, b, n);
    for (int i = 0; i < n; ++i) memcpy(coeffs + i * n, b[i], sizeof(int) * n);
    free_int_array(b, n);
    entropy_free(e);
}

void ref_zigzag(int n, const int *coeffs, int *zz) {
    int **b = alloc_int_array(n, n);
    for (int i = 0; i < n; ++i) memcpy(b[i], coeffs + i * n, sizeof(int) * n);
    block_to_zigzag(b, zz, n);
    free_int_array(b, n);
}

/* The reference pipeline's per-block size (tests/test_entropy.c:329-341):
 * run_length_encode -> build_huffman_codes -> get_encoded_size, use_huffman = 1.
 * Also returns the block's Huffman code lengths by symbol value (for the
 * fixtures; ties make individual lengths order-dependent, their sum is not). */
int ref_huffman_bits(int n, const int *coeffs, int *nsym, int *ncodes) {
    int **b = alloc_int_array(n, n);
    for (int i = 0; i < n; ++i) memcpy(b[i], coeffs + i * n, sizeof(int) * n);
    EntropyContext *e = entropy_init(1);
    int cnt = run_length_encode(e, b, n);
    build_huffman_codes(e);
    int bits = get_encoded_size(e);
    if (nsym) *nsym = cnt;
    if (ncodes) *ncodes = e->huffman_size;
    entropy_free(e);
    free_int_array(b, n);
    return bits;
}
