/* tests/san/san_check.c -- SURVEY.md section 5 "race detection / sanitizers":
 * the CPU-side C of this repository built with -fsanitize=address,undefined
 * (-fno-sanitize-recover=all: any finding aborts) and exercised:
 *   - oracle/dct_oracle.c (the clean-room restatement, incl. its pthread plane
 *     loops) against
 *   - oracle/ref_driver.c + the reference's own src/{utils,dct,quantization,
 *     entropy}.c (compiled from /root/reference when present; -DNO_REF builds
 *     the oracle half alone),
 * bit for bit, over every block size class (1..128, edited public tables),
 * every quality class, both adaptive modes, the plane loops at 1 and 4 threads,
 * run-length coding and the per-block Huffman size.  Test infrastructure
 * (tests/test_sanitizers.py builds and runs it); not product code. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dct_oracle.h"

#ifndef NO_REF
void ref_dct_matrix(int n, double *d);
void ref_quant_tables(int n, int quality, int adaptive, double *q, double *dq, int *clamped_quality);
void ref_forward_tables(int n, const double *d, const double *t, const double *x, double *out);
void ref_inverse_tables(int n, const double *d, const double *t, const double *x, double *out);
double ref_variance(int n, const double *x);
void ref_quantize(int n, int quality, int adaptive, double var, const double *c, int *q);
void ref_dequantize(int n, int quality, int adaptive, double var, const int *q, double *c);
long ref_forward_plane(unsigned char *px, int width, int height, int quality, int adaptive, int16_t *out,
                       int nthreads, int rows);
int ref_rle_encode(int n, const int *coeffs, int *values, int *runs);
int ref_huffman_bits(int n, const int *coeffs, int *nsym, int *ncodes);
#endif

static int fails = 0;
#define CHECK(cond, ...)                       \
    do {                                       \
        if (!(cond)) {                         \
            fprintf(stderr, __VA_ARGS__);      \
            fputc('\n', stderr);               \
            ++fails;                           \
        }                                      \
    } while (0)

static uint64_t rng = 0x9E3779B97F4A7C15ULL;
static double urand(void) {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return (double)(rng >> 11) / 9007199254740992.0;
}

static void transforms(int n, int edit) {
    size_t nn = (size_t)n * n;
    double *d = malloc(nn * sizeof *d), *t = malloc(nn * sizeof *t), *x = malloc(nn * sizeof *x);
    double *a = malloc(nn * sizeof *a), *b = malloc(nn * sizeof *b);
    orc_dct_matrix(n, d);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) t[(size_t)i * n + j] = d[(size_t)j * n + i] * (edit ? 1.0 + 1e-3 * (i + j) : 1.0);
    for (size_t e = 0; e < nn; ++e) x[e] = (double)(int)(urand() * 256) - 128.0 + (edit ? urand() : 0.0);
    orc_forward_tables(n, d, t, x, a);
    orc_inverse_tables(n, d, t, a, b);
#ifndef NO_REF
    double *rd = malloc(nn * sizeof *rd), *ra = malloc(nn * sizeof *ra), *rb = malloc(nn * sizeof *rb);
    ref_dct_matrix(n, rd);
    CHECK(!memcmp(rd, d, nn * sizeof *d), "dct_matrix differs at n=%d", n);
    ref_forward_tables(n, d, t, x, ra);
    ref_inverse_tables(n, d, t, ra, rb);
    CHECK(!memcmp(ra, a, nn * sizeof *a), "forward differs at n=%d edit=%d", n, edit);
    CHECK(!memcmp(rb, b, nn * sizeof *b), "inverse differs at n=%d edit=%d", n, edit);
    CHECK(ref_variance(n, x) == orc_variance(n, x), "variance differs at n=%d", n);
    free(rd), free(ra), free(rb);
#endif
    free(d), free(t), free(x), free(a), free(b);
}

static void quantization(int n, int quality, int adaptive) {
    size_t nn = (size_t)n * n;
    double *q = malloc(nn * sizeof *q), *dq = malloc(nn * sizeof *dq), *c = malloc(nn * sizeof *c);
    double *o = malloc(nn * sizeof *o);
    int *qi = malloc(nn * sizeof *qi);
    const int ql = orc_clamp_quality(quality);
    orc_quant_matrix(n, ql, q);
    orc_dequant_matrix(n, q, dq);
    for (size_t e = 0; e < nn; ++e) c[e] = (urand() - 0.5) * 2048.0;
    const double var = urand() * 3000.0;
    orc_quantize(n, q, adaptive, var, c, qi);
    orc_dequantize(n, dq, adaptive, var, qi, o);
#ifndef NO_REF
    double *rq = malloc(nn * sizeof *rq), *rdq = malloc(nn * sizeof *rdq), *ro = malloc(nn * sizeof *ro);
    int *rqi = malloc(nn * sizeof *rqi), cq = 0;
    ref_quant_tables(n, quality, adaptive, rq, rdq, &cq);
    CHECK(cq == ql && !memcmp(rq, q, nn * sizeof *q), "quant table differs n=%d q=%d", n, quality);
    ref_quantize(n, quality, adaptive, var, c, rqi);
    CHECK(!memcmp(rqi, qi, nn * sizeof *qi), "quantize differs n=%d q=%d a=%d", n, quality, adaptive);
    ref_dequantize(n, quality, adaptive, var, rqi, ro);
    CHECK(!memcmp(ro, o, nn * sizeof *o), "dequantize differs n=%d q=%d a=%d", n, quality, adaptive);
    free(rq), free(rdq), free(ro), free(rqi);
#endif
    free(q), free(dq), free(c), free(o), free(qi);
}

static void planes(int kind, int quality, int adaptive, int threads) {
    const int w = 8 * 37, h = 8 * 19;
    const long nb = (long)(w / 8) * (h / 8);
    uint8_t *px = malloc((size_t)w * h);
    int16_t *co = malloc((size_t)nb * 64 * sizeof *co);
    orc_synth_plane(1234 + (uint64_t)kind, kind, w, h, px, w);
    CHECK(orc_forward_plane(px, w, w, h, quality, adaptive, co, NULL, threads) == 0, "forward_plane rc");
    double *var = malloc((size_t)nb * sizeof *var), *rec = malloc((size_t)nb * 64 * sizeof *rec);
    orc_plane_variance(px, w, w, h, var);
    orc_inverse_plane(co, adaptive ? var : NULL, (int)nb, quality, adaptive, rec);
    uint32_t *off = malloc((size_t)(nb + 1) * sizeof *off), *sym = malloc((size_t)nb * 64 * sizeof *sym);
    uint32_t *bits = malloc((size_t)nb * sizeof *bits);
    const long total = orc_rle_encode_plane(co, nb, off, sym);
    CHECK(total >= nb && total <= nb * 64, "rle total %ld", total);
    orc_huffman_bits_plane(co, nb, bits);
#ifndef NO_REF
    int16_t *rco = malloc((size_t)nb * 64 * sizeof *rco);
    ref_forward_plane(px, w, h, quality, adaptive, rco, threads, 0);
    CHECK(!memcmp(rco, co, (size_t)nb * 64 * sizeof *co), "forward_plane differs kind=%d q=%d a=%d t=%d", kind,
          quality, adaptive, threads);
    int vals[64], runs[64], oc[64], ov[64], orr[64], blk[64];
    for (long b = 0; b < nb; b += 7) {
        for (int k = 0; k < 64; ++k) blk[k] = co[b * 64 + k];
        const int rn = ref_rle_encode(8, blk, vals, runs), on = orc_rle_encode(8, blk, ov, orr);
        CHECK(rn == on && !memcmp(vals, ov, sizeof(int) * rn) && !memcmp(runs, orr, sizeof(int) * rn),
              "rle differs at block %ld", b);
        orc_rle_decode(8, ov, orr, on, oc);
        CHECK(!memcmp(oc, blk, sizeof blk), "rle round trip differs at block %ld", b);
        CHECK((uint32_t)ref_huffman_bits(8, blk, NULL, NULL) == bits[b], "huffman bits differ at block %ld", b);
    }
    free(rco);
#endif
    free(px), free(co), free(var), free(rec), free(off), free(sym), free(bits);
}

int main(void) {
    const int sizes[] = {1, 2, 3, 7, 8, 16, 31, 64, 65, 100, 128};
    for (size_t i = 0; i < sizeof sizes / sizeof *sizes; ++i) {
        transforms(sizes[i], 0);
        transforms(sizes[i], 1);
    }
    const int qs[] = {0, 1, 10, 49, 50, 51, 90, 100, 101};
    for (size_t i = 0; i < sizeof qs / sizeof *qs; ++i)
        for (int n = 1; n <= 16; n *= 2)
            for (int a = 0; a < 2; ++a) quantization(n == 16 ? 8 : n, qs[i], a);
    for (int kind = 0; kind < 4; ++kind)
        for (int a = 0; a < 2; ++a) {
            planes(kind, 50, a, 1);
            planes(kind, 90, a, 4);
        }
    printf("san_check: %d failure(s)\n", fails);
    return fails ? 1 : 0;
}
