/*
 * host/block_pipeline_mt.c -- the per-block pipeline of host/block_pipeline.c
 * (the reference's tests/test_entropy.c:300-373 loop: pixels-128 -> dct_forward
 * -> calculate_block_variance -> quantize -> dequantize -> dct_inverse) over
 * every 8x8 block of a u8 plane, from T pthreads sharing ONE DCTContext and ONE
 * QuantContext, as the reference API permits (no mutable global state,
 * src/quantization.c:8; SURVEY 8(b) ran 8 pthreads over one context).  Linked
 * against libdct_amd.so instead of src/{dct,quantization}.c.
 *
 *   block_pipeline_mt <pixels.u8> <width> <height> <quality> <adaptive> <threads> <reps> <out> [forward]
 *
 * With "forward" the pipeline stops after quantize (the four calls of the
 * reference's forward loop, tests/test_entropy.c:300-316; recon reads 0).
 * Thread t takes block rows t, t + T, ...; every rep repeats the whole plane.
 * <out> receives, per block in raster order, the 64 quantized ints (int32) and
 * the 64 reconstructed doubles (dct_inverse output, before + 128).  While the
 * workers run (after each has made one warm-up call), the main thread draws
 * glibc rand() from seed 1 and checks the sequence against one drawn before any
 * library call: the library must not touch the host's random stream.
 * Prints key:value lines (pipelines_per_s = blocks x reps / wall seconds).
 */
#define _POSIX_C_SOURCE 200112L
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "dct.h"
#include "quantization.h"

typedef struct {
    const unsigned char *px;
    int width, height, threads, reps, tid, forward_only;
    DCTContext *dct;
    QuantContext *qc;
    int32_t *q_out;
    double *r_out;
    pthread_barrier_t *bar;
} Job;

static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static int g_finished = 0;

static int workers_finished(void) {
    pthread_mutex_lock(&g_mu);
    const int n = g_finished;
    pthread_mutex_unlock(&g_mu);
    return n;
}

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

static void pipeline(Job *j, int by, int bx, double **c, int **q, double **dq, double **rec) {
    double **x = create_block_from_pixels((unsigned char *)j->px, j->width, 8 * by, 8 * bx, 8);
    dct_forward(j->dct, x, c);
    const double var = calculate_block_variance(x, 8);
    quantize(j->qc, c, q, var);
    if (!j->forward_only) {
        dequantize(j->qc, q, dq, var);
        dct_inverse(j->dct, dq, rec);
    }
    const long b = (long)by * (j->width / 8) + bx;
    for (int i = 0; i < 8; ++i)
        for (int k = 0; k < 8; ++k) {
            j->q_out[b * 64 + i * 8 + k] = q[i][k];
            j->r_out[b * 64 + i * 8 + k] = rec[i][k];
        }
    free_array(x, 8);
}

static void *worker(void *arg) {
    Job *j = (Job *)arg;
    double **c = alloc_array(8, 8), **dq = alloc_array(8, 8), **rec = alloc_array(8, 8);
    int **q = alloc_int_array(8, 8);
    pipeline(j, 0, 0, c, q, dq, rec); /* warm-up: this thread's first calls */
    pthread_barrier_wait(j->bar);     /* the main thread reseeds rand() now */
    pthread_barrier_wait(j->bar);
    for (int r = 0; r < j->reps; ++r)
        for (int by = j->tid; by < j->height / 8; by += j->threads)
            for (int bx = 0; bx < j->width / 8; ++bx) pipeline(j, by, bx, c, q, dq, rec);
    free_array(c, 8);
    free_array(dq, 8);
    free_array(rec, 8);
    free_int_array(q, 8);
    pthread_mutex_lock(&g_mu);
    ++g_finished;
    pthread_mutex_unlock(&g_mu);
    return NULL;
}

int main(int argc, char **argv) {
    if (argc != 9 && argc != 10) {
        fprintf(stderr, "usage: %s pixels width height quality adaptive threads reps out [forward]\n", argv[0]);
        return 2;
    }
    const int w = atoi(argv[2]), h = atoi(argv[3]), quality = atoi(argv[4]), adaptive = atoi(argv[5]);
    const int threads = atoi(argv[6]), reps = atoi(argv[7]);
    const int forward_only = argc == 10 && strcmp(argv[9], "forward") == 0;
    if (w <= 0 || h <= 0 || w % 8 || h % 8 || threads < 1 || threads > 64 || reps < 1) return 2;
    unsigned char *px = malloc((size_t)w * h);
    FILE *f = fopen(argv[1], "rb");
    if (!f || fread(px, 1, (size_t)w * h, f) != (size_t)w * h) return 3;
    fclose(f);

    enum { kDraws = 1 << 21 };
    int *want = malloc(sizeof(int) * kDraws);
    srand(1);
    for (int i = 0; i < kDraws; ++i) want[i] = rand();

    const long nblk = (long)(w / 8) * (h / 8);
    int32_t *q_out = calloc((size_t)nblk * 64, sizeof(int32_t));
    double *r_out = calloc((size_t)nblk * 64, sizeof(double));
    DCTContext *dct = dct_init(8);
    QuantContext *qc = quant_init(8, quality, adaptive);
    pthread_barrier_t bar;
    pthread_barrier_init(&bar, NULL, (unsigned)threads + 1);
    pthread_t th[64];
    Job jobs[64];
    for (int t = 0; t < threads; ++t) {
        jobs[t] = (Job){px, w, h, threads, reps, t, forward_only, dct, qc, q_out, r_out, &bar};
        pthread_create(&th[t], NULL, worker, &jobs[t]);
    }
    pthread_barrier_wait(&bar); /* every worker has made its first calls */
    srand(1);
    long draws = 0, bad = 0;
    const double t0 = now();
    pthread_barrier_wait(&bar);
    /* draw rand() while the workers run: the library's steady-state calls must leave it alone */
    while (draws < kDraws && workers_finished() < threads) {
        for (int k = 0; k < 256 && draws < kDraws; ++k, ++draws) bad += rand() != want[draws];
        struct timespec ts = {0, 100000};
        nanosleep(&ts, NULL);
    }
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    const double el = now() - t0;
    for (int k = 0; k < 1024 && draws < kDraws; ++k, ++draws) bad += rand() != want[draws];

    FILE *o = fopen(argv[8], "wb");
    if (!o) return 4;
    for (long b = 0; b < nblk; ++b) {
        fwrite(q_out + b * 64, sizeof(int32_t), 64, o);
        fwrite(r_out + b * 64, sizeof(double), 64, o);
    }
    fclose(o);
    printf("threads:%d\n", threads);
    printf("blocks:%ld\n", nblk * reps);
    printf("seconds:%.6f\n", el);
    printf("pipelines_per_s:%.1f\n", nblk * reps / el);
    printf("calls_per_s:%.1f\n", (forward_only ? 3.0 : 5.0) * nblk * reps / el);
    printf("rand_draws:%ld\n", draws);
    printf("rand_ok:%d\n", bad == 0);
    dct_free(dct);
    quant_free(qc);
    free(px);
    free(want);
    free(q_out);
    free(r_out);
    return 0;
}
