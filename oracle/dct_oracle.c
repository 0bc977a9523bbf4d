/*
 * oracle/dct_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker / CPU baseline).
 *
 * A clean-room, flat-array CPU restatement of the reference hot path
 * (erkinov-wtf/dct: src/dct.c + src/quantization.c) that follows the
 * reference's floating-point operation ORDER exactly, so that its results are
 * bit-identical to the reference's.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library.  The product (dct_amd/)
 * never links or calls it.
 *
 * Pinned: tests/test_oracle.py checks every function below against golden
 * vectors produced by the reference itself (compiled from /root/reference by
 * oracle/Makefile into oracle/_ref/, fixtures in tests/golden/).
 *
 * Build: -std=c99 -O2 -ffp-contract=off (the reference's -std=c99 already
 * implies no contraction under gcc; we make it explicit).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "dct_oracle.h"

/* include/dct.h:15 -- the literal the reference uses for pi. */
#define ORC_PI 3.14159265358979323846

/* src/quantization.c:8-17 -- JPEG Annex K luminance table. */
static const int orc_luma[64] = {
    16, 11, 10, 16, 24, 40, 51, 61,     12, 12, 14, 19, 26, 58, 60, 55,
    14, 13, 16, 24, 40, 57, 69, 56,     14, 17, 22, 29, 51, 87, 80, 62,
    18, 22, 37, 56, 68, 109, 103, 77,   24, 35, 55, 64, 81, 104, 113, 92,
    49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};

/* src/dct.c:17-30: D[i][j] = alpha_i * cos(PI*(2j+1)*i / (2N)).
 * The expression is evaluated as in the reference: (PI*(2j+1))*i, then the
 * quotient by (2.0*N); alpha_0 = 1/sqrt(N), alpha_i = sqrt(2/N). */
void orc_dct_matrix(int n, double *d) {
    for (int i = 0; i < n; ++i) {
        double a = (i == 0) ? 1.0 / sqrt(n) : sqrt(2.0 / n);
        for (int j = 0; j < n; ++j) d[i * n + j] = a * cos((ORC_PI * (2 * j + 1) * i) / (2.0 * n));
    }
}

/* src/quantization.c:51-99 (scale factor :55-60; 8x8 JPEG table :63-77; radial
 * formula for other sizes :80-96).  Quality is NOT clamped here (quant_init
 * clamps, :26-31). */
void orc_quant_matrix(int n, int quality, double *q) {
    double s;
    if (quality < 50)
        s = 5000.0 / quality;
    else
        s = 200.0 - 2 * quality;
    s /= 100.0;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            double v;
            if (n == 8)
                v = orc_luma[i * 8 + j] * s;
            else
                v = (1.0 + sqrt((double)(i * i + j * j))) * s * 8.0;
            if (v < 1.0) v = 1.0;
            if (v > 255.0) v = 255.0;
            q[i * n + j] = v;
        }
}

/* src/quantization.c:101-111: dequant = 1.0 / Q. */
void orc_dequant_matrix(int n, const double *q, double *dq) {
    for (int k = 0; k < n * n; ++k) dq[k] = 1.0 / q[k];
}

/* src/quantization.c:26-31 */
int orc_clamp_quality(int quality) {
    if (quality < 1) quality = 1;
    if (quality > 100) quality = 100;
    return quality;
}

/* src/dct.c:52-77 with the context's two public tables as given: temp = X * T
 * (T = ctx->transposed_dct, :61), out = D * temp (D = ctx->dct_matrix, :72),
 * k ascending, each accumulator starting at 0.0, separate multiply and add;
 * any n (temp on the heap, as the reference allocates it, :54). */
static void orc_forward_core(int n, const double *d, const double *t, const double *x, double *out, double *tmp) {
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            double acc = 0.0;
            for (int k = 0; k < n; ++k) acc += x[(size_t)i * n + k] * t[(size_t)k * n + j];
            tmp[(size_t)i * n + j] = acc;
        }
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            double acc = 0.0;
            for (int k = 0; k < n; ++k) acc += d[(size_t)i * n + k] * tmp[(size_t)k * n + j];
            out[(size_t)i * n + j] = acc;
        }
}

void orc_forward_tables(int n, const double *d, const double *t, const double *x, double *out) {
    double *tmp = malloc(sizeof(double) * (size_t)n * n);
    if (!tmp) abort();
    orc_forward_core(n, d, t, x, out, tmp);
    free(tmp);
}

/* src/dct.c:80-105 with the public tables as given: temp = T * C (:89),
 * out = temp * D (:100). */
void orc_inverse_tables(int n, const double *d, const double *t, const double *c, double *out) {
    double *tmp = malloc(sizeof(double) * (size_t)n * n);
    if (!tmp) abort();
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            double acc = 0.0;
            for (int k = 0; k < n; ++k) acc += t[(size_t)i * n + k] * c[(size_t)k * n + j];
            tmp[(size_t)i * n + j] = acc;
        }
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            double acc = 0.0;
            for (int k = 0; k < n; ++k) acc += tmp[(size_t)i * n + k] * d[(size_t)k * n + j];
            out[(size_t)i * n + j] = acc;
        }
    free(tmp);
}

static double *orc_transposed(int n, const double *d) {
    double *t = malloc(sizeof(double) * (size_t)n * n);
    if (!t) abort();
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) t[(size_t)i * n + j] = d[(size_t)j * n + i]; /* src/dct.c:33-37 */
    return t;
}

/* The context dct_init builds: T = D^T exactly (src/dct.c:33-37). */
void orc_forward(int n, const double *d, const double *x, double *out) {
    double *t = orc_transposed(n, d);
    orc_forward_tables(n, d, t, x, out);
    free(t);
}

/* 8x8 forward for the plane loops: T and temp on the stack. */
static void orc_forward8(const double *d, const double *x, double *out) {
    double t[64], tmp[64];
    for (int i = 0; i < 8; ++i)
        for (int j = 0; j < 8; ++j) t[i * 8 + j] = d[j * 8 + i];
    orc_forward_core(8, d, t, x, out, tmp);
}

void orc_inverse(int n, const double *d, const double *c, double *out) {
    double *t = orc_transposed(n, d);
    orc_inverse_tables(n, d, t, c, out);
    free(t);
}

/* src/quantization.c:153-169: row-major sum / sum of squares, mean = sum/count,
 * var = sum_sq/count - mean^2. */
double orc_variance(int n, const double *x) {
    double s = 0.0, s2 = 0.0;
    int cnt = n * n;
    for (int k = 0; k < cnt; ++k) {
        s += x[k];
        s2 += x[k] * x[k];
    }
    double mean = s / cnt;
    return (s2 / cnt) - (mean * mean);
}

/* src/quantization.c:171-211: per-block matrix.  nv = fmin(1, fmax(0.1, var/1000));
 * quantize: src=Q, scale = 2-nv, clamp >= 1; dequantize: src=1/Q, scale = 1/(2-nv).
 * Element (0,0) keeps the source value. */
void orc_adjust(int n, const double *src, double variance, int is_quantize, double *m) {
    double nv = fmin(1.0, fmax(0.1, variance / 1000.0));
    double scale = is_quantize ? 2.0 - nv : 1.0 / (2.0 - nv);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            double v;
            if (i == 0 && j == 0) {
                v = src[0];
            } else {
                v = src[i * n + j] * scale;
                if (is_quantize && v < 1.0) v = 1.0;
            }
            m[i * n + j] = v;
        }
}

/* src/quantization.c:113-131: q = (int) round(c / M). */
void orc_quantize(int n, const double *qm, int adaptive, double variance, const double *c, int *q) {
    double adj[64 * 64];
    const double *m = qm;
    if (adaptive) {
        orc_adjust(n, qm, variance, 1, adj);
        m = adj;
    }
    for (int k = 0; k < n * n; ++k) q[k] = (int)round(c[k] / m[k]);
}

/* src/quantization.c:133-151: non-adaptive dq = q * (1/Q) (the reference's
 * dequant table -- bug-compatible); adaptive dq = q * (1.0 / M)
 * with M = adjust(1/Q, var, 0). */
void orc_dequantize(int n, const double *dqm, int adaptive, double variance, const int *q, double *c) {
    double adj[64 * 64];
    if (adaptive) {
        orc_adjust(n, dqm, variance, 0, adj);
        for (int k = 0; k < n * n; ++k) c[k] = q[k] * (1.0 / adj[k]);
    } else {
        for (int k = 0; k < n * n; ++k) c[k] = q[k] * dqm[k];
    }
}

/* src/dct.c:109-120: x = (double)pixel - 128.0 from a row-major plane. */
void orc_block_from_pixels(const uint8_t *px, long stride, int row0, int col0, int n, double *x) {
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) x[i * n + j] = (double)px[(long)(row0 + i) * stride + (col0 + j)] - 128.0;
}

/* ---------------------------------------------------------------------------
 * Plane drivers: the per-block pipeline of tests/test_entropy.c:300-316
 * (pixels-128 -> dct_forward -> variance -> quantize) applied to every 8x8 block
 * of a plane in raster order; blocks are emitted as [by][bx][8][8] int16.
 * ------------------------------------------------------------------------- */
typedef struct {
    const uint8_t *px;
    long stride;
    int bw, bh, quality, adaptive;
    int16_t *out;
    double *fout; /* optional float-coefficient output [nblk][64] */
    int row_lo, row_hi;
    double d[64], q[64];
} orc_job;

static void orc_rows(orc_job *jb) {
    double x[64], c[64];
    int qi[64];
    for (int by = jb->row_lo; by < jb->row_hi; ++by)
        for (int bx = 0; bx < jb->bw; ++bx) {
            long b = (long)by * jb->bw + bx;
            orc_block_from_pixels(jb->px, jb->stride, by * 8, bx * 8, 8, x);
            orc_forward8(jb->d, x, c);
            if (jb->fout) memcpy(jb->fout + b * 64, c, sizeof c);
            if (jb->out) {
                double var = jb->adaptive ? orc_variance(8, x) : 0.0;
                orc_quantize(8, jb->q, jb->adaptive, var, c, qi);
                for (int k = 0; k < 64; ++k) jb->out[b * 64 + k] = (int16_t)qi[k];
            }
        }
}

static void *orc_thread(void *arg) {
    orc_rows((orc_job *)arg);
    return NULL;
}

int orc_forward_plane(const uint8_t *px, long stride, int width, int height, int quality, int adaptive,
                      int16_t *out, double *fout, int nthreads) {
    if (width % 8 || height % 8 || nthreads < 1) return -1;
    int bw = width / 8, bh = height / 8;
    if (nthreads > bh) nthreads = bh > 0 ? bh : 1;
    orc_job *jobs = calloc((size_t)nthreads, sizeof *jobs);
    pthread_t *th = calloc((size_t)nthreads, sizeof *th);
    if (!jobs || !th) return -2;
    for (int t = 0; t < nthreads; ++t) {
        orc_job *jb = &jobs[t];
        jb->px = px;
        jb->stride = stride;
        jb->bw = bw;
        jb->bh = bh;
        jb->quality = orc_clamp_quality(quality);
        jb->adaptive = adaptive;
        jb->out = out;
        jb->fout = fout;
        jb->row_lo = (int)((long)bh * t / nthreads);
        jb->row_hi = (int)((long)bh * (t + 1) / nthreads);
        orc_dct_matrix(8, jb->d);
        orc_quant_matrix(8, jb->quality, jb->q);
    }
    for (int t = 1; t < nthreads; ++t) pthread_create(&th[t], NULL, orc_thread, &jobs[t]);
    orc_rows(&jobs[0]);
    for (int t = 1; t < nthreads; ++t) pthread_join(th[t], NULL);
    free(jobs);
    free(th);
    return 0;
}

/* Inverse pipeline of tests/test_entropy.c:350-393 per block:
 * dequantize(q, var) -> dct_inverse -> recon = out + 128 (double, unclamped).
 * `var` per block is needed for adaptive mode (the forward pass's variance). */
int orc_inverse_plane(const int16_t *coef, const double *var, int nblocks, int quality, int adaptive,
                      double *recon) {
    double d[64], q[64], dq[64], c[64], o[64];
    int qi[64];
    orc_dct_matrix(8, d);
    orc_quant_matrix(8, orc_clamp_quality(quality), q);
    orc_dequant_matrix(8, q, dq);
    for (long b = 0; b < nblocks; ++b) {
        for (int k = 0; k < 64; ++k) qi[k] = coef[b * 64 + k];
        orc_dequantize(8, dq, adaptive, var ? var[b] : 0.0, qi, c);
        orc_inverse(8, d, c, o);
        for (int k = 0; k < 64; ++k) recon[b * 64 + k] = o[k];
    }
    return 0;
}

/* Per-block variance of a plane (adaptive side-channel for the inverse). */
int orc_plane_variance(const uint8_t *px, long stride, int width, int height, double *var) {
    double x[64];
    int bw = width / 8, bh = height / 8;
    for (int by = 0; by < bh; ++by)
        for (int bx = 0; bx < bw; ++bx) {
            orc_block_from_pixels(px, stride, by * 8, bx * 8, 8, x);
            var[(long)by * bw + bx] = orc_variance(8, x);
        }
    return 0;
}

/* ---------------------------------------------------------------------------
 * Synthetic frames.  A counter-based splitmix64 (Steele et al. 2014) so that the
 * host, the tests and the device generator (dct_amd/csrc/synth.hip) agree bit
 * for bit without shipping data.  All arithmetic is integer.
 * ------------------------------------------------------------------------- */
static uint64_t orc_mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
uint64_t orc_splitmix(uint64_t seed, uint64_t i) { return orc_mix(seed + (i + 1) * 0x9E3779B97F4A7C15ULL); }

/* kind: 0 uniform, 1 smooth (bilinear random lattice + small noise),
 *       2 constant 8x8 blocks, 3 extremes (each pixel 0 or 255) */
uint8_t orc_synth_pixel(uint64_t seed, int kind, int width, int x, int y) {
    uint64_t idx = (uint64_t)y * (uint64_t)width + (uint64_t)x;
    switch (kind) {
    case 0:
        return (uint8_t)(orc_splitmix(seed, idx) & 0xFF);
    case 1: {
        int cx = x >> 4, cy = y >> 4, fx = x & 15, fy = y & 15;
        uint64_t s2 = seed ^ 0x5DEECE66DULL;
        int gw = (width >> 4) + 2;
        int v00 = (int)(orc_splitmix(s2, (uint64_t)cy * gw + cx) & 0xFF);
        int v01 = (int)(orc_splitmix(s2, (uint64_t)cy * gw + cx + 1) & 0xFF);
        int v10 = (int)(orc_splitmix(s2, (uint64_t)(cy + 1) * gw + cx) & 0xFF);
        int v11 = (int)(orc_splitmix(s2, (uint64_t)(cy + 1) * gw + cx + 1) & 0xFF);
        int top = v00 * (16 - fx) + v01 * fx, bot = v10 * (16 - fx) + v11 * fx;
        int v = (top * (16 - fy) + bot * fy + 128) >> 8;
        int noise = (int)(orc_splitmix(seed, idx) & 7) - 3;
        v += noise;
        return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
    }
    case 2: {
        uint64_t b = (uint64_t)(y >> 3) * (uint64_t)((width + 7) >> 3) + (uint64_t)(x >> 3);
        return (uint8_t)(orc_splitmix(seed, b) & 0xFF);
    }
    default:
        return (orc_splitmix(seed, idx) & 1) ? 255 : 0;
    }
}

void orc_synth_plane(uint64_t seed, int kind, int width, int height, uint8_t *px, long stride) {
    for (int y = 0; y < height; ++y)
        for (int x = 0; x < width; ++x) px[(long)y * stride + x] = orc_synth_pixel(seed, kind, width, x, y);
}

/* ---- zigzag + run-length symbols ------------------------- */

/* src/entropy.c:158-178: order[k] = natural (row-major) index of the k-th
 * element of the zigzag traversal (anti-diagonals; even sums walk up-right
 * from the row maximum, odd sums walk down-left from the row minimum). */
void orc_zigzag_order(int n, int *order) {
    int k = 0;
    for (int sum = 0; sum <= 2 * (n - 1); ++sum) {
        if (sum % 2 == 0) {
            for (int i = sum < n ? sum : n - 1; i >= 0 && sum - i < n; --i) order[k++] = i * n + (sum - i);
        } else {
            for (int i = sum < n ? 0 : sum - n + 1; i < n && sum - i >= 0; ++i) order[k++] = i * n + (sum - i);
        }
    }
}

/* src/entropy.c:216-256: one (value, run) symbol per nonzero zigzag element,
 * the run counting the zeros before it, and always a symbol for the LAST
 * element -- whose run also counts itself when it is zero.  Returns the count. */
int orc_rle_encode(int n, const int *coeffs, int *values, int *runs) {
    int order[64 * 64];
    orc_zigzag_order(n, order);
    int count = 0, zeros = 0, size = n * n;
    for (int i = 0; i < size; ++i) {
        int v = coeffs[order[i]];
        if (v != 0 || i == size - 1) {
            if (i == size - 1 && v == 0) zeros++;
            values[count] = v;
            runs[count] = zeros;
            count++;
            zeros = 0;
        } else {
            zeros++;
        }
    }
    return count;
}

/* src/entropy.c:327-351 (run_length_decode): skip `run` zeros, place the value
 * (dropped when past the end), then undo the zigzag (:183-210). */
void orc_rle_decode(int n, const int *values, const int *runs, int count, int *coeffs) {
    int order[64 * 64], zz[64 * 64];
    int size = n * n, pos = 0;
    orc_zigzag_order(n, order);
    for (int i = 0; i < size; ++i) zz[i] = 0;
    for (int i = 0; i < count; ++i) {
        pos += runs[i];
        if (pos < size) zz[pos++] = values[i];
    }
    for (int i = 0; i < size; ++i) coeffs[order[i]] = zz[i];
}

/* Batched form of the device format (include/dct_amd.h, dctq_rle_*):
 * offsets[b] = symbols before block b (offsets[nblk] = total), symbol =
 * (uint16)value | run << 16, blocks in order.  Returns the total. */
long orc_rle_encode_plane(const int16_t *coef, long nblk, uint32_t *offsets, uint32_t *symbols) {
    long total = 0;
    int c[64], v[64], r[64];
    for (long b = 0; b < nblk; ++b) {
        for (int k = 0; k < 64; ++k) c[k] = coef[b * 64 + k];
        int cnt = orc_rle_encode(8, c, v, r);
        if (offsets) offsets[b] = (uint32_t)total;
        if (symbols)
            for (int k = 0; k < cnt; ++k) symbols[total + k] = (uint32_t)(uint16_t)(int16_t)v[k] | ((uint32_t)r[k] << 16);
        total += cnt;
    }
    if (offsets) offsets[nblk] = (uint32_t)total;
    return total;
}

/* ---- per-block Huffman size ------------------------------
 * src/entropy.c:261-328 build_huffman_codes + :363-399 get_encoded_size for the
 * symbols of one block, as the pipeline calls them (tests/test_entropy.c:
 * 329-341, use_huffman = 1).  Restated with the reference's own heap
 * discipline (pq_push :36-46 sifts up past strictly larger parents; pq_pop
 * :48-77 moves the last node to the root and sifts down to the strictly
 * smaller child, left first), leaves pushed in increasing symbol index
 * (value + max|value| + 1), each merge popping left then right, so the tree --
 * and every individual code length -- is the reference's. */
typedef struct { unsigned freq; int value, left, right; } orc_hnode;

static void orc_pq_push(int *heap, int *size, const orc_hnode *nodes, int node) {
    int i = (*size)++;
    while (i > 0 && nodes[heap[(i - 1) / 2]].freq > nodes[node].freq) {
        heap[i] = heap[(i - 1) / 2];
        i = (i - 1) / 2;
    }
    heap[i] = node;
}

static int orc_pq_pop(int *heap, int *size, const orc_hnode *nodes) {
    int top = heap[0];
    heap[0] = heap[--(*size)];
    int i = 0;
    while (i * 2 + 1 < *size) {
        int s = i, l = 2 * i + 1, r = 2 * i + 2;
        if (l < *size && nodes[heap[l]].freq < nodes[heap[s]].freq) s = l;
        if (r < *size && nodes[heap[r]].freq < nodes[heap[s]].freq) s = r;
        if (s == i) break;
        int t = heap[i];
        heap[i] = heap[s];
        heap[s] = t;
        i = s;
    }
    return top;
}

/* depth of every leaf (generate_codes :99-122: the code of a leaf is its path) */
static void orc_depths(const orc_hnode *nodes, int node, int depth, int *len_of_value, int off) {
    if (nodes[node].left < 0 && nodes[node].right < 0) {
        len_of_value[nodes[node].value + off] = depth;
        return;
    }
    if (nodes[node].left >= 0) orc_depths(nodes, nodes[node].left, depth + 1, len_of_value, off);
    if (nodes[node].right >= 0) orc_depths(nodes, nodes[node].right, depth + 1, len_of_value, off);
}

int orc_huffman_bits(const int *coeffs) {
    int v[64], r[64];
    int cnt = orc_rle_encode(8, coeffs, v, r);
    int maxs = 0;
    for (int k = 0; k < cnt; ++k) maxs = abs(v[k]) > maxs ? abs(v[k]) : maxs;
    int nsym = 2 * maxs + 2, off = maxs + 1;
    unsigned *freq = (unsigned *)calloc((size_t)nsym, sizeof(unsigned));
    int *len = (int *)calloc((size_t)nsym, sizeof(int));
    orc_hnode *nodes = (orc_hnode *)malloc(sizeof(orc_hnode) * (size_t)(2 * nsym));
    int *heap = (int *)malloc(sizeof(int) * (size_t)nsym);
    for (int k = 0; k < cnt; ++k) freq[v[k] + off]++;
    int nn = 0, size = 0;
    for (int i = 0; i < nsym; ++i)
        if (freq[i]) {
            nodes[nn] = (orc_hnode){freq[i], i - off, -1, -1};
            orc_pq_push(heap, &size, nodes, nn++);
        }
    while (size > 1) {
        int a = orc_pq_pop(heap, &size, nodes), b = orc_pq_pop(heap, &size, nodes);
        nodes[nn] = (orc_hnode){nodes[a].freq + nodes[b].freq, -1, a, b};
        orc_pq_push(heap, &size, nodes, nn++);
    }
    orc_depths(nodes, orc_pq_pop(heap, &size, nodes), 0, len, off);
    int bits = 0;
    for (int k = 0; k < cnt; ++k) bits += len[v[k] + off] + 8;  /* code length + 8 run bits */
    free(freq);
    free(len);
    free(nodes);
    free(heap);
    return bits;
}

void orc_huffman_bits_plane(const int16_t *coef, long nblk, uint32_t *bits) {
    int c[64];
    for (long b = 0; b < nblk; ++b) {
        for (int k = 0; k < 64; ++k) c[k] = coef[b * 64 + k];
        bits[b] = (uint32_t)orc_huffman_bits(c);
    }
}
