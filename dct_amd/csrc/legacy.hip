// dct_amd/csrc/legacy.hip -- the reference's per-block API (include/dct.h,
// include/quantization.h, include/utils.h) as a drop-in, backed by the GPU.
//
// Each call marshals its row-pointer arrays into one staging buffer, runs a
// small exact kernel that repeats the reference's fp64 arithmetic in the same
// order (this file is compiled with -ffp-contract=off), and copies the result
// back -- bit-identical to src/dct.c and src/quantization.c for any block size
// up to 64.  It is a drop-in for callers that stay per-block; frame-level
// callers should use include/dct_amd.h (one launch per plane).
//
// Conventions kept from the reference: no return codes; failures print to
// stderr and exit(EXIT_FAILURE) (src/utils.c:10-12, src/dct.c:9-12); contexts
// and matrices are plain malloc'd row-pointer arrays with public fields.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "dct.h"
#include "dctq_internal.h"
#include "host_tables.h"
#include "quantization.h"
#include "utils.h"

namespace {

[[noreturn]] void die(const char *what, hipError_t e = hipSuccess) {
    if (e != hipSuccess)
        fprintf(stderr, "%s failed: %s\n", what, hipGetErrorString(e));
    else
        fprintf(stderr, "%s\n", what);
    exit(EXIT_FAILURE);
}
#define LCHK(call, what)                          \
    do {                                          \
        hipError_t e_ = (call);                   \
        if (e_ != hipSuccess) die(what, e_);      \
    } while (0)

constexpr int kMaxN = 64;

// ---------------------------------------------------------------- kernels
// src/dct.c:52-77 -- one workgroup per block; temp in LDS.
__global__ void k_forward(int n, const double *__restrict__ d, const double *__restrict__ in, double *__restrict__ out) {
    extern __shared__ double tmp[];
    const int nn = n * n;
    for (int e = threadIdx.x; e < nn; e += blockDim.x) {
        const int i = e / n, j = e % n;
        double acc = 0.0;
        for (int k = 0; k < n; ++k) acc += in[i * n + k] * d[j * n + k];  // input[i][k] * D^T[k][j]
        tmp[e] = acc;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < nn; e += blockDim.x) {
        const int i = e / n, j = e % n;
        double acc = 0.0;
        for (int k = 0; k < n; ++k) acc += d[i * n + k] * tmp[k * n + j];
        out[e] = acc;
    }
}

// src/dct.c:80-105
__global__ void k_inverse(int n, const double *__restrict__ d, const double *__restrict__ in, double *__restrict__ out) {
    extern __shared__ double tmp[];
    const int nn = n * n;
    for (int e = threadIdx.x; e < nn; e += blockDim.x) {
        const int i = e / n, j = e % n;
        double acc = 0.0;
        for (int k = 0; k < n; ++k) acc += d[k * n + i] * in[k * n + j];  // D^T[i][k] * input[k][j]
        tmp[e] = acc;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < nn; e += blockDim.x) {
        const int i = e / n, j = e % n;
        double acc = 0.0;
        for (int k = 0; k < n; ++k) acc += tmp[i * n + k] * d[k * n + j];
        out[e] = acc;
    }
}

// src/quantization.c:171-211 element (i,j) of the adjusted matrix.
__device__ double adjusted(const double *src, int e, double variance, int is_quantize) {
    const double nv = fmin(1.0, fmax(0.1, variance / 1000.0));
    const double scale = is_quantize ? 2.0 - nv : 1.0 / (2.0 - nv);
    if (e == 0) return src[0];
    double v = src[e] * scale;
    if (is_quantize && v < 1.0) v = 1.0;
    return v;
}

// src/quantization.c:113-131 (mode 0), :133-151 (mode 1), :171-211 (mode 2),
// src/dct.c:123-129 (mode 3: (int) round(c)).
__global__ void k_elementwise(int mode, int nn, const double *__restrict__ m, int adaptive, double variance,
                              const double *__restrict__ din, const int *__restrict__ iin, double *__restrict__ dout,
                              int *__restrict__ iout) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nn) return;
    switch (mode) {
    case 0: {
        const double mm = adaptive ? adjusted(m, e, variance, 1) : m[e];
        iout[e] = (int)round(din[e] / mm);
        break;
    }
    case 1:
        dout[e] = iin[e] * (adaptive ? 1.0 / adjusted(m, e, variance, 0) : m[e]);
        break;
    case 2:
        dout[e] = adjusted(m, e, variance, adaptive);  // `adaptive` carries is_quantize here
        break;
    default:
        iout[e] = (int)round(din[e]);
        break;
    }
}

// src/quantization.c:153-169 -- sequential row-major sums (order matters for non-integer input).
__global__ void k_variance(int nn, const double *__restrict__ x, double *__restrict__ out) {
    double s = 0.0, s2 = 0.0;
    for (int k = 0; k < nn; ++k) {
        s += x[k];
        s2 += x[k] * x[k];
    }
    const double mean = s / nn;
    out[0] = (s2 / nn) - (mean * mean);
}

// ---------------------------------------------------------------- staging
struct Staging {
    void *dev = nullptr;
    size_t bytes = 0;
    std::vector<unsigned char> host;
    void *get(size_t need) {
        if (need > bytes) {
            if (dev) (void)hipFree(dev);
            LCHK(hipMalloc(&dev, need), "hipMalloc(legacy staging)");
            bytes = need;
        }
        if (host.size() < need) host.resize(need);
        return dev;
    }
};
thread_local Staging g_stage;

void pack(double **a, int n, double *dst) {
    for (int i = 0; i < n; ++i) memcpy(dst + i * n, a[i], sizeof(double) * n);
}
void unpack(const double *src, int n, double **a) {
    for (int i = 0; i < n; ++i) memcpy(a[i], src + i * n, sizeof(double) * n);
}

void check_n(int n) {
    if (n < 1 || n > kMaxN) die("block_size out of the supported range 1..64");
}

void transform(DCTContext *ctx, double **input, double **output, bool fwd) {
    DCTQ_ENTRY;  // HIP calls below must not touch the host's rand() stream
    const int n = ctx->block_size, nn = n * n;
    check_n(n);
    const size_t bytes = sizeof(double) * 3 * nn;
    double *dev = (double *)g_stage.get(bytes);
    double *h = (double *)g_stage.host.data();
    pack(ctx->dct_matrix, n, h);
    pack(input, n, h + nn);
    LCHK(hipMemcpy(dev, h, sizeof(double) * 2 * nn, hipMemcpyHostToDevice), "hipMemcpy");
    const int threads = nn < 256 ? ((nn + 63) / 64) * 64 : 256;
    if (fwd)
        hipLaunchKernelGGL(k_forward, dim3(1), dim3(threads), sizeof(double) * nn, 0, n, dev, dev + nn, dev + 2 * nn);
    else
        hipLaunchKernelGGL(k_inverse, dim3(1), dim3(threads), sizeof(double) * nn, 0, n, dev, dev + nn, dev + 2 * nn);
    LCHK(hipGetLastError(), "kernel launch");
    LCHK(hipMemcpy(h + 2 * nn, dev + 2 * nn, sizeof(double) * nn, hipMemcpyDeviceToHost), "hipMemcpy");
    unpack(h + 2 * nn, n, output);
}

// One elementwise launch over an n x n block; inputs/outputs as flat host arrays.
void elementwise(int mode, int n, double **m, int flag, double variance, const double *din, const int *iin,
                 double *dout, int *iout) {
    DCTQ_ENTRY;  // HIP calls below must not touch the host's rand() stream
    const int nn = n * n;
    const size_t bytes = sizeof(double) * 3 * nn + sizeof(int) * 2 * nn;
    unsigned char *dev = (unsigned char *)g_stage.get(bytes);
    unsigned char *h = g_stage.host.data();
    double *hm = (double *)h, *hd = hm + nn;
    int *hi = (int *)(hd + 2 * nn);
    pack(m, n, hm);
    if (din) memcpy(hd, din, sizeof(double) * nn);
    if (iin) memcpy(hi, iin, sizeof(int) * nn);
    LCHK(hipMemcpy(dev, h, bytes, hipMemcpyHostToDevice), "hipMemcpy");
    double *dm = (double *)dev, *dd = dm + nn, *ddo = dd + nn;
    int *di = (int *)(ddo + nn), *dio = di + nn;
    hipLaunchKernelGGL(k_elementwise, dim3((nn + 255) / 256), dim3(256), 0, 0, mode, nn, dm, flag, variance, dd, di,
                       ddo, dio);
    LCHK(hipGetLastError(), "kernel launch");
    LCHK(hipMemcpy(h, dev, bytes, hipMemcpyDeviceToHost), "hipMemcpy");
    if (dout) memcpy(dout, (double *)h + 2 * nn, sizeof(double) * nn);
    if (iout) memcpy(iout, (int *)((double *)h + 3 * nn) + nn, sizeof(int) * nn);
}

}  // namespace

extern "C" {

// ------------------------------------------------------------- utils.h
double **alloc_array(int rows, int cols) {
    double **a = (double **)malloc(sizeof(double *) * (size_t)(rows > 0 ? rows : 1));
    if (!a) die("Memory allocation failed, when creating new 2D array");
    for (int i = 0; i < rows; ++i) {
        a[i] = (double *)calloc((size_t)(cols > 0 ? cols : 1), sizeof(double));
        if (!a[i]) die("Memory allocation failed, when creating new 2D array");
    }
    return a;
}

void free_array(double **array, int rows) {
    if (!array) return;
    for (int i = 0; i < rows; ++i) free(array[i]);
    free(array);
}

int **alloc_int_array(int rows, int cols) {
    int **a = (int **)malloc(sizeof(int *) * (size_t)(rows > 0 ? rows : 1));
    if (!a) die("Memory allocation failed, when creating new 2D integer array");
    for (int i = 0; i < rows; ++i) {
        a[i] = (int *)calloc((size_t)(cols > 0 ? cols : 1), sizeof(int));
        if (!a[i]) die("Memory allocation failed, when creating new 2D integer array");
    }
    return a;
}

void free_int_array(int **array, int rows) {
    if (!array) return;
    for (int i = 0; i < rows; ++i) free(array[i]);
    free(array);
}

// ------------------------------------------------------------- dct.h
DCTContext *dct_init(int block_size) {
    DCTContext *ctx = (DCTContext *)malloc(sizeof(DCTContext));
    if (!ctx) die("Memory allocation failed, when creating new context");
    check_n(block_size);
    ctx->block_size = block_size;
    ctx->dct_matrix = alloc_array(block_size, block_size);
    ctx->transposed_dct = alloc_array(block_size, block_size);
    std::vector<double> d((size_t)block_size * block_size);
    dctq_host::dct_matrix(block_size, d.data());
    for (int i = 0; i < block_size; ++i)
        for (int j = 0; j < block_size; ++j) {
            ctx->dct_matrix[i][j] = d[(size_t)i * block_size + j];
            ctx->transposed_dct[j][i] = d[(size_t)i * block_size + j];
        }
    return ctx;
}

void dct_free(DCTContext *ctx) {
    if (!ctx) return;
    free_array(ctx->dct_matrix, ctx->block_size);
    free_array(ctx->transposed_dct, ctx->block_size);
    free(ctx);
}

void dct_forward(DCTContext *ctx, double **input, double **output) { transform(ctx, input, output, true); }

void dct_inverse(DCTContext *ctx, double **input, double **output) { transform(ctx, input, output, false); }

double **create_block_from_pixels(unsigned char *pixels, int width, int row_start, int col_start, int block_size) {
    // Marshalling only (gather of host bytes into a host row-pointer array); the
    // arithmetic "- 128" is exact.  Batched callers never come here: the
    // dct_amd.h kernels read pixels straight from HBM.
    double **block = alloc_array(block_size, block_size);
    for (int i = 0; i < block_size; ++i)
        for (int j = 0; j < block_size; ++j)
            block[i][j] = (double)pixels[(long)(row_start + i) * width + (col_start + j)] - 128.0;
    return block;
}

void copy_block_to_coefficients(double **block, int **coefficients, int block_size) {
    check_n(block_size);
    std::vector<double> in((size_t)block_size * block_size);
    std::vector<int> out(in.size());
    pack(block, block_size, in.data());
    double **dummy = block;  // unused table slot
    elementwise(3, block_size, dummy, 0, 0.0, in.data(), nullptr, nullptr, out.data());
    for (int i = 0; i < block_size; ++i) memcpy(coefficients[i], &out[(size_t)i * block_size], sizeof(int) * block_size);
}

// ------------------------------------------------------------- quantization.h
QuantContext *quant_init(int block_size, int quality, int adaptive) {
    QuantContext *ctx = (QuantContext *)malloc(sizeof(QuantContext));
    if (!ctx) die("Memory allocation failed when creating quantization context");
    quality = dctq_host::clamp_quality(quality);
    ctx->block_size = block_size;
    ctx->quality = quality;
    ctx->adaptive = adaptive;
    ctx->quant_matrix = generate_quant_matrix(block_size, quality);
    ctx->dequant_matrix = generate_dequant_matrix(ctx->quant_matrix, block_size);
    return ctx;
}

void quant_free(QuantContext *ctx) {
    if (!ctx) return;
    free_array(ctx->quant_matrix, ctx->block_size);
    free_array(ctx->dequant_matrix, ctx->block_size);
    free(ctx);
}

double **generate_quant_matrix(int block_size, int quality) {
    double **m = alloc_array(block_size, block_size);
    std::vector<double> q((size_t)block_size * block_size);
    dctq_host::quant_matrix(block_size, quality, q.data());
    unpack(q.data(), block_size, m);
    return m;
}

double **generate_dequant_matrix(double **quant_matrix, int block_size) {
    double **m = alloc_array(block_size, block_size);
    for (int i = 0; i < block_size; ++i)
        for (int j = 0; j < block_size; ++j) m[i][j] = 1.0 / quant_matrix[i][j];
    return m;
}

void quantize(QuantContext *ctx, double **dct_coeffs, int **quant_coeffs, double block_variance) {
    const int n = ctx->block_size;
    check_n(n);
    std::vector<double> in((size_t)n * n);
    std::vector<int> out(in.size());
    pack(dct_coeffs, n, in.data());
    elementwise(0, n, ctx->quant_matrix, ctx->adaptive, block_variance, in.data(), nullptr, nullptr, out.data());
    for (int i = 0; i < n; ++i) memcpy(quant_coeffs[i], &out[(size_t)i * n], sizeof(int) * n);
}

void dequantize(QuantContext *ctx, int **quant_coeffs, double **dct_coeffs, double block_variance) {
    const int n = ctx->block_size;
    check_n(n);
    std::vector<int> in((size_t)n * n);
    std::vector<double> out(in.size());
    for (int i = 0; i < n; ++i) memcpy(&in[(size_t)i * n], quant_coeffs[i], sizeof(int) * n);
    elementwise(1, n, ctx->dequant_matrix, ctx->adaptive, block_variance, nullptr, in.data(), out.data(), nullptr);
    unpack(out.data(), n, dct_coeffs);
}

double calculate_block_variance(double **block, int block_size) {
    DCTQ_ENTRY;  // HIP calls below must not touch the host's rand() stream
    check_n(block_size);
    const int nn = block_size * block_size;
    double *dev = (double *)g_stage.get(sizeof(double) * (nn + 1));
    double *h = (double *)g_stage.host.data();
    pack(block, block_size, h);
    LCHK(hipMemcpy(dev, h, sizeof(double) * nn, hipMemcpyHostToDevice), "hipMemcpy");
    hipLaunchKernelGGL(k_variance, dim3(1), dim3(1), 0, 0, nn, dev, dev + nn);
    LCHK(hipGetLastError(), "kernel launch");
    double v = 0.0;
    LCHK(hipMemcpy(&v, dev + nn, sizeof(double), hipMemcpyDeviceToHost), "hipMemcpy");
    return v;
}

double **adjust_matrix_for_block(QuantContext *ctx, double variance, int is_quantize) {
    const int n = ctx->block_size;
    check_n(n);
    double **m = alloc_array(n, n);
    std::vector<double> out((size_t)n * n);
    elementwise(2, n, is_quantize ? ctx->quant_matrix : ctx->dequant_matrix, is_quantize, variance, nullptr, nullptr,
                out.data(), nullptr);
    unpack(out.data(), n, m);
    return m;
}

}  // extern "C"
