// dct_amd/csrc/legacy.hip -- the reference's per-block API (include/dct.h,
// include/quantization.h, include/utils.h) as a drop-in, backed by the GPU.
//
// Each call marshals its row-pointer arrays into one pinned, device-mapped
// staging buffer, runs a small exact kernel that reads it over the host link,
// repeats the reference's fp64 arithmetic in the same order (this file is
// compiled with -ffp-contract=off) and writes the result back into it --
// bit-identical to src/dct.c and src/quantization.c for any block size
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
// src/dct.c:52-77 (forward) and :80-105 (inverse) -- one workgroup per block.
// `d` and `in` live in pinned host memory (zero-copy staging, see Staging): the
// workgroup first copies them into LDS in one parallel round trip over the host
// link (d stays in host memory when 3 n^2 doubles exceed kLdsTables), then runs
// both passes from LDS and writes `out` straight back to host memory.
constexpr int kLdsTables = 48 * 1024;
__device__ __forceinline__ const double *stage_in(const double *__restrict__ src, double *dst, int nn) {
    for (int e = threadIdx.x; e < nn; e += blockDim.x) dst[e] = src[e];
    return dst;
}

template <bool FWD>
__global__ void k_transform(int n, const double *__restrict__ dh, const double *__restrict__ inh,
                            double *__restrict__ out) {
    extern __shared__ double lds[];
    const int nn = n * n;
    const bool dl = 3 * nn * (int)sizeof(double) <= kLdsTables;
    double *tmp = lds, *in = lds + nn;
    const double *d = dl ? stage_in(dh, lds + 2 * nn, nn) : dh;
    stage_in(inh, in, nn);
    __syncthreads();
    for (int e = threadIdx.x; e < nn; e += blockDim.x) {
        const int i = e / n, j = e % n;
        double acc = 0.0;
        if (FWD)
            for (int k = 0; k < n; ++k) acc += in[i * n + k] * d[j * n + k];  // input[i][k] * D^T[k][j]
        else
            for (int k = 0; k < n; ++k) acc += d[k * n + i] * in[k * n + j];  // D^T[i][k] * input[k][j]
        tmp[e] = acc;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < nn; e += blockDim.x) {
        const int i = e / n, j = e % n;
        double acc = 0.0;
        if (FWD)
            for (int k = 0; k < n; ++k) acc += d[i * n + k] * tmp[k * n + j];
        else
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

// src/quantization.c:153-169 -- sequential row-major sums (order matters for
// non-integer input), after one parallel copy of the block into LDS.
__global__ void k_variance(int nn, const double *__restrict__ xh, double *__restrict__ out) {
    extern __shared__ double x[];
    stage_in(xh, x, nn);
    __syncthreads();
    if (threadIdx.x != 0) return;
    double s = 0.0, s2 = 0.0;
    for (int k = 0; k < nn; ++k) {
        s += x[k];
        s2 += x[k] * x[k];
    }
    const double mean = s / nn;
    out[0] = (s2 / nn) - (mean * mean);
}

// ---------------------------------------------------------------- staging
// Zero-copy: one pinned, device-mapped host buffer per thread.  A call packs its
// row-pointer arrays into it, launches one kernel that reads its inputs from it
// and writes its outputs back into it over the host link, and synchronizes: no
// memcpy calls (each was a synchronous round trip through the driver).
struct Staging {
    unsigned char *host = nullptr;  // pinned host memory
    unsigned char *dev = nullptr;   // the same pages as seen by the device
    size_t bytes = 0;
    unsigned char *get(size_t need) {
        if (need > bytes) {
            if (host) (void)hipHostFree(host);
            host = nullptr;
            LCHK(hipHostMalloc((void **)&host, need, hipHostMallocMapped), "hipHostMalloc(legacy staging)");
            LCHK(hipHostGetDevicePointer((void **)&dev, host, 0), "hipHostGetDevicePointer");
            bytes = need;
        }
        return host;
    }
};
thread_local Staging g_stage;

void finish(const char *what) {
    LCHK(hipGetLastError(), what);
    LCHK(hipStreamSynchronize(nullptr), "hipStreamSynchronize");
}

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
    double *h = (double *)g_stage.get(sizeof(double) * 3 * nn);
    const double *dv = (const double *)g_stage.dev;
    pack(ctx->dct_matrix, n, h);
    pack(input, n, h + nn);
    const int threads = nn < 256 ? ((nn + 63) / 64) * 64 : 256;
    const size_t lds = sizeof(double) * (3 * nn * sizeof(double) <= (size_t)kLdsTables ? 3 * nn : 2 * nn);
    if (fwd)
        hipLaunchKernelGGL(k_transform<true>, dim3(1), dim3(threads), lds, 0, n, dv, dv + nn, (double *)dv + 2 * nn);
    else
        hipLaunchKernelGGL(k_transform<false>, dim3(1), dim3(threads), lds, 0, n, dv, dv + nn, (double *)dv + 2 * nn);
    finish("transform launch");
    unpack(h + 2 * nn, n, output);
}

// One elementwise launch over an n x n block; inputs/outputs as flat host arrays.
void elementwise(int mode, int n, double **m, int flag, double variance, const double *din, const int *iin,
                 double *dout, int *iout) {
    DCTQ_ENTRY;  // HIP calls below must not touch the host's rand() stream
    const int nn = n * n;
    const size_t bytes = sizeof(double) * 3 * nn + sizeof(int) * 2 * nn;
    unsigned char *h = g_stage.get(bytes);
    double *hm = (double *)h, *hd = hm + nn;
    int *hi = (int *)(hd + 2 * nn);
    pack(m, n, hm);
    if (din) memcpy(hd, din, sizeof(double) * nn);
    if (iin) memcpy(hi, iin, sizeof(int) * nn);
    double *dm = (double *)g_stage.dev, *dd = dm + nn, *ddo = dd + nn;
    int *di = (int *)(ddo + nn), *dio = di + nn;
    hipLaunchKernelGGL(k_elementwise, dim3((nn + 255) / 256), dim3(256), 0, 0, mode, nn, dm, flag, variance, dd, di,
                       ddo, dio);
    finish("elementwise launch");
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
    double *h = (double *)g_stage.get(sizeof(double) * (nn + 1));
    double *dv = (double *)g_stage.dev;
    pack(block, block_size, h);
    const int threads = nn < 256 ? ((nn + 63) / 64) * 64 : 256;
    hipLaunchKernelGGL(k_variance, dim3(1), dim3(threads), sizeof(double) * nn, 0, nn, dv, dv + nn);
    finish("variance launch");
    return h[nn];
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
