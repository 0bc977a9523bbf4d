// dct_amd/csrc/legacy.hip -- the reference's per-block API (include/dct.h,
// include/quantization.h, include/utils.h) as a drop-in, backed by the GPU.
//
// Each call marshals its row-pointer arrays into one pinned, device-mapped
// staging buffer (or, for large blocks, a device scratch buffer), runs a small
// exact kernel, repeats the reference's fp64 arithmetic in the same order (this
// file is compiled with -ffp-contract=off) and copies the result back --
// bit-identical to src/dct.c and src/quantization.c for any block size.  It is a drop-in for callers that stay per-block; frame-level
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

#include <atomic>
#include <chrono>
#include <mutex>
#include <optional>
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

// ---------------------------------------------------------------- kernels
// src/dct.c:52-77 (forward) and :80-105 (inverse).  Both passes of both
// transforms are Z[i][j] = ((0 + X[i][0] Y[0][j]) + X[i][1] Y[1][j]) + ...:
//   forward: temp = input * T (T = ctx->transposed_dct, :61), out = D * temp (:72)
//   inverse: temp = T * input (:89),                    out = temp * D (:100)
// with D = ctx->dct_matrix -- the two PUBLIC tables exactly as the caller holds
// them (a caller may have edited either).  Separate multiply and add (this file
// is compiled with -ffp-contract=off), k ascending, accumulators from +0.0.
__device__ __forceinline__ double dot_ordered(const double *x, const double *y, int n, int i, int j) {
    double acc = 0.0;
    for (int k = 0; k < n; ++k) acc += x[i * n + k] * y[k * n + j];
    return acc;
}

// One-workgroup kernels end by writing `seq` to the calling lane's done flag in
// pinned host memory, after every output of the workgroup has reached the host
// (each thread's system-scope fence, then the barrier): the calling thread spins
// on that flag instead of a stream synchronize (finish()).  The flag address goes
// through a VGPR so the store is a vector store.
__device__ __forceinline__ void signal_done(uint32_t *done, uint32_t seq) {
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) {
        asm volatile("" : "+v"(done));
        __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Small blocks (4 n^2 doubles <= kLdsBytes: n <= 32, the codec's n = 8): ONE
// workgroup per call, its D, T and input staged in LDS from the pinned zero-copy
// buffer in one parallel round trip over the host link, the result written
// straight back to it.
constexpr int kLdsBytes = 32 * 1024;
template <bool FWD>
__device__ __forceinline__ void transform_body(int n, const double *__restrict__ dh, const double *__restrict__ th,
                                               const double *__restrict__ inh, double *__restrict__ out, double *lds) {
    const int nn = n * n;
    double *d = lds, *t = lds + nn, *in = lds + 2 * nn, *tmp = lds + 3 * nn;
    for (int e = threadIdx.x; e < nn; e += blockDim.x) {
        d[e] = dh[e];
        t[e] = th[e];
        in[e] = inh[e];
    }
    __syncthreads();
    for (int e = threadIdx.x; e < nn; e += blockDim.x)
        tmp[e] = FWD ? dot_ordered(in, t, n, e / n, e % n) : dot_ordered(t, in, n, e / n, e % n);
    __syncthreads();
    for (int e = threadIdx.x; e < nn; e += blockDim.x)
        out[e] = FWD ? dot_ordered(d, tmp, n, e / n, e % n) : dot_ordered(tmp, d, n, e / n, e % n);
}

template <bool FWD>
__global__ void k_transform_small(int n, const double *__restrict__ dh, const double *__restrict__ th,
                                  const double *__restrict__ inh, double *__restrict__ out, uint32_t *done,
                                  uint32_t seq) {
    extern __shared__ double lds[];
    transform_body<FWD>(n, dh, th, inh, out, lds);
    signal_done(done, seq);
}

// n == 8, the codec's block (round 6): the 64-value inputs travel as kernel
// arguments, which the runtime writes into device memory with the dispatch, so the
// kernel reads them without a round trip over the host link; only the outputs and
// the done flag cross it (posted writes).
struct Vals64 {
    double v[64];
};
struct Ints64 {
    int v[64];
};
template <bool FWD>
__global__ void k_transform8(Vals64 d, Vals64 t, Vals64 in, double *__restrict__ out, uint32_t *done, uint32_t seq) {
    __shared__ double lds[4 * 64];
    transform_body<FWD>(8, d.v, t.v, in.v, out, lds);
    signal_done(done, seq);
}

// Any n (the reference takes any block size, src/dct.c:7-40): the packed
// tables and input are copied to device memory once, each pass is its own
// launch over all n^2 elements, one element per thread.
__global__ void k_pass(int n, const double *__restrict__ x, const double *__restrict__ y, double *__restrict__ z) {
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < (long long)n * n) z[e] = dot_ordered(x, y, n, (int)(e / n), (int)(e % n));
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
__device__ __forceinline__ void elementwise_one(int mode, int e, const double *__restrict__ m, int adaptive,
                                                double variance, const double *__restrict__ din,
                                                const int *__restrict__ iin, double *__restrict__ dout,
                                                int *__restrict__ iout) {
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

__global__ void k_elementwise(int mode, int nn, const double *__restrict__ m, int adaptive, double variance,
                              const double *__restrict__ din, const int *__restrict__ iin, double *__restrict__ dout,
                              int *__restrict__ iout, uint32_t *done, uint32_t seq) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < nn) elementwise_one(mode, e, m, adaptive, variance, din, iin, dout, iout);
    if (done) signal_done(done, seq);  // one-workgroup launches only (n <= 16)
}

__global__ void k_elementwise8(int mode, int adaptive, double variance, Vals64 m, Vals64 din, Ints64 iin,
                               double *__restrict__ dout, int *__restrict__ iout, uint32_t *done, uint32_t seq) {
    if (threadIdx.x < 64) elementwise_one(mode, threadIdx.x, m.v, adaptive, variance, din.v, iin.v, dout, iout);
    signal_done(done, seq);
}

// src/quantization.c:153-169 -- sequential row-major sums (order matters for
// non-integer input), one thread; small blocks first copied from the zero-copy
// buffer into LDS by the whole workgroup (one parallel round trip over the
// host link), large ones read from device scratch.
__device__ __forceinline__ void variance_body(int nn, const double *__restrict__ xh, double *__restrict__ out,
                                              double *x) {
    for (int e = threadIdx.x; e < nn; e += blockDim.x) x[e] = xh[e];
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = 0.0, s2 = 0.0;
        for (int k = 0; k < nn; ++k) {
            s += x[k];
            s2 += x[k] * x[k];
        }
        const double mean = s / nn;
        out[0] = (s2 / nn) - (mean * mean);
    }
}

__global__ void k_variance_small(int nn, const double *__restrict__ xh, double *__restrict__ out, uint32_t *done,
                                 uint32_t seq) {
    extern __shared__ double x[];
    variance_body(nn, xh, out, x);
    signal_done(done, seq);
}

__global__ void k_variance8(Vals64 xv, double *__restrict__ out, uint32_t *done, uint32_t seq) {
    __shared__ double x[64];
    variance_body(64, xv.v, out, x);
    signal_done(done, seq);
}

__global__ void k_variance(int nn, const double *__restrict__ x, double *__restrict__ out) {
    double s = 0.0, s2 = 0.0;
    for (int k = 0; k < nn; ++k) {
        s += x[k];
        s2 += x[k] * x[k];
    }
    const double mean = s / nn;
    out[0] = (s2 / nn) - (mean * mean);
}

// ---------------------------------------------------------------- lanes
// The reference API is reentrant and keeps no mutable global state (its only
// static, src/quantization.c:8, is const; SURVEY 8(b) ran 8 pthreads over one
// context), so calls from different host threads must overlap here too.  Each
// thread gets one LANE per device: its own non-blocking stream, a pinned,
// device-mapped staging buffer (zero-copy: a call packs its row-pointer arrays
// into it, the kernel reads its inputs from it and writes its outputs back into
// it over the host link -- no memcpy calls), a done flag in pinned coherent host
// memory (finish_signalled) and, for large blocks, a device scratch buffer.  No
// lock is held in
// steady state: only a thread's FIRST call on a device (it creates the lane's
// stream and launches on it first, which is where libhsa may call srand/rand)
// and a buffer's growth (a HIP allocation) take the rand isolation lock
// (dctq_internal.h), like the batched entry points' first calls.
//
// Lanes are never freed: a thread that exits hands its lanes to a pool (no HIP
// call runs in a thread-exit destructor) and the next thread that needs a lane
// on that device takes it, so a host that keeps spawning threads holds at most
// as many lanes as it ever had threads alive at once.
constexpr size_t kStageMin = 64 * 1024;  // every n <= 32 call fits without growing
struct Lane {
    int device = -1;
    hipStream_t stream = nullptr;
    unsigned char *host = nullptr;  // pinned host memory
    unsigned char *hdev = nullptr;  // the same pages as seen by the device
    size_t host_bytes = 0;
    unsigned char *scratch = nullptr;
    size_t scratch_bytes = 0;
    uint32_t *done_host = nullptr;  // the one-workgroup kernels' completion flag (signal_done)
    uint32_t *done_dev = nullptr;
    uint32_t seq = 0;               // the value the next call's kernel writes there
    uint32_t since_sync = 0;        // calls since the lane's stream was last synchronized
    unsigned char *stage(size_t need) {
        if (need > host_bytes) {
            DCTQ_ENTRY;  // an allocation: may reach the runtime's rand()
            if (host) (void)hipHostFree(host);
            host = nullptr;
            const size_t bytes = need > kStageMin ? need : kStageMin;
            // coherent: the kernel's outputs reach host memory before its done flag does
            LCHK(hipHostMalloc((void **)&host, bytes, hipHostMallocMapped | hipHostMallocCoherent),
                 "hipHostMalloc(legacy staging)");
            LCHK(hipHostGetDevicePointer((void **)&hdev, host, 0), "hipHostGetDevicePointer");
            host_bytes = bytes;
        }
        return host;
    }
    unsigned char *dscratch(size_t need) {
        if (need > scratch_bytes) {
            DCTQ_ENTRY;
            if (scratch) (void)hipFree(scratch);
            scratch = nullptr;
            LCHK(hipMalloc((void **)&scratch, need), "hipMalloc(legacy scratch)");
            scratch_bytes = need;
        }
        return scratch;
    }
};

__global__ void k_nop() {}

std::mutex g_pool_mu;
std::vector<Lane *> g_pool;        // lanes of threads that have exited
std::atomic<int> g_lanes_made{0};  // lanes ever created (diagnostics: dctq_diag_legacy_lanes)

struct ThreadLanes {
    std::vector<Lane *> lanes;
    ~ThreadLanes() {
        std::lock_guard<std::mutex> g(g_pool_mu);
        for (Lane *l : lanes) g_pool.push_back(l);
    }
};
thread_local ThreadLanes t_lanes;

// This thread's lane on the current device, made (or taken from the pool) on
// its first call there.
Lane &lane() {
    std::optional<dctq::RandIsolation> iso;
    if (!dctq::runtime_started()) iso.emplace();  // this hipGetDevice may initialise the runtime
    int d = 0;
    LCHK(hipGetDevice(&d), "hipGetDevice");
    dctq::note_runtime_started();
    for (Lane *l : t_lanes.lanes)
        if (l->device == d) return *l;
    if (!iso) iso.emplace();
    Lane *l = nullptr;
    {
        std::lock_guard<std::mutex> g(g_pool_mu);
        for (size_t i = 0; i < g_pool.size(); ++i)
            if (g_pool[i]->device == d) {
                l = g_pool[i];
                g_pool.erase(g_pool.begin() + (long)i);
                break;
            }
    }
    if (!l) {
        l = new Lane();
        l->device = d;
        g_lanes_made.fetch_add(1, std::memory_order_relaxed);
        LCHK(hipStreamCreateWithFlags(&l->stream, hipStreamNonBlocking), "hipStreamCreateWithFlags(legacy lane)");
        (void)l->stage(kStageMin);
        LCHK(hipHostMalloc((void **)&l->done_host, 64, hipHostMallocMapped | hipHostMallocCoherent),
             "hipHostMalloc(legacy done flag)");
        LCHK(hipHostGetDevicePointer((void **)&l->done_dev, l->done_host, 0), "hipHostGetDevicePointer");
        __atomic_store_n(l->done_host, 0u, __ATOMIC_RELEASE);
        hipLaunchKernelGGL(k_nop, dim3(1), dim3(64), 0, l->stream);  // the stream's first queue, under isolation
        LCHK(hipGetLastError(), "legacy lane launch");
        LCHK(hipStreamSynchronize(l->stream), "hipStreamSynchronize");
    }
    t_lanes.lanes.push_back(l);
    return *l;
}

void finish(const Lane &ln, const char *what) {
    LCHK(hipGetLastError(), what);
    LCHK(hipStreamSynchronize(ln.stream), "hipStreamSynchronize");
}

// The call's one-workgroup kernel writes ln.seq to the done flag after its outputs
// (signal_done): the calling thread spins on the flag over the host link instead of
// a stream synchronize.  Fallbacks: past 50 ms of spinning (a slow device, or a
// launch that failed without an error code) the stream is synchronized and the flag
// must then be there; and every 1024 calls the stream is synchronized anyway, so the
// runtime retires the lane's launches.
void finish_signalled(Lane &ln, const char *what) {
    LCHK(hipGetLastError(), what);
    const uint32_t want = ln.seq;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 0; __atomic_load_n(ln.done_host, __ATOMIC_ACQUIRE) != want; ++i) {
        if ((i & 1023u) == 1023u && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(50)) {
            LCHK(hipStreamSynchronize(ln.stream), "hipStreamSynchronize");
            if (__atomic_load_n(ln.done_host, __ATOMIC_ACQUIRE) != want) die("legacy kernel finished without signalling");
            break;
        }
        __builtin_ia32_pause();
    }
    if (++ln.since_sync >= 1024u) {
        ln.since_sync = 0;
        LCHK(hipStreamSynchronize(ln.stream), "hipStreamSynchronize");
    }
}

void pack(double **a, int n, double *dst) {
    for (int i = 0; i < n; ++i) memcpy(dst + (size_t)i * n, a[i], sizeof(double) * n);
}
void unpack(const double *src, int n, double **a) {
    for (int i = 0; i < n; ++i) memcpy(a[i], src + (size_t)i * n, sizeof(double) * n);
}

void check_n(int n) {
    if (n < 1 || n > 46340) die("block_size out of the supported range 1..46340");  // n^2 fits an int
}

void transform(DCTContext *ctx, double **input, double **output, bool fwd) {
    const int n = ctx->block_size;
    check_n(n);
    const size_t nn = (size_t)n * n;
    Lane &ln = lane();
    if (n == 8) {
        Vals64 d, t, in;
        pack(ctx->dct_matrix, 8, d.v);
        pack(ctx->transposed_dct, 8, t.v);
        pack(input, 8, in.v);
        double *h = (double *)ln.stage(sizeof(double) * 64);
        if (fwd)
            hipLaunchKernelGGL(k_transform8<true>, dim3(1), dim3(64), 0, ln.stream, d, t, in, (double *)ln.hdev,
                               ln.done_dev, ++ln.seq);
        else
            hipLaunchKernelGGL(k_transform8<false>, dim3(1), dim3(64), 0, ln.stream, d, t, in, (double *)ln.hdev,
                               ln.done_dev, ++ln.seq);
        finish_signalled(ln, "transform launch");
        unpack(h, 8, output);
        return;
    }
    if (4 * nn * sizeof(double) <= (size_t)kLdsBytes) {
        double *h = (double *)ln.stage(sizeof(double) * 4 * nn);
        const double *dv = (const double *)ln.hdev;
        pack(ctx->dct_matrix, n, h);
        pack(ctx->transposed_dct, n, h + nn);
        pack(input, n, h + 2 * nn);
        const int threads = nn < 256 ? (int)((nn + 63) / 64) * 64 : 256;
        const size_t lds = sizeof(double) * 4 * nn;
        if (fwd)
            hipLaunchKernelGGL(k_transform_small<true>, dim3(1), dim3(threads), lds, ln.stream, n, dv, dv + nn,
                               dv + 2 * nn, (double *)dv + 3 * nn, ln.done_dev, ++ln.seq);
        else
            hipLaunchKernelGGL(k_transform_small<false>, dim3(1), dim3(threads), lds, ln.stream, n, dv, dv + nn,
                               dv + 2 * nn, (double *)dv + 3 * nn, ln.done_dev, ++ln.seq);
        finish_signalled(ln, "transform launch");
        unpack(h + 3 * nn, n, output);
        return;
    }
    // any n: D | T | input | temp | output in device scratch
    std::vector<double> h(3 * nn);
    pack(ctx->dct_matrix, n, h.data());
    pack(ctx->transposed_dct, n, h.data() + nn);
    pack(input, n, h.data() + 2 * nn);
    double *d = (double *)ln.dscratch(sizeof(double) * 5 * nn), *t = d + nn, *in = d + 2 * nn, *tmp = d + 3 * nn,
           *out = d + 4 * nn;
    LCHK(hipMemcpyAsync(d, h.data(), sizeof(double) * 3 * nn, hipMemcpyHostToDevice, ln.stream),
         "hipMemcpy(legacy transform in)");
    const unsigned grid = (unsigned)((nn + 255) / 256);
    if (fwd) {
        hipLaunchKernelGGL(k_pass, dim3(grid), dim3(256), 0, ln.stream, n, in, t, tmp);
        hipLaunchKernelGGL(k_pass, dim3(grid), dim3(256), 0, ln.stream, n, d, tmp, out);
    } else {
        hipLaunchKernelGGL(k_pass, dim3(grid), dim3(256), 0, ln.stream, n, t, in, tmp);
        hipLaunchKernelGGL(k_pass, dim3(grid), dim3(256), 0, ln.stream, n, tmp, d, out);
    }
    LCHK(hipGetLastError(), "transform launch");
    LCHK(hipMemcpyAsync(h.data(), out, sizeof(double) * nn, hipMemcpyDeviceToHost, ln.stream),
         "hipMemcpy(legacy transform out)");
    LCHK(hipStreamSynchronize(ln.stream), "hipStreamSynchronize");
    unpack(h.data(), n, output);
}

// One elementwise launch over an n x n block; inputs/outputs as flat host arrays.
void elementwise(int mode, int n, double **m, int flag, double variance, const double *din, const int *iin,
                 double *dout, int *iout) {
    const int nn = n * n;
    const size_t bytes = sizeof(double) * 3 * (size_t)nn + sizeof(int) * 2 * (size_t)nn;
    Lane &ln = lane();
    if (n == 8) {
        Vals64 mv, dv{};
        Ints64 iv{};
        pack(m, 8, mv.v);
        if (din) memcpy(dv.v, din, sizeof dv.v);
        if (iin) memcpy(iv.v, iin, sizeof iv.v);
        unsigned char *h = ln.stage(sizeof(double) * 64 + sizeof(int) * 64);
        double *ddo = (double *)ln.hdev;
        int *dio = (int *)(ddo + 64);
        hipLaunchKernelGGL(k_elementwise8, dim3(1), dim3(64), 0, ln.stream, mode, flag, variance, mv, dv, iv, ddo, dio,
                           ln.done_dev, ++ln.seq);
        finish_signalled(ln, "elementwise launch");
        if (dout) memcpy(dout, h, sizeof(double) * 64);
        if (iout) memcpy(iout, h + sizeof(double) * 64, sizeof(int) * 64);
        return;
    }
    unsigned char *h = ln.stage(bytes);
    double *hm = (double *)h, *hd = hm + nn;
    int *hi = (int *)(hd + 2 * nn);
    pack(m, n, hm);
    if (din) memcpy(hd, din, sizeof(double) * nn);
    if (iin) memcpy(hi, iin, sizeof(int) * nn);
    double *dm = (double *)ln.hdev, *dd = dm + nn, *ddo = dd + nn;
    int *di = (int *)(ddo + nn), *dio = di + nn;
    const unsigned grid = (unsigned)((nn + 255) / 256);
    const bool one = grid == 1;  // n <= 16: one workgroup, which signals its own completion
    hipLaunchKernelGGL(k_elementwise, dim3(grid), dim3(256), 0, ln.stream, mode, nn, dm, flag, variance, dd, di, ddo,
                       dio, one ? ln.done_dev : nullptr, one ? ++ln.seq : 0u);
    if (one)
        finish_signalled(ln, "elementwise launch");
    else
        finish(ln, "elementwise launch");
    if (dout) memcpy(dout, (double *)h + 2 * nn, sizeof(double) * nn);
    if (iout) memcpy(iout, (int *)((double *)h + 3 * nn) + nn, sizeof(int) * nn);
}

}  // namespace

// Lanes created so far and lanes waiting in the pool (threads that exited), for the
// diagnostic library's dctq_diag_legacy_lanes (tests: a host that keeps spawning
// threads holds at most as many lanes as it had threads alive at once).
void dctq::legacy_lane_counts(int *made, int *pooled) {
    *made = g_lanes_made.load(std::memory_order_relaxed);
    std::lock_guard<std::mutex> g(g_pool_mu);
    *pooled = (int)g_pool.size();
}

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
    check_n(block_size);
    const size_t nn = (size_t)block_size * block_size;
    Lane &ln = lane();
    if (block_size == 8) {
        Vals64 xv;
        pack(block, 8, xv.v);
        double *hs = (double *)ln.stage(sizeof(double));
        hipLaunchKernelGGL(k_variance8, dim3(1), dim3(64), 0, ln.stream, xv, (double *)ln.hdev, ln.done_dev, ++ln.seq);
        finish_signalled(ln, "variance launch");
        return hs[0];
    }
    if (nn * sizeof(double) <= (size_t)kLdsBytes) {
        double *hs = (double *)ln.stage(sizeof(double) * (nn + 1));
        double *dv = (double *)ln.hdev;
        pack(block, block_size, hs);
        const int threads = nn < 256 ? (int)((nn + 63) / 64) * 64 : 256;
        hipLaunchKernelGGL(k_variance_small, dim3(1), dim3(threads), sizeof(double) * nn, ln.stream, (int)nn, dv,
                           dv + nn, ln.done_dev, ++ln.seq);
        finish_signalled(ln, "variance launch");
        return hs[nn];
    }
    std::vector<double> h(nn + 1);
    pack(block, block_size, h.data());
    double *dv = (double *)ln.dscratch(sizeof(double) * (nn + 1));
    LCHK(hipMemcpyAsync(dv, h.data(), sizeof(double) * nn, hipMemcpyHostToDevice, ln.stream),
         "hipMemcpy(variance in)");
    hipLaunchKernelGGL(k_variance, dim3(1), dim3(1), 0, ln.stream, (int)nn, dv, dv + nn);
    LCHK(hipGetLastError(), "variance launch");
    LCHK(hipMemcpyAsync(h.data() + nn, dv + nn, sizeof(double), hipMemcpyDeviceToHost, ln.stream),
         "hipMemcpy(variance out)");
    LCHK(hipStreamSynchronize(ln.stream), "hipStreamSynchronize");
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
