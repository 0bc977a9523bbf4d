// tools/ubench/hbm_mix.hip -- hardware ceilings for the forward kernel's traffic
// (64 B read : 128 B written per block), independent of the kernel's own access
// pattern:
//   copy  : the guide's float4 copy (MI355X_MICROARCH.md: 6.29 TB/s = 79 %), 1:1
//   read  : read-only stream;  write : write-only stream
//   s12   : flat 1:2 stream, per wave 4 KiB in (4 x 1 KiB loads) and 8 KiB out
//           (8 x 1 KiB stores), one wave-batch per wave (non-persistent grid) or a
//           persistent grid-stride loop
//   rows  : the forward kernel's movement: lane-per-block 8 x 8-B pixel-row loads
//           of a 4K plane stack, LDS stage, 8 x 1 KiB stores per 64-block batch,
//           non-persistent or persistent
// Each variant with plain / non-temporal loads and stores.  96 4K luma planes =
// 12 441 600 blocks = the bench step's block count (796 MB in, 1.59 GB out).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench/hbm_mix tools/ubench/hbm_mix.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <vector>
#include <functional>

typedef unsigned int u2v __attribute__((ext_vector_type(2)));
typedef unsigned int u4v __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

template <int NT>
__device__ __forceinline__ u4v ld16(const u4v *p) {
    if (NT) return __builtin_nontemporal_load(p);
    return *p;
}
template <int NT>
__device__ __forceinline__ void st16(u4v *p, u4v v) {
    if (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// ---- float4 copy: each thread U uint4, coalesced (stride = blockDim)
template <int LN, int SN, int U>
__global__ __launch_bounds__(256) void k_copy(const u4v *__restrict__ in, u4v *__restrict__ out, size_t n16) {
    const size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x;
    u4v v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = base + u * 256 < n16 ? ld16<LN>(in + base + u * 256) : u4v{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (base + u * 256 < n16) st16<SN>(out + base + u * 256, v[u]);
}

template <int LN, int U>
__global__ __launch_bounds__(256) void k_read(const u4v *__restrict__ in, u4v *__restrict__ out, size_t n16) {
    const size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x;
    u4v acc = {0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (base + u * 256 < n16) acc ^= ld16<LN>(in + base + u * 256);
    if (acc.x == 0x12345678u && acc.y == 0x9abcdef0u) out[base] = acc;
}

template <int SN, int U>
__global__ __launch_bounds__(256) void k_write(u4v *__restrict__ out, size_t n16) {
    const size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (base + u * 256 < n16) st16<SN>(out + base + u * 256, u4v{(unsigned)base, (unsigned)u, 7u, 9u});
}

// ---- flat 1:2: wave-batch b reads in[b*4K .. +4K) and writes out[b*8K .. +8K)
template <int LN, int SN>
__device__ __forceinline__ void s12_batch(const u4v *__restrict__ in, u4v *__restrict__ out, uint32_t b, int lane) {
    u4v v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = ld16<LN>(in + (size_t)b * 256 + k * 64 + lane);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        st16<SN>(out + (size_t)b * 512 + k * 64 + lane, v[k]);
        st16<SN>(out + (size_t)b * 512 + (k + 4) * 64 + lane, v[k] ^ u4v{1, 0, 0, 0});
    }
}
template <int LN, int SN>
__global__ __launch_bounds__(256) void k_s12_np(const u4v *__restrict__ in, u4v *__restrict__ out, uint32_t nb) {
    const uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b < nb) s12_batch<LN, SN>(in, out, b, threadIdx.x & 63);
}
template <int LN, int SN>
__global__ __launch_bounds__(256) void k_s12_ps(const u4v *__restrict__ in, u4v *__restrict__ out, uint32_t nb) {
    for (uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6); b < nb; b += gridDim.x * 4)
        s12_batch<LN, SN>(in, out, b, threadIdx.x & 63);
}

// ---- the forward kernel's movement (rows of a W x H plane stack, 64-block batches)
struct Geo {
    const uint8_t *src;
    uint32_t bw, per_frame;
    uint32_t stride;
    size_t fstride;
};
template <int LN, int SN>
__device__ __forceinline__ void rows_batch(const Geo &g, char *coef, uint32_t b, int lane, char *ws) {
    const uint32_t n = b * 64 + lane;
    const uint32_t f = n / g.per_frame, rem = n - f * g.per_frame, by = rem / g.bw, bx = rem - by * g.bw;
    const uint8_t *p = g.src + f * g.fstride + (size_t)by * 8 * g.stride + bx * 8;
    uint2 r[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        if (LN) {
            const u2v t = __builtin_nontemporal_load((const u2v *)(p + k * g.stride));
            r[k] = make_uint2(t.x, t.y);
        } else {
            r[k] = *(const uint2 *)(p + k * g.stride);
        }
    }
    uint2 *mine = reinterpret_cast<uint2 *>(ws + lane * 136);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        mine[2 * k] = r[k];
        mine[2 * k + 1] = make_uint2(r[k].x ^ 1, r[k].y);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // stores retired before the stage is re-read (see DESIGN)
    __builtin_amdgcn_wave_barrier();
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(coef + (size_t)b * 8192, 0, 8192, 0x00020000);
    u4v val[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int m = k * 64 + lane, bl = m >> 3;
        const uint2 *s2 = reinterpret_cast<const uint2 *>(ws + bl * 136 + (m & 7) * 16);
        val[k] = u4v{s2[0].x, s2[0].y, s2[1].x, s2[1].y};
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) __builtin_amdgcn_raw_buffer_store_b128(val[k], rc, lane * 16, k * 1024, SN ? 2 : 0);
}
template <int LN, int SN>
__global__ __launch_bounds__(256) void k_rows_np(Geo g, char *coef, uint32_t nb) {
    __shared__ uint4 st[256 * 136 / 16];
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t b = blockIdx.x * 4 + wv;
    if (b < nb) rows_batch<LN, SN>(g, coef, b, threadIdx.x & 63, reinterpret_cast<char *>(st) + wv * 8704);
}
template <int LN, int SN>
__global__ __launch_bounds__(256) void k_rows_ps(Geo g, char *coef, uint32_t nb) {
    __shared__ uint4 st[256 * 136 / 16];
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint32_t b = blockIdx.x * 4 + wv; b < nb; b += gridDim.x * 4)
        rows_batch<LN, SN>(g, coef, b, threadIdx.x & 63, reinterpret_cast<char *>(st) + wv * 8704);
}

struct Case {
    const char *name;
    double bytes;
    std::vector<float> ms;
};

int main(int argc, char **argv) {
    const int passes = argc > 1 ? atoi(argv[1]) : 2;
    const uint32_t W = 3840, H = 2160, F = 96;
    const uint32_t bw = W / 8, per = bw * (H / 8);
    const size_t nblk = (size_t)per * F;  // 12 441 600
    const uint32_t nb = (uint32_t)(nblk / 64);
    const size_t in_bytes = nblk * 64, out_bytes = nblk * 128;
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint8_t *src;
    char *dst;
    CHECK(hipMalloc(&src, in_bytes));
    CHECK(hipMalloc(&dst, out_bytes));
    CHECK(hipMemset(src, 7, in_bytes));
    CHECK(hipMemset(dst, 0, out_bytes));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    printf("CUs %d, %zu blocks, in %.1f MB, out %.1f MB\n", cus, nblk, in_bytes / 1e6, out_bytes / 1e6);

    const u4v *in16 = (const u4v *)src;
    u4v *out16 = (u4v *)dst;
    const size_t n16_in = in_bytes / 16, n16_out = out_bytes / 16;
    Geo g{src, bw, per, W, (size_t)W * H};
    const int G4 = cus * 4;  // persistent grid: 4 WGs (16 waves) per CU
    const double b12 = (double)nblk * 192;

    struct Item {
        const char *name;
        double bytes;
        std::function<void()> fn;
    };
    std::vector<Item> items = {
        {"copy  plain/plain U1 (guide float4 copy)", 2.0 * in_bytes,
         [&] { hipLaunchKernelGGL((k_copy<0, 0, 1>), dim3((n16_in + 255) / 256), dim3(256), 0, 0, in16, out16, n16_in); }},
        {"copy  plain/plain U4", 2.0 * in_bytes,
         [&] { hipLaunchKernelGGL((k_copy<0, 0, 4>), dim3((n16_in + 1023) / 1024), dim3(256), 0, 0, in16, out16, n16_in); }},
        {"copy  nt/nt U4", 2.0 * in_bytes,
         [&] { hipLaunchKernelGGL((k_copy<1, 1, 4>), dim3((n16_in + 1023) / 1024), dim3(256), 0, 0, in16, out16, n16_in); }},
        {"read  plain U4 (out-size buffer)", (double)out_bytes,
         [&] { hipLaunchKernelGGL((k_read<0, 4>), dim3((n16_out + 1023) / 1024), dim3(256), 0, 0, (const u4v *)dst, out16, n16_out); }},
        {"read  nt U4", (double)out_bytes,
         [&] { hipLaunchKernelGGL((k_read<1, 4>), dim3((n16_out + 1023) / 1024), dim3(256), 0, 0, (const u4v *)dst, out16, n16_out); }},
        {"write plain U4", (double)out_bytes,
         [&] { hipLaunchKernelGGL((k_write<0, 4>), dim3((n16_out + 1023) / 1024), dim3(256), 0, 0, out16, n16_out); }},
        {"write nt U4", (double)out_bytes,
         [&] { hipLaunchKernelGGL((k_write<1, 4>), dim3((n16_out + 1023) / 1024), dim3(256), 0, 0, out16, n16_out); }},
        {"s12   plain/plain non-persistent", b12,
         [&] { hipLaunchKernelGGL((k_s12_np<0, 0>), dim3((nb + 3) / 4), dim3(256), 0, 0, in16, out16, nb); }},
        {"s12   nt/plain non-persistent", b12,
         [&] { hipLaunchKernelGGL((k_s12_np<1, 0>), dim3((nb + 3) / 4), dim3(256), 0, 0, in16, out16, nb); }},
        {"s12   plain/nt non-persistent", b12,
         [&] { hipLaunchKernelGGL((k_s12_np<0, 1>), dim3((nb + 3) / 4), dim3(256), 0, 0, in16, out16, nb); }},
        {"s12   nt/nt non-persistent", b12,
         [&] { hipLaunchKernelGGL((k_s12_np<1, 1>), dim3((nb + 3) / 4), dim3(256), 0, 0, in16, out16, nb); }},
        {"s12   plain/plain persistent 4 WG/CU", b12,
         [&] { hipLaunchKernelGGL((k_s12_ps<0, 0>), dim3(G4), dim3(256), 0, 0, in16, out16, nb); }},
        {"s12   nt/nt persistent 4 WG/CU", b12,
         [&] { hipLaunchKernelGGL((k_s12_ps<1, 1>), dim3(G4), dim3(256), 0, 0, in16, out16, nb); }},
        {"rows  plain/plain non-persistent", b12,
         [&] { hipLaunchKernelGGL((k_rows_np<0, 0>), dim3((nb + 3) / 4), dim3(256), 0, 0, g, dst, nb); }},
        {"rows  nt/plain non-persistent", b12,
         [&] { hipLaunchKernelGGL((k_rows_np<1, 0>), dim3((nb + 3) / 4), dim3(256), 0, 0, g, dst, nb); }},
        {"rows  nt/nt non-persistent", b12,
         [&] { hipLaunchKernelGGL((k_rows_np<1, 1>), dim3((nb + 3) / 4), dim3(256), 0, 0, g, dst, nb); }},
        {"rows  plain/plain persistent", b12,
         [&] { hipLaunchKernelGGL((k_rows_ps<0, 0>), dim3(G4), dim3(256), 0, 0, g, dst, nb); }},
        {"rows  nt/plain persistent", b12,
         [&] { hipLaunchKernelGGL((k_rows_ps<1, 0>), dim3(G4), dim3(256), 0, 0, g, dst, nb); }},
        {"rows  nt/nt persistent (= v2 movement)", b12,
         [&] { hipLaunchKernelGGL((k_rows_ps<1, 1>), dim3(G4), dim3(256), 0, 0, g, dst, nb); }},
    };
    std::vector<std::vector<float>> ms(items.size());
    for (auto &it : items) it.fn();
    CHECK(hipDeviceSynchronize());
    for (int p = 0; p < passes; ++p)
        for (size_t i = 0; i < items.size(); ++i)
            for (int r = 0; r < 5; ++r) {
                CHECK(hipEventRecord(e0));
                items[i].fn();
                CHECK(hipEventRecord(e1));
                CHECK(hipEventSynchronize(e1));
                float t;
                CHECK(hipEventElapsedTime(&t, e0, e1));
                ms[i].push_back(t);
            }
    CHECK(hipGetLastError());
    for (size_t i = 0; i < items.size(); ++i) {
        std::vector<float> v = ms[i];
        std::sort(v.begin(), v.end());
        const double med = v[v.size() / 2], best = v[0];
        printf("%-44s median %8.1f us  %6.0f GB/s %5.1f %%   best %5.1f %%\n", items[i].name, med * 1e3,
               items[i].bytes / med / 1e6, items[i].bytes / med / 1e6 / 80.0, items[i].bytes / best / 1e6 / 80.0);
    }
    return 0;
}
