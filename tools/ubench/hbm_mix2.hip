// tools/ubench/hbm_mix2.hip -- is the 1:2 read:write mix's ~70 % of 8 TB/s a
// property of the mix itself?  Same byte counts as the bench step (796 MB read,
// 1.59 GB written), all samples printed (sorted), these forms:
//   phased    : a read-only kernel over the input, then a write-only kernel over
//               the output, inside one event pair (mixing at kernel granularity)
//   s12 WGk   : flat 1:2 stream (4 KiB in, 8 KiB out per wave-batch), persistent
//               grid of k workgroups (4 waves) per CU
//   s12 Rr    : r consecutive wave-batches per iteration: r*4 KiB loaded, then
//               r*8 KiB stored
//   s12 cont  : each wave sweeps ONE contiguous run of batches (in-flight window
//               spread over the whole buffers instead of a compact front)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench/hbm_mix2 tools/ubench/hbm_mix2.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <functional>
#include <vector>

typedef unsigned int u4v __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

__global__ __launch_bounds__(256) void k_read(const u4v *__restrict__ in, u4v *__restrict__ out, size_t n16) {
    const size_t base = (size_t)blockIdx.x * 1024 + threadIdx.x;
    u4v acc = {0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < 4; ++u)
        if (base + u * 256 < n16) acc ^= __builtin_nontemporal_load(in + base + u * 256);
    if (acc.x == 0x12345678u && acc.y == 0x9abcdef0u) out[base] = acc;
}

__global__ __launch_bounds__(256) void k_write(u4v *__restrict__ out, size_t n16) {
    const size_t base = (size_t)blockIdx.x * 1024 + threadIdx.x;
#pragma unroll
    for (int u = 0; u < 4; ++u)
        if (base + u * 256 < n16) out[base + u * 256] = u4v{(unsigned)base, (unsigned)u, 7u, 9u};
}

template <int R, int SN>
__device__ __forceinline__ void s12_run(const u4v *__restrict__ in, u4v *__restrict__ out, uint32_t b, uint32_t nb,
                                        int lane) {
    u4v v[R][4];
#pragma unroll
    for (int j = 0; j < R; ++j)
#pragma unroll
        for (int k = 0; k < 4; ++k)
            v[j][k] = b + j < nb ? __builtin_nontemporal_load(in + (size_t)(b + j) * 256 + k * 64 + lane) : u4v{0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < R; ++j)
        if (b + j < nb)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                u4v *o = out + (size_t)(b + j) * 512 + k * 64 + lane;
                if (SN) {
                    __builtin_nontemporal_store(v[j][k], o);
                    __builtin_nontemporal_store(v[j][k] ^ u4v{1, 0, 0, 0}, o + 256);
                } else {
                    o[0] = v[j][k];
                    o[256] = v[j][k] ^ u4v{1, 0, 0, 0};
                }
            }
}

// grid-stride over groups of R batches
template <int R, int SN>
__global__ __launch_bounds__(256) void k_s12(const u4v *__restrict__ in, u4v *__restrict__ out, uint32_t nb) {
    const int lane = threadIdx.x & 63;
    for (uint32_t b = (blockIdx.x * 4 + (threadIdx.x >> 6)) * R; b < nb; b += gridDim.x * 4 * R)
        s12_run<R, SN>(in, out, b, nb, lane);
}

// each wave one contiguous run of batches
__global__ __launch_bounds__(256) void k_s12_cont(const u4v *__restrict__ in, u4v *__restrict__ out, uint32_t nb) {
    const int lane = threadIdx.x & 63;
    const uint32_t tw = gridDim.x * 4, w = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t per = (nb + tw - 1) / tw;
    for (uint32_t i = 0; i < per; ++i) {
        const uint32_t b = w * per + i;
        if (b < nb) s12_run<1, 1>(in, out, b, nb, lane);
    }
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 8;
    const size_t nblk = 12441600;
    const uint32_t nb = (uint32_t)(nblk / 64);
    const size_t in_bytes = nblk * 64, out_bytes = nblk * 128;
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    char *src, *dst;
    CHECK(hipMalloc(&src, in_bytes));
    CHECK(hipMalloc(&dst, out_bytes));
    CHECK(hipMemset(src, 7, in_bytes));
    CHECK(hipMemset(dst, 0, out_bytes));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const u4v *in16 = (const u4v *)src;
    u4v *out16 = (u4v *)dst;
    const size_t n16_in = in_bytes / 16, n16_out = out_bytes / 16;
    const double b12 = (double)nblk * 192;
    struct Item {
        const char *name;
        double bytes;
        std::function<void()> fn;
    };
    std::vector<Item> items = {
        {"phased: read kernel then write kernel", b12,
         [&] {
             hipLaunchKernelGGL(k_read, dim3((n16_in + 1023) / 1024), dim3(256), 0, 0, in16, out16, n16_in);
             hipLaunchKernelGGL(k_write, dim3((n16_out + 1023) / 1024), dim3(256), 0, 0, out16, n16_out);
         }},
        {"read only (input)", (double)in_bytes,
         [&] { hipLaunchKernelGGL(k_read, dim3((n16_in + 1023) / 1024), dim3(256), 0, 0, in16, out16, n16_in); }},
        {"write only (output)", (double)out_bytes,
         [&] { hipLaunchKernelGGL(k_write, dim3((n16_out + 1023) / 1024), dim3(256), 0, 0, out16, n16_out); }},
        {"s12 nt/nt WG1", b12, [&] { hipLaunchKernelGGL((k_s12<1, 1>), dim3(cus), dim3(256), 0, 0, in16, out16, nb); }},
        {"s12 nt/nt WG2", b12, [&] { hipLaunchKernelGGL((k_s12<1, 1>), dim3(cus * 2), dim3(256), 0, 0, in16, out16, nb); }},
        {"s12 nt/nt WG4", b12, [&] { hipLaunchKernelGGL((k_s12<1, 1>), dim3(cus * 4), dim3(256), 0, 0, in16, out16, nb); }},
        {"s12 nt/nt WG8", b12, [&] { hipLaunchKernelGGL((k_s12<1, 1>), dim3(cus * 8), dim3(256), 0, 0, in16, out16, nb); }},
        {"s12 nt/plain WG4", b12, [&] { hipLaunchKernelGGL((k_s12<1, 0>), dim3(cus * 4), dim3(256), 0, 0, in16, out16, nb); }},
        {"s12 nt/nt R2 WG4", b12, [&] { hipLaunchKernelGGL((k_s12<2, 1>), dim3(cus * 4), dim3(256), 0, 0, in16, out16, nb); }},
        {"s12 nt/nt R4 WG2", b12, [&] { hipLaunchKernelGGL((k_s12<4, 1>), dim3(cus * 2), dim3(256), 0, 0, in16, out16, nb); }},
        {"s12 nt/nt R4 WG4", b12, [&] { hipLaunchKernelGGL((k_s12<4, 1>), dim3(cus * 4), dim3(256), 0, 0, in16, out16, nb); }},
        {"s12 nt/plain R4 WG4", b12, [&] { hipLaunchKernelGGL((k_s12<4, 0>), dim3(cus * 4), dim3(256), 0, 0, in16, out16, nb); }},
        {"s12 cont WG4", b12, [&] { hipLaunchKernelGGL(k_s12_cont, dim3(cus * 4), dim3(256), 0, 0, in16, out16, nb); }},
    };
    for (auto &it : items) it.fn();
    CHECK(hipDeviceSynchronize());
    std::vector<std::vector<float>> ms(items.size());
    for (int r = 0; r < reps; ++r)
        for (size_t i = 0; i < items.size(); ++i) {
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
        printf("%-40s median %7.1f us %5.1f %% |", items[i].name, v[v.size() / 2] * 1e3,
               items[i].bytes / v[v.size() / 2] / 1e6 / 80.0);
        for (float t : v) printf(" %.1f", items[i].bytes / t / 1e6 / 80.0);
        printf("\n");
    }
    return 0;
}
