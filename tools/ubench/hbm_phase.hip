// tools/ubench/hbm_phase.hip -- chip-wide read / write phases inside one
// persistent launch (hbm_mix2: a read kernel followed by a write kernel moves
// the 1:2 traffic at 82 % of 8 TB/s, a mixed stream at 71-74 %).  Each wave
// loads R 64-block batches (R x 4 KiB, 16 B per lane per load) into registers,
// the grid meets at a barrier, every wave stores its R x 8 KiB, waits for its
// stores, meets again.  Barrier: one device-scope counter, one arrival per
// workgroup, polled by one lane with s_sleep; bounded polls (a barrier that
// times out just proceeds -- this is a timing probe, outputs are not checked).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench/hbm_phase tools/ubench/hbm_phase.hip
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

__device__ __forceinline__ void grid_barrier(unsigned *ctr, unsigned target, unsigned *timeouts) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        int polls = 0;
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(2);
            if (++polls > 2000000) {
                atomicAdd(timeouts, 1u);
                break;
            }
        }
    }
    __syncthreads();
}

// BAR: 0 = no barriers (control), 1 = barrier after loads and after stores, 2 = only after loads
template <int R, int AUX, int BAR>
__global__ __launch_bounds__(512) void k_phase(const u4v *__restrict__ in, char *__restrict__ out, uint32_t nb,
                                               unsigned *ctr, unsigned *timeouts) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t tw = gridDim.x * 8;
    const uint32_t w = blockIdx.x * 8 + wv;
    const uint32_t ncyc = (nb + tw * R - 1) / (tw * R);
    unsigned gen = 0;
    for (uint32_t cyc = 0; cyc < ncyc; ++cyc) {
        const uint32_t b0 = (cyc * tw + w) * R;
        u4v v[R][4];
#pragma unroll
        for (int j = 0; j < R; ++j)
#pragma unroll
            for (int k = 0; k < 4; ++k)
                v[j][k] = b0 + j < nb ? __builtin_nontemporal_load(in + (size_t)(b0 + j) * 256 + k * 64 + lane)
                                      : u4v{0, 0, 0, 0};
        if (BAR) {
            __builtin_amdgcn_s_waitcnt(0x0F70);
            grid_barrier(ctr, (++gen) * gridDim.x, timeouts);
        }
#pragma unroll
        for (int j = 0; j < R; ++j)
            if (b0 + j < nb) {
                const __amdgpu_buffer_rsrc_t rc =
                    __builtin_amdgcn_make_buffer_rsrc(out + (size_t)(b0 + j) * 8192, 0, 8192, 0x00020000);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    __builtin_amdgcn_raw_buffer_store_b128(v[j][k], rc, lane * 16, k * 1024, AUX);
                    __builtin_amdgcn_raw_buffer_store_b128(v[j][k] ^ u4v{1, 0, 0, 0}, rc, lane * 16, (k + 4) * 1024, AUX);
                }
            }
        if (BAR == 1) {
            __builtin_amdgcn_s_waitcnt(0x0F70);
            grid_barrier(ctr, (++gen) * gridDim.x, timeouts);
        }
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
    unsigned *ctr;
    CHECK(hipMalloc(&src, in_bytes));
    CHECK(hipMalloc(&dst, out_bytes));
    CHECK(hipMalloc(&ctr, 64));
    CHECK(hipMemset(src, 7, in_bytes));
    CHECK(hipMemset(dst, 0, out_bytes));
    CHECK(hipMemset(ctr, 0, 64));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const u4v *in16 = (const u4v *)src;
    const double b12 = (double)nblk * 192;
    struct Item {
        const char *name;
        std::function<void()> fn;
    };
#define PH(R, AUX, BAR, WG)                                                                                  \
    [&] {                                                                                                    \
        CHECK(hipMemsetAsync(ctr, 0, 8, 0));                                                                 \
        hipLaunchKernelGGL((k_phase<R, AUX, BAR>), dim3(cus * (WG)), dim3(512), 0, 0, in16, dst, nb, ctr, ctr + 1); \
    }
    std::vector<Item> items = {
        {"R4 nt    no barrier  1WG", PH(4, 2, 0, 1)}, {"R4 plain no barrier  1WG", PH(4, 0, 0, 1)},
        {"R4 nt    phased      1WG", PH(4, 2, 1, 1)}, {"R4 plain phased      1WG", PH(4, 0, 1, 1)},
        {"R8 nt    no barrier  1WG", PH(8, 2, 0, 1)}, {"R8 plain no barrier  1WG", PH(8, 0, 0, 1)},
        {"R8 nt    phased      1WG", PH(8, 2, 1, 1)}, {"R8 plain phased      1WG", PH(8, 0, 1, 1)},
        {"R8 nt    load-bar    1WG", PH(8, 2, 2, 1)}, {"R8 plain load-bar    1WG", PH(8, 0, 2, 1)},
        {"R4 nt    phased      2WG", PH(4, 2, 1, 2)}, {"R4 plain phased      2WG", PH(4, 0, 1, 2)},
    };
    for (auto &it : items) it.fn();
    CHECK(hipDeviceSynchronize());
    std::vector<std::vector<float>> ms(items.size());
    for (int r = 0; r < reps; ++r)
        for (size_t i = 0; i < items.size(); ++i) {
            items[i].fn();  // includes the counter reset
            CHECK(hipEventRecord(e0));
            items[i].fn();
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float t;
            CHECK(hipEventElapsedTime(&t, e0, e1));
            ms[i].push_back(t);
        }
    CHECK(hipGetLastError());
    unsigned h[2];
    CHECK(hipMemcpy(h, ctr, 8, hipMemcpyDeviceToHost));
    printf("barrier timeouts in the last run: %u\n", h[1]);
    for (size_t i = 0; i < items.size(); ++i) {
        std::vector<float> v = ms[i];
        std::sort(v.begin(), v.end());
        printf("%-26s median %7.1f us %5.1f %% |", items[i].name, v[v.size() / 2] * 1e3, b12 / v[v.size() / 2] / 1e6 / 80.0);
        for (float t : v) printf(" %.1f", b12 / t / 1e6 / 80.0);
        printf("\n");
    }
    return 0;
}
