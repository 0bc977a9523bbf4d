// tools/ubench/hbm_mix3.hip -- the forward kernel's data movement with R
// consecutive 64-block batches per wave iteration (hbm_mix2: a flat 1:2 stream
// with 16 KiB loaded then 32 KiB stored per wave reached 74.7 % with plain
// stores vs 71 % for one batch at a time).  Row form: lane-per-block 8 x 8-B
// pixel-row loads of a 96 x 4K luma stack, the next group's rows prefetched into
// registers while the current group is "computed" (BURN dependent VALU ops per
// batch, ~the real kernel's per-batch VALU work) and staged through LDS, then
// 8 x 1 KiB stores per batch.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench/hbm_mix3 tools/ubench/hbm_mix3.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <functional>
#include <vector>

typedef unsigned int u2v __attribute__((ext_vector_type(2)));
typedef unsigned int u4v __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

struct Geo {
    const uint8_t *src;
    uint32_t bw, per_frame, stride;
    size_t fstride;
};

__device__ __forceinline__ void load_rows(const Geo &g, uint32_t n, uint2 (&r)[8]) {
    const uint32_t f = n / g.per_frame, rem = n - f * g.per_frame, by = rem / g.bw, bx = rem - by * g.bw;
    const uint8_t *p = g.src + f * g.fstride + (size_t)by * 8 * g.stride + bx * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const u2v t = __builtin_nontemporal_load((const u2v *)(p + k * g.stride));
        r[k] = make_uint2(t.x, t.y);
    }
}

// R batches per iteration; AUX = store cache policy (0 plain, 2 nt); BURN = VALU
// chain length per batch (4 independent chains)
template <int R, int AUX, int BURN>
__global__ __launch_bounds__(256) void k_mv(Geo g, char *coef, uint32_t nb) {
    __shared__ uint4 st[256 * 136 / 16];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    char *ws = reinterpret_cast<char *>(st) + wv * 8704;
    const uint32_t step = gridDim.x * 4 * R;
    uint32_t b0 = (blockIdx.x * 4 + wv) * R;
    uint2 nxt[R][8];
#pragma unroll
    for (int j = 0; j < R; ++j) load_rows(g, (b0 + j < nb ? b0 + j : 0) * 64 + lane, nxt[j]);
    for (; b0 < nb; b0 += step) {
        uint2 cur[R][8];
#pragma unroll
        for (int j = 0; j < R; ++j)
#pragma unroll
            for (int k = 0; k < 8; ++k) cur[j][k] = nxt[j][k];
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const uint32_t bn = b0 + step + j;
            load_rows(g, (bn < nb ? bn : 0) * 64 + lane, nxt[j]);
        }
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const uint32_t b = b0 + j;
            uint2 x[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) x[k] = cur[j][k];
            float a0 = __uint_as_float(x[0].x & 0x3fffffff), a1 = __uint_as_float(x[1].x & 0x3fffffff),
                  a2 = __uint_as_float(x[2].x & 0x3fffffff), a3 = __uint_as_float(x[3].x & 0x3fffffff);
#pragma unroll
            for (int i = 0; i < BURN / 4; ++i) {
                a0 = __builtin_fmaf(a0, 0.999f, 1e-3f);
                a1 = __builtin_fmaf(a1, 0.999f, 1e-3f);
                a2 = __builtin_fmaf(a2, 0.999f, 1e-3f);
                a3 = __builtin_fmaf(a3, 0.999f, 1e-3f);
            }
            x[0].x ^= __float_as_uint(a0 + a1 + a2 + a3) & 1u;
            if (j == 0)  // the prefetch rows consumed before the stores (as fdct8_batch does)
                asm volatile("" : "+v"(nxt[0][0]), "+v"(nxt[R - 1][7])::"memory");
            __builtin_amdgcn_s_waitcnt(0x0F70);  // LDS reuse after stores: retire them (see DESIGN)
            uint2 *mine = reinterpret_cast<uint2 *>(ws + lane * 136);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                mine[2 * k] = x[k];
                mine[2 * k + 1] = make_uint2(x[k].x ^ 1, x[k].y);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (b < nb) {
                const __amdgpu_buffer_rsrc_t rc =
                    __builtin_amdgcn_make_buffer_rsrc(coef + (size_t)b * 8192, 0, 8192, 0x00020000);
                u4v val[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const int m = k * 64 + lane, bl = m >> 3;
                    const uint2 *s2 = reinterpret_cast<const uint2 *>(ws + bl * 136 + (m & 7) * 16);
                    val[k] = u4v{s2[0].x, s2[0].y, s2[1].x, s2[1].y};
                }
#pragma unroll
                for (int k = 0; k < 8; ++k) __builtin_amdgcn_raw_buffer_store_b128(val[k], rc, lane * 16, k * 1024, AUX);
            }
        }
    }
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 8;
    const uint32_t W = 3840, H = 2160, F = 96;
    const uint32_t bw = W / 8, per = bw * (H / 8);
    const size_t nblk = (size_t)per * F;
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
    Geo g{src, bw, per, W, (size_t)W * H};
    const double b12 = (double)nblk * 192;
    struct Item {
        const char *name;
        std::function<void()> fn;
    };
#define MV(R, AUX, BURN, WG) \
    [&] { hipLaunchKernelGGL((k_mv<R, AUX, BURN>), dim3(cus * (WG)), dim3(256), 0, 0, g, dst, nb); }
    std::vector<Item> items = {
        {"R1 nt    burn0   4WG", MV(1, 2, 0, 4)},   {"R1 plain burn0   4WG", MV(1, 0, 0, 4)},
        {"R2 nt    burn0   4WG", MV(2, 2, 0, 4)},   {"R2 plain burn0   4WG", MV(2, 0, 0, 4)},
        {"R4 nt    burn0   2WG", MV(4, 2, 0, 2)},   {"R4 plain burn0   2WG", MV(4, 0, 0, 2)},
        {"R4 plain burn0   4WG", MV(4, 0, 0, 4)},
        {"R1 nt    burn400 4WG", MV(1, 2, 400, 4)}, {"R1 plain burn400 4WG", MV(1, 0, 400, 4)},
        {"R2 nt    burn400 3WG", MV(2, 2, 400, 3)}, {"R2 plain burn400 3WG", MV(2, 0, 400, 3)},
        {"R4 nt    burn400 2WG", MV(4, 2, 400, 2)}, {"R4 plain burn400 2WG", MV(4, 0, 400, 2)},
        {"R1 nt    burn800 4WG", MV(1, 2, 800, 4)}, {"R1 plain burn800 4WG", MV(1, 0, 800, 4)},
        {"R4 plain burn800 2WG", MV(4, 0, 800, 2)},
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
        printf("%-24s median %7.1f us %5.1f %% |", items[i].name, v[v.size() / 2] * 1e3, b12 / v[v.size() / 2] / 1e6 / 80.0);
        for (float t : v) printf(" %.1f", b12 / t / 1e6 / 80.0);
        printf("\n");
    }
    return 0;
}
