// tools/ubench/move5.hip -- round 4: the forward's data movement against the flat
// 1:2 stream, across grid sizes and batches per iteration, on the bench step's
// exact bytes (64 4K luma planes + 128 1080p chroma planes, uniform random
// pixels, 12.44 M blocks: 796 MB read, 1.59 GB written), steady state (one
// untimed launch of a case, then B2B timed launches back to back), interleaved
// rounds, HIP events, medians.
//   LOAD 0: flat, 4 x 16 B per lane per batch (the planes read as one array)
//   LOAD 1: pixel rows, 8 x 8 B per lane (lane-per-block: the product's loads)
//   STAGE 0: stores straight from the loaded registers (flat only)
//   STAGE 1: through a per-wave LDS stage at the product's 136-B pitch
//   NB: batches per wave iteration (all NB batches' loads, then all their stores)
//   MULT: grid = CUs x 4 WG x MULT (the product launches x8)
// Every case prefetches the next iteration's inputs before the current stores,
// as fdct8_quant_v3 does; loads nt, stores nt (the product's policies).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench/move5 tools/ubench/move5.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <functional>
#include <string>
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

struct Plane {
    const uint8_t *src;
    uint32_t bw, per_frame, stride, nbatch;
    size_t fstride;
};
struct Geo {
    Plane p[2];
    const uint8_t *flat;
    uint32_t nbatch;  // p[0].nbatch + p[1].nbatch
};

__device__ __forceinline__ const uint8_t *blk(const Plane &g, uint32_t n) {
    const uint32_t f = n / g.per_frame, rem = n - f * g.per_frame, by = rem / g.bw, bx = rem - by * g.bw;
    return g.src + f * g.fstride + (size_t)by * 8 * g.stride + bx * 8;
}

template <int LOAD>
struct In;
template <>
struct In<0> {
    u4v v[4];
};
template <>
struct In<1> {
    uint2 r[8];
};

template <int LOAD>
__device__ __forceinline__ void load_batch(const Geo &g, uint32_t b, int lane, In<LOAD> &in) {
    if constexpr (LOAD == 0) {
        const u4v *s = reinterpret_cast<const u4v *>(g.flat) + (size_t)b * 256;
#pragma unroll
        for (int k = 0; k < 4; ++k) in.v[k] = __builtin_nontemporal_load(s + k * 64 + lane);
    } else {
        const int pl = b >= g.p[0].nbatch;
        const Plane &P = pl ? g.p[1] : g.p[0];
        const uint8_t *px = blk(P, (b - (pl ? g.p[0].nbatch : 0)) * 64 + lane);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const u2v t = __builtin_nontemporal_load((const u2v *)(px + k * P.stride));
            in.r[k] = make_uint2(t.x, t.y);
        }
    }
}

template <int LOAD>
__device__ __forceinline__ void pin(In<LOAD> &in) {
    if constexpr (LOAD == 0) {
        asm volatile("" : "+v"(in.v[0]), "+v"(in.v[1]), "+v"(in.v[2]), "+v"(in.v[3])::"memory");
    } else {
        asm volatile("" : "+v"(in.r[0]), "+v"(in.r[1]), "+v"(in.r[2]), "+v"(in.r[3]), "+v"(in.r[4]), "+v"(in.r[5]),
                     "+v"(in.r[6]), "+v"(in.r[7])::"memory");
    }
}

__device__ double g_tab[128];  // stands in for the plan's exact tables (fdct8_quant_v3's LDS copy)

// TAB 1: every workgroup starts as fdct8_quant_v3 does -- 1 KiB of tables from
// global memory into LDS, then __syncthreads -- before its first batch's loads
template <int LOAD, int STAGE, int NB, int TAB = 0>
__global__ __launch_bounds__(256) void k_mv(Geo g, char *coef) {
    __shared__ uint4 st[(STAGE ? NB * 256 * 136 / 16 : 1) + 96];  // + the product's 1.5 KiB of tables/scratch
    if (TAB) {
        double *t = reinterpret_cast<double *>(st + (STAGE ? NB * 256 * 136 / 16 : 1));
        for (int i = threadIdx.x; i < 128; i += blockDim.x) t[i] = g_tab[i];
        __syncthreads();
    }
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t step = gridDim.x * 4;
    uint32_t it = blockIdx.x * 4 + wv;  // iteration unit: NB consecutive batches
    const uint32_t nit = g.nbatch / NB;
    In<LOAD> nxt[NB];
    if (it < nit)
#pragma unroll
        for (int j = 0; j < NB; ++j) load_batch<LOAD>(g, it * NB + j, lane, nxt[j]);
#pragma unroll
    for (int j = 0; j < NB; ++j) pin<LOAD>(nxt[j]);
    for (; it < nit; it += step) {
        In<LOAD> cur[NB];
#pragma unroll
        for (int j = 0; j < NB; ++j) cur[j] = nxt[j];
        if (it + step < nit)
#pragma unroll
            for (int j = 0; j < NB; ++j) load_batch<LOAD>(g, (it + step) * NB + j, lane, nxt[j]);
        if constexpr (STAGE == 0) {
#pragma unroll
            for (int j = 0; j < NB; ++j) {
                const __amdgpu_buffer_rsrc_t rc =
                    __builtin_amdgcn_make_buffer_rsrc(coef + (size_t)(it * NB + j) * 8192, 0, 8192, 0x00020000);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    __builtin_amdgcn_raw_buffer_store_b128(cur[j].v[k], rc, lane * 16, k * 1024, 2);
                    __builtin_amdgcn_raw_buffer_store_b128(cur[j].v[k] ^ u4v{1, 0, 0, 0}, rc, lane * 16, (k + 4) * 1024, 2);
                }
            }
            continue;
        } else {
#pragma unroll
            for (int j = 0; j < NB; ++j) {
                char *ws = reinterpret_cast<char *>(st) + (wv * NB + j) * 8704;
                uint2 *mine = reinterpret_cast<uint2 *>(ws + lane * 136);
                if constexpr (LOAD == 0) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        mine[4 * k] = make_uint2(cur[j].v[k].x, cur[j].v[k].y);
                        mine[4 * k + 1] = make_uint2(cur[j].v[k].z, cur[j].v[k].w);
                        mine[4 * k + 2] = make_uint2(cur[j].v[k].x ^ 1, cur[j].v[k].y);
                        mine[4 * k + 3] = make_uint2(cur[j].v[k].z, cur[j].v[k].w);
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        mine[2 * k] = cur[j].r[k];
                        mine[2 * k + 1] = make_uint2(cur[j].r[k].y, cur[j].r[k].x);
                    }
                }
            }
            // the product's fence: the prefetch wait before the stage read-back
#pragma unroll
            for (int j = 0; j < NB; ++j) pin<LOAD>(nxt[j]);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int j = 0; j < NB; ++j) {
                const char *ws = reinterpret_cast<const char *>(st) + (wv * NB + j) * 8704;
                u4v val[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const int m = k * 64 + lane, bl = m >> 3;
                    const uint2 *s2 = reinterpret_cast<const uint2 *>(ws + bl * 136 + (m & 7) * 16);
                    val[k] = u4v{s2[0].x, s2[0].y, s2[1].x, s2[1].y};
                }
                const __amdgpu_buffer_rsrc_t rc =
                    __builtin_amdgcn_make_buffer_rsrc(coef + (size_t)(it * NB + j) * 8192, 0, 8192, 0x00020000);
#pragma unroll
                for (int k = 0; k < 8; ++k) __builtin_amdgcn_raw_buffer_store_b128(val[k], rc, lane * 16, k * 1024, 2);
            }
        }
    }
}

// Dynamic batch assignment (round 4): a persistent grid whose waves take the next
// 64-block batch from a device counter (one vector atomic per batch, issued one
// batch ahead so its latency hides behind the current batch), the rest as the
// rows8 staged case.  The counters reset themselves: the last wave to finish
// (the `fin` counter) zeroes both, so back-to-back launches need no memset.
__global__ __launch_bounds__(256) void k_dyn(Geo g, char *coef, uint32_t *ctr) {
    __shared__ uint4 st[256 * 136 / 16 + 96];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t n = g.nbatch;
    auto grab = [&]() -> uint32_t {
        uint32_t v = 0;
        if (lane == 0) v = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return __builtin_amdgcn_readfirstlane(v);
    };
    uint32_t cur = grab();
    uint32_t nx = grab();
    In<1> nxt;
    if (cur < n) load_batch<1>(g, cur, lane, nxt);
    pin<1>(nxt);
    char *ws = reinterpret_cast<char *>(st) + wv * 8704;
    while (cur < n) {
        In<1> c = nxt;
        const uint32_t nn = grab();  // the batch after next: its latency hides behind this batch
        if (nx < n) load_batch<1>(g, nx, lane, nxt);
        uint2 *mine = reinterpret_cast<uint2 *>(ws + lane * 136);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            mine[2 * k] = c.r[k];
            mine[2 * k + 1] = make_uint2(c.r[k].y, c.r[k].x);
        }
        pin<1>(nxt);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        u4v val[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int m = k * 64 + lane, bl = m >> 3;
            const uint2 *s2 = reinterpret_cast<const uint2 *>(ws + bl * 136 + (m & 7) * 16);
            val[k] = u4v{s2[0].x, s2[0].y, s2[1].x, s2[1].y};
        }
        const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(coef + (size_t)cur * 8192, 0, 8192, 0x00020000);
#pragma unroll
        for (int k = 0; k < 8; ++k) __builtin_amdgcn_raw_buffer_store_b128(val[k], rc, lane * 16, k * 1024, 2);
        cur = nx;
        nx = nn;
    }
    if (lane == 0) {
        const uint32_t waves = gridDim.x * 4;
        if (__hip_atomic_fetch_add(ctr + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == waves - 1) {
            __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(ctr + 1, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

__global__ void k_fill(uint32_t *p, size_t n, uint32_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull + seed;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = (uint32_t)(z ^ (z >> 31));
    }
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
    const int B2B = argc > 2 ? atoi(argv[2]) : 3;
    const uint32_t FY = 64, FC = 128;
    const size_t ybytes = (size_t)3840 * 2160 * FY, cbytes = (size_t)1920 * 1080 * FC;
    const size_t nblk = (ybytes + cbytes) / 64;
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint8_t *src;
    char *dst;
    CHECK(hipMalloc(&src, ybytes + cbytes));
    CHECK(hipMalloc(&dst, nblk * 128));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint32_t *)src, (ybytes + cbytes) / 4, 12345u);
    CHECK(hipMemset(dst, 0, nblk * 128));
    CHECK(hipDeviceSynchronize());
    Geo g;
    g.p[0] = Plane{src, 480, 129600, 3840, (uint32_t)(ybytes / 4096), (size_t)3840 * 2160};
    g.p[1] = Plane{src + ybytes, 240, 32400, 1920, (uint32_t)(cbytes / 4096), (size_t)1920 * 1080};
    g.flat = src;
    g.nbatch = g.p[0].nbatch + g.p[1].nbatch;  // 194400: divisible by 1, 2, 4
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const double bytes = (double)nblk * 192;
    struct Item {
        std::string name;
        std::function<void()> fn;
    };
    std::vector<Item> items;
    auto add = [&](const char *nm, auto kern, int mult) {
        int per = 0;
        CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, 256, 0));
        const int grid = cus * 4 * mult;  // the product: CUs x 4 resident x 8
        char buf[96];
        snprintf(buf, sizeof buf, "%s x%d (%d WG/CU res)", nm, mult, per);
        items.push_back({buf, [=] { hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, g, dst); }});
    };
    // round 4, second call: the grid multiplier past x8 (the dynamic counter of k_dyn ran at 12 % of 8 TB/s:
    // one address takes ~80 M atomics/s, profiles/r04/move5_grid.log -- dropped from the list)
    for (int m : {4, 8, 12, 16, 24, 32, 48}) {
        add("flat16 staged NB1", k_mv<0, 1, 1>, m);
        add("rows8  staged NB1", k_mv<1, 1, 1>, m);
    }
    add("flat16 direct NB4", k_mv<0, 0, 4>, 1);
    add("flat16 direct NB1", k_mv<0, 0, 1>, 1);
    for (int w = 0; w < 300; ++w) items[w % items.size()].fn();  // clock pre-warm
    CHECK(hipDeviceSynchronize());
    std::vector<std::vector<float>> us(items.size());
    for (int r = 0; r < reps; ++r)
        for (size_t i = 0; i < items.size(); ++i) {
            items[i].fn();
            CHECK(hipEventRecord(e0));
            for (int k = 0; k < B2B; ++k) items[i].fn();
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float t;
            CHECK(hipEventElapsedTime(&t, e0, e1));
            us[i].push_back(t * 1e3f / B2B);
        }
    CHECK(hipGetLastError());
    printf("%zu blocks, %.1f MB read + %.1f MB written per launch, %d CUs, %d rounds x %d b2b\n", nblk, nblk * 64 / 1e6,
           nblk * 128 / 1e6, cus, reps, B2B);
    for (size_t i = 0; i < items.size(); ++i) {
        std::vector<float> v = us[i];
        std::sort(v.begin(), v.end());
        const float med = v[v.size() / 2];
        printf("%-40s median %7.1f us %5.1f %% of 8 TB/s | min %7.1f\n", items[i].name.c_str(), med,
               bytes / (med * 1e-6) / 8e12 * 100.0, v[0]);
    }
    return 0;
}
