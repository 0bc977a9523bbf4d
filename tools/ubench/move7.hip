// tools/ubench/move7.hip -- round 4: the forward's pixel loads as 16 B per lane
// (1 KiB per instruction, as the flat stream) instead of 8 B per lane (512 B).
// rows8:  lane b loads the 8 rows of block b, 8 x 8 B (the product's loads)
// pair16: lane (p, h) loads row 2j + h of blocks 2p, 2p + 1 (16 B) for j = 0..3:
//         4 x 1 KiB per batch; the rows go through the wave's LDS stage (4 KiB, row
//         r of block b at r * 512 + 8 b: b128 writes and b64 reads conflict-free)
//         into the lane-per-block registers, then the same 136-B stage and stores.
//         Pairs of blocks never straddle a block row here (480 / 240 blocks per row).
// rows8 direct: no stage, each lane stores its block (8 x 16 B at a 128-B lane stride).
// flat staged: the flat stream's loads with the product's stage and stores.
// Same bytes, method and items as move6 (steady state, interleaved, HIP events).
// Build: hipcc --offload-arch=gfx950 -O3 -Iinclude -Ldct_amd -ldct_amd_diag
//        -Wl,-rpath,'$ORIGIN/../../dct_amd' -o tools/ubench/move7 tools/ubench/move7.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <functional>
#include <string>
#include <vector>

#include "dct_amd.h"
extern "C" int dctq_diag_movement_grid_planes(const dctq_plan *plan, const dctq_plane *planes, int nplanes,
                                              int16_t *const *coef, int grid_mult, void *stream);
extern "C" int dctq_diag_stream(int kind, const void *src, void *dst, long long blocks, void *stream);

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
#define DCHECK(x)                                                   \
    do {                                                            \
        int r_ = (x);                                               \
        if (r_) {                                                   \
            fprintf(stderr, "%s:%d %s = %d\n", __FILE__, __LINE__, #x, r_); \
            exit(1);                                                \
        }                                                           \
    } while (0)

struct Plane {
    const uint8_t *src;
    char *dst;
    uint32_t bw, per_frame, stride, nbatch;
    size_t fstride;
};
struct Geo {
    Plane p[2];
    uint32_t nbatch;
};

__device__ __forceinline__ const uint8_t *blk(const Plane &g, uint32_t n) {
    const uint32_t f = n / g.per_frame, rem = n - f * g.per_frame, by = rem / g.bw, bx = rem - by * g.bw;
    return g.src + f * g.fstride + (size_t)by * 8 * g.stride + bx * 8;
}

__device__ __forceinline__ void load_rows(const Geo &g, uint32_t b, int lane, uint2 (&r)[8]) {
    const int pl = b >= g.p[0].nbatch;
    const Plane &P = pl ? g.p[1] : g.p[0];
    const uint8_t *px = blk(P, (b - (pl ? g.p[0].nbatch : 0)) * 64 + lane);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const u2v t = __builtin_nontemporal_load((const u2v *)(px + k * P.stride));
        r[k] = make_uint2(t.x, t.y);
    }
}

__device__ __forceinline__ void pin(uint2 (&r)[8]) {
    asm volatile("" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]),
                 "+v"(r[7])::"memory");
}

// move5's k_mv<1, 1, 1>: rows8 loads, the product's 136-B LDS stage, 8 x 1 KiB nt stores
__global__ __launch_bounds__(256) void k_rows8(Geo g) {
    __shared__ uint4 st[256 * 136 / 16 + 96];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t step = gridDim.x * 4;
    uint32_t it = blockIdx.x * 4 + wv;
    uint2 nxt[8];
    if (it < g.nbatch) load_rows(g, it, lane, nxt);
    pin(nxt);
    char *ws = reinterpret_cast<char *>(st) + wv * 8704;
    for (; it < g.nbatch; it += step) {
        uint2 cur[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) cur[k] = nxt[k];
        if (it + step < g.nbatch) load_rows(g, it + step, lane, nxt);
        uint2 *mine = reinterpret_cast<uint2 *>(ws + lane * 136);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            mine[2 * k] = cur[k];
            mine[2 * k + 1] = make_uint2(cur[k].y, cur[k].x);
        }
        pin(nxt);
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
        const int pl = it >= g.p[0].nbatch;
        const Plane &P = pl ? g.p[1] : g.p[0];
        const uint32_t lb = it - (pl ? g.p[0].nbatch : 0);
        const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(P.dst + (size_t)lb * 8192, 0, 8192, 0x00020000);
#pragma unroll
        for (int k = 0; k < 8; ++k) __builtin_amdgcn_raw_buffer_store_b128(val[k], rc, lane * 16, k * 1024, 2);
    }
}

__device__ __forceinline__ void load_pairs(const Geo &g, uint32_t b, int lane, u4v (&r)[4]) {
    const int pl = b >= g.p[0].nbatch;
    const Plane &P = pl ? g.p[1] : g.p[0];
    const int p = lane & 31, h = lane >> 5;
    const uint8_t *px = blk(P, (b - (pl ? g.p[0].nbatch : 0)) * 64 + 2 * p) + h * P.stride;
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = __builtin_nontemporal_load((const u4v *)(px + 2 * j * P.stride));
}

__device__ __forceinline__ void pin4(u4v (&r)[4]) {
    asm volatile("" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3])::"memory");
}

template <int XPOSE>
__global__ __launch_bounds__(256) void k_pair16(Geo g) {
    __shared__ uint4 st[256 * 136 / 16 + 96];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t step = gridDim.x * 4;
    uint32_t it = blockIdx.x * 4 + wv;
    u4v nxt[4];
    if (it < g.nbatch) load_pairs(g, it, lane, nxt);
    pin4(nxt);
    char *ws = reinterpret_cast<char *>(st) + wv * 8704;
    for (; it < g.nbatch; it += step) {
        uint2 cur[8];
        {
            // rows -> LDS (row r at r * 512, 16 B per lane), then lane-per-block
            const int p = lane & 31, h = lane >> 5;
#pragma unroll
            for (int j = 0; j < 4; ++j) *reinterpret_cast<u4v *>(ws + (2 * j + h) * 512 + p * 16) = nxt[j];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int k = 0; k < 8; ++k) cur[k] = *reinterpret_cast<const uint2 *>(ws + k * 512 + lane * 8);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        if (it + step < g.nbatch) load_pairs(g, it + step, lane, nxt);
        uint2 *mine = reinterpret_cast<uint2 *>(ws + lane * 136);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            mine[2 * k] = cur[k];
            mine[2 * k + 1] = make_uint2(cur[k].y, cur[k].x);
        }
        pin4(nxt);
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
        const int pl = it >= g.p[0].nbatch;
        const Plane &P = pl ? g.p[1] : g.p[0];
        const uint32_t lb = it - (pl ? g.p[0].nbatch : 0);
        const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(P.dst + (size_t)lb * 8192, 0, 8192, 0x00020000);
#pragma unroll
        for (int k = 0; k < 8; ++k) __builtin_amdgcn_raw_buffer_store_b128(val[k], rc, lane * 16, k * 1024, 2);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

// rows8 loads, no stage: lane b stores its own block's 128 B as 8 x 16 B (instruction k
// writes bytes 16k.. of every block: 64 x 16 B at a 128-B stride)
__global__ __launch_bounds__(256) void k_rows8_direct(Geo g) {
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t step = gridDim.x * 4;
    uint32_t it = blockIdx.x * 4 + wv;
    uint2 nxt[8];
    if (it < g.nbatch) load_rows(g, it, lane, nxt);
    pin(nxt);
    for (; it < g.nbatch; it += step) {
        uint2 cur[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) cur[k] = nxt[k];
        if (it + step < g.nbatch) load_rows(g, it + step, lane, nxt);
        pin(nxt);
        const int pl = it >= g.p[0].nbatch;
        const Plane &P = pl ? g.p[1] : g.p[0];
        const uint32_t lb = it - (pl ? g.p[0].nbatch : 0);
        const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(P.dst + (size_t)lb * 8192, 0, 8192, 0x00020000);
#pragma unroll
        for (int k = 0; k < 8; ++k)
            __builtin_amdgcn_raw_buffer_store_b128(u4v{cur[k].x, cur[k].y, cur[k].y, cur[k].x}, rc, lane * 128, k * 16, 2);
    }
}

// flat loads (4 x 16 B per lane = the batch's 4 KiB of pixels in order), the product's
// 136-B stage writes and 8 x 1 KiB stores: rows8 with the load shape of the flat stream
__global__ __launch_bounds__(256) void k_flat_staged(const u4v *src, Geo g) {
    __shared__ uint4 st[256 * 136 / 16 + 96];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t step = gridDim.x * 4;
    uint32_t it = blockIdx.x * 4 + wv;
    u4v nxt[4];
    if (it < g.nbatch)
#pragma unroll
        for (int j = 0; j < 4; ++j) nxt[j] = __builtin_nontemporal_load(src + (size_t)it * 256 + j * 64 + lane);
    pin4(nxt);
    char *ws = reinterpret_cast<char *>(st) + wv * 8704;
    for (; it < g.nbatch; it += step) {
        uint2 cur[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            cur[2 * j] = make_uint2(nxt[j].x, nxt[j].y);
            cur[2 * j + 1] = make_uint2(nxt[j].z, nxt[j].w);
        }
        if (it + step < g.nbatch)
#pragma unroll
            for (int j = 0; j < 4; ++j) nxt[j] = __builtin_nontemporal_load(src + (size_t)(it + step) * 256 + j * 64 + lane);
        uint2 *mine = reinterpret_cast<uint2 *>(ws + lane * 136);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            mine[2 * k] = cur[k];
            mine[2 * k + 1] = make_uint2(cur[k].y, cur[k].x);
        }
        pin4(nxt);
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
        const int pl = it >= g.p[0].nbatch;
        const Plane &P = pl ? g.p[1] : g.p[0];
        const uint32_t lb = it - (pl ? g.p[0].nbatch : 0);
        const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(P.dst + (size_t)lb * 8192, 0, 8192, 0x00020000);
#pragma unroll
        for (int k = 0; k < 8; ++k) __builtin_amdgcn_raw_buffer_store_b128(val[k], rc, lane * 16, k * 1024, 2);
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
    const size_t nby = ybytes / 64, nbc = cbytes / 64, nblk = nby + nbc;
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint8_t *src;
    char *out1, *outY, *outC;
    CHECK(hipMalloc(&src, ybytes + cbytes));
    CHECK(hipMalloc(&out1, nblk * 128));
    CHECK(hipMalloc(&outY, nby * 128));
    CHECK(hipMalloc(&outC, nbc * 128));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint32_t *)src, (ybytes + cbytes) / 4, 12345u);
    CHECK(hipDeviceSynchronize());
    Geo g1, g2;
    g1.p[0] = Plane{src, out1, 480, 129600, 3840, (uint32_t)(ybytes / 4096), (size_t)3840 * 2160};
    g1.p[1] = Plane{src + ybytes, out1 + nby * 128, 240, 32400, 1920, (uint32_t)(cbytes / 4096), (size_t)1920 * 1080};
    g1.nbatch = g1.p[0].nbatch + g1.p[1].nbatch;
    g2 = g1;
    g2.p[0].dst = outY;
    g2.p[1].dst = outC;
    dctq_plan *plan = nullptr;
    DCHECK(dctq_plan_create(50, 0, &plan));
    dctq_plane planes[2] = {{src, 3840, (long long)3840 * 2160, 3840, 2160, (int)FY},
                            {src + ybytes, 1920, (long long)1920 * 1080, 1920, 1080, (int)FC}};
    int16_t *c1[2] = {(int16_t *)out1, (int16_t *)(out1 + nby * 128)};
    int16_t *c2[2] = {(int16_t *)outY, (int16_t *)outC};
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const double bytes = (double)nblk * 192;
    struct Item {
        std::string name;
        std::function<void()> fn;
    };
    std::vector<Item> items;
    for (int m : {16, 32}) {
        items.push_back({"rows8 2out x" + std::to_string(m),
                         [=] { hipLaunchKernelGGL(k_rows8, dim3(cus * 4 * m), dim3(256), 0, 0, g2); }});
        items.push_back({"pair16 2out x" + std::to_string(m),
                         [=] { hipLaunchKernelGGL(k_pair16<0>, dim3(cus * 4 * m), dim3(256), 0, 0, g2); }});
    }
    for (int m : {16, 32}) {
        items.push_back({"rows8 direct x" + std::to_string(m),
                         [=] { hipLaunchKernelGGL(k_rows8_direct, dim3(cus * 4 * m), dim3(256), 0, 0, g2); }});
        items.push_back({"flat staged x" + std::to_string(m),
                         [=] { hipLaunchKernelGGL(k_flat_staged, dim3(cus * 4 * m), dim3(256), 0, 0, (const u4v *)src, g2); }});
    }
    items.push_back({"fwd 2out", [=] { DCHECK(dctq_forward_quant_planes(plan, planes, 2, c2, nullptr, nullptr)); }});
    items.push_back({"mv 2out x16", [=] { DCHECK(dctq_diag_movement_grid_planes(plan, planes, 2, c2, 16, nullptr)); }});
    for (int k : {0, 7})
        items.push_back({"flat kind " + std::to_string(k),
                         [=] { DCHECK(dctq_diag_stream(k, src, out1, (long long)nblk / 64 * 64, nullptr)); }});
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
    printf("%zu blocks, %d CUs, %d rounds x %d b2b\n", nblk, cus, reps, B2B);
    for (size_t i = 0; i < items.size(); ++i) {
        std::vector<float> v = us[i];
        std::sort(v.begin(), v.end());
        const float med = v[v.size() / 2];
        printf("%-16s median %7.1f us %5.1f %% of 8 TB/s | min %7.1f\n", items[i].name.c_str(), med,
               bytes / (med * 1e-6) / 8e12 * 100.0, v[0]);
    }
    dctq_plan_destroy(plan);
    return 0;
}
