// tools/ubench/move8.hip -- round 4: what separates the forward's movement
// (rows8 loads, LDS stage, 1 KiB stores, next batch prefetched) from the flat
// 1:2 stream that beats it by 2-4 % on median boxes (dctq_diag_stream kind 7: 16-B
// loads, stores straight from the loaded registers, no prefetch, one batch per wave).
// One kernel template over the three differences, same bytes and buffers:
//   LOAD  0 rows8 (8 x 8 B per lane: block rows) / 1 flat16 (4 x 16 B per lane: NOT the
//         batch's blocks, the bytes in memory order) / 2 pair16 (16 B per lane: row 2j + h of
//         blocks 2p, 2p + 1, transposed through the stage into lane-per-block rows, move7) /
//         3 flat16 loads with pair16's LDS transpose (the instruction mix of a design that loads a
//         contiguous block row and transposes it; the data are not blocks)
//   STAGE 0 stores from registers (flat16 only) / 1 the product's 136-B stage
//   PF    0 load at the loop top / 1 next batch prefetched before the stores
// on grids of CUs x 4 x {16, 32, 48} workgroups of 4 waves, writing the outputs of two
// allocations (g2, as bench.py) or one (out1 right after the pixels, outZ allocated last); steady state,
// interleaved rounds, HIP events, medians (as move6/move7).  ORD: the order of the 8 x 1 KiB
// stores (chunks 0..7, or 0, 4, 1, 5, .. as dctq_diag_stream).  profiles/r04/move8_*.log.
// Build: hipcc --offload-arch=gfx950 -O3 -Iinclude -Ldct_amd -ldct_amd_diag
//        -Wl,-rpath,'$ORIGIN/../../dct_amd' -o tools/ubench/move8 tools/ubench/move8.hip
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


__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// the batch's 4 KiB: rows8 -> 8 x uint2 per lane (row k of block lane); flat16 ->
// 4 x 16 B per lane (piece j * 64 + lane of the batch's bytes in the source order)
template <int LOAD>
__device__ __forceinline__ void load_batch(const Geo &g, const u4v *flat, uint32_t b, int lane, u4v (&r)[4]) {
    if constexpr (LOAD == 0) {
        uint2 rows[8];
        load_rows(g, b, lane, rows);
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = u4v{rows[2 * j].x, rows[2 * j].y, rows[2 * j + 1].x, rows[2 * j + 1].y};
    } else if constexpr (LOAD == 1 || LOAD == 3) {
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = __builtin_nontemporal_load(flat + (size_t)b * 256 + j * 64 + lane);
    } else {  // pair16: lane (p, h) loads row 2j + h of blocks 2p, 2p + 1
        const int pl = b >= g.p[0].nbatch;
        const Plane &P = pl ? g.p[1] : g.p[0];
        const int p = lane & 31, h = lane >> 5;
        const uint8_t *px = blk(P, (b - (pl ? g.p[0].nbatch : 0)) * 64 + 2 * p) + h * P.stride;
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = __builtin_nontemporal_load((const u4v *)(px + 2 * j * P.stride));
    }
}

__device__ __forceinline__ void pin4(u4v (&r)[4]) {
    asm volatile("" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3])::"memory");
}

template <int LOAD, int STAGE, int PF, int ORD = 0>
__global__ __launch_bounds__(256) void k_move(Geo g, const u4v *flat) {
    __shared__ uint4 st[256 * 136 / 16 + 96];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t step = gridDim.x * 4;
    uint32_t it = blockIdx.x * 4 + wv;
    u4v nxt[4];
    if (PF && it < g.nbatch) load_batch<LOAD>(g, flat, it, lane, nxt);
    if (PF) pin4(nxt);
    char *ws = reinterpret_cast<char *>(st) + wv * 8704;
    for (; it < g.nbatch; it += step) {
        u4v cur[4];
        if (PF) {
#pragma unroll
            for (int j = 0; j < 4; ++j) cur[j] = nxt[j];
            if (it + step < g.nbatch) load_batch<LOAD>(g, flat, it + step, lane, nxt);
        } else {
            load_batch<LOAD>(g, flat, it, lane, cur);
        }
        if constexpr (LOAD >= 2) {  // rows -> LDS (row r at r * 512), then lane-per-block rows
            const int p = lane & 31, h = lane >> 5;
#pragma unroll
            for (int j = 0; j < 4; ++j) *reinterpret_cast<u4v *>(ws + (2 * j + h) * 512 + p * 16) = cur[j];
            wsync();
            uint2 rw[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) rw[k] = *reinterpret_cast<const uint2 *>(ws + k * 512 + lane * 8);
#pragma unroll
            for (int j = 0; j < 4; ++j) cur[j] = u4v{rw[2 * j].x, rw[2 * j].y, rw[2 * j + 1].x, rw[2 * j + 1].y};
            wsync();
        }
        const int pl = it >= g.p[0].nbatch;
        const Plane &P = pl ? g.p[1] : g.p[0];
        const uint32_t lb = it - (pl ? g.p[0].nbatch : 0);
        const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(P.dst + (size_t)lb * 8192, 0, 8192, 0x00020000);
        u4v val[8];
        if constexpr (STAGE) {
            uint2 *mine = reinterpret_cast<uint2 *>(ws + lane * 136);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                mine[4 * j] = make_uint2(cur[j].x, cur[j].y);
                mine[4 * j + 1] = make_uint2(cur[j].y, cur[j].x);
                mine[4 * j + 2] = make_uint2(cur[j].z, cur[j].w);
                mine[4 * j + 3] = make_uint2(cur[j].w, cur[j].z);
            }
            if (PF) pin4(nxt);
            wsync();
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int m = k * 64 + lane, bl = m >> 3;
                const uint2 *s2 = reinterpret_cast<const uint2 *>(ws + bl * 136 + (m & 7) * 16);
                val[k] = u4v{s2[0].x, s2[0].y, s2[1].x, s2[1].y};
            }
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                val[j] = cur[j];
                val[j + 4] = cur[j] ^ u4v{1, 0, 0, 0};
            }
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {  // ORD 0: chunks 0..7; ORD 1: 0, 4, 1, 5, 2, 6, 3, 7 (dctq_diag_stream's order)
            const int k = ORD ? (i >> 1) + 4 * (i & 1) : i;
            __builtin_amdgcn_raw_buffer_store_b128(val[k], rc, lane * 16, k * 1024, 2);
        }
        if (STAGE) wsync();
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
    char *out1, *outY, *outC, *outZ;
    CHECK(hipMalloc(&src, ybytes + cbytes));
    CHECK(hipMalloc(&out1, nblk * 128));
    CHECK(hipMalloc(&outY, nby * 128));
    CHECK(hipMalloc(&outC, nbc * 128));
    CHECK(hipMalloc(&outZ, nblk * 128));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint32_t *)src, (ybytes + cbytes) / 4, 12345u);
    CHECK(hipDeviceSynchronize());
    Geo g2;
    g2.p[0] = Plane{src, outY, 480, 129600, 3840, (uint32_t)(ybytes / 4096), (size_t)3840 * 2160};
    g2.p[1] = Plane{src + ybytes, outC, 240, 32400, 1920, (uint32_t)(cbytes / 4096), (size_t)1920 * 1080};
    g2.nbatch = g2.p[0].nbatch + g2.p[1].nbatch;
    // g1: both planes' outputs in out1 (allocated right after the pixels, as dctq_diag_stream's
    // dst in this program); gz: in outZ (allocated last)
    Geo g1 = g2, gz = g2;
    g1.p[0].dst = out1;
    g1.p[1].dst = out1 + nby * 128;
    gz.p[0].dst = outZ;
    gz.p[1].dst = outZ + nby * 128;
    const u4v *flat = (const u4v *)src;
    dctq_plan *plan = nullptr;
    DCHECK(dctq_plan_create(50, 0, &plan));
    dctq_plane planes[2] = {{src, 3840, (long long)3840 * 2160, 3840, 2160, (int)FY},
                            {src + ybytes, 1920, (long long)1920 * 1080, 1920, 1080, (int)FC}};
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
        const dim3 gr(cus * 4 * m);
        const std::string x = " x" + std::to_string(m);
        items.push_back({"rows8  stage pf" + x, [=] { hipLaunchKernelGGL((k_move<0, 1, 1>), gr, dim3(256), 0, 0, g2, flat); }});
        items.push_back({"rows8  stage nopf" + x, [=] { hipLaunchKernelGGL((k_move<0, 1, 0>), gr, dim3(256), 0, 0, g2, flat); }});
        items.push_back({"flat16 stage nopf" + x, [=] { hipLaunchKernelGGL((k_move<1, 1, 0>), gr, dim3(256), 0, 0, g2, flat); }});
        items.push_back({"flat16 xpose stage nopf" + x, [=] { hipLaunchKernelGGL((k_move<3, 1, 0>), gr, dim3(256), 0, 0, g2, flat); }});
        items.push_back({"flat16 xpose stage pf" + x, [=] { hipLaunchKernelGGL((k_move<3, 1, 1>), gr, dim3(256), 0, 0, g2, flat); }});
        items.push_back({"pair16 stage nopf" + x, [=] { hipLaunchKernelGGL((k_move<2, 1, 0>), gr, dim3(256), 0, 0, g2, flat); }});
    }
    items.push_back({"fwd q50", [=] { DCHECK(dctq_forward_quant_planes(plan, planes, 2, c2, nullptr, nullptr)); }});
    items.push_back({"diag flat kind 7 (1 out)", [=] { DCHECK(dctq_diag_stream(7, src, out1, (long long)nblk / 64 * 64, nullptr)); }});
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
        printf("%-26s median %7.1f us %5.1f %% of 8 TB/s | min %7.1f\n", items[i].name.c_str(), med,
               bytes / (med * 1e-6) / 8e12 * 100.0, v[0]);
    }
    dctq_plan_destroy(plan);
    return 0;
}
