// tools/ubench/hbm_mix4.hip -- where do the 2-3 points between a flat 1:2
// stream (hbm_mix2: 71-73 % of 8 TB/s) and the forward kernel's row-form
// movement (68 %) go?  One persistent grid-stride kernel (4 WG/CU), per
// 64-block batch 4 KiB read / 8 KiB written, combinations of
//   LOAD 0: flat, 4 x 16 B per lane (1 KiB contiguous per instruction)
//   LOAD 1: pixel rows, 8 x 8 B per lane (lane-per-block, 512 B per instruction)
//   LOAD 2: pixel rows as 4 x 16 B per lane (2 rows x 512 B per instruction)
//   STAGE 0: stores straight from the loaded registers (flat only)
//   STAGE 1: through the per-wave LDS stage (136-B pitch), vmcnt(0) first
//   AUX: store policy 0 plain / 2 nt (loads are nt)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench/hbm_mix4 tools/ubench/hbm_mix4.hip
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

__device__ __forceinline__ const uint8_t *blk(const Geo &g, uint32_t n) {
    const uint32_t f = n / g.per_frame, rem = n - f * g.per_frame, by = rem / g.bw, bx = rem - by * g.bw;
    return g.src + f * g.fstride + (size_t)by * 8 * g.stride + bx * 8;
}

template <int LOAD, int STAGE, int AUX>
__global__ __launch_bounds__(256) void k_mx(Geo g, char *coef, uint32_t nb) {
    __shared__ uint4 st[256 * 136 / 16];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    char *ws = reinterpret_cast<char *>(st) + wv * 8704;
    for (uint32_t b = blockIdx.x * 4 + wv; b < nb; b += gridDim.x * 4) {
        const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(coef + (size_t)b * 8192, 0, 8192, 0x00020000);
        if (LOAD == 0) {
            u4v v[4];
            const u4v *in = reinterpret_cast<const u4v *>(g.src) + (size_t)b * 256;
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = __builtin_nontemporal_load(in + k * 64 + lane);
            if (STAGE == 0) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    __builtin_amdgcn_raw_buffer_store_b128(v[k], rc, lane * 16, k * 1024, AUX);
                    __builtin_amdgcn_raw_buffer_store_b128(v[k] ^ u4v{1, 0, 0, 0}, rc, lane * 16, (k + 4) * 1024, AUX);
                }
                continue;
            }
            __builtin_amdgcn_s_waitcnt(0x0F70);
            u4v *mine = reinterpret_cast<u4v *>(ws + lane * 136);
            // 8 x 8 B per lane = 4 x 16 B; write as 16-B pairs at the 136-B pitch (b64 writes)
            uint2 *m2 = reinterpret_cast<uint2 *>(mine);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                m2[4 * k] = make_uint2(v[k].x, v[k].y);
                m2[4 * k + 1] = make_uint2(v[k].z, v[k].w);
                m2[4 * k + 2] = make_uint2(v[k].x ^ 1, v[k].y);
                m2[4 * k + 3] = make_uint2(v[k].z, v[k].w);
            }
        } else {
            uint2 r[8];
            if (LOAD == 1) {
                const uint8_t *p = blk(g, b * 64 + lane);
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const u2v t = __builtin_nontemporal_load((const u2v *)(p + k * g.stride));
                    r[k] = make_uint2(t.x, t.y);
                }
            } else {
                // lane l: blocks 2(l&31), 2(l&31)+1 of pixel row 2k + (l>>5), redistributed via LDS
                const uint8_t *p = blk(g, b * 64 + 2 * (lane & 31)) + (lane >> 5) * g.stride;
                u4v t[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) t[k] = __builtin_nontemporal_load((const u4v *)(p + 2 * k * g.stride));
                __builtin_amdgcn_s_waitcnt(0x0F70);
                char *wi = ws;  // 4 KiB input image in the stage area (read before the stage is written)
#pragma unroll
                for (int k = 0; k < 4; ++k) *reinterpret_cast<u4v *>(wi + k * 1024 + lane * 16) = t[k];
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int k = 0; k < 8; ++k) r[k] = *reinterpret_cast<const uint2 *>(wi + k * 512 + lane * 8);
                __builtin_amdgcn_s_waitcnt(0xC07F);
                __builtin_amdgcn_wave_barrier();
            }
            __builtin_amdgcn_s_waitcnt(0x0F70);
            uint2 *mine = reinterpret_cast<uint2 *>(ws + lane * 136);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                mine[2 * k] = r[k];
                mine[2 * k + 1] = make_uint2(r[k].x ^ 1, r[k].y);
            }
        }
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
#pragma unroll
        for (int k = 0; k < 8; ++k) __builtin_amdgcn_raw_buffer_store_b128(val[k], rc, lane * 16, k * 1024, AUX);
    }
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
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
#define MX(L, S, A) [&] { hipLaunchKernelGGL((k_mx<L, S, A>), dim3(cus * 4), dim3(256), 0, 0, g, dst, nb); }
    std::vector<Item> items = {
        {"flat16 direct  nt", MX(0, 0, 2)}, {"flat16 direct  plain", MX(0, 0, 0)},
        {"flat16 staged  nt", MX(0, 1, 2)}, {"flat16 staged  plain", MX(0, 1, 0)},
        {"rows8  staged  nt", MX(1, 1, 2)}, {"rows8  staged  plain", MX(1, 1, 0)},
        {"rows16 staged  nt", MX(2, 1, 2)}, {"rows16 staged  plain", MX(2, 1, 0)},
    };
    // steady state (profiles/r02/clock_ramp.md, policy_b2b.md): ~300 launches of clock pre-warm, then
    // per sample one untimed launch of the same case followed by B2B timed launches back to back
    const int B2B = argc > 2 ? atoi(argv[2]) : 1;
    for (int w = 0; w < (B2B > 1 ? 300 : 1); ++w) items[w % items.size()].fn();
    CHECK(hipDeviceSynchronize());
    std::vector<std::vector<float>> ms(items.size());
    for (int r = 0; r < reps; ++r)
        for (size_t i = 0; i < items.size(); ++i) {
            if (B2B > 1) items[i].fn();
            CHECK(hipEventRecord(e0));
            for (int k = 0; k < B2B; ++k) items[i].fn();
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float t;
            CHECK(hipEventElapsedTime(&t, e0, e1));
            ms[i].push_back(t / B2B);
        }
    CHECK(hipGetLastError());
    for (size_t i = 0; i < items.size(); ++i) {
        std::vector<float> v = ms[i];
        std::sort(v.begin(), v.end());
        printf("%-22s median %7.1f us %5.1f %% |", items[i].name, v[v.size() / 2] * 1e3, b12 / v[v.size() / 2] / 1e6 / 80.0);
        for (float t : v) printf(" %.1f", b12 / t / 1e6 / 80.0);
        printf("\n");
    }
    return 0;
}
