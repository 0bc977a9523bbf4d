#pragma clang diagnostic ignored "-Wunused-value"
// tools/ubench/stream_ceiling3.hip -- memory ceiling of the fused round trip's
// traffic (64 B in, 128 + 256 B out per block) with no math: lane-per-block nt
// row loads, LDS-staged 1 KiB nt stores for the int16 and fp32 outputs, same
// persistent grid and occupancy as roundtrip8; plus the ideal coalesced 1:6 stream.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef unsigned int u2v __attribute__((ext_vector_type(2)));
typedef unsigned int u4v __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256, 4) void kRT(const uint8_t *src, int bw, int nblk, int per_frame, long long stride,
                                              long long fstride, char *coef, char *recon) {
    __shared__ uint4 st[256 * 136 / 16];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nb = (nblk + 63) / 64, step = gridDim.x * 4;
    char *ws = reinterpret_cast<char *>(st) + wv * 8704;
    for (int b = blockIdx.x * 4 + wv; b < nb; b += step) {
        int n = b * 64 + lane;
        int f = n / per_frame, rem = n - f * per_frame, by = rem / bw, bx = rem - by * bw;
        const uint8_t *p = src + f * fstride + (long long)by * 8 * stride + bx * 8;
        uint2 r[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) { u2v t = __builtin_nontemporal_load((const u2v *)(p + k * stride)); r[k] = make_uint2(t.x, t.y); }
        uint2 *mine = reinterpret_cast<uint2 *>(ws + lane * 136);
#pragma unroll
        for (int k = 0; k < 8; ++k) { mine[2 * k] = r[k]; mine[2 * k + 1] = make_uint2(r[k].x ^ 1, r[k].y); }
        __builtin_amdgcn_s_waitcnt(0x0F70);
        __builtin_amdgcn_wave_barrier();
        const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(coef + (size_t)b * 8192, 0, 8192, 0x00020000);
        u4v val[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            int m = k * 64 + lane, bl = m >> 3;
            const uint2 *s2 = reinterpret_cast<const uint2 *>(ws + bl * 136 + (m & 7) * 16);
            val[k] = u4v{s2[0].x, s2[0].y, s2[1].x, s2[1].y};
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) __builtin_amdgcn_raw_buffer_store_b128(val[k], rc, lane * 16, k * 1024, 2);
        // two 8 KiB recon halves from the same stage (content irrelevant)
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            __builtin_amdgcn_s_waitcnt(0x0F70);
            __builtin_amdgcn_wave_barrier();
            const __amdgpu_buffer_rsrc_t rr =
                __builtin_amdgcn_make_buffer_rsrc(recon + (size_t)b * 16384 + half * 8192, 0, 8192, 0x00020000);
            u4v rv[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int bl = 4 * k + (lane >> 4);
                const uint4 t = *reinterpret_cast<const uint4 *>(ws + bl * 272 + (lane & 15) * 16);
                rv[k] = u4v{t.x ^ half, t.y, t.z, t.w};
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) __builtin_amdgcn_raw_buffer_store_b128(rv[k], rr, lane * 16, k * 1024, 2);
        }
    }
}

template <int R>
__global__ __launch_bounds__(256) void kD(const uint4 *src, size_t n16, uint4 *dst) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, step = (size_t)gridDim.x * blockDim.x;
    for (; i < n16; i += step) {
        const u4v v = __builtin_nontemporal_load((const u4v *)(src + i));
#pragma unroll
        for (int r = 0; r < R; ++r)
            __builtin_nontemporal_store((u4v){v.x ^ r, v.y, v.z, v.w}, (u4v *)(dst + r * n16 + i));
    }
}

#define TIME(label, bytes, launch)                                                         \
    {                                                                                      \
        float best = 1e9;                                                                  \
        for (int rep = 0; rep < 8; ++rep) {                                                \
            hipEventRecord(e0); launch; hipEventRecord(e1); hipEventSynchronize(e1);       \
            float ms; hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;           \
        }                                                                                  \
        printf("%-48s %8.1f us %7.0f GB/s %5.1f %%\n", label, best * 1e3, (bytes) / best / 1e6,   \
               (bytes) / best / 1e6 / 80.0);                                               \
    }

int main() {
    const int W = 3840, H = 2160, F = 64;
    const int bw = W / 8, per = bw * (H / 8), nblk = per * F;
    uint8_t *src; char *coef, *recon;
    hipMalloc(&src, (size_t)W * H * F);
    hipMalloc(&coef, (size_t)nblk * 128 + 8192);
    hipMalloc(&recon, (size_t)nblk * 256 + 16384);
    char *big;
    hipMalloc(&big, (size_t)nblk * 384);
    hipMemset(src, 7, (size_t)W * H * F);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    int ncu = 256;
    const double bytes = (double)nblk * 448;
    TIME("roundtrip pattern (no math), 4 WG/CU", bytes,
         hipLaunchKernelGGL(kRT, dim3(ncu * 4), dim3(256), 0, 0, src, bw, nblk, per, (long long)W,
                            (long long)W * H, coef, recon));
    const size_t n16 = (size_t)nblk * 64 / 16;
    TIME("ideal coalesced 1:6 (16 B in, 6 x 16 B out)", (double)n16 * 16 * 7,
         hipLaunchKernelGGL(kD<6>, dim3(ncu * 8), dim3(256), 0, 0, (const uint4 *)src, n16, (uint4 *)big));
    return 0;
}
