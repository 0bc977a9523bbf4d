// tools/ubench/stream_vs_valu.hip -- the fdct8 v2 data movement (nt row loads,
// LDS-staged 1 KiB stores) plus N dependent-free fp32 FMAs per block (per lane),
// to see how VALU load trades against HBM throughput on gfx950.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef unsigned int u2v __attribute__((ext_vector_type(2)));

template <int N>
__global__ __launch_bounds__(256) void kW(const uint8_t *src, int bw, int nblk, int per_frame, long long stride,
                                          long long fstride, uint4 *dst) {
    __shared__ uint2 st[256 * 17];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int nb = (nblk + 63) / 64, step = gridDim.x * 4;
    for (int b = blockIdx.x * 4 + wv; b < nb; b += step) {
        int n = b * 64 + lane;
        int f = n / per_frame, rem = n - f * per_frame, by = rem / bw, bx = rem - by * bw;
        const uint8_t *p = src + f * fstride + (long long)by * 8 * stride + bx * 8;
        uint2 r[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) { u2v t = __builtin_nontemporal_load((const u2v *)(p + k * stride)); r[k] = make_uint2(t.x, t.y); }
        float a[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] = __uint_as_float(r[k].x & 0x3fffffff);
#pragma unroll
        for (int i = 0; i < N / 8; ++i)
#pragma unroll
            for (int k = 0; k < 8; ++k) a[k] = __builtin_fmaf(a[k], 1.0001f, a[(k + 1) & 7]);
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k].y ^= __float_as_uint(a[k]);
        uint2 *mine = st + (wv * 64 + lane) * 17;
#pragma unroll
        for (int k = 0; k < 8; ++k) { mine[2 * k] = r[k]; mine[2 * k + 1] = make_uint2(r[k].x ^ 1, r[k].y); }
        __builtin_amdgcn_wave_barrier();
        uint4 *d = dst + (size_t)b * 512;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            int m = k * 64 + lane, bl = m >> 3;
            uint2 lo = st[(wv * 64 + bl) * 17 + (m & 7) * 2], hi = st[(wv * 64 + bl) * 17 + (m & 7) * 2 + 1];
            d[m] = make_uint4(lo.x, lo.y, hi.x, hi.y);
        }
    }
}

#define RUN(N)                                                                                            \
    {                                                                                                     \
        float best = 1e9;                                                                                 \
        for (int rep = 0; rep < 8; ++rep) {                                                               \
            hipEventRecord(e0);                                                                           \
            hipLaunchKernelGGL(kW<N>, dim3(1024), dim3(256), 0, 0, src, bw, nblk, per, (long long)W, (long long)W * H, dst); \
            hipEventRecord(e1); hipEventSynchronize(e1);                                                  \
            float ms; hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;                         \
        }                                                                                                 \
        printf("N=%5d fma/lane/batch (%.0f VALU cyc/wave at 2.4):  %7.1f us  %6.0f GB/s\n", N, N * 2.4, best * 1e3, (double)nblk * 192 / best / 1e6); \
    }

int main() {
    const int W = 3840, H = 2160, F = 64;
    const int bw = W / 8, per = bw * (H / 8), nblk = per * F;
    uint8_t *src; uint4 *dst;
    hipMalloc(&src, (size_t)W * H * F);
    hipMalloc(&dst, (size_t)nblk * 128);
    hipMemset(src, 7, (size_t)W * H * F);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    RUN(0) RUN(256) RUN(512) RUN(768) RUN(1024) RUN(1280) RUN(1536) RUN(2048)
    return 0;
}
