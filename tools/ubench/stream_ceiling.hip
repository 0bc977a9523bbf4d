// tools/ubench/stream_ceiling.hip -- memory-side speed of light for the DCT+quant
// traffic shape (read 64 B/block, write 128 B/block), no arithmetic:
//  A) lane-per-block: 8 x 8-byte row loads per lane (block addressing of a 4K plane
//     stack), LDS-staged 16-byte stores (the fdct8 v2 data movement, math removed);
//  B) same, but loads 16 B per lane (two blocks' rows) -- wider requests;
//  C) flat 1:2 stream: 16 B loads, 2 x 16 B stores per lane, grid-stride.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ __launch_bounds__(256) void kA(const uint8_t *src, int bw, int nblk, int per_frame, long long stride,
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
        for (int k = 0; k < 8; ++k) r[k] = *(const uint2 *)(p + k * stride);
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

__global__ __launch_bounds__(256) void kC(const uint4 *src, size_t n16, uint4 *dst) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, step = (size_t)gridDim.x * blockDim.x;
    for (; i < n16; i += step) {
        uint4 v = src[i];
        dst[2 * i] = v;
        dst[2 * i + 1] = make_uint4(v.x ^ 1, v.y, v.z, v.w);
    }
}

int main() {
    const int W = 3840, H = 2160, F = 64;
    const int bw = W / 8, per = bw * (H / 8), nblk = per * F;
    uint8_t *src; uint4 *dst;
    hipMalloc(&src, (size_t)W * H * F);
    hipMalloc(&dst, (size_t)nblk * 128);
    hipMemset(src, 7, (size_t)W * H * F);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    double bytes = (double)nblk * 192;
    for (int grid : {1024, 2048, 4096}) {
        float best = 1e9;
        for (int rep = 0; rep < 6; ++rep) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(kA, dim3(grid), dim3(256), 0, 0, src, bw, nblk, per, (long long)W, (long long)W * H, dst);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;
        }
        printf("A lane-per-block pattern grid=%d: %.1f us  %.0f GB/s\n", grid, best * 1e3, bytes / best / 1e6);
    }
    for (int grid : {1024, 2048, 4096, 8192}) {
        float best = 1e9;
        for (int rep = 0; rep < 6; ++rep) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(kC, dim3(grid), dim3(256), 0, 0, (const uint4 *)src, (size_t)nblk * 64 / 16, dst);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;
        }
        printf("C flat 1:2 stream grid=%d: %.1f us  %.0f GB/s\n", grid, best * 1e3, bytes / best / 1e6);
    }
    return 0;
}
