// tools/ubench/loop_order.hip -- loop orderings for a prefetching streaming
// kernel on gfx950 with ~2.5K cycles of VALU per 64-block batch:
//  P: prefetch next batch's rows at the top, stage + store at the end (fdct8 v2)
//  D: deferred stores -- at the top store the PREVIOUS batch from the LDS stage,
//     then prefetch, compute, stage (stores retire a whole batch before the wait)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef unsigned int u2v __attribute__((ext_vector_type(2)));
typedef unsigned int u4v __attribute__((ext_vector_type(4)));
constexpr int NF = 1024;

__device__ __forceinline__ void ld(const uint8_t *src, int n, int nblk, int bw, int per, long long stride, long long fs, uint2 (&r)[8]) {
    n = n < nblk ? n : 0;
    int f = n / per, rem = n - f * per, by = rem / bw, bx = rem - by * bw;
    const uint8_t *p = src + f * fs + (long long)by * 8 * stride + bx * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) { u2v t = __builtin_nontemporal_load((const u2v *)(p + k * stride)); r[k] = make_uint2(t.x, t.y); }
}
__device__ __forceinline__ void work(uint2 (&r)[8], uint2 *mine) {
    float a[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = __uint_as_float(r[k].x & 0x3fffffff);
#pragma unroll
    for (int i = 0; i < NF / 8; ++i)
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] = __builtin_fmaf(a[k], 1.0001f, a[(k + 1) & 7]);
#pragma unroll
    for (int k = 0; k < 8; ++k) { mine[2 * k] = make_uint2(r[k].x, r[k].y ^ __float_as_uint(a[k])); mine[2 * k + 1] = r[k]; }
}
__device__ __forceinline__ void store(const uint2 *st, int wv, int lane, uint32_t b, int nblk, int16_t *dst) {
    uint32_t left = nblk - b * 64, bytes = (left < 64 ? left : 64) * 128;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((char *)dst + (size_t)b * 8192, (short)0, (int)bytes, 0x00020000);
    u4v val[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        int m = k * 64 + lane, bl = m >> 3;
        uint2 lo = st[(wv * 64 + bl) * 17 + (m & 7) * 2], hi = st[(wv * 64 + bl) * 17 + (m & 7) * 2 + 1];
        val[k] = u4v{lo.x, lo.y, hi.x, hi.y};
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) __builtin_amdgcn_raw_buffer_store_b128(val[k], rs, lane * 16, k * 1024, 0);
}

__global__ __launch_bounds__(256, 4) void kP(const uint8_t *src, int bw, int nblk, int per, long long stride, long long fs, int16_t *dst) {
    __shared__ uint2 st[256 * 17];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t nb = (nblk + 63) / 64, step = gridDim.x * 4;
    uint32_t b = blockIdx.x * 4 + wv;
    uint2 nxt[8];
    ld(src, b * 64 + lane, nblk, bw, per, stride, fs, nxt);
    for (; b < nb; b += step) {
        uint2 cur[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) cur[k] = nxt[k];
        ld(src, (b + step) * 64 + lane, nblk, bw, per, stride, fs, nxt);
        work(cur, st + (wv * 64 + lane) * 17);
        __builtin_amdgcn_wave_barrier();
        store(st, wv, lane, b, nblk, dst);
    }
}
__global__ __launch_bounds__(256, 4) void kD(const uint8_t *src, int bw, int nblk, int per, long long stride, long long fs, int16_t *dst) {
    __shared__ uint2 st[256 * 17];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t nb = (nblk + 63) / 64, step = gridDim.x * 4;
    uint32_t b = blockIdx.x * 4 + wv;
    uint2 nxt[8];
    ld(src, b * 64 + lane, nblk, bw, per, stride, fs, nxt);
    bool have = false;
    uint32_t prev = 0;
    for (; b < nb; b += step) {
        if (have) store(st, wv, lane, prev, nblk, dst);   // previous batch leaves first
        uint2 cur[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) cur[k] = nxt[k];
        ld(src, (b + step) * 64 + lane, nblk, bw, per, stride, fs, nxt);
        work(cur, st + (wv * 64 + lane) * 17);
        __builtin_amdgcn_wave_barrier();
        have = true;
        prev = b;
    }
    if (have) store(st, wv, lane, prev, nblk, dst);
}

int main() {
    const int W = 3840, H = 2160, F = 64;
    const int bw = W / 8, per = bw * (H / 8), nblk = per * F;
    uint8_t *src; int16_t *dst;
    hipMalloc(&src, (size_t)W * H * F);
    hipMalloc(&dst, (size_t)nblk * 128);
    hipMemset(src, 7, (size_t)W * H * F);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int rep = 0; rep < 3; ++rep)
    for (int which = 0; which < 2; ++which) {
        float best = 1e9;
        for (int i = 0; i < 6; ++i) {
            hipEventRecord(e0);
            if (which == 0) hipLaunchKernelGGL(kP, dim3(1024), dim3(256), 0, 0, src, bw, nblk, per, (long long)W, (long long)W * H, dst);
            else hipLaunchKernelGGL(kD, dim3(1024), dim3(256), 0, 0, src, bw, nblk, per, (long long)W, (long long)W * H, dst);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;
        }
        printf("%s  %7.1f us  %6.0f GB/s\n", which ? "D deferred stores" : "P prefetch/store ", best * 1e3, (double)nblk * 192 / best / 1e6);
    }
    return 0;
}
