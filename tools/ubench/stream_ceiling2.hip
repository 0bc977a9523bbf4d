// tools/ubench/stream_ceiling2.hip -- what limits the 64 B-in / 128 B-out stream:
// cache policy of the loads/stores, and the read:write mix.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef unsigned int u2v __attribute__((ext_vector_type(2)));
typedef unsigned int u4v __attribute__((ext_vector_type(4)));

template <int NTL, int NTS>
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
        for (int k = 0; k < 8; ++k) {
            if (NTL) { u2v t = __builtin_nontemporal_load((const u2v *)(p + k * stride)); r[k] = make_uint2(t.x, t.y); }
            else r[k] = *(const uint2 *)(p + k * stride);
        }
        uint2 *mine = st + (wv * 64 + lane) * 17;
#pragma unroll
        for (int k = 0; k < 8; ++k) { mine[2 * k] = r[k]; mine[2 * k + 1] = make_uint2(r[k].x ^ 1, r[k].y); }
        __builtin_amdgcn_wave_barrier();
        uint4 *d = dst + (size_t)b * 512;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            int m = k * 64 + lane, bl = m >> 3;
            uint2 lo = st[(wv * 64 + bl) * 17 + (m & 7) * 2], hi = st[(wv * 64 + bl) * 17 + (m & 7) * 2 + 1];
            uint4 v = make_uint4(lo.x, lo.y, hi.x, hi.y);
            if (NTS) __builtin_nontemporal_store((u4v){v.x, v.y, v.z, v.w}, (u4v *)(d + m)); else d[m] = v;
        }
    }
}

// ideal 1:R stream: coalesced 16 B loads, R coalesced 16 B stores into R separate regions
template <int R, int NTS>
__global__ __launch_bounds__(256) void kD(const uint4 *src, size_t n16, uint4 *dst) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, step = (size_t)gridDim.x * blockDim.x;
    for (; i < n16; i += step) {
        uint4 v = src[i];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            uint4 w = make_uint4(v.x ^ r, v.y, v.z, v.w);
            if (NTS) __builtin_nontemporal_store((u4v){w.x, w.y, w.z, w.w}, (u4v *)(dst + r * n16 + i)); else dst[r * n16 + i] = w;
        }
    }
}
__global__ __launch_bounds__(256) void kRead(const uint4 *src, size_t n16, uint32_t *out) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, step = (size_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    for (; i < n16; i += step) { uint4 v = src[i]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
    if (acc == 0x12345678) out[0] = acc;
}
__global__ __launch_bounds__(256) void kWrite(uint4 *dst, size_t n16) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, step = (size_t)gridDim.x * blockDim.x;
    for (; i < n16; i += step) dst[i] = make_uint4(i, 1, 2, 3);
}

#define TIME(label, bytes, launch)                                                         \
    {                                                                                      \
        float best = 1e9;                                                                  \
        for (int rep = 0; rep < 6; ++rep) {                                                \
            hipEventRecord(e0); launch; hipEventRecord(e1); hipEventSynchronize(e1);       \
            float ms; hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;           \
        }                                                                                  \
        printf("%-40s %8.1f us %7.0f GB/s\n", label, best * 1e3, (bytes) / best / 1e6);    \
    }

int main() {
    const int W = 3840, H = 2160, F = 64;
    const int bw = W / 8, per = bw * (H / 8), nblk = per * F;
    uint8_t *src; uint4 *dst; uint32_t *o;
    hipMalloc(&src, (size_t)W * H * F);
    hipMalloc(&dst, (size_t)nblk * 128 * 2);
    hipMalloc(&o, 64);
    hipMemset(src, 7, (size_t)W * H * F);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const double b192 = (double)nblk * 192;
    const size_t n16 = (size_t)nblk * 64 / 16;
    const int g = 2048;
    TIME("A  (plain loads, plain stores)", b192, hipLaunchKernelGGL((kA<0, 0>), dim3(g), dim3(256), 0, 0, src, bw, nblk, per, (long long)W, (long long)W * H, dst));
    TIME("A  nt stores", b192, hipLaunchKernelGGL((kA<0, 1>), dim3(g), dim3(256), 0, 0, src, bw, nblk, per, (long long)W, (long long)W * H, dst));
    TIME("A  nt loads", b192, hipLaunchKernelGGL((kA<1, 0>), dim3(g), dim3(256), 0, 0, src, bw, nblk, per, (long long)W, (long long)W * H, dst));
    TIME("A  nt loads + nt stores", b192, hipLaunchKernelGGL((kA<1, 1>), dim3(g), dim3(256), 0, 0, src, bw, nblk, per, (long long)W, (long long)W * H, dst));
    TIME("D  1:2 coalesced", b192, hipLaunchKernelGGL((kD<2, 0>), dim3(g), dim3(256), 0, 0, (const uint4 *)src, n16, dst));
    TIME("D  1:2 coalesced nt stores", b192, hipLaunchKernelGGL((kD<2, 1>), dim3(g), dim3(256), 0, 0, (const uint4 *)src, n16, dst));
    TIME("D  1:1 copy", (double)nblk * 128, hipLaunchKernelGGL((kD<1, 0>), dim3(g), dim3(256), 0, 0, (const uint4 *)src, n16, dst));
    TIME("read only", (double)nblk * 64, hipLaunchKernelGGL(kRead, dim3(g), dim3(256), 0, 0, (const uint4 *)src, n16, o));
    TIME("write only", (double)nblk * 128, hipLaunchKernelGGL(kWrite, dim3(g), dim3(256), 0, 0, dst, n16 * 2));
    return 0;
}
