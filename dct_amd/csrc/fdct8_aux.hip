// dct_amd/csrc/fdct8_aux.hip -- synth_kernel: the counter-based synthetic frame
// generator (bench inputs made on the device; the oracle regenerates any frame on
// the host).  The lane-per-block fp64 float-forward / inverse kernels that used to
// live here are the diagnostic library's variant 1 now (fdct8_diag.hip).
#include "dctq_internal.h"

namespace dctq {

// ---------------------------------------------------------------------------
// Synthetic frames: the same counter-based splitmix64 as oracle/dct_oracle.c
// (orc_synth_pixel); integer-only so host and device agree bit for bit.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t splitmix(uint64_t seed, uint64_t i) { return mix64(seed + (i + 1) * 0x9E3779B97F4A7C15ULL); }

__device__ __forceinline__ uint32_t synth_pixel(uint64_t seed, int kind, int width, int x, int y) {
    const uint64_t idx = (uint64_t)y * (uint64_t)width + (uint64_t)x;
    switch (kind) {
    case 0:
        return (uint32_t)(splitmix(seed, idx) & 0xFF);
    case 1: {
        const int cx = x >> 4, cy = y >> 4, fx = x & 15, fy = y & 15;
        const uint64_t s2 = seed ^ 0x5DEECE66DULL;
        const int gw = (width >> 4) + 2;
        const int v00 = (int)(splitmix(s2, (uint64_t)cy * gw + cx) & 0xFF);
        const int v01 = (int)(splitmix(s2, (uint64_t)cy * gw + cx + 1) & 0xFF);
        const int v10 = (int)(splitmix(s2, (uint64_t)(cy + 1) * gw + cx) & 0xFF);
        const int v11 = (int)(splitmix(s2, (uint64_t)(cy + 1) * gw + cx + 1) & 0xFF);
        const int top = v00 * (16 - fx) + v01 * fx, bot = v10 * (16 - fx) + v11 * fx;
        int v = (top * (16 - fy) + bot * fy + 128) >> 8;
        v += (int)(splitmix(seed, idx) & 7) - 3;
        return (uint32_t)(v < 0 ? 0 : v > 255 ? 255 : v);
    }
    case 2: {
        const uint64_t b = (uint64_t)(y >> 3) * (uint64_t)((width + 7) >> 3) + (uint64_t)(x >> 3);
        return (uint32_t)(splitmix(seed, b) & 0xFF);
    }
    default:
        return (splitmix(seed, idx) & 1) ? 255u : 0u;
    }
}

__global__ void synth_kernel(uint64_t seed, int kind, uint8_t *dst, long long stride, long long frame_stride,
                             int width, int height) {
    const int x4 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
    const int y = blockIdx.y;
    const int f = blockIdx.z;
    if (x4 >= width) return;
    uint32_t w = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) w |= synth_pixel(seed + f, kind, width, x4 + k, y) << (8 * k);
    *reinterpret_cast<uint32_t *>(dst + (long long)f * frame_stride + (long long)y * stride + x4) = w;
}

hipError_t launch_synth(uint64_t seed, int kind, uint8_t *dst, long long stride, long long frame_stride, int width,
                        int height, int nframes, hipStream_t stream) {
    const dim3 block(256), grid((width / 4 + 255) / 256, height, nframes);
    hipLaunchKernelGGL(synth_kernel, grid, block, 0, stream, seed, kind, dst, stride, frame_stride, width, height);
    return hipGetLastError();
}

}  // namespace dctq
