// dct_amd/csrc/fdct8_aux.hip -- the other batched 8x8 kernels:
//   * fdct8_float_kernel: forward DCT to float coefficients (dct_forward,
//     src/dct.c:52-77, without quantization), fp64 butterfly, one fp32 rounding.
//   * idct8_kernel: dequantize (src/quantization.c:133-151, incl. the
//     non-adaptive 1/Q multiplier) + dct_inverse (src/dct.c:80-105) + 128.
//   * synth_kernel: the counter-based synthetic frame generator.
// Same lane-per-block layout as fdct8.hip.
#include "aan_f64.h"
#include "dctq_internal.h"

namespace dctq {

constexpr int kThreadsAux = 256;

__global__ __launch_bounds__(kThreadsAux) void fdct8_float_kernel(PlaneArgs p, const DevTables *__restrict__ dev,
                                                                  float *__restrict__ coef) {
    const uint32_t n = blockIdx.x * kThreadsAux + threadIdx.x;
    if (n >= (uint32_t)p.nblk) return;
    const uint32_t f = fdiv(n, p.div_frame);
    const uint32_t rem = n - f * (uint32_t)p.nblk_frame;
    const uint32_t by = fdiv(rem, p.div_bw), bx = rem - by * (uint32_t)p.bw;
    const uint8_t *px = p.src + (long long)f * p.frame_stride + (long long)(by * 8) * p.stride + (long long)bx * 8;
    double v[8][8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const uint2 row = *reinterpret_cast<const uint2 *>(px + r * p.stride);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            v[r][k] = (double)((row.x >> (8 * k)) & 0xFFu) - 128.0;
            v[r][k + 4] = (double)((row.y >> (8 * k)) & 0xFFu) - 128.0;
        }
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) aan8_d(v[r][0], v[r][1], v[r][2], v[r][3], v[r][4], v[r][5], v[r][6], v[r][7]);
#pragma unroll
    for (int c = 0; c < 8; ++c) aan8_d(v[0][c], v[1][c], v[2][c], v[3][c], v[4][c], v[5][c], v[6][c], v[7][c]);
    float4 *dst = reinterpret_cast<float4 *>(coef + (size_t)n * 64);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int c = 4 * q;
        dst[q] = make_float4((float)(v[c >> 3][c & 7] * dev->s2[c]), (float)(v[(c + 1) >> 3][(c + 1) & 7] * dev->s2[c + 1]),
                             (float)(v[(c + 2) >> 3][(c + 2) & 7] * dev->s2[c + 2]),
                             (float)(v[(c + 3) >> 3][(c + 3) & 7] * dev->s2[c + 3]));
    }
}

template <bool ADAPTIVE>
__global__ __launch_bounds__(kThreadsAux) void idct8_kernel(const DevTables *__restrict__ dev,
                                                            const int16_t *__restrict__ coef,
                                                            const int32_t *__restrict__ var_num, long long nblk,
                                                            float *__restrict__ recon) {
    const long long n = (long long)blockIdx.x * kThreadsAux + threadIdx.x;
    if (n >= nblk) return;
    const int4 *src = reinterpret_cast<const int4 *>(coef + n * 64);
    double v[8][8];
    // dequantize and fold the A^T input scale S_i S_j:
    //   non-adaptive: q * (1/Q)            (src/quantization.c:139,144 -- reference semantics)
    //   adaptive:     q * Q * (2 - nv), DC: q * Q  (= q * 1.0/M of :137,144,193)
    double sc = 1.0;
    if (ADAPTIVE) {
        const double var = (double)var_num[n] / 4096.0;
        sc = 2.0 - fmin(1.0, fmax(0.1, var / 1000.0));
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int4 w = src[q];
        const int32_t ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            const int c = 8 * q + 2 * h;
            const double lo = (double)(int16_t)(ww[h] & 0xFFFF), hi = (double)(int16_t)((uint32_t)ww[h] >> 16);
            if (ADAPTIVE) {
                v[c >> 3][c & 7] = lo * dev->qscale[c] * (c == 0 ? 1.0 : sc);
                v[(c + 1) >> 3][(c + 1) & 7] = hi * dev->qscale[c + 1] * sc;
            } else {
                v[c >> 3][c & 7] = lo * dev->iscale[c];
                v[(c + 1) >> 3][(c + 1) & 7] = hi * dev->iscale[c + 1];
            }
        }
    }
#pragma unroll
    for (int c = 0; c < 8; ++c) aan8t_d(v[0][c], v[1][c], v[2][c], v[3][c], v[4][c], v[5][c], v[6][c], v[7][c]);
#pragma unroll
    for (int r = 0; r < 8; ++r) aan8t_d(v[r][0], v[r][1], v[r][2], v[r][3], v[r][4], v[r][5], v[r][6], v[r][7]);
    float4 *dst = reinterpret_cast<float4 *>(recon + n * 64);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int c = 4 * q;
        dst[q] = make_float4((float)(v[c >> 3][c & 7] + 128.0), (float)(v[(c + 1) >> 3][(c + 1) & 7] + 128.0),
                             (float)(v[(c + 2) >> 3][(c + 2) & 7] + 128.0), (float)(v[(c + 3) >> 3][(c + 3) & 7] + 128.0));
    }
}

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

hipError_t launch_fdct8_float(const PlaneArgs &p, const DevTables *dev, float *coef, hipStream_t stream) {
    hipLaunchKernelGGL(fdct8_float_kernel, dim3((p.nblk + kThreadsAux - 1) / kThreadsAux), dim3(kThreadsAux), 0,
                       stream, p, dev, coef);
    return hipGetLastError();
}

hipError_t launch_idct8(const DevTables *dev, int adaptive, const int16_t *coef, const int32_t *var_num,
                        long long nblk, float *recon, hipStream_t stream) {
    const dim3 grid((unsigned)((nblk + kThreadsAux - 1) / kThreadsAux)), block(kThreadsAux);
    if (adaptive)
        hipLaunchKernelGGL(idct8_kernel<true>, grid, block, 0, stream, dev, coef, var_num, nblk, recon);
    else
        hipLaunchKernelGGL(idct8_kernel<false>, grid, block, 0, stream, dev, coef, var_num, nblk, recon);
    return hipGetLastError();
}

hipError_t launch_synth(uint64_t seed, int kind, uint8_t *dst, long long stride, long long frame_stride, int width,
                        int height, int nframes, hipStream_t stream) {
    const dim3 block(256), grid((width / 4 + 255) / 256, height, nframes);
    hipLaunchKernelGGL(synth_kernel, grid, block, 0, stream, seed, kind, dst, stride, frame_stride, width, height);
    return hipGetLastError();
}

}  // namespace dctq
