#pragma clang diagnostic ignored "-Wunused-value"
#pragma clang diagnostic ignored "-Wunused-result"
// tools/ubench/stream_ceiling4.hip -- the write side of the 64 B-in / 128 B-out
// stream: what write pattern gets closest to the HBM peak, and does it carry
// over to the lane-per-block 1:2 mix of fdct8_quant_v2 (no math)?
//   W*: write-only sweeps of 1.06 GB (the coefficient array of 64 4K luma planes)
//   M*: the v2 data movement (8 x 8 B nt row loads per lane, LDS stage,
//       8 x 1 KiB stores per 64-block batch) under mappings / policies
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench/stream_ceiling4 tools/ubench/stream_ceiling4.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
typedef unsigned int u2v __attribute__((ext_vector_type(2)));
typedef unsigned int u4v __attribute__((ext_vector_type(4)));

// batch index for wave `w` (of TW) at iteration `it`; MAP 0 = grid-stride,
// MAP 1 = each XCD (WG % 8) sweeps a contiguous 1/8 of the batches,
// MAP 2 = each wave sweeps a contiguous run of batches
template <int MAP>
__device__ __forceinline__ bool batch_of(int nb, int it, int &b) {
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int G = gridDim.x;
    if (MAP == 0) {
        b = (blockIdx.x * 4 + wv) + it * G * 4;
        return b < nb;
    } else if (MAP == 1) {
        const int x = blockIdx.x & 7, j = blockIdx.x >> 3, G8 = G >> 3;
        const int lo = (int)((long long)nb * x / 8), hi = (int)((long long)nb * (x + 1) / 8);
        b = lo + (j * 4 + wv) + it * G8 * 4;
        return b < hi;
    } else if (MAP == 3) {
        const int w = blockIdx.x * 4 + wv, TW = G * 4;
        b = ((it >> 2) * TW + w) * 4 + (it & 3);
        return b < nb;
    } else {
        const int TW = G * 4, w = blockIdx.x * 4 + wv;
        const int per = (nb + TW - 1) / TW;
        b = w * per + it;
        return it < per && b < nb;
    }
}

// write-only: CH KiB contiguous per wave-iteration, 1 KiB (16 B/lane) per store
template <int CH, int AUX, int MAP>
__global__ __launch_bounds__(256) void kW(char *dst, int nchunk) {
    const int lane = threadIdx.x & 63;
    int c;
    for (int it = 0; batch_of<MAP>(nchunk, it, c); ++it) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst + (size_t)c * CH * 1024, 0, CH * 1024, 0x00020000);
#pragma unroll
        for (int k = 0; k < CH; ++k)
            __builtin_amdgcn_raw_buffer_store_b128(u4v{(unsigned)c, (unsigned)k, (unsigned)lane, 7u}, rs, lane * 16, k * 1024, AUX);
    }
}

// write-only, 4 B per lane (256 B per store), 8 KiB per wave-iteration
template <int AUX>
__global__ __launch_bounds__(256) void kW4(char *dst, int nchunk) {
    const int lane = threadIdx.x & 63;
    int c;
    for (int it = 0; batch_of<0>(nchunk, it, c); ++it) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst + (size_t)c * 8192, 0, 8192, 0x00020000);
#pragma unroll
        for (int k = 0; k < 32; ++k) __builtin_amdgcn_raw_buffer_store_b32((unsigned)(c + k), rs, lane * 4, k * 256, AUX);
    }
}

// the v2 data movement: B batches of 64 blocks per iteration
template <int AUX, int MAP, int NTL>
__global__ __launch_bounds__(256, 4) void kM(const uint8_t *src, int bw, int nblk, int per_frame, long long stride,
                                             long long fstride, char *coef) {
    __shared__ uint4 st[256 * 136 / 16];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nb = (nblk + 63) / 64;
    char *ws = reinterpret_cast<char *>(st) + wv * 8704;
    int b;
    for (int it = 0; batch_of<MAP>(nb, it, b); ++it) {
        int n = b * 64 + lane;
        int f = n / per_frame, rem = n - f * per_frame, by = rem / bw, bx = rem - by * bw;
        const uint8_t *p = src + f * fstride + (long long)by * 8 * stride + bx * 8;
        uint2 r[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (NTL) { u2v t = __builtin_nontemporal_load((const u2v *)(p + k * stride)); r[k] = make_uint2(t.x, t.y); }
            else r[k] = *(const uint2 *)(p + k * stride);
        }
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
        for (int k = 0; k < 8; ++k) __builtin_amdgcn_raw_buffer_store_b128(val[k], rc, lane * 16, k * 1024, AUX);
    }
}


// write-only, CH KiB per wave-iteration in groups of 8 KiB separated by s_sleep (models compute between batches)
template <int CH, int AUX, int SL>
__global__ __launch_bounds__(256) void kWs(char *dst, int nchunk) {
    const int lane = threadIdx.x & 63;
    int c;
    for (int it = 0; batch_of<0>(nchunk, it, c); ++it) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst + (size_t)c * CH * 1024, 0, CH * 1024, 0x00020000);
#pragma unroll
        for (int k = 0; k < CH; ++k) {
            if (k % 8 == 0 && SL) __builtin_amdgcn_s_sleep(SL);
            __builtin_amdgcn_raw_buffer_store_b128(u4v{(unsigned)c, (unsigned)k, (unsigned)lane, 7u}, rs, lane * 16, k * 1024, AUX);
        }
    }
}

// v2 movement, WG-cooperative: the 4 waves stage 4 consecutive batches (32 KiB
// of output) in the WG's stage; after a barrier, MODE 0: wave (it % 4) stores all
// 32 KiB; MODE 1: every wave stores 1 KiB chunks w, w+4, ... (interleaved);
// MODE 2: every wave stores its own 8 KiB (= kM, plus the barrier)
template <int AUX, int MODE>
__global__ __launch_bounds__(256, 4) void kMC(const uint8_t *src, int bw, int nblk, int per_frame, long long stride,
                                              long long fstride, char *coef) {
    __shared__ uint4 st[256 * 136 / 16];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nb = (nblk + 63) / 64;
    char *ws = reinterpret_cast<char *>(st) + wv * 8704;
    const int nwg = nb / 4;  // assume divisible
    int it = 0;
    for (int gb = blockIdx.x; gb < nwg; gb += gridDim.x, ++it) {
        const int b = gb * 4 + wv;
        int n = b * 64 + lane;
        int f = n / per_frame, rem = n - f * per_frame, by = rem / bw, bx = rem - by * bw;
        const uint8_t *p = src + f * fstride + (long long)by * 8 * stride + bx * 8;
        uint2 r[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) { u2v t = __builtin_nontemporal_load((const u2v *)(p + k * stride)); r[k] = make_uint2(t.x, t.y); }
        __builtin_amdgcn_s_waitcnt(0x0F70);
        __syncthreads();  // previous iteration's stage reads done
        uint2 *mine = reinterpret_cast<uint2 *>(ws + lane * 136);
#pragma unroll
        for (int k = 0; k < 8; ++k) { mine[2 * k] = r[k]; mine[2 * k + 1] = make_uint2(r[k].x ^ 1, r[k].y); }
        __syncthreads();
        const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(coef + (size_t)gb * 32768, 0, 32768, 0x00020000);
        if (MODE == 0) {
            if (wv == (it & 3)) {
#pragma unroll
                for (int h = 0; h < 4; ++h) {
                    const char *wsh = reinterpret_cast<char *>(st) + h * 8704;
                    u4v val[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        int m = k * 64 + lane, bl = m >> 3;
                        const uint2 *s2 = reinterpret_cast<const uint2 *>(wsh + bl * 136 + (m & 7) * 16);
                        val[k] = u4v{s2[0].x, s2[0].y, s2[1].x, s2[1].y};
                    }
#pragma unroll
                    for (int k = 0; k < 8; ++k) __builtin_amdgcn_raw_buffer_store_b128(val[k], rc, lane * 16, h * 8192 + k * 1024, AUX);
                }
            }
        } else {
            u4v val[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int ch = MODE == 1 ? k * 4 + wv : wv * 8 + k;  // 1 KiB chunk of the WG's 32 KiB
                const char *wsh = reinterpret_cast<char *>(st) + (ch >> 3) * 8704;
                int m = (ch & 7) * 64 + lane, bl = m >> 3;
                const uint2 *s2 = reinterpret_cast<const uint2 *>(wsh + bl * 136 + (m & 7) * 16);
                val[k] = u4v{s2[0].x, s2[0].y, s2[1].x, s2[1].y};
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int ch = MODE == 1 ? k * 4 + wv : wv * 8 + k;
                __builtin_amdgcn_raw_buffer_store_b128(val[k], rc, lane * 16, ch * 1024, AUX);
            }
        }
    }
}


// Phase-aligned 1:2 stream (no math): every wave issues its loads only in the
// chip-wide READ window and its stores only in the WRITE window of a period
// derived from s_memrealtime (100 MHz), so the HBM controllers see long
// read-only and write-only stretches.  R consecutive 64-block batches per
// wave-iteration (R*4 KiB in, R*8 KiB out, the output built from registers).
template <int R>
__global__ __launch_bounds__(256) void kPh(const uint8_t *src, int bw, int nblk, int per_frame, long long stride,
                                           long long fstride, char *coef, int period, int rwin) {
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nb = (nblk + 63) / 64, TW = gridDim.x * 4, w = blockIdx.x * 4 + wv;
    for (int b0 = w * R; b0 < nb; b0 += TW * R) {
        while ((int)(__builtin_amdgcn_s_memrealtime() % (unsigned long long)period) >= rwin) __builtin_amdgcn_s_sleep(2);
        uint2 r[R][8];
#pragma unroll
        for (int j = 0; j < R; ++j) {
            int n = (b0 + j) * 64 + lane;
            int f = n / per_frame, rem = n - f * per_frame, by = rem / bw, bx = rem - by * bw;
            const uint8_t *p = src + f * fstride + (long long)by * 8 * stride + bx * 8;
#pragma unroll
            for (int k = 0; k < 8; ++k) { u2v t = __builtin_nontemporal_load((const u2v *)(p + k * stride)); r[j][k] = make_uint2(t.x, t.y); }
        }
        __builtin_amdgcn_s_waitcnt(0x0F70);
        while ((int)(__builtin_amdgcn_s_memrealtime() % (unsigned long long)period) < rwin) __builtin_amdgcn_s_sleep(2);
        const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(coef + (size_t)b0 * 8192, 0, R * 8192, 0x00020000);
#pragma unroll
        for (int j = 0; j < R; ++j)
#pragma unroll
            for (int k = 0; k < 8; ++k)
                __builtin_amdgcn_raw_buffer_store_b128(u4v{r[j][k].x, r[j][k].y, r[j][(k + 1) & 7].x, (unsigned)k}, rc, lane * 16, (j * 8 + k) * 1024, 2);
    }
}


// v2 movement with the pixel rows fetched by LDS-DMA: 4 global_load_lds_dwordx4
// (1 KiB each = pixel rows 2k, 2k+1 of the batch's 64 blocks) into a per-wave
// 4 KiB input tile, then ds_read_b64 per lane per row (requires the batch's
// block-row splits at even block offsets: true for 3840 and 1920 wide planes)
template <int AUX, int WGS>
__global__ __launch_bounds__(256, WGS) void kMG(const uint8_t *src, int bw, int nblk, int per_frame, long long stride,
                                                long long fstride, char *coef) {
    __shared__ uint4 st[256 * 136 / 16];
    __shared__ uint4 inb[4 * 256];  // 4 KiB per wave
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nb = (nblk + 63) / 64;
    char *ws = reinterpret_cast<char *>(st) + wv * 8704;
    char *wi = reinterpret_cast<char *>(inb) + wv * 4096;
    int b;
    for (int it = 0; batch_of<0>(nb, it, b); ++it) {
        // lane l loads 16 B = blocks 2(l&31), 2(l&31)+1 of pixel row 2k + (l>>5)
        const int n = b * 64 + 2 * (lane & 31);
        int f = n / per_frame, rem = n - f * per_frame, by = rem / bw, bx = rem - by * bw;
        const uint8_t *p = src + f * fstride + (long long)(by * 8 + (lane >> 5)) * stride + bx * 8;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            __builtin_amdgcn_global_load_lds((const void *)(p + 2 * k * stride), (__attribute__((address_space(3))) void *)(wi + k * 1024), 16, 0, 2);
        __builtin_amdgcn_s_waitcnt(0x0F70);
        uint2 r[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] = *reinterpret_cast<const uint2 *>(wi + k * 512 + lane * 8);
        uint2 *mine = reinterpret_cast<uint2 *>(ws + lane * 136);
#pragma unroll
        for (int k = 0; k < 8; ++k) { mine[2 * k] = r[k]; mine[2 * k + 1] = make_uint2(r[k].x ^ 1, r[k].y); }
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
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
        for (int k = 0; k < 8; ++k) __builtin_amdgcn_raw_buffer_store_b128(val[k], rc, lane * 16, k * 1024, AUX);
    }
}

// v2 movement with 16-B row loads: lane l reads 16 B (2 blocks of one pixel
// row, rows 2k + (l>>5)) into registers, then writes them to the stage's
// input area; per-lane rows come back through LDS (the glds variant's data
// path, register-staged)
template <int AUX>
__global__ __launch_bounds__(256, 3) void kM16(const uint8_t *src, int bw, int nblk, int per_frame, long long stride,
                                              long long fstride, char *coef) {
    __shared__ uint4 st[256 * 136 / 16];
    __shared__ uint4 inb[4 * 256];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nb = (nblk + 63) / 64;
    char *ws = reinterpret_cast<char *>(st) + wv * 8704;
    char *wi = reinterpret_cast<char *>(inb) + wv * 4096;
    int b;
    for (int it = 0; batch_of<0>(nb, it, b); ++it) {
        const int n = b * 64 + 2 * (lane & 31);
        int f = n / per_frame, rem = n - f * per_frame, by = rem / bw, bx = rem - by * bw;
        const uint8_t *p = src + f * fstride + (long long)(by * 8 + (lane >> 5)) * stride + bx * 8;
        u4v t[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) t[k] = __builtin_nontemporal_load((const u4v *)(p + 2 * k * stride));
#pragma unroll
        for (int k = 0; k < 4; ++k) *reinterpret_cast<u4v *>(wi + k * 1024 + lane * 16) = t[k];
        __builtin_amdgcn_s_waitcnt(0xC07F);
        uint2 r[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] = *reinterpret_cast<const uint2 *>(wi + k * 512 + lane * 8);
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
        for (int k = 0; k < 8; ++k) __builtin_amdgcn_raw_buffer_store_b128(val[k], rc, lane * 16, k * 1024, AUX);
    }
}


// v2 movement with the pixel rows of a batch CONTIGUOUS in memory (a tile-major
// input layout the API does not have: load r = bytes [4096 b + 512 r, +512)):
// does the 2-D row gather (8 rows 3840 B apart) cost anything?
template <int AUX>
__global__ __launch_bounds__(256, 4) void kMT(const uint8_t *src, int nblk, char *coef) {
    __shared__ uint4 st[256 * 136 / 16];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nb = (nblk + 63) / 64;
    char *ws = reinterpret_cast<char *>(st) + wv * 8704;
    int b;
    for (int it = 0; batch_of<0>(nb, it, b); ++it) {
        const uint8_t *p = src + (size_t)b * 4096 + lane * 8;
        uint2 r[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) { u2v t = __builtin_nontemporal_load((const u2v *)(p + k * 512)); r[k] = make_uint2(t.x, t.y); }
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
        for (int k = 0; k < 8; ++k) __builtin_amdgcn_raw_buffer_store_b128(val[k], rc, lane * 16, k * 1024, AUX);
    }
}

// the inverse kernel's shape: 16-B contiguous loads of 8 KiB per 64 blocks (int16
// coefficients), 16 KiB of 1 KiB stores (fp32): 1:2 like the forward, double the bytes
template <int AUX>
__global__ __launch_bounds__(256, 4) void kInv(const char *src, int nblk, char *dst) {
    const int lane = threadIdx.x & 63;
    const int nb = (nblk + 63) / 64;
    int b;
    for (int it = 0; batch_of<0>(nb, it, b); ++it) {
        const u4v *p = reinterpret_cast<const u4v *>(src + (size_t)b * 8192) + lane;
        u4v v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = __builtin_nontemporal_load(p + k * 64);
        const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(dst + (size_t)b * 16384, 0, 16384, 0x00020000);
#pragma unroll
        for (int k = 0; k < 16; ++k)
            __builtin_amdgcn_raw_buffer_store_b128(u4v{v[k & 7][0] ^ k, v[k & 7][1], v[k & 7][2], v[k & 7][3]}, rc, lane * 16, k * 1024, AUX);
    }
}


// the paired inverse kernel's data movement exactly (idct8_pair, no math): 32-block
// batches, lane (h, j) loads rows 4h..4h+3 of block j (4 x 16 B, plain loads) of
// the int16 coefficients, writes 128 B of its block's fp32 rows to the stage
// (pitch 272), and the wave stores the stage as 8 x 1 KiB nt stores (8 KiB out)
__global__ __launch_bounds__(256, 4) void kInvExact(const char *src, int nblk, char *dst) {
    __shared__ uint4 st[4 * 32 * 272 / 16];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5, j = lane & 31;
    const int nb = (nblk + 31) / 32;
    char *base = reinterpret_cast<char *>(st) + wv * 32 * 272;
    int b;
    for (int it = 0; batch_of<0>(nb, it, b); ++it) {
        const uint4 *p = reinterpret_cast<const uint4 *>(src + ((size_t)b * 32 + j) * 128) + 4 * h;
        uint4 r[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) r[k] = p[k];
        char *mine = base + j * 272 + h * 128;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            *reinterpret_cast<uint4 *>(mine + k * 32) = r[k];
            *reinterpret_cast<uint4 *>(mine + k * 32 + 16) = make_uint4(r[k].y, r[k].x, r[k].w, r[k].z);
        }
        __builtin_amdgcn_s_waitcnt(0x0F70);
        __builtin_amdgcn_wave_barrier();
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst + (size_t)b * 32 * 256, 0, 8192, 0x00020000);
        u4v val[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int bl = 4 * k + (lane >> 4);
            const uint4 t = *reinterpret_cast<const uint4 *>(base + bl * 272 + (lane & 15) * 16);
            val[k] = u4v{t.x, t.y, t.z, t.w};
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) __builtin_amdgcn_raw_buffer_store_b128(val[k], rs, lane * 16, k * 1024, 2);
    }
}

// read-only sweep, 16 B/lane nt, 8 KiB per wave-iteration
template <int MAP>
__global__ __launch_bounds__(256) void kR(const char *src, int nchunk, unsigned *out) {
    const int lane = threadIdx.x & 63;
    unsigned acc = 0;
    int c;
    for (int it = 0; batch_of<MAP>(nchunk, it, c); ++it) {
        const u4v *p = reinterpret_cast<const u4v *>(src + (size_t)c * 8192) + lane;
        u4v v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = __builtin_nontemporal_load(p + k * 64);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc ^= v[k].x ^ v[k].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

static hipEvent_t e0, e1;
#define TIME(label, bytes, launch)                                                                   \
    {                                                                                                \
        float best = 1e9, sum = 0;                                                                   \
        for (int rep = 0; rep < 10; ++rep) {                                                         \
            hipEventRecord(e0); launch; hipEventRecord(e1); hipEventSynchronize(e1);                 \
            float ms; hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms; if (rep >= 2) sum += ms; \
        }                                                                                            \
        printf("%-52s best %8.1f us %5.1f %%  mean %5.1f %%\n", label, best * 1e3, (bytes) / best / 1e6 / 80.0, \
               (bytes) / (sum / 8) / 1e6 / 80.0);                                                    \
        fflush(stdout);                                                                              \
    }

int main() {
    const int W = 3840, H = 2160, F = 64;
    const int bw = W / 8, per = bw * (H / 8), nblk = per * F, nb = nblk / 64;
    uint8_t *src; char *dst; unsigned *o;
    hipMalloc(&src, (size_t)W * H * F);
    hipMalloc(&dst, (size_t)nblk * 128 + (1 << 20));
    hipMalloc(&o, 64);
    hipMemset(src, 7, (size_t)W * H * F);
    hipMemset(dst, 0, (size_t)nblk * 128);
    hipEventCreate(&e0); hipEventCreate(&e1);
    int ncu = 0; hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const double wb = (double)nblk * 128, mb = (double)nblk * 192;
    const int g4 = ncu * 4, g8 = ncu * 8;
    const long long ls = W, lf = (long long)W * H;
    printf("CUs %d, %d blocks, write %.2f GB\n", ncu, nblk, wb / 1e9);
    if (getenv("ROUND1")) {
    TIME("W 8K plain grid-stride 16w/CU", wb, hipLaunchKernelGGL((kW<8, 0, 0>), dim3(g4), dim3(256), 0, 0, dst, nb));
    TIME("W 8K nt    grid-stride 16w/CU", wb, hipLaunchKernelGGL((kW<8, 2, 0>), dim3(g4), dim3(256), 0, 0, dst, nb));
    TIME("W 8K sc0nt grid-stride 16w/CU", wb, hipLaunchKernelGGL((kW<8, 3, 0>), dim3(g4), dim3(256), 0, 0, dst, nb));
    TIME("W 8K sc1   grid-stride 16w/CU", wb, hipLaunchKernelGGL((kW<8, 16, 0>), dim3(g4), dim3(256), 0, 0, dst, nb));
    TIME("W 8K nt    grid-stride 32w/CU", wb, hipLaunchKernelGGL((kW<8, 2, 0>), dim3(g8), dim3(256), 0, 0, dst, nb));
    TIME("W 8K plain grid-stride 32w/CU", wb, hipLaunchKernelGGL((kW<8, 0, 0>), dim3(g8), dim3(256), 0, 0, dst, nb));
    TIME("W 8K nt    xcd-contig 16w/CU", wb, hipLaunchKernelGGL((kW<8, 2, 1>), dim3(g4), dim3(256), 0, 0, dst, nb));
    TIME("W 8K plain xcd-contig 16w/CU", wb, hipLaunchKernelGGL((kW<8, 0, 1>), dim3(g4), dim3(256), 0, 0, dst, nb));
    TIME("W 8K nt    wave-contig 16w/CU", wb, hipLaunchKernelGGL((kW<8, 2, 2>), dim3(g4), dim3(256), 0, 0, dst, nb));
    TIME("W 8K plain wave-contig 16w/CU", wb, hipLaunchKernelGGL((kW<8, 0, 2>), dim3(g4), dim3(256), 0, 0, dst, nb));
    TIME("W 2K nt    grid-stride 16w/CU", wb, hipLaunchKernelGGL((kW<2, 2, 0>), dim3(g4), dim3(256), 0, 0, dst, nb * 4));
    TIME("W 32K nt   grid-stride 16w/CU", wb, hipLaunchKernelGGL((kW<32, 2, 0>), dim3(g4), dim3(256), 0, 0, dst, nb / 4));
    TIME("W 32K plain grid-stride 16w/CU", wb, hipLaunchKernelGGL((kW<32, 0, 0>), dim3(g4), dim3(256), 0, 0, dst, nb / 4));
    TIME("W dword plain 8K 16w/CU", wb, hipLaunchKernelGGL((kW4<0>), dim3(g4), dim3(256), 0, 0, dst, nb));
    TIME("W dword nt 8K 16w/CU", wb, hipLaunchKernelGGL((kW4<2>), dim3(g4), dim3(256), 0, 0, dst, nb));
    TIME("R 8K nt grid-stride 16w/CU", wb, hipLaunchKernelGGL((kR<0>), dim3(g4), dim3(256), 0, 0, dst, nb, o));
    TIME("R 8K nt xcd-contig 16w/CU", wb, hipLaunchKernelGGL((kR<1>), dim3(g4), dim3(256), 0, 0, dst, nb, o));
    TIME("M v2 movement nt/nt grid-stride", mb, hipLaunchKernelGGL((kM<2, 0, 1>), dim3(g4), dim3(256), 0, 0, src, bw, nblk, per, ls, lf, dst));
    TIME("M v2 movement nt/sc0nt grid-stride", mb, hipLaunchKernelGGL((kM<3, 0, 1>), dim3(g4), dim3(256), 0, 0, src, bw, nblk, per, ls, lf, dst));
    TIME("M v2 movement nt/nt xcd-contig", mb, hipLaunchKernelGGL((kM<2, 1, 1>), dim3(g4), dim3(256), 0, 0, src, bw, nblk, per, ls, lf, dst));
    TIME("M v2 movement nt/nt wave-contig", mb, hipLaunchKernelGGL((kM<2, 2, 1>), dim3(g4), dim3(256), 0, 0, src, bw, nblk, per, ls, lf, dst));
    TIME("M v2 movement plain/nt grid-stride", mb, hipLaunchKernelGGL((kM<2, 0, 0>), dim3(g4), dim3(256), 0, 0, src, bw, nblk, per, ls, lf, dst));
    TIME("M v2 movement nt/plain grid-stride", mb, hipLaunchKernelGGL((kM<0, 0, 1>), dim3(g4), dim3(256), 0, 0, src, bw, nblk, per, ls, lf, dst));
    TIME("M v2 movement nt/nt grid-stride (repeat)", mb, hipLaunchKernelGGL((kM<2, 0, 1>), dim3(g4), dim3(256), 0, 0, src, bw, nblk, per, ls, lf, dst));

    }
    printf("--- same-box reference\n");
    TIME("M v2 movement nt/nt grid-stride", mb, hipLaunchKernelGGL((kM<2, 0, 1>), dim3(g4), dim3(256), 0, 0, src, bw, nblk, per, ls, lf, dst));
    TIME("W 8K nt    runs-of-4 16w/CU", wb, hipLaunchKernelGGL((kW<8, 2, 3>), dim3(g4), dim3(256), 0, 0, dst, nb));
    TIME("MT tile-major contiguous input, 4 WG/CU", mb, hipLaunchKernelGGL((kMT<2>), dim3(g4), dim3(256), 0, 0, src, nblk, dst));
    TIME("M v2 movement nt/nt grid-stride (again)", mb, hipLaunchKernelGGL((kM<2, 0, 1>), dim3(g4), dim3(256), 0, 0, src, bw, nblk, per, ls, lf, dst));
    {   // inverse shape over 64 x 4K luma blocks: 128 B in (int16), 256 B out (fp32)
        char *big; hipMalloc(&big, (size_t)nblk * 256 + (1 << 20));
        TIME("Inv shape 16B loads 8K + 16K stores (384 B/blk)", (double)nblk * 384, hipLaunchKernelGGL((kInv<2>), dim3(g4), dim3(256), 0, 0, dst, nblk, big));
        TIME("InvExact idct8_pair movement (384 B/blk)", (double)nblk * 384, hipLaunchKernelGGL(kInvExact, dim3(g4), dim3(256), 0, 0, dst, nblk, big));
        TIME("M v2 movement nt/nt grid-stride (again)", mb, hipLaunchKernelGGL((kM<2, 0, 1>), dim3(g4), dim3(256), 0, 0, src, bw, nblk, per, ls, lf, dst));
        TIME("InvExact idct8_pair movement (384 B/blk) again", (double)nblk * 384, hipLaunchKernelGGL(kInvExact, dim3(g4), dim3(256), 0, 0, dst, nblk, big));
        hipFree(big);
    }
    TIME("MG glds rows, 3 WG/CU", mb, hipLaunchKernelGGL((kMG<2, 3>), dim3(ncu * 3), dim3(256), 0, 0, src, bw, nblk, per, ls, lf, dst));
    TIME("MG glds rows, 2 WG/CU", mb, hipLaunchKernelGGL((kMG<2, 2>), dim3(ncu * 2), dim3(256), 0, 0, src, bw, nblk, per, ls, lf, dst));
    TIME("M16 16B reg rows via LDS, 3 WG/CU", mb, hipLaunchKernelGGL((kM16<2>), dim3(ncu * 3), dim3(256), 0, 0, src, bw, nblk, per, ls, lf, dst));
    TIME("M v2 movement, 3 WG/CU", mb, hipLaunchKernelGGL((kM<2, 0, 1>), dim3(ncu * 3), dim3(256), 0, 0, src, bw, nblk, per, ls, lf, dst));
    TIME("M v2 movement, 2 WG/CU", mb, hipLaunchKernelGGL((kM<2, 0, 1>), dim3(ncu * 2), dim3(256), 0, 0, src, bw, nblk, per, ls, lf, dst));
    if (getenv("PHASE")) {  // negative result: phase-aligned windows lose (47-71 %%)
        const int cfg[][3] = {{2, 1500, 500}, {2, 1600, 500}, {2, 1800, 600}, {2, 2400, 800}, {2, 1200, 400},
                              {4, 3000, 1000}, {4, 3200, 1000}, {4, 3600, 1200}, {1, 800, 260}, {1, 1000, 330}};
        for (auto &c : cfg) {
            char lab[96];
            snprintf(lab, sizeof lab, "Ph R=%d period %d read %d (%dw/CU)", c[0], c[1], c[2], 16);
            if (c[0] == 1) TIME(lab, mb, hipLaunchKernelGGL((kPh<1>), dim3(g4), dim3(256), 0, 0, src, bw, nblk, per, ls, lf, dst, c[1], c[2]))
            else if (c[0] == 2) TIME(lab, mb, hipLaunchKernelGGL((kPh<2>), dim3(g4), dim3(256), 0, 0, src, bw, nblk, per, ls, lf, dst, c[1], c[2]))
            else TIME(lab, mb, hipLaunchKernelGGL((kPh<4>), dim3(g4), dim3(256), 0, 0, src, bw, nblk, per, ls, lf, dst, c[1], c[2]))
        }
        TIME("Ph R=2 period 1500 read 500, 32w/CU", mb, hipLaunchKernelGGL((kPh<2>), dim3(g8), dim3(256), 0, 0, src, bw, nblk, per, ls, lf, dst, 1500, 500));
    }
    TIME("M v2 movement nt/nt grid-stride (repeat)", mb, hipLaunchKernelGGL((kM<2, 0, 1>), dim3(g4), dim3(256), 0, 0, src, bw, nblk, per, ls, lf, dst));
    {   // chroma geometry: 128 planes of 1920x1080 (4 147 200 blocks)
        const int cw = 1920, ch = 1080, cbw = cw / 8, cper = cbw * (ch / 8), cn = cper * 128;
        TIME("M v2 movement nt/nt chroma 128x1920x1080", (double)cn * 192, hipLaunchKernelGGL((kM<2, 0, 1>), dim3(g4), dim3(256), 0, 0, src, cbw, cn, cper, (long long)cw, (long long)cw * ch, dst));
    }
    return 0;
}
