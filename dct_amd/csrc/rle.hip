// dct_amd/csrc/rle.hip -- zigzag + run-length symbols of quantized blocks on the GPU
// (shrink the coefficient planes before the xGMI gather).
//
// Per block this is exactly the reference's run_length_encode
// (src/entropy.c:216-256 over block_to_zigzag :158-178): one symbol per
// nonzero zigzag element, its run = zeros before it, plus always a symbol for
// the last element (7,7), whose run also counts itself when it is zero.  So a
// block has exactly 1 + nnz(first 63 zigzag elements) symbols.  Blocks are
// concatenated in order; symbol = (uint16)value | run << 16.
//
// Layout choices (DESIGN.md "RLE"): one WAVE per block -- lane i holds zigzag
// element i, so "nonzero" is a ballot, a symbol's index is mbcnt of that ballot,
// its run is the distance to the previous set bit, and the symbols of a block
// are written by consecutive lanes to consecutive addresses.
//   dctq_rle_count : lane-per-block counts, wave-scanned per 64-block tile, a
//                    one-workgroup scan of the tile totals, a fix-up pass.
//   dctq_rle_emit  : the symbols (one wave per tile, block by block).
//   dctq_rle_decode: run_length_decode (:327-351) + zigzag_to_block (:183-210),
//                    one wave per tile through a 64-entry LDS row.
#include "dctq_internal.h"

namespace dctq {

// zigzag position k -> natural index (src/entropy.c:158-178 for n = 8)
__constant__ uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
// natural index -> zigzag position
__constant__ uint8_t kUnzigzag[64] = {0,  1,  5,  6,  14, 15, 27, 28, 2,  4,  7,  13, 16, 26, 29, 42,
                                      3,  8,  12, 17, 25, 30, 41, 43, 9,  11, 18, 24, 31, 40, 44, 53,
                                      10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60,
                                      21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63};

constexpr int kRleWaves = 4;
constexpr int kRleThreads = 64 * kRleWaves;
constexpr int kScanThreads = 1024;

__device__ __forceinline__ uint64_t lane_mask_below(int lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }

// Inclusive wave scan (DPP row shifts + row broadcasts: VALU only, no LDS).
__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t e) {
    e += __builtin_amdgcn_update_dpp(0u, e, 0x111, 0xF, 0xF, false);  // row_shr:1
    e += __builtin_amdgcn_update_dpp(0u, e, 0x112, 0xF, 0xF, false);  // row_shr:2
    e += __builtin_amdgcn_update_dpp(0u, e, 0x114, 0xF, 0xF, false);  // row_shr:4
    e += __builtin_amdgcn_update_dpp(0u, e, 0x118, 0xF, 0xF, false);  // row_shr:8
    e += __builtin_amdgcn_update_dpp(0u, e, 0x142, 0xA, 0xF, false);  // row_bcast:15
    e += __builtin_amdgcn_update_dpp(0u, e, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return e;
}

// Nonzero int16 halves of a dword (0, 1 or 2).
__device__ __forceinline__ uint32_t nz16(uint32_t w) { return ((w & 0xFFFFu) != 0u) + ((w >> 16) != 0u); }

// ---- count: tile t = blocks [64t, 64t+64), one wave, lane j = block 64t+j:
// count = 1 + nnz(the block's first 63 zigzag elements) = 1 + nnz(all) - (c[63] != 0),
// tile-local exclusive offsets by a wave scan, tile total -> tiles[t].
__global__ __launch_bounds__(kRleThreads) void rle_count_kernel(const int16_t *__restrict__ coef, long long nblk,
                                                                uint32_t *__restrict__ offsets,
                                                                uint32_t *__restrict__ tiles, long long ntiles) {
    const int lane = threadIdx.x & 63;
    const long long t = (long long)blockIdx.x * kRleWaves + (threadIdx.x >> 6);
    if (t >= ntiles) return;
    const long long b = t * 64 + lane;
    uint32_t cnt = 0;
    if (b < nblk) {
        const uint4 *src = reinterpret_cast<const uint4 *>(coef + b * 64);
        uint4 q[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) q[k] = src[k];
        uint32_t nz = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) nz += nz16(q[k].x) + nz16(q[k].y) + nz16(q[k].z) + nz16(q[k].w);
        cnt = 1u + nz - ((q[7].w >> 16) != 0u);
    }
    const uint32_t inc = wave_inclusive_scan(cnt);
    if (b < nblk) offsets[b] = inc - cnt;
    if (lane == 63) tiles[t] = inc;
}

// ---- exclusive scan of the tile totals in place (one workgroup), total -> offsets[nblk]
__global__ __launch_bounds__(kScanThreads) void rle_scan_tiles_kernel(uint32_t *__restrict__ tiles, long long ntiles,
                                                                      uint32_t *__restrict__ total_out) {
    __shared__ uint32_t part[kScanThreads];
    const int tid = threadIdx.x;
    const long long per = (ntiles + kScanThreads - 1) / kScanThreads;
    const long long lo = tid * per, hi = lo + per < ntiles ? lo + per : ntiles;
    uint32_t s = 0;
    for (long long i = lo; i < hi; ++i) s += tiles[i];
    part[tid] = s;
    __syncthreads();
    for (int d = 1; d < kScanThreads; d <<= 1) {  // Hillis-Steele inclusive scan
        const uint32_t add = tid >= d ? part[tid - d] : 0u;
        __syncthreads();
        part[tid] += add;
        __syncthreads();
    }
    uint32_t acc = part[tid] - s;  // exclusive prefix of this thread's range
    for (long long i = lo; i < hi; ++i) {
        const uint32_t v = tiles[i];
        tiles[i] = acc;
        acc += v;
    }
    if (tid == kScanThreads - 1) *total_out = part[tid];
}

__global__ __launch_bounds__(kRleThreads) void rle_fixup_kernel(uint32_t *__restrict__ offsets,
                                                                const uint32_t *__restrict__ tiles, long long nblk) {
    const long long b = (long long)blockIdx.x * kRleThreads + threadIdx.x;
    if (b < nblk) offsets[b] += tiles[b >> 6];
}

// ---- emit: one wave per 64-block tile; lane i holds zigzag element i of the
// current block; the tile's offsets come in with one coalesced load and are
// read per block with readlane; 8 blocks' gathers are in flight at a time.
constexpr int kGroup = 8;

__global__ __launch_bounds__(kRleThreads) void rle_emit_kernel(const int16_t *__restrict__ coef, long long nblk,
                                                               const uint32_t *__restrict__ offsets,
                                                               uint32_t *__restrict__ symbols, long long ntiles) {
    const int lane = threadIdx.x & 63;
    const long long stride = (long long)gridDim.x * kRleWaves;
    const int nat = kZigzag[lane];
    const uint64_t below = lane_mask_below(lane);
    for (long long t = (long long)blockIdx.x * kRleWaves + (threadIdx.x >> 6); t < ntiles; t += stride) {
        const long long b0 = t * 64;
        const int nb = nblk - b0 < 64 ? (int)(nblk - b0) : 64;
        const uint32_t offv = lane < nb ? offsets[b0 + lane] : 0u;
        for (int g = 0; g < nb; g += kGroup) {
            int16_t v[kGroup];
#pragma unroll
            for (int u = 0; u < kGroup; ++u) v[u] = coef[(b0 + (g + u < nb ? g + u : g)) * 64 + nat];
#pragma unroll
            for (int u = 0; u < kGroup; ++u) {
                if (g + u >= nb) break;
                const uint32_t o = __builtin_amdgcn_readlane(offv, g + u);
                const bool emit = v[u] != 0 || lane == 63;
                const uint64_t prev = __builtin_amdgcn_ballot_w64(emit) & below;
                const int p = prev ? 63 - __builtin_clzll(prev) : -1;
                const uint32_t runlen = (uint32_t)(lane - p - 1) + (lane == 63 && v[u] == 0 ? 1u : 0u);
                if (emit) symbols[o + (uint32_t)__builtin_popcountll(prev)] = (uint32_t)(uint16_t)v[u] | (runlen << 16);
            }
        }
    }
}

// ---- decode: one wave per 64-block tile, groups of 8 blocks: the symbol loads
// of a group are in flight together (each block's range from readlane of the
// tile's coalesced offsets); each block is rebuilt in the wave's 64-entry LDS
// row (zeroed, symbols scattered to their zigzag positions -- LDS writes of one
// wave are performed in order), read back in natural order, and the group's 8
// blocks are stored as 128-B rows.
//
// LDS loads and the store-data race (fdct8.hip v2 / DESIGN.md): the previous
// group's stores may still be reading their data VGPRs when this group's LDS
// reads return, so those 8 registers are kept live across the reads (the LDS
// reads cannot land in them); the stores' address operands are loop-invariant
// (voff) or scalar.
__global__ __launch_bounds__(kRleThreads) void rle_decode_kernel(const uint32_t *__restrict__ symbols,
                                                                 const uint32_t *__restrict__ offsets, long long nblk,
                                                                 int16_t *__restrict__ coef, long long ntiles) {
    __shared__ int16_t row[kRleWaves][64];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const long long stride = (long long)gridDim.x * kRleWaves;
    const int zpos = kUnzigzag[lane];
    uint32_t voff = (uint32_t)lane * 2u;
    uint32_t outv[kGroup];
#pragma unroll
    for (int u = 0; u < kGroup; ++u) outv[u] = 0;
    for (long long t = (long long)blockIdx.x * kRleWaves + wv; t < ntiles; t += stride) {
        const long long b0 = t * 64;
        const int nb = nblk - b0 < 64 ? (int)(nblk - b0) : 64;
        const uint32_t offv = offsets[b0 + (lane < nb ? lane : nb)];  // lane nb: the end of the tile
        for (int g = 0; g < nb; g += kGroup) {
            uint32_t sy[kGroup], cnt[kGroup];
#pragma unroll
            for (int u = 0; u < kGroup; ++u) {
                const int jb = g + u < nb ? g + u : nb - 1;
                const uint32_t o0 = __builtin_amdgcn_readlane(offv, jb), o1 = __builtin_amdgcn_readlane(offv, jb + 1);
                cnt[u] = g + u < nb ? o1 - o0 : 0u;
                sy[u] = (uint32_t)lane < cnt[u] ? symbols[o0 + lane] : 0u;
            }
#pragma unroll
            for (int u = 0; u < kGroup; ++u) asm volatile("" : "+v"(outv[u]));
            uint32_t val[kGroup];
#pragma unroll
            for (int u = 0; u < kGroup; ++u) {
                const uint32_t e = wave_inclusive_scan((uint32_t)lane < cnt[u] ? (sy[u] >> 16) + 1u : 0u);
                row[wv][lane] = 0;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const uint32_t pos = e - 1u;  // run_length_decode: pos += run; zigzag[pos++] = value (dropped past the end)
                if ((uint32_t)lane < cnt[u] && pos < 64u) row[wv][pos] = (int16_t)(sy[u] & 0xFFFFu);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                val[u] = (uint32_t)(uint16_t)row[wv][zpos];
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
#pragma unroll
            for (int u = 0; u < kGroup; ++u) asm volatile("" ::"v"(outv[u]));
#pragma unroll
            for (int u = 0; u < kGroup; ++u) {
                outv[u] = val[u];
                if (g + u < nb) {
                    const __amdgpu_buffer_rsrc_t rs =
                        __builtin_amdgcn_make_buffer_rsrc(coef + (b0 + g + u) * 64, (short)0, 128, 0x00020000);
                    __builtin_amdgcn_raw_buffer_store_b16((uint16_t)outv[u], rs, voff, 0, 0);
                }
            }
            asm volatile("" : "+v"(voff));
        }
    }
}

static unsigned grid_for(long long waves_wanted, int num_cus) {
    long long g = (waves_wanted + kRleWaves - 1) / kRleWaves;
    const long long cap = (long long)num_cus * 16;
    return (unsigned)(g < 1 ? 1 : g > cap ? cap : g);
}

size_t rle_workspace_bytes(long long nblk) { return (size_t)((nblk + 63) / 64) * sizeof(uint32_t); }

hipError_t launch_rle_count(const int16_t *coef, long long nblk, uint32_t *offsets, void *ws, hipStream_t stream) {
    const long long ntiles = (nblk + 63) / 64;
    uint32_t *tiles = (uint32_t *)ws;
    hipLaunchKernelGGL(rle_count_kernel, dim3((unsigned)((ntiles + kRleWaves - 1) / kRleWaves)), dim3(kRleThreads), 0,
                       stream, coef, nblk, offsets, tiles, ntiles);
    hipLaunchKernelGGL(rle_scan_tiles_kernel, dim3(1), dim3(kScanThreads), 0, stream, tiles, ntiles, offsets + nblk);
    hipLaunchKernelGGL(rle_fixup_kernel, dim3((unsigned)((nblk + kRleThreads - 1) / kRleThreads)), dim3(kRleThreads),
                       0, stream, offsets, (const uint32_t *)tiles, nblk);
    return hipGetLastError();
}

hipError_t launch_rle_emit(const int16_t *coef, long long nblk, const uint32_t *offsets, uint32_t *symbols,
                           hipStream_t stream, int num_cus) {
    const long long ntiles = (nblk + 63) / 64;
    hipLaunchKernelGGL(rle_emit_kernel, dim3(grid_for(ntiles, num_cus)), dim3(kRleThreads), 0, stream, coef, nblk,
                       offsets, symbols, ntiles);
    return hipGetLastError();
}

hipError_t launch_rle_decode(const uint32_t *symbols, const uint32_t *offsets, long long nblk, int16_t *coef,
                             hipStream_t stream, int num_cus) {
    const long long ntiles = (nblk + 63) / 64;
    hipLaunchKernelGGL(rle_decode_kernel, dim3(grid_for(ntiles, num_cus)), dim3(kRleThreads), 0, stream, symbols,
                       offsets, nblk, coef, ntiles);
    return hipGetLastError();
}

}  // namespace dctq
