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
#include "scan_core.h"

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

__device__ __forceinline__ uint64_t lane_mask_below(int lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }

// Nonzero int16 halves of a dword (0, 1 or 2).
__device__ __forceinline__ uint32_t nz16(uint32_t w) { return ((w & 0xFFFFu) != 0u) + ((w >> 16) != 0u); }

// ---- count: tile t = blocks [64t, 64t+64), one wave, grid-stride with the
// next tile's 8 KiB prefetched in registers.
// count = 1 + nnz(first 63 zigzag elements) = 1 + nnz(all) - (c[63] != 0).
// The tile is read with 1 KiB-contiguous loads: chunk m = 64k + lane holds 16 B
// of block 8k + lane/8, so load k covers blocks 8k..8k+7 in groups of 8 lanes.
// A wave scan of load k's per-lane contributions (the +1 and the c[63]
// exclusion fall on each group's last lane) gives, at lane 8q+7, the count of
// blocks 8k..8k+q inclusive; the block's exclusive tile offset follows with the
// running total of loads 0..k-1.  No cross-lane data movement beyond DPP and no
// LDS, so no store-data hazard.  Writes tile-local offsets and tiles[t].
__global__ __launch_bounds__(kRleThreads) void rle_count_kernel(const int16_t *__restrict__ coef, long long nblk,
                                                                uint32_t *__restrict__ offsets,
                                                                uint32_t *__restrict__ tiles, long long ntiles) {
    const int lane = threadIdx.x & 63;
    const long long stride = (long long)gridDim.x * kRleWaves;
    long long t = (long long)blockIdx.x * kRleWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (t >= ntiles) return;
    auto load_tile = [&](long long tt, uint4 (&q)[8]) {
        const long long r = nblk - tt * 64;
        const int nb = r < 64 ? (int)r : 64;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<int16_t *>(coef) + tt * 64 * 64, (short)0, nb * 128, 0x00020000);  // past the tail: zeros
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, k * 1024, 2 /* nt */);
            q[k] = make_uint4(v[0], v[1], v[2], v[3]);
        }
    };
    uint4 nxt[8];
    load_tile(t, nxt);
    for (; t < ntiles; t += stride) {
        uint4 q[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) q[k] = nxt[k];
        if (t + stride < ntiles) load_tile(t + stride, nxt);
        const long long b0 = t * 64;
        const int nb = nblk - b0 < 64 ? (int)(nblk - b0) : 64;
        uint32_t run = 0;  // blocks 0..8k-1 of the tile
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            uint32_t e = nz16(q[k].x) + nz16(q[k].y) + nz16(q[k].z) + nz16(q[k].w);
            const int blk = 8 * k + (lane >> 3);
            if ((lane & 7) == 7) e = blk < nb ? e + 1u - ((q[k].w >> 16) != 0u) : 0u;
            const uint32_t inc = wave_inclusive_scan(e);
            // lane 8q: exclusive sum = count of blocks 8k..8k+q-1; row_shr:7 brings it to
            // lane 8q+7 (same 16-lane row), which writes block 8k+q's tile offset
            const uint32_t before = __builtin_amdgcn_update_dpp(0u, inc - e, 0x117, 0xF, 0xF, false);
            if ((lane & 7) == 7 && blk < nb) offsets[b0 + blk] = run + before;
            run += __builtin_amdgcn_readlane(inc, 63);
        }
        if (lane == 0) tiles[t] = run;
    }
}

// ---- exclusive scan of the tile totals in place (one workgroup of 1024), total -> *total_out.
// Chunks of 8192 totals: each thread scans 8 consecutive values (two 16-B loads,
// coalesced), a wave scan and a 16-entry LDS scan combine the threads, the
// running carry crosses chunks; the next chunk's loads are issued first.
constexpr int kScanThreads = 1024;
constexpr int kScanPer = 8;

__global__ __launch_bounds__(kScanThreads) void rle_scan_tiles_kernel(uint32_t *__restrict__ tiles, long long ntiles,
                                                                      uint32_t *__restrict__ total_out) {
    __shared__ uint32_t wsum[kScanThreads / 64];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const long long chunk = (long long)kScanThreads * kScanPer;
    auto load = [&](long long c0, uint32_t (&v)[kScanPer]) {
#pragma unroll
        for (int i = 0; i < kScanPer; ++i) {
            const long long idx = c0 + (long long)tid * kScanPer + i;
            v[i] = idx < ntiles ? tiles[idx] : 0u;
        }
    };
    uint32_t carry = 0, nxt[kScanPer];
    load(0, nxt);
    for (long long c0 = 0; c0 < ntiles; c0 += chunk) {
        uint32_t v[kScanPer];
#pragma unroll
        for (int i = 0; i < kScanPer; ++i) v[i] = nxt[i];
        if (c0 + chunk < ntiles) load(c0 + chunk, nxt);
        uint32_t s = 0;
#pragma unroll
        for (int i = 0; i < kScanPer; ++i) s += v[i];
        const uint32_t inc = wave_inclusive_scan(s);
        if (lane == 63) wsum[wv] = inc;
        __syncthreads();
        uint32_t wpre = 0, ctot = 0;
#pragma unroll
        for (int w = 0; w < kScanThreads / 64; ++w) {
            const uint32_t x = wsum[w];
            wpre += w < wv ? x : 0u;
            ctot += x;
        }
        __syncthreads();  // wsum is rewritten by the next chunk
        uint32_t acc = carry + wpre + inc - s;
#pragma unroll
        for (int i = 0; i < kScanPer; ++i) {
            const long long idx = c0 + (long long)tid * kScanPer + i;
            if (idx < ntiles) tiles[idx] = acc;
            acc += v[i];
        }
        carry += ctot;
    }
    if (tid == 0) *total_out = carry;
}

__global__ __launch_bounds__(kRleThreads) void rle_fixup_kernel(uint32_t *__restrict__ offsets,
                                                                const uint32_t *__restrict__ tiles, long long nblk) {
    const long long b = (long long)blockIdx.x * kRleThreads + threadIdx.x;
    if (b < nblk) offsets[b] += tiles[b >> 6];
}

// ---- emit: one wave per 64-block tile; lane i holds zigzag element i of the
// current block.  Blocks are processed in groups of kEmitGroup whose 2-byte
// gathers (one 128-B line per block) are issued one group ahead, across tile
// boundaries too, so a wave always has a group of loads in flight while it
// emits the previous one.  Offsets arrive per tile with one coalesced load and
// are read per block with readlane.  All loads are VMEM (ordered against the
// symbol stores' data reads), so no store-data hazard arises.
constexpr int kEmitGroup = 16;
constexpr int kGroup = 8;  // decode: blocks per group

__device__ __forceinline__ int tile_blocks(long long t, long long nblk) {
    const long long r = nblk - t * 64;
    return r < 64 ? (int)r : 64;
}

__device__ __forceinline__ void emit_gather(const int16_t *coef, long long t, int g, int nb, int nat,
                                            int16_t (&v)[kEmitGroup]) {
    const int16_t *base = coef + t * 64 * 64 + nat;
#pragma unroll
    for (int u = 0; u < kEmitGroup; ++u) {
        const int jb = g + u < nb ? g + u : nb - 1;
        v[u] = base[(long long)jb * 64];
    }
}

__global__ __launch_bounds__(kRleThreads) void rle_emit_kernel(const int16_t *__restrict__ coef, long long nblk,
                                                               const uint32_t *__restrict__ offsets,
                                                               uint32_t *__restrict__ symbols, long long ntiles) {
    const int lane = threadIdx.x & 63;
    const long long stride = (long long)gridDim.x * kRleWaves;
    const int nat = kZigzag[lane];
    const uint64_t below = lane_mask_below(lane);
    long long t = (long long)blockIdx.x * kRleWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (t >= ntiles) return;
    int g = 0, nb = tile_blocks(t, nblk);
    uint32_t offv = offsets[t * 64 + (lane < nb ? lane : nb - 1)];
    int16_t v[kEmitGroup];
    emit_gather(coef, t, 0, nb, nat, v);
    for (;;) {
        // the next group (possibly the first of the wave's next tile), requested before this one is emitted
        long long tn = t;
        int gn = g + kEmitGroup, nbn = nb;
        if (gn >= nb) {
            tn = t + stride;
            gn = 0;
            nbn = tn < ntiles ? tile_blocks(tn, nblk) : 1;
        }
        int16_t vn[kEmitGroup];
        uint32_t offn = offv;
        if (tn < ntiles) {
            emit_gather(coef, tn, gn, nbn, nat, vn);
            if (gn == 0) offn = offsets[tn * 64 + (lane < nbn ? lane : nbn - 1)];
        }
#pragma unroll
        for (int u = 0; u < kEmitGroup; ++u) {
            if (g + u >= nb) break;
            const uint32_t o = __builtin_amdgcn_readlane(offv, g + u);
            const bool emit = v[u] != 0 || lane == 63;
            const uint64_t prev = __builtin_amdgcn_ballot_w64(emit) & below;
            const int p = prev ? 63 - __builtin_clzll(prev) : -1;
            const uint32_t runlen = (uint32_t)(lane - p - 1) + (lane == 63 && v[u] == 0 ? 1u : 0u);
            if (emit) symbols[o + (uint32_t)__builtin_popcountll(prev)] = (uint32_t)(uint16_t)v[u] | (runlen << 16);
        }
        if (tn >= ntiles) break;
        t = tn;
        g = gn;
        nb = nbn;
        offv = offn;
#pragma unroll
        for (int u = 0; u < kEmitGroup; ++u) v[u] = vn[u];
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

hipError_t launch_rle_count(const int16_t *coef, long long nblk, uint32_t *offsets, void *ws, hipStream_t stream,
                            int num_cus) {
    const long long ntiles = (nblk + 63) / 64;
    uint32_t *tiles = (uint32_t *)ws;
    hipLaunchKernelGGL(rle_count_kernel, dim3(grid_for(ntiles, num_cus)), dim3(kRleThreads), 0, stream, coef, nblk,
                       offsets, tiles, ntiles);
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
