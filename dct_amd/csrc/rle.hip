// dct_amd/csrc/rle.hip -- zigzag + run-length symbols of quantized blocks on the GPU
// (shrink the coefficient planes before the xGMI gather).
//
// Per block this is exactly the reference's run_length_encode
// (src/entropy.c:216-256 over block_to_zigzag :158-178): one symbol per
// nonzero zigzag element, its run = zeros before it, plus always a symbol for
// the last element (7,7), whose run also counts itself when it is zero.  So a
// block has exactly 1 + nnz(first 63 zigzag elements) symbols.  Blocks are
// concatenated in order.  Two symbol formats (round 5):
//   W = 4 (uint32): (uint16)value | run << 16 -- any int16 value;
//   W = 2 (uint16): (run & 63) << 10 | (value & 0x3FF) -- |value| <= 511, which a
//         plan guarantees when its Q table bounds every quantized coefficient there
//         (api.hip symbol_bytes; q <= 90 of the standard table): 2 B per symbol,
//         so dense noise's 45.7 symbols per block take 91 B instead of 183 B --
//         less than the 128 B of int16 coefficients they shrink.
//         Runs are 0..63 except in the one symbol of an all-zero block, (0, 64),
//         which packs to 0x0000: no other symbol does (a zero value only ends a
//         block, and then its run counts itself, >= 1).
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
#include "zigzag.h"

namespace dctq {

constexpr int kCountPolicy = kNtAux;  // count's tile loads: non-temporal (read once)
constexpr int kRleWaves = 4;
constexpr int kRleThreads = 64 * kRleWaves;

// A symbol of value v (int16 bits in the low half of `v16`) and run r in format W.
template <int W>
__device__ __forceinline__ uint32_t pack_sym(uint32_t v16, uint32_t r) {
    if constexpr (W == 4) return (v16 & 0xFFFFu) | (r << 16);
    else return ((r & 63u) << 10) | (v16 & 0x3FFu);  // (0, 64) -> 0x0000
}
// ... and back: the run, and the value as int16 bits (sign-extended from 10 bits for W = 2)
template <int W>
__device__ __forceinline__ uint32_t sym_run(uint32_t s) {
    if constexpr (W == 4) return s >> 16;
    else return (s & 0xFFFFu) ? (s >> 10) & 0x3Fu : 64u;
}
template <int W>
__device__ __forceinline__ int16_t sym_value(uint32_t s) {
    if constexpr (W == 4) return (int16_t)(s & 0xFFFFu);
    else return (int16_t)((int32_t)(s << 22) >> 22);
}

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
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, k * 1024, kCountPolicy);
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

// ---- exclusive scan of the tile totals in place, segment by segment: one
// workgroup of 1024 per segment of 8192 tiles (each thread scans 8 consecutive
// totals from two 16-B loads, a wave scan and a 16-entry LDS pass combine the
// threads); the segment's sum -> segs[s].  The segments' own prefix is added in
// the fix-up, which also writes the grand total.
constexpr int kScanThreads = 1024;
constexpr int kScanPer = 8;
constexpr int kSegTilesLog2 = 13;  // 1024 * 8 tiles per segment

__global__ __launch_bounds__(kScanThreads) void rle_scan_tiles_kernel(uint32_t *__restrict__ tiles, long long ntiles,
                                                                      uint32_t *__restrict__ segs) {
    __shared__ uint32_t wsum[kScanThreads / 64];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const long long c0 = (long long)blockIdx.x << kSegTilesLog2;
    const long long i0 = c0 + (long long)tid * kScanPer;
    uint32_t v[kScanPer];
    if (i0 + kScanPer <= ntiles) {
        const uint4 a = *reinterpret_cast<const uint4 *>(tiles + i0), b = *reinterpret_cast<const uint4 *>(tiles + i0 + 4);
        v[0] = a.x, v[1] = a.y, v[2] = a.z, v[3] = a.w, v[4] = b.x, v[5] = b.y, v[6] = b.z, v[7] = b.w;
    } else {
#pragma unroll
        for (int i = 0; i < kScanPer; ++i) v[i] = i0 + i < ntiles ? tiles[i0 + i] : 0u;
    }
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
    uint32_t acc = wpre + inc - s;
    uint32_t out[kScanPer];
#pragma unroll
    for (int i = 0; i < kScanPer; ++i) {
        out[i] = acc;
        acc += v[i];
    }
    if (i0 + kScanPer <= ntiles) {
        *reinterpret_cast<uint4 *>(tiles + i0) = make_uint4(out[0], out[1], out[2], out[3]);
        *reinterpret_cast<uint4 *>(tiles + i0 + 4) = make_uint4(out[4], out[5], out[6], out[7]);
    } else {
#pragma unroll
        for (int i = 0; i < kScanPer; ++i)
            if (i0 + i < ntiles) tiles[i0 + i] = out[i];
    }
    if (tid == 0) segs[blockIdx.x] = ctot;
}

// offsets[b] += tile prefix (within its segment) + the segment's prefix, for
// blocks b of one plane whose tiles start at global tile tile0 (0 for a plain
// coefficient array; the encoder runs one fix-up per plane).  The <= 128 segment
// sums are scanned into LDS by the first wave; total_out (if set) gets the
// grand total.
__global__ __launch_bounds__(kRleThreads) void rle_fixup_kernel(uint32_t *__restrict__ offsets,
                                                                const uint32_t *__restrict__ tiles,
                                                                const uint32_t *__restrict__ segs, int nsegs,
                                                                long long nblk, long long tile0,
                                                                uint32_t *__restrict__ total_out) {
    __shared__ uint32_t segpre[129];
    const int lane = threadIdx.x & 63;
    if (threadIdx.x < 64) {  // exclusive prefix of the segment sums, two per lane
        const uint32_t a = 2 * lane < nsegs ? segs[2 * lane] : 0u, b = 2 * lane + 1 < nsegs ? segs[2 * lane + 1] : 0u;
        const uint32_t inc = wave_inclusive_scan(a + b);
        segpre[2 * lane] = inc - a - b;
        segpre[2 * lane + 1] = inc - b;
        if (lane == 63) segpre[128] = inc;
    }
    __syncthreads();
    const long long b = (long long)blockIdx.x * kRleThreads + threadIdx.x;
    if (b < nblk) {
        const long long t = tile0 + (b >> 6);
        offsets[b] += tiles[t] + segpre[t >> kSegTilesLog2];
    }
    if (total_out && blockIdx.x == 0 && threadIdx.x == 0) *total_out = segpre[128];
}

// ---- emit: one wave per 64-block tile, lane i = zigzag element i of the
// current block.
//
// Address throughput, not bytes, bounded the first versions: a CU's texture
// addresser takes ~2 lane-addresses per cycle (measured: 2-byte gathers + 4-byte
// symbol stores ran at 2.1-2.2 lane-addresses/cycle for dense and sparse
// symbol streams alike).  So the tile's 8 KiB comes in with eight 1 KiB loads
// (8 lane-addresses per block instead of 64), goes to LDS, and each block's
// zigzag element per lane is an LDS read.  All 64 LDS reads of a tile happen
// before its first symbol store, after a vmcnt(0) at the top of the tile that
// retires the previous tile's stores (store-data hazard); the next
// tile's loads are in flight meanwhile.  Per block (~14 VALU): E = ballot(emit);
// the symbol's index is mbcnt(E); its run is lane - 63 + clz64(((E << 1) | 1) &
// lanes <= i), the sentinel bit 0 standing for "no earlier symbol".  Only the
// emitting lanes store (exec mask).
__device__ __forceinline__ int tile_blocks(long long t, long long nblk) {
    const long long r = nblk - t * 64;
    return r < 0 ? 0 : r < 64 ? (int)r : 64;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const int16_t *coef, long long t, int nb) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<int16_t *>(coef) + (nb ? t * 64 * 64 : 0), (short)0, nb * 128,
                                             0x00020000);
}

typedef uint32_t u4r __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// zigzag position -> natural index as a compile-time table (register indexing
// in the lane-per-block walk below must resolve statically)
constexpr uint8_t kZzStatic[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                   12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                   35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                   58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
constexpr int kEmitPitch = 144;  // LDS bytes per block (128 + 16: lane-per-block row reads are conflict-free)
constexpr int kEmitLds = 64 * kEmitPitch;
constexpr uint32_t kLaneWalkMax = 2048;  // symbols of a tile the lane-per-block path stages
static_assert(kLaneWalkMax <= kEmitLds / 4 && kLaneWalkMax <= 2048, "two flush rounds of 1 024");
// 2-byte symbols: every tile fits the staging (64 x 64 symbols + one unit of padding in the
// 9 KiB), so every tile takes the lane-per-block path -- dense ones too: -5.8 % on the bench's
// encode step against the wave path above 2 048 (profiles/r05/encode_walk4k_ab.log)
constexpr uint32_t kLaneWalkMax2 = kLaneWalkMax ? 4096u : 0u;
static_assert(2 * kLaneWalkMax2 + 2 <= kEmitLds, "2-byte staging (one unit of padding) fits the tile's LDS");
constexpr int kMaxChunks = 16;  // chunks of 64 symbols per flush round

// A tile whose symbols fit the wave's LDS (natural content: ~6 symbols per
// block) is walked lane-per-block: lane b reads block b's row, walks its 64
// zigzag elements in registers (~6 VALU per element, no cross-lane work) and
// writes its symbols at offsets[b] - offsets[64t] into LDS, which then leaves
// as coalesced dword stores.  Denser tiles take the wave-per-block path.
template <int W>
__device__ __forceinline__ void emit_lane_walk(const char *lt, char *ls, int lane, uint32_t base) {
    uint32_t z[32];  // block `lane`, natural order, two elements per dword
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const u4r v = *reinterpret_cast<const u4r *>(lt + lane * kEmitPitch + 16 * k);
        z[4 * k] = v[0], z[4 * k + 1] = v[1], z[4 * k + 2] = v[2], z[4 * k + 3] = v[3];
    }
    wave_sync_lds();  // every lane's row is in registers before the symbols overwrite the tile
    // Branch-free: every element writes its would-be symbol at the block's next
    // slot, which advances only past a nonzero -- a zero's write is overwritten
    // by the next symbol (the last element always is one), so the slots
    // [base, base + count) end up exactly the block's symbols.
    uint32_t pos = base, run = 0;
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        const int c = kZzStatic[i];
        const uint32_t w = z[c >> 1];
        const bool nz = (c & 1) ? w > 0xFFFFu : (w & 0xFFFFu) != 0u;
        // the last element's run counts itself when zero
        const uint32_t r = (i == 63 && !nz) ? run + 1u : run;
        if constexpr (W == 4) {  // (uint16)value | run << 16
            const uint32_t sym = __builtin_amdgcn_perm(r, w, (c & 1) ? 0x05040302u : 0x05040100u);
            *reinterpret_cast<uint32_t *>(ls + pos * 4u) = sym;
        } else {
            *reinterpret_cast<uint16_t *>(ls + pos * 2u) = (uint16_t)pack_sym<2>((c & 1) ? w >> 16 : w, r);
        }
        pos += nz ? 1u : 0u;
        run = nz ? 0u : run + 1u;
    }
}

template <int W>
__global__ __launch_bounds__(kRleThreads, 4) void rle_emit_kernel(const int16_t *__restrict__ coef, long long nblk,
                                                               const uint32_t *__restrict__ offsets,
                                                               void *__restrict__ symbols, long long ntiles,
                                                               unsigned long long capacity) {
    __shared__ u4r tiles_lds[kRleWaves][kEmitLds / 16];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const long long stride = (long long)gridDim.x * kRleWaves;
    const uint32_t zoff = 2u * kZigzag[lane];
    const uint64_t upto = ~0ull >> (63 - lane);  // lanes 0..lane
    const uint32_t upto_lo = (uint32_t)upto, upto_hi = (uint32_t)(upto >> 32);
    const long long noffs = nblk + 1;  // offsets[nblk] = end of the last block's symbols
    const __amdgpu_buffer_rsrc_t roff = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint32_t *>(offsets), (short)0, (int)(noffs * 4 < 0x7FFFFFFF ? noffs * 4 : 0x7FFFFFFF), 0x00020000);
    long long t = (long long)blockIdx.x * kRleWaves + wv;
    if (t >= ntiles) return;
    u4r nq[8];
    uint32_t noff, nend;
    auto load_tile = [&](long long tt) {  // past the last tile: everything clipped, no traffic
        const int nb = tile_blocks(tt, nblk);
        const __amdgpu_buffer_rsrc_t rs = tile_rsrc(coef, tt, nb);
#pragma unroll
        for (int k = 0; k < 8; ++k) nq[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, k * 1024, 2 /* nt */);
        noff = __builtin_amdgcn_raw_buffer_load_b32(roff, tt < ntiles ? (uint32_t)(tt * 64 + lane) * 4u : 0xFFFFFFF0u,
                                                    0, 0);
        nend = __builtin_amdgcn_raw_buffer_load_b32(roff, tt < ntiles ? (uint32_t)(tt * 64 + nb) * 4u : 0xFFFFFFF0u,
                                                    0, 0);
    };
    load_tile(t);
    char *lt = reinterpret_cast<char *>(tiles_lds[wv]);
    // chunk k*64 + lane of the tile = block 8k + lane/8, bytes 16*(lane%8) of its row
    const uint32_t wr = (uint32_t)(lane >> 3) * kEmitPitch + 16u * (lane & 7);
    for (; t < ntiles; t += stride) {
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this tile's loads and the previous tile's stores
        const uint32_t offv = noff;
        const uint32_t o0 = __builtin_amdgcn_readlane(offv, 0);
        const uint32_t nsym = __builtin_amdgcn_readfirstlane(nend) - o0;
#pragma unroll
        for (int k = 0; k < 8; ++k) *reinterpret_cast<u4r *>(lt + 8 * k * kEmitPitch + wr) = nq[k];
        load_tile(t + stride);
        wave_sync_lds();
        const int nb = tile_blocks(t, nblk);
        // the tile's symbols start at offsets[64t]: a per-tile descriptor keeps the
        // 32-bit voffset small (the stream itself may exceed 4 GiB); symbols at or
        // past `capacity` are dropped by num_records
        const unsigned long long room = capacity > o0 ? capacity - o0 : 0ull;
        if (W == 2 && nsym <= kLaneWalkMax2) {
            // 2-B symbols: the tile's stream is staged one unit late when it starts at an
            // odd unit, so LDS dword j is global dword (o0 - pad) / 2 + j.  Whole dwords go
            // out as b32 through a descriptor that ends at the last whole one; the (at most
            // two) dwords shared with a neighbour tile or cut by `capacity` are written as
            // their one unit by lane 0 afterwards (values read with the chunks, before any
            // store: store-data hazard)
            const uint32_t pad = o0 & 1u;
            if (lane < nb) emit_lane_walk<2>(lt, lt, lane, offv - o0 + pad);
            wave_sync_lds();
            const unsigned long long first = o0 - pad;  // even: the descriptor base is 4-B aligned
            const unsigned long long cap = capacity > first ? capacity - first : 0ull;  // units below capacity
            const uint32_t end = (uint32_t)(cap < pad + nsym ? cap : pad + nsym);      // units [pad, end) land
            uint16_t *base16 = reinterpret_cast<uint16_t *>(symbols) + first;
            const __amdgpu_buffer_rsrc_t rfull =
                __builtin_amdgcn_make_buffer_rsrc(base16, (short)0, (int)((end & ~1u) * 2u), 0x00020000);
            const __amdgpu_buffer_rsrc_t redge = __builtin_amdgcn_make_buffer_rsrc(base16, (short)0, (int)(end * 2u),
                                                                                  0x00020000);
            const bool head = pad && end > 1u, tail = (end & 1u) && end - 1u >= pad;  // wave-uniform
            const uint16_t *l16 = reinterpret_cast<const uint16_t *>(lt);
            const uint32_t uhead = head ? l16[1] : 0u, utail = tail ? l16[end - 1u] : 0u;
            const uint32_t ndw = end >> 1;  // whole dwords (dword 0 is not one when pad)
#pragma unroll
            for (int r = 0; r < (int)((kLaneWalkMax2 / 2 + 1 + 1023) / 1024); ++r) {
                if (r * 1024 >= (int)ndw) break;
                if (r) __builtin_amdgcn_s_waitcnt(0x0F70);
                uint32_t v[kMaxChunks];
#pragma unroll
                for (int j = 0; j < kMaxChunks; ++j)
                    v[j] = *reinterpret_cast<const uint32_t *>(lt + ((r * kMaxChunks + j) * 64 + lane) * 4);
#pragma unroll
                for (int g = 0; g < kMaxChunks; g += 4)
                    if ((r * kMaxChunks + g) * 64 < (int)ndw) {
#pragma unroll
                        for (int j = g; j < g + 4; ++j) {
                            const uint32_t d = (uint32_t)((r * kMaxChunks + j) * 64 + lane);
                            if (r || j || lane || !pad)  // dword 0 holds a neighbour's unit when pad
                                __builtin_amdgcn_raw_buffer_store_b32(v[j], rfull, d * 4u, 0, 0);
                        }
                    }
            }
            if (lane == 0) {
                if (head) __builtin_amdgcn_raw_buffer_store_b16((uint16_t)uhead, redge, 2u, 0, 0);
                if (tail) __builtin_amdgcn_raw_buffer_store_b16((uint16_t)utail, redge, (end - 1u) * 2u, 0, 0);
            }
            continue;
        }
        if (W == 4 && nsym <= kLaneWalkMax) {
            if (lane < nb) emit_lane_walk<4>(lt, lt, lane, offv - o0);
            wave_sync_lds();
            const uint32_t nrec = (uint32_t)(room < nsym ? room : nsym) * 4u;
            const __amdgpu_buffer_rsrc_t rsym = __builtin_amdgcn_make_buffer_rsrc(
                reinterpret_cast<uint32_t *>(symbols) + o0, (short)0, (int)nrec, 0x00020000);
            // all LDS reads of a round first, then its stores (store-data hazard):
            // chunks of 64 symbols in guarded groups of 4, the tail clipped by num_records;
            // a second round (past 1 024 symbols) starts after a vmcnt(0)
#pragma unroll
            for (int r = 0; r < (int)((kLaneWalkMax + 1023) / 1024); ++r) {
                if (r * 1024 >= (int)nsym) break;
                if (r) __builtin_amdgcn_s_waitcnt(0x0F70);
                uint32_t v[kMaxChunks];
#pragma unroll
                for (int j = 0; j < kMaxChunks; ++j)
                    v[j] = *reinterpret_cast<const uint32_t *>(lt + ((r * kMaxChunks + j) * 64 + lane) * 4);
#pragma unroll
                for (int g = 0; g < kMaxChunks; g += 4)
                    if ((r * kMaxChunks + g) * 64 < (int)nsym) {
#pragma unroll
                        for (int j = g; j < g + 4; ++j)
                            __builtin_amdgcn_raw_buffer_store_b32(v[j], rsym, ((r * kMaxChunks + j) * 64 + lane) * 4,
                                                                  0, 0);
                    }
            }
            continue;
        }
        uint32_t z[32];  // two blocks' elements per register (64 live VGPRs would halve the occupancy)
#pragma unroll
        for (int u = 0; u < 32; ++u)
            z[u] = (uint32_t)*reinterpret_cast<const uint16_t *>(lt + 2 * u * kEmitPitch + zoff) |
                   ((uint32_t)*reinterpret_cast<const uint16_t *>(lt + (2 * u + 1) * kEmitPitch + zoff) << 16);
        const __amdgpu_buffer_rsrc_t rsym = __builtin_amdgcn_make_buffer_rsrc(
            reinterpret_cast<char *>(symbols) + o0 * (unsigned long long)W, (short)0,
            (int)((room < 4096ull ? room : 4096ull) * W), 0x00020000);
#pragma unroll
        for (int u = 0; u < 64; ++u) {
            const uint32_t val = (u & 1) ? z[u >> 1] >> 16 : z[u >> 1] & 0xFFFFu;
            const bool emit = val != 0u || lane == 63;
            const uint64_t E = __builtin_amdgcn_ballot_w64(emit);
            const uint64_t E2 = (E << 1) | 1ull;  // SALU; bit 0: "no earlier symbol"
            const uint64_t prev =
                (uint64_t)(upto_lo & (uint32_t)E2) | ((uint64_t)(upto_hi & (uint32_t)(E2 >> 32)) << 32);
            uint32_t runlen = (uint32_t)(lane - 63 + __builtin_clzll(prev));
            if (lane == 63 && val == 0u) runlen += 1u;  // the last symbol's run counts itself (src/entropy.c:231-233)
            const uint32_t idx =
                __builtin_amdgcn_mbcnt_hi((uint32_t)(E >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)E, 0u));
            const uint32_t o = __builtin_amdgcn_readlane(offv, u);
            // exec-masked: only emitting lanes reach the addresser (-4 % dense, -6 % sparse
            // against unconditional stores aimed past num_records, tools/rle_ab.py); the
            // vmcnt(0) at the top of the next tile is explicit, so LLVM's waitcnt
            // placement around predicated stores does not matter here
            if (emit && u < nb) {
                if constexpr (W == 4)
                    __builtin_amdgcn_raw_buffer_store_b32(pack_sym<4>(val, runlen), rsym, (o - o0 + idx) * 4u, 0, 0);
                else
                    __builtin_amdgcn_raw_buffer_store_b16((uint16_t)pack_sym<2>(val, runlen), rsym, (o - o0 + idx) * 2u, 0,
                                                          0);
            }
        }
    }
}

// ---- decode: one wave per 64-block tile, rebuilt 32 blocks at a time in a
// natural-order LDS copy (8 waves/SIMD) and written as 1 KiB stores (8
// lane-addresses per block).  Each half takes one of three paths by its symbol
// count: lane (<= 240), walk (<= kDecWalkMax) or quad (denser halves);
// all three place each symbol at zigzag position pos (run_length_decode: pos +=
// run; zigzag[pos++] = value, dropped past the end, src/entropy.c:327-351) of
// its block's natural-order row (zigzag_to_block, :183-210, through an LDS copy
// of the order).  Every symbol load goes through a buffer descriptor whose
// num_records ends at the half's last symbol, so no path reads past the
// stream.  Each half tile's LDS work starts after a vmcnt(0) that retires the
// previous half's stores (store-data hazard); no store is issued inside the half.
constexpr int kHalf = 32;

// offv: lane b holds offsets[64t + b] (b < nb); oend = offsets[64t + nb], the end
// of the tile's symbols (lane 64 does not exist, and readlane(64) would wrap).
__device__ __forceinline__ uint32_t off_at(uint32_t offv, uint32_t oend, int b) {
    return b < 64 ? __builtin_amdgcn_readlane(offv, b) : oend;
}

// Walk path (a half tile of at most kDecWalkMax symbols): lane i < 32 rebuilds
// block h+i on its own -- its symbols as 16-B loads (four per lane-address,
// the next kDecBatch in flight while these are placed), each value written at
// zigzag[pos] of its row in a zeroed natural-order half tile (pos += run; put
// while pos < 64; pos++).  The row pitch is 144 B: a symbol past position 63
// or past the block's count lands in the row's 16-B padding, so placement is
// branch-free.  A block's count is clamped to 64, which bounds the walk for
// any offsets.  Denser halves take the scan-and-scatter path (pitch 128).
// 4.5 KiB per wave keeps 8 waves/SIMD.
//
// Lane path (a half tile of at most kDecLaneMax symbols: natural content): the
// half's symbols come in as coalesced dword loads and go to LDS behind the
// zeroed half tile (pitch 128), and lane i < 32 walks block h+i's symbols from
// there, clamped to the half's symbols.  Faster than the walk path at this
// density (one coalesced load per 64 symbols instead of per-lane 16-B loads).
//
// 4 KiB + 960 B per wave keeps 8 waves/SIMD (the scan path needs them).
constexpr uint32_t kDecLaneMax = 240, kDecWalkMax = 1024;
constexpr int kDecPitch = 144;
constexpr int kDecBatch = 16;  // symbols per lane per step
constexpr int kDecLds = kHalf * 128 + 240 * 4;  // >= kHalf * kDecPitch
static_assert(kDecLds >= kHalf * kDecPitch, "walk path tile");

// 2-B symbols widened to the 4-B format in registers: the decode paths below then
// run unchanged.  Units sit two per dword; a lane whose units start at an odd unit
// loads from the dword before and shifts by 16 bits (v_alignbit).
__device__ __forceinline__ uint32_t widen16(uint32_t u) {
    return pack_sym<4>((uint32_t)(uint16_t)sym_value<2>(u), sym_run<2>(u));
}
// units [u, u + 2N) from dword-aligned `d` (N + 1 dwords: d[0] holds unit u & ~1)
template <int N>
__device__ __forceinline__ void align_units(const uint32_t (&d)[N + 1], uint32_t odd, uint32_t (&out)[N]) {
#pragma unroll
    for (int k = 0; k < N; ++k) out[k] = __builtin_amdgcn_alignbit(d[k + 1], d[k], odd * 16u);
}

// (the 2-byte instantiation asks for 7 waves/SIMD: at 8 the register allocator spilled two
// VGPRs; at 7 it fits in 61, so it still runs 8)
template <int W>
__global__ __launch_bounds__(kRleThreads, W == 4 ? 8 : 7) void rle_decode_kernel(const void *__restrict__ symbols,
                                                                 const uint32_t *__restrict__ offsets, long long nblk,
                                                                 int16_t *__restrict__ coef, long long ntiles) {
    __shared__ u4r wave_lds[kRleWaves][kDecLds / 16];
    __shared__ uint8_t zz[64];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (threadIdx.x < 64) zz[threadIdx.x] = kZigzag[threadIdx.x];
    __syncthreads();
    const long long stride = (long long)gridDim.x * kRleWaves;
    char *lt = reinterpret_cast<char *>(wave_lds[wv]);
    uint32_t *lsym = reinterpret_cast<uint32_t *>(lt + kHalf * 128);
    for (long long t = (long long)blockIdx.x * kRleWaves + wv; t < ntiles; t += stride) {
        const long long b0 = t * 64;
        const int nb = tile_blocks(t, nblk);
        const uint32_t offv = offsets[b0 + (lane < nb ? lane : nb)];  // lanes >= nb: the end of the tile
        const uint32_t oend = offsets[b0 + nb];
        // per-lane block symbol count (lane b: block b of the tile)
        const uint32_t nxt_off = (uint32_t)__shfl_down((int)offv, 1);
        const uint32_t cnt_lane = (lane == 63 ? oend : nxt_off) - offv;
        for (int h = 0; h < nb; h += kHalf) {
            const int he = nb < h + kHalf ? nb : h + kHalf;
            const uint32_t s0 = __builtin_amdgcn_readlane(offv, h), nh = off_at(offv, oend, he) - s0;
            const bool lane_path = kDecLaneMax && nh <= kDecLaneMax;
            const bool walk = !lane_path && kDecWalkMax && nh <= kDecWalkMax;
            if (lane_path) {
                const __amdgpu_buffer_rsrc_t rsy = __builtin_amdgcn_make_buffer_rsrc(
                    const_cast<char *>(reinterpret_cast<const char *>(symbols)) + (unsigned long long)s0 * W, (short)0,
                    (int)(nh * W), 0x00020000);
                uint32_t v[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {  // past nh: clipped to 0, no traffic
                    if constexpr (W == 4)
                        v[j] = __builtin_amdgcn_raw_buffer_load_b32(rsy, (j * 64 + lane) * 4, 0, 0);
                    else
                        v[j] = widen16(__builtin_amdgcn_raw_buffer_load_b16(rsy, (j * 64 + lane) * 2, 0, 0));
                }
                // block h+i's start and count, to lane i
                const uint32_t my_off = (uint32_t)__shfl((int)offv, (lane + h) & 63);
                const uint32_t my_cnt = (uint32_t)__shfl((int)cnt_lane, (lane + h) & 63);
                // vmcnt(0): these loads, and the previous half's stores before any LDS read (store-data hazard)
                __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (j < 3 || lane < 48) lsym[j * 64 + lane] = v[j];
#pragma unroll
                for (int k = 0; k < 4; ++k) reinterpret_cast<u4r *>(lt)[k * 64 + lane] = u4r{0u, 0u, 0u, 0u};
                wave_sync_lds();
                // a block's symbols must lie inside the half's (bounds the walk for any offsets)
                const uint32_t base = my_off - s0;
                const uint32_t cnt =
                    lane < he - h && base <= nh ? (my_cnt < nh - base ? my_cnt : nh - base) : 0u;
                int16_t *row = reinterpret_cast<int16_t *>(lt + (lane & 31) * 128);
                uint32_t pos = 0;
                for (uint32_t i = 0; i < cnt; ++i) {
                    const uint32_t sym = lsym[base + i];
                    pos += sym >> 16;
                    if (pos < 64u) row[zz[pos]] = (int16_t)(sym & 0xFFFFu);
                    pos += 1u;
                }
            } else if (walk) {
                // the half's symbols; loads past them (any lane, any offsets) are clipped to 0.
                // 2-B units: the descriptor starts at the even unit at or before s0 and ends on
                // a whole dword (one unit past the half at most: inside the stream's 4-B-aligned
                // allocation)
                const uint32_t pad = W == 2 ? (s0 & 1u) : 0u;
                const __amdgpu_buffer_rsrc_t rsy = __builtin_amdgcn_make_buffer_rsrc(
                    const_cast<char *>(reinterpret_cast<const char *>(symbols)) + (unsigned long long)(s0 - pad) * W,
                    (short)0, (int)(W == 4 ? nh * 4u : ((pad + nh + 1u) & ~1u) * 2u), 0x00020000);
                const uint32_t my_off = (uint32_t)__shfl((int)offv, (lane + h) & 63);
                const uint32_t my_cnt = (uint32_t)__shfl((int)cnt_lane, (lane + h) & 63);
                const uint32_t cnt = lane < he - h ? (my_cnt < 64u ? my_cnt : 64u) : 0u;
                const uint32_t urel = my_off - s0 + pad;  // the block's first unit from the descriptor base
                const uint32_t rel = W == 4 ? (my_off - s0) * 4u : (urel & ~1u) * 2u, odd = urel & 1u;
                auto load_batch = [&](uint32_t i, u4r (&q)[kDecBatch / 4]) {
                    if constexpr (W == 4) {
#pragma unroll
                        for (int k = 0; k < kDecBatch / 4; ++k)
                            q[k] = i + 4 * k < cnt
                                       ? __builtin_amdgcn_raw_buffer_load_b128(rsy, rel + (i + 4 * k) * 4u, 0, 0)
                                       : u4r{0u, 0u, 0u, 0u};
                    } else {  // kDecBatch units = 8 dwords, from 9 aligned ones
                        uint32_t d[kDecBatch / 2 + 1];
#pragma unroll
                        for (int k = 0; k < kDecBatch / 8; ++k) {
                            // dwords 4k..4k+3 hold units i + 8k - odd .. i + 8k - odd + 7
                            const u4r t = i + 8 * k < cnt + odd
                                              ? __builtin_amdgcn_raw_buffer_load_b128(rsy, rel + (i + 8 * k) * 2u, 0, 0)
                                              : u4r{0u, 0u, 0u, 0u};
                            d[4 * k] = t[0], d[4 * k + 1] = t[1], d[4 * k + 2] = t[2], d[4 * k + 3] = t[3];
                        }
                        d[kDecBatch / 2] = odd && i + kDecBatch - 1 < cnt
                                               ? __builtin_amdgcn_raw_buffer_load_b32(rsy, rel + (i + kDecBatch) * 2u, 0, 0)
                                               : 0u;
                        uint32_t a[kDecBatch / 2];
                        align_units<kDecBatch / 2>(d, odd, a);
#pragma unroll
                        for (int k = 0; k < kDecBatch / 4; ++k)
                            q[k] = u4r{widen16(a[2 * k]), widen16(a[2 * k] >> 16), widen16(a[2 * k + 1]),
                                       widen16(a[2 * k + 1] >> 16)};
                    }
                };
                u4r cur[kDecBatch / 4];
                load_batch(0, cur);
                // vmcnt(0) before any LDS read into registers: the previous half's stores
                // (store-data hazard); the walk's own loads are in the same count
                __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll
                for (int k = 0; k < 5; ++k)
                    if (k < 4 || lane < 32) reinterpret_cast<u4r *>(lt)[k * 64 + lane] = u4r{0u, 0u, 0u, 0u};
                wave_sync_lds();
                char *row = lt + (lane & 31) * kDecPitch;
                uint32_t pos = 0;
                for (uint32_t i = 0; __builtin_amdgcn_ballot_w64(i < cnt); i += kDecBatch) {
                    u4r nxt[kDecBatch / 4];
                    load_batch(i + kDecBatch, nxt);
#pragma unroll
                    for (int j = 0; j < kDecBatch; ++j) {
                        const uint32_t sym = cur[j >> 2][j & 3];
                        pos += sym >> 16;
                        const bool put = pos < 64u && i + j < cnt;
                        const uint32_t at = put ? 2u * zz[pos < 64u ? pos : 63u] : 128u;  // 128: the padding
                        *reinterpret_cast<int16_t *>(row + at) = (int16_t)(sym & 0xFFFFu);
                        pos += 1u;
                    }
#pragma unroll
                    for (int k = 0; k < kDecBatch / 4; ++k) cur[k] = nxt[k];
                }
            } else {
                // Quad path: 4 blocks per step, one per 16-lane row; lane s of a row holds its
                // block's symbols 4s..4s+3 (one 16-B load: 4 symbols per lane-address). Positions:
                // a 4-element prefix in the lane, then a row-segmented DPP scan of the lane totals.
                const uint32_t pad = W == 2 ? (s0 & 1u) : 0u;  // as the walk path
                const __amdgpu_buffer_rsrc_t rsy = __builtin_amdgcn_make_buffer_rsrc(
                    const_cast<char *>(reinterpret_cast<const char *>(symbols)) + (unsigned long long)(s0 - pad) * W,
                    (short)0, (int)(W == 4 ? nh * 4u : ((pad + nh + 1u) & ~1u) * 2u), 0x00020000);
                const int r = lane >> 4, s4 = 4 * (lane & 15);
                auto group_load = [&](int g, u4r &q, uint32_t &cnt) {
                    const int b = h + 4 * g + r;  // this row's block (past `he`: none)
                    const uint32_t ob = (uint32_t)__shfl((int)offv, b & 63);
                    const uint32_t cb = (uint32_t)__shfl((int)cnt_lane, b & 63);
                    cnt = b < he ? (cb < 64u ? cb : 64u) : 0u;
                    if constexpr (W == 4) {
                        q = (uint32_t)s4 < cnt ? __builtin_amdgcn_raw_buffer_load_b128(rsy, (ob - s0 + s4) * 4u, 0, 0)
                                               : u4r{0u, 0u, 0u, 0u};
                    } else {  // units s4..s4+3 = 2 dwords, from 3 aligned ones
                        const uint32_t u = ob - s0 + pad + (uint32_t)s4, odd = u & 1u;
                        uint32_t d[3] = {0u, 0u, 0u};
                        if ((uint32_t)s4 < cnt) {
                            const auto t = __builtin_amdgcn_raw_buffer_load_b96(rsy, (u & ~1u) * 2u, 0, 0);
                            d[0] = t[0], d[1] = t[1], d[2] = t[2];
                        }
                        uint32_t a[2];
                        align_units<2>(d, odd, a);
                        q = u4r{widen16(a[0]), widen16(a[0] >> 16), widen16(a[1]), widen16(a[1] >> 16)};
                    }
                };
                const int ng = (he - h + 3) >> 2;
                u4r q;
                uint32_t cnt;
                group_load(0, q, cnt);
                // vmcnt(0) before any LDS read into registers: the previous half's stores (store-data hazard)
                __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll
                for (int k = 0; k < 5; ++k)
                    if (k < 4 || lane < 32) reinterpret_cast<u4r *>(lt)[k * 64 + lane] = u4r{0u, 0u, 0u, 0u};
                wave_sync_lds();
                for (int g = 0; g < ng; ++g) {
                    u4r nq;
                    uint32_t ncnt;
                    group_load(g + 1 < ng ? g + 1 : g, nq, ncnt);
                    uint32_t p[4], run = 0;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        run += (uint32_t)s4 + j < cnt ? (q[j] >> 16) + 1u : 0u;
                        p[j] = run;
                    }
                    uint32_t incl = run;  // row-segmented inclusive scan of the lane totals
                    incl += __builtin_amdgcn_update_dpp(0u, incl, 0x111, 0xF, 0xF, false);  // row_shr:1
                    incl += __builtin_amdgcn_update_dpp(0u, incl, 0x112, 0xF, 0xF, false);  // row_shr:2
                    incl += __builtin_amdgcn_update_dpp(0u, incl, 0x114, 0xF, 0xF, false);  // row_shr:4
                    incl += __builtin_amdgcn_update_dpp(0u, incl, 0x118, 0xF, 0xF, false);  // row_shr:8
                    const uint32_t before = incl - run;
                    char *row = lt + (4 * g + r) * kDecPitch;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const uint32_t pos = before + p[j] - 1u;
                        const bool put = (uint32_t)s4 + j < cnt && pos < 64u;
                        const uint32_t at = put ? 2u * zz[pos < 64u ? pos : 63u] : 128u;  // 128: the padding
                        *reinterpret_cast<int16_t *>(row + at) = (int16_t)(q[j] & 0xFFFFu);
                    }
                    q = nq;
                    cnt = ncnt;
                }
            }
            wave_sync_lds();
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the walk's last (clipped) loads before the read-out
            u4r val[4];
            const int pitch = lane_path ? 128 : kDecPitch;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                val[k] = *reinterpret_cast<const u4r *>(lt + (8 * k + (lane >> 3)) * pitch + 16 * (lane & 7));
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc(coef + (b0 + h) * 64, (short)0, (he - h) * 128, 0x00020000);
#pragma unroll
            for (int k = 0; k < 4; ++k) __builtin_amdgcn_raw_buffer_store_b128(val[k], rs, lane * 16, k * 1024, kNtAux);
        }
    }
}

// Grid = at most per_cu workgroups per CU (far more than are resident: the queued ones refill retiring
// slots at once, which evens out tiles of unequal symbol counts).  Against 16 per CU, one box
// (profiles/r02/grid_mult_ab.log, tools/rle_ab.py): count -3 to -5 % at 128, emit -1 to -8 % and decode
// 0 to -9 % at 64 (128 is one tile per wave at 64 4K frames; it loses 11 % on constant-block decode).
static unsigned grid_for(long long waves_wanted, int num_cus, int per_cu) {
    long long g = (waves_wanted + kRleWaves - 1) / kRleWaves;
    const long long cap = (long long)num_cus * per_cu;
    return (unsigned)(g < 1 ? 1 : g > cap ? cap : g);
}

// tile totals, then (16-B aligned) the segment sums
size_t rle_scan_workspace_bytes(long long ntiles) { return (size_t)((ntiles + 3) / 4 * 4) * 4 + 128 * 4; }
size_t rle_workspace_bytes(long long nblk) { return rle_scan_workspace_bytes((nblk + 63) / 64); }

// Scan of ntiles tile totals in ws (in place, by segment); then per plane
// launch_rle_fixup.
hipError_t launch_rle_scan(void *ws, long long ntiles, hipStream_t stream) {
    const int nsegs = (int)((ntiles + (1 << kSegTilesLog2) - 1) >> kSegTilesLog2);  // <= 128 for < 2^26 blocks
    uint32_t *tiles = (uint32_t *)ws;
    hipLaunchKernelGGL(rle_scan_tiles_kernel, dim3(nsegs), dim3(kScanThreads), 0, stream, tiles, ntiles,
                       tiles + (ntiles + 3) / 4 * 4);
    return hipGetLastError();
}

hipError_t launch_rle_fixup(uint32_t *offsets, long long nblk, const void *ws, long long ntiles, long long tile0,
                            uint32_t *total_out, hipStream_t stream) {
    const int nsegs = (int)((ntiles + (1 << kSegTilesLog2) - 1) >> kSegTilesLog2);
    const uint32_t *tiles = (const uint32_t *)ws;
    hipLaunchKernelGGL(rle_fixup_kernel, dim3((unsigned)((nblk + kRleThreads - 1) / kRleThreads)), dim3(kRleThreads),
                       0, stream, offsets, tiles, tiles + (ntiles + 3) / 4 * 4, nsegs, nblk, tile0, total_out);
    return hipGetLastError();
}

hipError_t launch_rle_count(const int16_t *coef, long long nblk, uint32_t *offsets, void *ws, hipStream_t stream,
                            int num_cus) {
    const long long ntiles = (nblk + 63) / 64;
    hipLaunchKernelGGL(rle_count_kernel, dim3(grid_for(ntiles, num_cus, 128)), dim3(kRleThreads), 0, stream, coef, nblk,
                       offsets, (uint32_t *)ws, ntiles);
    hipError_t e = launch_rle_scan(ws, ntiles, stream);
    if (e != hipSuccess) return e;
    return launch_rle_fixup(offsets, nblk, ws, ntiles, 0, offsets + nblk, stream);
}

hipError_t launch_rle_emit(const int16_t *coef, long long nblk, const uint32_t *offsets, void *symbols,
                           int symbol_bytes, unsigned long long capacity, hipStream_t stream, int num_cus) {
    const long long ntiles = (nblk + 63) / 64;
    // 2-byte emit: up to 1 024 workgroups per CU (about one tile per wave on the bench step):
    // -2.3..-2.9 % on the encode step against 64 (round 6, profiles/r06/rle_grid_ab/, tools/enc_ab.py);
    // the 4-byte emit was 5 % slower that way (tools/rle_ab.py), and the decoders 5-17 %, so they keep 64
    if (symbol_bytes == 2)
        hipLaunchKernelGGL(rle_emit_kernel<2>, dim3(grid_for(ntiles, num_cus, 1024)), dim3(kRleThreads), 0, stream, coef,
                           nblk, offsets, symbols, ntiles, capacity);
    else
        hipLaunchKernelGGL(rle_emit_kernel<4>, dim3(grid_for(ntiles, num_cus, 64)), dim3(kRleThreads), 0, stream, coef,
                           nblk, offsets, symbols, ntiles, capacity);
    return hipGetLastError();
}

hipError_t launch_rle_decode(const void *symbols, int symbol_bytes, const uint32_t *offsets, long long nblk,
                             int16_t *coef, hipStream_t stream, int num_cus) {
    const long long ntiles = (nblk + 63) / 64;
    if (symbol_bytes == 2)
        hipLaunchKernelGGL(rle_decode_kernel<2>, dim3(grid_for(ntiles, num_cus, 64)), dim3(kRleThreads), 0, stream,
                           symbols, offsets, nblk, coef, ntiles);
    else
        hipLaunchKernelGGL(rle_decode_kernel<4>, dim3(grid_for(ntiles, num_cus, 64)), dim3(kRleThreads), 0, stream,
                           symbols, offsets, nblk, coef, ntiles);
    return hipGetLastError();
}

}  // namespace dctq
