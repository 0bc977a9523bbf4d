// dct_amd/csrc/huffman.hip -- per-block Huffman size estimate on the GPU
// (SURVEY 8(f)4): for every quantized block, the bit count the reference's
// pipeline reports after coding that block on its own
// (tests/test_entropy.c:329-341):
//   run_length_encode (src/entropy.c:216-256) -> build_huffman_codes (:261-328)
//   -> get_encoded_size (:363-399) = sum over symbols of (len(code) + 8).
//
// What is computed, and why it is exact:
//  * The symbols of a block are its nonzero coefficients of zigzag positions
//    0..62 plus the last element (7,7), zero or not (rle.hip).  Frequencies do
//    not depend on order, so the multiset of symbol values is "every nonzero
//    coefficient, plus a value 0 once if c[63] == 0" -- no zigzag needed.
//  * build_huffman_codes merges the two minimum-frequency nodes of a binary heap
//    until one is left (src/entropy.c:26-77 pops a true minimum every time), so
//    its tree is a Huffman tree and sum(freq * depth) -- the code bits -- is the
//    optimum, the same for every tie order.  A single distinct value is a lone
//    leaf at depth 0 (code "", 0 bits).  Hence
//        bits = 8 * count + WPL(frequencies)
//    and WPL = the sum of the internal node weights of ANY Huffman merge order.
//  * The GPU merges in weight buckets: cnt[w] = nodes of weight w.  Scanning w
//    upward, the nodes of bucket w pair up among themselves (new weight 2w), an
//    odd one left over waits as `pending` and merges with one node of the next
//    non-empty bucket w' (new weight pending + w').  New weights are always above
//    the current bucket, every merge takes the two smallest nodes, and weights
//    never exceed count <= 64.
// The oracle restates the reference's heap literally (oracle/dct_oracle.c,
// orc_huffman_bits) and is pinned to the compiled reference; the GPU result is
// compared with it (tests/test_gpu_parity.py::test_huffman_bits*).
//
// Layout: one LANE per block (64 blocks per wave).  The wave's tile (8 KiB)
// arrives in LDS by LDS-DMA, the next one while the current one is processed.
// Dense tiles whose every block's values span < 64 integers (q50 noise) count
// their values in a workgroup-shared byte region and merge in registers
// (narrow_leaves / narrow_merge).  Other tiles sort each lane's values with a
// Batcher odd-even merge network in registers (equal values become adjacent;
// zeros map to the top and are dropped) -- all 64, or, when every block of the
// tile has at most 16 / 32 nonzero coefficients (natural content), just those,
// compacted through LDS -- add one count per run length into the same shared
// region (Hist), and run the bucket merge there.  VALU- and LDS-latency-bound
// at 3 waves/SIMD.
#include <type_traits>

#include "dctq_internal.h"
#include "fdct8_core.h"


namespace dctq {

constexpr int kHufWaves = 4;
constexpr int kHufThreads = 64 * kHufWaves;
// The wave's tile stage: 64 blocks x 128 B, 16-B piece k of block b at
// b * 128 + 16 * (k ^ ((b >> 1) & 7)) -- the XOR swizzle makes the lane-per-block
// ds_read_b128 of tile_row conflict-free (each 16-lane group of a b128 read
// covers 16 distinct 16-B bank groups) with no padding, so the tile can arrive
// by LDS-DMA (1 KiB contiguous per instruction; each lane picks its source piece).
// 9 KiB per wave: the sparse paths reuse it for their compacted keys (up to 33 slots
// of 256 B), huffman_from_pixels for the forward's stage (64 x kPitch2 + 128 B).
constexpr int kHufWaveLds = 9 * 1024;
// The narrow path's value counters and every path's weight histogram, one region
// shared by the workgroup's waves: byte  row * 256 + lane * 4 + wave  is wave `wave`'s
// 8-bit counter `row` of lane `lane` (counts never exceed 64).  Every lane owns
// a dword per row (conflict-free banks), the wave owns a byte of it (its adds
// are 1 << 8 * wave), and one v_perm builds a dword address from a value (byte
// 1 = the row, byte 0 = lane * 4).  Rows 0..63: value vmin + row; then rows 0..64: leaf / node weight.
constexpr int kHufCtrBytes = 65 * 256;

__device__ __forceinline__ void cas(uint32_t &a, uint32_t &b) {
    const uint32_t lo = a < b ? a : b, hi = a < b ? b : a;
    a = lo;
    b = hi;
}

// Batcher's odd-even merge sort of N registers (N = 16, 32, 64: 63, 191, 543
// compare-exchanges), fully unrolled so every index is a compile-time register.
template <int N>
__device__ __forceinline__ void sort_net(uint32_t (&a)[N]) {
#pragma unroll
    for (int p = 1; p < N; p <<= 1)
#pragma unroll
        for (int k = p; k >= 1; k >>= 1)
#pragma unroll
            for (int j = k % p; j + k < N; j += 2 * k)
#pragma unroll
                for (int i = 0; i < k; ++i)
                    if (i + j + k < N && (i + j) / (2 * p) == (i + j + k) / (2 * p)) cas(a[i + j], a[i + j + k]);
}

// The sparse and dense paths' weight histogram lives in the workgroup's shared
// byte region (kHufCtrBytes), like the narrow path's counters: byte
// w * 256 + lane * 4 + wave is the wave's count of nodes of weight w (<= 65) for
// that lane -- conflict-free, and the tile stage is free for the next tile's DMA as
// soon as the row (or the compacted keys) are in registers.  Every bucket is read
// AND cleared when the merge processes it, so the region stays zeroed between tiles.
struct Hist {
    char *ctr;
    uint32_t base, sh;  // lane * 4, 8 * wave
    __device__ __forceinline__ uint32_t *at(uint32_t w) const { return reinterpret_cast<uint32_t *>(ctr + (w << 8) + base); }
    __device__ __forceinline__ void add(uint32_t w, uint32_t n) const {
        __hip_atomic_fetch_add(at(w), n << sh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
    __device__ __forceinline__ uint32_t peek(uint32_t w) const { return (*at(w) >> sh) & 0xFFu; }
    __device__ __forceinline__ uint32_t take(uint32_t w) const {  // read and clear the wave's byte
        uint32_t keep = ~(0xFFu << sh);
        asm volatile("" : "+v"(keep));  // rematerialised per use (a hoisted copy spills in the fused kernel)
        return (__hip_atomic_fetch_and(at(w), keep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT) >> sh) & 0xFFu;
    }
};

// Occupancy of the lane's histogram: bit w-1 set while bucket w may hold nodes
// (the merge jumps from one occupied bucket to the next).  Occ64 is one uint64;
// Occ32x2 two 32-bit halves, for the fused kernel: there the zero high half of
// the first eight marks was a 64-bit constant it spilled (and the reload waited
// for every load in flight, the next batch's rows included).  The standalone
// kernel keeps Occ64 (the halves measured +2.6 % on extreme input there).
struct Occ64 {
    uint64_t m = 0;
    __device__ __forceinline__ void first8(uint32_t w, uint32_t n) { m |= n ? 1ull << (w - 1) : 0ull; }
    __device__ __forceinline__ bool any() const { return m != 0; }
    __device__ __forceinline__ void set(uint32_t w) { m |= 1ull << (w - 1); }
    __device__ __forceinline__ uint32_t pop() {
        const uint32_t w = (uint32_t)__builtin_ctzll(m) + 1u;
        m &= m - 1ull;
        return w;
    }
};
struct Occ32x2 {
    uint32_t lo = 0, hi = 0;  // buckets 1..32, 33..64
    __device__ __forceinline__ void first8(uint32_t w, uint32_t n) { lo |= n ? 1u << (w - 1) : 0u; }
    __device__ __forceinline__ bool any() const { return (lo | hi) != 0; }
    __device__ __forceinline__ void set(uint32_t w) {  // w in 1..64
        if (w <= 32)
            lo |= 1u << (w - 1);
        else
            hi |= 1u << (w - 33);
    }
    __device__ __forceinline__ uint32_t pop() {  // lowest occupied bucket, cleared
        if (lo) {
            const uint32_t w = (uint32_t)__builtin_ctz(lo) + 1u;
            lo &= lo - 1u;
            return w;
        }
        const uint32_t w = (uint32_t)__builtin_ctz(hi) + 33u;
        hi &= hi - 1u;
        return w;
    }
};

constexpr uint32_t kSent = 0xFFFFFFFFu;  // a zero coefficient (dropped)

// Sort key of coefficient i of a block held as 32 dwords (two int16 each):
// value*65536 - 1 as uint32 -- injective, and 0 -> kSent, which sorts last.
__device__ __forceinline__ uint32_t key_of(const uint32_t (&d)[32], int i) {
    return ((i & 1) ? (d[i >> 1] & 0xFFFF0000u) : (d[i >> 1] << 16)) - 1u;
}

// Runs of equal values in the sorted registers -> one histogram count per
// distinct value at its frequency; `nodes` += distinct values.
template <int N, bool kMax>
__device__ __forceinline__ void runs_to_hist(const uint32_t (&a)[N], const Hist &h, uint32_t &nodes,
                                             uint32_t &lmax) {
    // branch-free: every element adds (end ? 1 : 0) at its run length, so no
    // per-element exec mask is live (64 of them spilled to SGPR lanes)
    // a[] is sorted with kSent (max) last: a run ends where the next key differs,
    // and a kSent run is never one (the element after a kSent is kSent)
    uint32_t run = 1;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const uint32_t end = (i + 1 < N ? a[i] != a[i + 1 < N ? i + 1 : N - 1] : a[i] != kSent) ? 1u : 0u;
        h.add(run, end);
        if (kMax) lmax = end && run > lmax ? run : lmax;
        nodes += end;
        run = end ? 1u : run + 1u;
    }
}

// Sparse waves (every block of the tile has <= N nonzero coefficients): the
// nonzero values, compacted into the lane's LDS column (dword k*64 + lane:
// conflict-free), come back as N registers padded with kSent and take the
// N-network instead of the 64-one.
// The lane's 64 coefficients from its row of the tile stage, as 32 dwords.
// FWD: the row sits where the forward core left it (huffman_from_pixels_kernel):
// lane * kPitch2, 8-byte aligned, unswizzled.
template <bool FWD = false>
__device__ __forceinline__ void tile_row(const char *mine, int lane, uint32_t (&d)[32]) {
    if constexpr (FWD) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint2 w = *reinterpret_cast<const uint2 *>(mine + lane * kPitch2 + 8 * k);
            d[2 * k] = w.x;
            d[2 * k + 1] = w.y;
        }
        return;
    }
    // the row's address, made opaque per call: eight hoisted loop-invariant piece
    // addresses spilled; recomputed it is one v_xor per piece
    int row = (lane << 7) | (((lane >> 1) & 7) << 4);
    asm volatile("" : "+v"(row));
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint4 w = *reinterpret_cast<const uint4 *>(mine + (row ^ (k << 4)));
        d[4 * k] = w.x;
        d[4 * k + 1] = w.y;
        d[4 * k + 2] = w.z;
        d[4 * k + 3] = w.w;
    }
}

// Tile t (blocks 64t .. 64t + nb - 1) into the wave's stage by LDS-DMA: chunk c
// (1 KiB of LDS) holds blocks 8c .. 8c + 7, lane l the piece (l & 7) ^ ((b >> 1) & 7)
// of block b = 8c + (l >> 3) (the swizzle of tile_row).  No VGPRs, no ds_write:
// the next tile streams in while the narrow path works on this one.  The caller
// has retired its reads of the stage (lgkmcnt(0)); the data is there after
// vmcnt(0).  Blocks past the end are zeroed by the loop (the tail tile only).
__device__ __forceinline__ void tile_dma(const int16_t *coef, long long t, long long nblk, char *mine, int lane) {
    typedef int i4 __attribute__((ext_vector_type(4)));
    const long long left = nblk - t * 64;
    const int nb = left < 64 ? (int)left : 64;
    const uint64_t a = (uint64_t)(coef + t * 64 * 64);
    const i4 rs = {(int)(uint32_t)a, (int)((a >> 32) & 0xFFFFu), nb * 128, 0x00020000};  // as make_buffer_rsrc
    // piece (l & 7) ^ (b >> 1 & 7) of block b = 8c + (l >> 3) sits at byte 1024 c + (base ^ 64 (c & 1))
    int base = ((lane >> 3) << 7) | (((lane & 7) ^ (lane >> 4)) << 4);
    asm volatile("" : "+v"(base));  // computed here: eight loop-invariant offsets hoisted out of the loop spilled
    const uint32_t lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char *)mine;
    // Inline asm, not __builtin_amdgcn_raw_ptr_buffer_load_lds: LLVM's waitcnt pass
    // cannot tell an LDS-DMA from the workgroup's other LDS traffic and puts a
    // vmcnt(0) before the next LDS instruction -- the narrow path's first counter
    // add would wait for the whole prefetch.  The stage is only read after the
    // explicit vmcnt(0) at the top of the next tile, and M0 is restored.
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        uint32_t save;
        asm volatile(
            "s_mov_b32 %0, m0\n\t"
            "s_mov_b32 m0, %1\n\t"
            "buffer_load_dwordx4 %2, %3, 0 offen nt lds\n\t"  // non-temporal: the tile is read once
            "s_mov_b32 m0, %0"
            : "=&s"(save)
            : "s"(lds + c * 1024), "v"(c * 1024 + (base ^ ((c & 1) << 6))), "s"(rs)
            : "memory");
    }
}

// Every path works on the row classify() read (d: the lane's 64 coefficients as 32
// dwords), so the tile is read out of LDS once per tile (round 6: -2 to -3 % on
// uniform input against a re-read per path, profiles/r06/huf_keep_row_ab; the row
// live across the path choice costs the dense path a few spilled loop invariants).
template <int N, bool FWD = false, typename NextTile>
__device__ __forceinline__ void sparse_runs(char *mine, const Hist &h, int lane, uint32_t &nodes, uint32_t &lmax,
                                            NextTile next_tile, const uint32_t (&d)[32]) {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): every lane has its row before the columns overwrite the tile
    __builtin_amdgcn_wave_barrier();
    // branch-free compaction: every value is written at the next slot, which advances
    // only past a nonzero (a zero's write is overwritten or lies past `pos`).  The
    // key is the value's raw 16 bits (zeros never reach the sort, and any injective
    // key groups equal values): ds_write_b16 / ds_write_b16_d16_hi straight from the
    // packed pair, and one packed min gives both nonzero flags.
    uint32_t pos = 0;
    uint32_t b[N];
    if constexpr (!FWD) {
        const uint32_t one2 = 0x00010001u;
#pragma unroll
        for (int h = 0; h < 32; ++h) {
            uint32_t nz2;  // (lo != 0, hi != 0) as 16-bit halves; inline asm: LLVM expands the packed min
            asm volatile("v_pk_min_u16 %0, %1, %2" : "=v"(nz2) : "v"(d[h]), "v"(one2));
            *reinterpret_cast<uint16_t *>(mine + (pos * 64 + lane) * 4) = (uint16_t)d[h];
            pos += nz2 & 0xFFFFu;
            *reinterpret_cast<uint16_t *>(mine + (pos * 64 + lane) * 4) = (uint16_t)(d[h] >> 16);
            pos += nz2 >> 16;
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int k = 0; k < N; ++k) {
            const uint32_t v = *reinterpret_cast<const uint16_t *>(mine + (k * 64 + lane) * 4);
            b[k] = (uint32_t)k < pos ? v : kSent;
        }
    } else {
        // the fused kernel (huffman_from_pixels) keeps 32-bit keys: with the 16-bit
        // stores its loop invariants spilled (12-14 VGPRs at its 168-register bound)
#pragma unroll
        for (int i = 0; i < 64; ++i) {
            const uint32_t v = key_of(d, i);
            *reinterpret_cast<uint32_t *>(mine + (pos * 64 + lane) * 4) = v;
            pos += v != kSent ? 1u : 0u;
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int k = 0; k < N; ++k) {
            const uint32_t v = *reinterpret_cast<const uint32_t *>(mine + (k * 64 + lane) * 4);
            b[k] = (uint32_t)k < pos ? v : kSent;
        }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the keys are in registers, the stage is free
    __builtin_amdgcn_wave_barrier();
    next_tile();
    sort_net<N>(b);
    runs_to_hist<N, false>(b, h, nodes, lmax);
}

template <bool FWD = false, typename NextTile>
__device__ __forceinline__ void dense_runs(char *mine, const Hist &h, int lane, uint32_t &nodes, uint32_t &lmax,
                                           NextTile next_tile, const uint32_t (&d)[32]) {
    uint32_t a[64];
#pragma unroll
    for (int h = 0; h < 32; ++h) {
        a[2 * h] = (d[h] << 16) - 1u;
        a[2 * h + 1] = (d[h] & 0xFFFF0000u) - 1u;
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the row is in registers, the stage is free
    __builtin_amdgcn_wave_barrier();
    next_tile();
    sort_net<64>(a);
    runs_to_hist<64, true>(a, h, nodes, lmax);
}

// Tiles whose every block's values (zeros included) span fewer than 64 integers
// (q50 noise, most natural content): no sort, and a merge in the shared byte
// region (kHufCtrBytes), left zeroed for the next tile:
//  1. count: one v_pk_add_u16 per coefficient pair (slot = value - vmin) and one
//     v_perm + ds_add per coefficient;
//  2. zeros are not symbols -- except one 0 when c[63] == 0 -- so the zero
//     counter is replaced with last_zero;
//  3. readout: each counter is read AND cleared by one ds_and_rtn (the wave's
//     byte only), and adds one leaf at its frequency to the weight histogram
//     (row 0 absorbs empty counters);
//  4. the weight rows are read back (and cleared) and merged in registers.
// narrow_leaves runs steps 1-3 and ISSUES the read-back of step 4 (its results
// stay in flight in NarrowLeaves until narrow_merge extracts the wave's bytes
// and runs the register merge).  A software-pipelined kernel loop that merged one
// tile while the next tile's LDS phases were in flight measured no faster
// (profiles/r03/huffman_restructure_ab.log).
// weight rows 17.. read back without waiting (q50 noise: largest leaf ~20; 6 or 8 rows measured the
// same or slower, profiles/r06/huf_keep_row_ab/heavy_rows_*.log)
constexpr int kHeavyRows = 4;
struct NarrowLeaves {
    uint32_t light[16];  // weight rows 1..16 as read (the wave's byte at 8 * wave)
    uint32_t heavy[kHeavyRows];  // weight rows 17..16 + kHeavyRows as read, when hrows > 16
    uint32_t hn, hs, hmn, hmx;  // leaves of the rows past those (read at once: rare): count, sum, min, max
    uint32_t count;      // symbols of the block
    uint32_t hrows;      // wave-uniform: 16 + kHeavyRows when heavy[] was read, else 16
};

template <typename NextTile>
__device__ __forceinline__ void narrow_leaves(char *ctr, int lane, int wv, int32_t vmin, uint32_t span,
                                              bool last_zero, NextTile next_tile, NarrowLeaves &L,
                                              const uint32_t (&d)[32]) {
    // the row is in registers and the stage is free: the next tile streams in meanwhile
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    next_tile();
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    const uint32_t base = (uint32_t)(lane * 4);  // byte 0 of the lane's dword in every row
    const uint32_t sh = 8u * (uint32_t)wv, inc = 1u << sh;  // the wave's byte of it
    uint32_t keep = ~(0xFFu << sh);
    asm volatile("" : "+v"(keep));  // rematerialised per tile: hoisted out of the kernel loop, the fused kernel spilled it
    const u16x2 off = {(unsigned short)(-vmin), (unsigned short)(-vmin)};
    auto at = [&](uint32_t row) { return reinterpret_cast<uint32_t *>(ctr + (row << 8) + base); };
    auto take_raw = [&](uint32_t row) {  // row's dword, the wave's byte cleared in LDS
        return __hip_atomic_fetch_and(at(row), keep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    };
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        const uint32_t sl = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, d[k]) + off);  // slots, < 64 each
        __hip_atomic_fetch_add(reinterpret_cast<uint32_t *>(ctr + __builtin_amdgcn_perm(sl, base, 0x0C0C0400u)), inc,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        __hip_atomic_fetch_add(reinterpret_cast<uint32_t *>(ctr + __builtin_amdgcn_perm(sl, base, 0x0C0C0600u)), inc,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
    // zeros: their count gives the symbol count; then only c[63] == 0 leaves one
    // (reading this counter first in the read-out batch instead, without a round trip
    // of its own, measured within noise: profiles/r06/huf_keep_row_ab/zero_in_batch_*.log)
    uint32_t zeros = 0;
    if (vmin <= 0 && vmin > -64) {
        const uint32_t z = (uint32_t)(-vmin);
        zeros = (take_raw(z) >> sh) & 0xFFu;
        if (last_zero) __hip_atomic_fetch_add(at(z), inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
    L.count = 64u - zeros + (last_zero ? 1u : 0u);
    // readout: every counter read and cleared, THEN the leaves added (the weight
    // histogram reuses the rows).  Only rows below the wave's largest span hold
    // counts (q50 noise: 32-40 of 64): the first nck wave-uniform chunks of 8 rows
    // (span conditions are monotone in the chunk).  Rows of skipped chunks are
    // never read, so nothing is materialised for them.
    // (4-row chunks: 3.5 % slower on uniform input, 16-row chunks the same as 8:
    // profiles/r06/huf_keep_row_ab/chunk_*.log)
    constexpr int CH = 8, NCH = 64 / CH;
    int nck = 1;
#pragma unroll
    for (int c8 = 1; c8 < NCH; ++c8) nck += __builtin_amdgcn_ballot_w64(span > (uint32_t)(CH * c8)) != 0 ? 1 : 0;
    uint32_t raw[64];
#pragma unroll
    for (int c8 = 0; c8 < NCH; ++c8) {
        if (c8 < nck) {
#pragma unroll
            for (int s_ = CH * c8; s_ < CH * c8 + CH; ++s_) raw[s_] = take_raw((uint32_t)s_);
        }
    }
    // A counter is kept as its leaf's address: one v_perm moves the wave's byte of
    // the returned dword into byte 1 (the row) over the lane's byte 0 -- no extract
    // -- and the largest address gives the largest leaf weight.
    const uint32_t leaf_sel = 0x0C0C0000u | ((4u + (uint32_t)wv) << 8);
    uint32_t amax = base;
#pragma unroll
    for (int c8 = 0; c8 < NCH; ++c8) {
        if (c8 < nck) {
#pragma unroll
            for (int s_ = CH * c8; s_ < CH * c8 + CH; ++s_) {
                const uint32_t a = __builtin_amdgcn_perm(raw[s_], base, leaf_sel);
                amax = a > amax ? a : amax;
                __hip_atomic_fetch_add(reinterpret_cast<uint32_t *>(ctr + a), inc, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WAVEFRONT);
            }
        }
    }
    const uint32_t lmax = amax >> 8;  // the largest leaf weight
    (void)take_raw(0);  // row 0: the empties
    // weight rows 1..16 issued together (independent reads, all in flight; their
    // results are used by narrow_merge), each row cleared
#pragma unroll
    for (int w = 1; w <= 16; ++w) L.light[w - 1] = take_raw((uint32_t)w);
    // rows 17..16 + kHeavyRows read unconditionally when the wave has a leaf there
    // (rows past a lane's largest leaf read as zero): no branch per row, so the
    // results stay in flight in registers
    L.hrows = __builtin_amdgcn_ballot_w64(lmax > 16) ? 16u + kHeavyRows : 16u;
    if (L.hrows > 16) {
#pragma unroll
        for (int r = 17; r <= 16 + kHeavyRows; ++r) L.heavy[r - 17] = take_raw((uint32_t)r);
    }
    // rows past those (a leaf of that many copies of one value): read one by one
    L.hn = 0;
    L.hs = 0;
    L.hmn = 0xFFu;
    L.hmx = 0;
    for (uint32_t r = 17 + kHeavyRows; __builtin_amdgcn_ballot_w64(r <= lmax); ++r) {
        const uint32_t k = (take_raw(r) >> sh) & 0xFFu;
        L.hn += k;
        L.hs += k * r;
        L.hmn = (k && L.hmn == 0xFFu) ? r : L.hmn;
        L.hmx = k ? r : L.hmx;
    }
}

// ---- merge in registers (no LDS round trip inside the merge; Python model:
// tests/test_oracle.py::register_merge_wpl).  Leaf weights <= 16 (their rows
// read back by narrow_leaves) are scanned w = 1..16 as the bucket merge.  A
// pending merge makes ONE node of weight p + w in (w, 2w), and successive ones
// are strictly heavier, so they are bits of a mask.  Nodes heavier than 16
// (leaves, pairs of w >= 9, pending merges) are at most 3, because all node
// weights add up to the symbol count (<= 65): their count, sum, min and max give
// them sorted, and with the pending node (the lightest) they finish in closed form.
// Returns the WPL.
__device__ __forceinline__ uint32_t narrow_merge(const NarrowLeaves &L, int wv) {
    const uint32_t sh = 8u * (uint32_t)wv;
    uint32_t cnt[17];
#pragma unroll
    for (int w = 1; w <= 16; ++w) cnt[w] = (L.light[w - 1] >> sh) & 0xFFu;
    // heavy leaves: rows 17..16 + kHeavyRows, then the rarer rows past them (all heavier)
    uint32_t hn = 0, hs = 0, hmn = 0xFFu, hmx = 0;
#pragma unroll
    for (int r = 17; r <= 16 + kHeavyRows; ++r) {
        if (L.hrows > 16) {
            const uint32_t k = (L.heavy[r - 17] >> sh) & 0xFFu;
            hn += k;
            hs += k * (uint32_t)r;
            hmn = (k && hmn == 0xFFu) ? (uint32_t)r : hmn;
            hmx = k ? (uint32_t)r : hmx;
        }
    }
    hn += L.hn;
    hs += L.hs;
    hmn = min(hmn, L.hmn);
    hmx = max(hmx, L.hmx);
    // p: the pending node's weight (0: none); pm: pending-merge nodes (bit = weight);
    // qp: pairs of w = 9..16 (weight 2w > 16, at most 3 per w because node weights
    // add up to <= 65) as 2-bit fields at 2 (w - 9), qs: their weights.
    // WPL = the sum of the internal nodes' weights = the sum of every node's weight
    // but the root's (each non-root node is a child of exactly one internal node),
    // so it needs no per-merge accounting: acc sums the nodes of every light bucket,
    // hs the heavy ones, fin the nodes of the closed-form finish, and the root
    // weighs `count`.
    uint32_t p = 0, pm = 0, acc = 0, qp = 0, qs = 0;
    // v_mad_u32_u24 with the bucket's weight as an inline constant: LLVM turns
    // (c & 1) * w into a compare and a select and c * w into v_mul_lo_u32 for
    // some w (it cannot see that c < 2^24)
    auto mad24 = [](uint32_t a, auto wc, uint32_t c) {
        uint32_t d;
        asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(d) : "v"(a), "n"(decltype(wc)::value), "v"(c));
        return d;
    };
    auto bucket = [&](auto wc) {
        constexpr uint32_t w = decltype(wc)::value;
        uint32_t c = cnt[w];
        if constexpr (w >= 3) c += (pm >> w) & 1u;  // p + w' >= 3
        acc = mad24(c, wc, acc);                   // bucket w's nodes
        const bool mp = min(p, c) != 0u;           // the pending node merges with one node of bucket w
        c -= mp ? 1u : 0u;
        pm |= mp ? (1u << w) << p : 0u;            // the merged node: weight p + w in (w, 2w), at most 31
        p = mad24(c & 1u, wc, mp ? 0u : p);        // c odd: one node of w waits (p was 0 or merged)
        const uint32_t pairs = c >> 1;
        if constexpr (2 * w <= 16) {
            cnt[2 * w] += pairs;
        } else {
            qp |= pairs << (2 * (w - 9));
            qs = mad24(pairs, std::integral_constant<uint32_t, 2 * w>{}, qs);
        }
    };
    bucket(std::integral_constant<uint32_t, 1>{});
    bucket(std::integral_constant<uint32_t, 2>{});
    bucket(std::integral_constant<uint32_t, 3>{});
    bucket(std::integral_constant<uint32_t, 4>{});
    bucket(std::integral_constant<uint32_t, 5>{});
    bucket(std::integral_constant<uint32_t, 6>{});
    bucket(std::integral_constant<uint32_t, 7>{});
    bucket(std::integral_constant<uint32_t, 8>{});
    bucket(std::integral_constant<uint32_t, 9>{});
    bucket(std::integral_constant<uint32_t, 10>{});
    bucket(std::integral_constant<uint32_t, 11>{});
    bucket(std::integral_constant<uint32_t, 12>{});
    bucket(std::integral_constant<uint32_t, 13>{});
    bucket(std::integral_constant<uint32_t, 14>{});
    bucket(std::integral_constant<uint32_t, 15>{});
    bucket(std::integral_constant<uint32_t, 16>{});
    // the heavy pairs: count, min, max
    const uint32_t qn = (uint32_t)__builtin_popcount(qp & 0x5555u) + 2u * (uint32_t)__builtin_popcount(qp & 0xAAAAu);
    const uint32_t qmn = qp ? 18u + 2u * ((uint32_t)__builtin_ctz(qp) >> 1) : 0xFFu;
    const uint32_t qmx = qp ? 18u + 2u * ((31u - (uint32_t)__builtin_clz(qp)) >> 1) : 0u;
    // the pending-merge nodes above 16 (<= 3 bits of pm, bits 17..31)
    {
        uint32_t b = pm & ~0x1FFFFu;
        const uint32_t n = (uint32_t)__builtin_popcount(b);
        const uint32_t lo = b ? (uint32_t)__builtin_ctz(b) : 0xFFu, hi = b ? 31u - (uint32_t)__builtin_clz(b) : 0u;
        const uint32_t mid = n == 3 ? (uint32_t)__builtin_ctz(b & (b - 1)) : 0u;
        hn += n + qn;
        hs += (n ? lo : 0u) + (n == 3 ? mid : 0u) + (n >= 2 ? hi : 0u) + qs;
        hmn = min(min(hmn, qmn), lo);
        hmx = max(max(hmx, qmx), hi);
    }
    // the heavy nodes sorted: h1 <= h2 <= h3 (h2 = h3 when there are two)
    const uint32_t h1 = hmn, h3 = hmx, h2 = hn == 3 ? hs - h1 - h3 : h3;
    uint32_t fin;
    if (p) {  // p < 17 <= h1: nodes p, h1, h2, h3
        const uint32_t s2 = p + h1;
        fin = hn == 3 ? 2 * s2 + 2 * h2 + h3 + min(s2, h3) : hn == 2 ? 2 * s2 + h2 : hn == 1 ? s2 : 0u;
    } else {
        fin = hn == 3 ? 2 * (h1 + h2) + h3 : hn == 2 ? h1 + h3 : 0u;
    }
    return acc + hs + fin - L.count;
}

// Non-temporal bits stores (written once, never re-read here): -1.6 to -2.9 % on every input, three
// passes on one box (profiles/r02/huffman_dma_ab.log).
constexpr int kHufBitsAux = kNtAux;
// A tile's classification (tile_row layout, blocks past the end zeroed).
struct TileClass {
    uint32_t nz;        // the lane's nonzero count (exact unless narrow: then 0, unused)
    bool last_zero;     // c[63] == 0: value 0 is a symbol once
    bool narrow;        // wave-uniform: a dense tile whose every block has its values (zeros included) within 64 integers
    int32_t vmin;
    uint32_t span;      // the lane's values (zeros included) lie in [vmin, vmin + span)
};

template <bool FWD = false>
__device__ __forceinline__ TileClass classify(const char *mine, int lane, int nb, uint32_t (&d)[32]) {
    TileClass c;
    c.nz = 0;
    c.narrow = false;
    c.vmin = 0;
    c.span = 64;
    {
        tile_row<FWD>(mine, lane, d);
        c.last_zero = (d[31] >> 16) == 0u;
        // Nonzeros of dwords [k0, k1): unsigned min(h, 1) is 1 for any nonzero half;
        // the packed 0/1 pairs summed three at a time as plain dwords (each half
        // stays below 2^16), then the two halves added.
        auto nonzeros = [&](auto k0c, auto k1c) {
            constexpr int k0 = decltype(k0c)::value, k1 = decltype(k1c)::value;
            typedef unsigned short u2 __attribute__((ext_vector_type(2)));
            const u2 one = {1, 1};
            const uint32_t one32 = __builtin_bit_cast(uint32_t, one);
            uint32_t m[k1 - k0];
#pragma unroll
            for (int k = k0; k < k1; ++k)  // inline asm: LLVM turns the packed min into compares and selects
                asm("v_pk_min_u16 %0, %1, %2" : "=v"(m[k - k0]) : "v"(d[k]), "v"(one32));
            uint32_t acc0 = 0, acc1 = 0;  // two chains: no dependent back-to-back adds
#pragma unroll
            for (int k = 0; k + 1 < k1 - k0; k += 4) {
                acc0 = m[k] + m[k + 1] + acc0;
                if (k + 3 < k1 - k0) acc1 = m[k + 2] + m[k + 3] + acc1;
            }
            const uint32_t acc = acc0 + acc1;
            return (acc & 0xFFFFu) + (acc >> 16);
        };
        // The span test (packed 16-bit min/max) runs first on tiles that look dense:
        // rows 0-1 (dwords 0..7) with more than 7 nonzeros in some lane.  A dense
        // tile of narrow span takes the narrow path, which counts its own symbols,
        // so its exact nonzero count is never needed; the estimate only picks a
        // path (every path gives the same sizes).
        auto span_test = [&] {
            typedef short s2 __attribute__((ext_vector_type(2)));
            s2 mn = __builtin_bit_cast(s2, d[0]), mx = mn;
#pragma unroll
            for (int k = 1; k < 32; ++k) {
                const s2 x = __builtin_bit_cast(s2, d[k]);
                mn = __builtin_elementwise_min(mn, x);
                mx = __builtin_elementwise_max(mx, x);
            }
            c.vmin = mn.x < mn.y ? mn.x : mn.y;
            const int32_t vmax = mx.x > mx.y ? mx.x : mx.y;
            c.span = (uint32_t)(vmax - c.vmin + 1);
            c.narrow = !__builtin_amdgcn_ballot_w64(lane < nb && vmax - c.vmin >= 64);
        };
        const bool looks_dense =
            __builtin_amdgcn_ballot_w64(nonzeros(std::integral_constant<int, 0>{}, std::integral_constant<int, 8>{}) > 7u) != 0;
        if (looks_dense) span_test();
        if (!c.narrow) {
            c.nz = nonzeros(std::integral_constant<int, 0>{}, std::integral_constant<int, 32>{});
            if (!looks_dense && __builtin_amdgcn_ballot_w64(c.nz > 32)) span_test();  // dense after all
        }
    }
    // the row stays in d for the paths; the compiler barrier keeps the paths' LDS
    // writes (compacted keys, counters) after these reads, as in the measured build
    asm volatile("" ::: "memory");
    return c;
}

// The sparse and dense paths of a tile that is not narrow: runs of equal values
// -> histogram of frequencies in the shared byte region (Hist), then the bucket
// merge; they call next_tile() as soon as the stage is free (keys or row in
// registers), so the next tile's DMA overlaps the sort and the merge.  Returns the
// bit counts.
template <bool FWD = false, typename NextTile>
__device__ __forceinline__ uint32_t sort_tile_bits(char *mine, char *ctr, int lane, int wv, int nb,
                                                   const TileClass &cl, NextTile next_tile, const uint32_t (&d)[32]) {
    const Hist h{ctr, (uint32_t)(lane * 4), 8u * (uint32_t)wv};
    const uint32_t nz = cl.nz;
    const bool last_zero = cl.last_zero;
    uint32_t count = nz + (last_zero ? 1u : 0u);  // symbols: the nonzeros, plus a 0 once if c[63] == 0
    uint32_t nodes = last_zero ? 1u : 0u;
    uint32_t lmax = last_zero ? 1u : 0u;  // the largest leaf weight (dense paths)
    const bool dense = __builtin_amdgcn_ballot_w64(nz > 32) != 0;
    const bool lane_merge = dense;  // the dense paths merge per lane (occupancy mask)
    uint32_t wpl = 0, pending = 0;
    if (!__builtin_amdgcn_ballot_w64(nz > 16))
        sparse_runs<16, FWD>(mine, h, lane, nodes, lmax, next_tile, d);
    else if (!__builtin_amdgcn_ballot_w64(nz > 32))
        sparse_runs<32, FWD>(mine, h, lane, nodes, lmax, next_tile, d);
    else
        dense_runs<FWD>(mine, h, lane, nodes, lmax, next_tile, d);
    if (last_zero) h.add(1, 1);
    // ---- bucket merge (see the header): wpl = sum of internal node weights.  Lanes
    // past the tail hold one leaf (the zero block's last 0) and run as any other,
    // so their bucket is cleared too.
    if (lane_merge) {
        // occupancy of the leaf buckets, read back up to the wave's largest leaf weight
        // (cheaper than marking every leaf; this wave's LDS atomics are already ordered)
        std::conditional_t<FWD, Occ32x2, Occ64> occ;
#pragma unroll
        for (uint32_t w = 1; w <= 8; ++w)  // independent reads, in flight together
            occ.first8(w, h.peek(w));
        for (uint32_t w = 9; __builtin_amdgcn_ballot_w64(w <= lmax); ++w)
            if (h.peek(w)) occ.set(w);
        // Each lane jumps to its own next occupied bucket (lowest bit of occ), so the
        // loop runs as many steps as the busiest lane has occupied buckets, not up to
        // its largest weight.  New weights (pending + w, 2w) are above w, so the scan
        // order is the bucket order; weights never exceed the symbol count (<= 64).
        // The lane is done when no bucket is left: its last node (the root) is then
        // `pending`, and every bucket it held nodes in was taken (cleared).  The step
        // cap only bounds the loop.
        for (int step = 0; step < 130 && __builtin_amdgcn_ballot_w64(occ.any()); ++step) {
            if (occ.any()) {
                const uint32_t w = occ.pop();  // bucket w is emptied by this step
                uint32_t c = h.take(w);
                if (pending && c) {
                    const uint32_t nw = pending + w;
                    wpl += nw;
                    h.add(nw, 1);
                    occ.set(nw);
                    --c;
                    pending = 0;
                }
                const uint32_t pairs = c >> 1;
                if (pairs) {
                    wpl += pairs * 2 * w;
                    h.add(2 * w, pairs);
                    occ.set(2 * w);
                }
                if (c & 1) pending = w;
            }
        }
    } else {
        // Sparse tiles (few weights): every weight in turn; bucket w+1 is taken at the
        // top of iteration w, so its LDS latency hides behind the iteration; the only
        // merges of iteration w that land on w+1 (pending 1 + w, and the pairs of
        // w = 1) are carried in a register.  A lane stops once its root is made; the
        // root's bucket (weight = count) may then be left, and is cleared after the loop.
        uint32_t cur = h.take(1);
        for (uint32_t w = 1; w <= 64 && __builtin_amdgcn_ballot_w64(nodes > 1); ++w) {
            const uint32_t nxt = w < 64 ? h.take(w + 1) : 0u;
            uint32_t c = cur, carry = 0;
            if (nodes > 1) {
                if (pending && c) {
                    const uint32_t nw = pending + w;
                    wpl += nw;
                    if (nw == w + 1)
                        carry = 1;
                    else
                        h.add(nw, 1);
                    --c;
                    --nodes;
                    pending = 0;
                }
                const uint32_t pairs = c >> 1;
                if (pairs) {
                    wpl += pairs * 2 * w;
                    nodes -= pairs;
                    if (w == 1)
                        carry += pairs;
                    else
                        h.add(2 * w, pairs);
                }
                if (c & 1) pending = w;
            }
            cur = nxt + carry;
        }
        (void)h.take(count);  // the root, or a lone leaf, if still stored
    }
    return 8u * count + wpl;
}

// One tile in the wave's stage (Huffman layout, blocks past the end zeroed): the
// bit count of every lane's block.  next_tile() is called once the stage may be
// overwritten (the next tile's DMA, or nothing).
template <bool FWD = false, typename NextTile>
__device__ __forceinline__ uint32_t tile_bits(char *mine, char *ctr, int lane, int wv, int nb, NextTile next_tile) {
    uint32_t row[32];
    const TileClass cl = classify<FWD>(mine, lane, nb, row);
    if (cl.narrow) {
        NarrowLeaves L;
        narrow_leaves(ctr, lane, wv, cl.vmin, cl.span, cl.last_zero, next_tile, L, row);  // the zero leaf included
        return 8u * L.count + narrow_merge(L, wv);
    }
    return sort_tile_bits<FWD>(mine, ctr, lane, wv, nb, cl, next_tile, row);
}

// The tie passes of huffman_from_pixels: passes of <= 8 entries run 8 lanes per entry
// (exact_grouped<8>): -4.1 % uniform, -3.1 % smooth; passes of 9..32 entries in one round of
// 4 / 2 lanes per entry (resolve_ties_compact WIDE = 3): -2.7 % on extreme q10 (~10 entries per
// batch), uniform q50 unchanged (profiles/r04/wide_groups_ab.log); no scratch at this kernel's
// 168-VGPR bound.
constexpr bool kHpGroup8 = true;
constexpr int kHpWide = 3;
// Launch bound of both kernels: 3 waves/SIMD (168 VGPRs; 4 spilled, profiles/r01).
constexpr int kHufMinWaves = 3;
// Workgroups per CU in the grid: 3 are resident (LDS-bound) and the rest queue behind them, so
// tiles of unequal cost balance (8: +1-2.5 %, 3: +3-4 %).
constexpr long long kHufGridPerCu = 16;
__global__ __launch_bounds__(kHufThreads, kHufMinWaves) void huffman_bits_kernel(const int16_t *__restrict__ coef, long long nblk,
                                                                   uint32_t *__restrict__ bits, long long ntiles) {
    // per wave: the tile stage (9 KiB), reused for the sparse keys; per workgroup: the counters and histograms
    __shared__ uint4 lds[kHufWaves * kHufWaveLds / 16];
    __shared__ uint4 ctr_lds[kHufCtrBytes / 16];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    char *mine = reinterpret_cast<char *>(lds) + wv * kHufWaveLds;
    char *ctr = reinterpret_cast<char *>(ctr_lds);
    // the narrow path leaves its rows cleared after every tile; LDS starts undefined
    for (int i = threadIdx.x; i < kHufCtrBytes / 16; i += kHufThreads) ctr_lds[i] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    const long long stride = (long long)gridDim.x * kHufWaves;
    long long t = (long long)blockIdx.x * kHufWaves + wv;
    auto store_bits = [&](uint32_t out, long long tt, int n) {
        const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(bits + tt * 64, (short)0, n * 4, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b32(out, rb, lane * 4, 0, kHufBitsAux);
    };
    if (t < ntiles) tile_dma(coef, t, nblk, mine, lane);
    for (; t < ntiles; t += stride) {
        const long long left = nblk - t * 64;
        const int nb = left < 64 ? (int)left : 64;
        // this tile's DMA has landed, and the previous tile's bits store has left
        // (one in-order vmcnt) before LDS reads land in VGPRs (the store-data hazard)
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
        __builtin_amdgcn_wave_barrier();
        if (nb < 64) {  // the launch's last tile: blocks past the end are empty (every path reads them)
            if (lane >= nb) {
#pragma unroll
                for (int k = 0; k < 8; ++k) *reinterpret_cast<uint4 *>(mine + lane * 128 + k * 16) = make_uint4(0, 0, 0, 0);
            }
            __builtin_amdgcn_s_waitcnt(0xC07F);
            __builtin_amdgcn_wave_barrier();
        }
        auto next_tile = [&] {
            if (t + stride < ntiles) tile_dma(coef, t + stride, nblk, mine, lane);
        };
        store_bits(tile_bits(mine, ctr, lane, wv, nb, next_tile), t, nb);
    }
}

hipError_t launch_huffman_bits(const int16_t *coef, long long nblk, uint32_t *bits, hipStream_t stream, int num_cus) {
    const long long ntiles = (nblk + 63) / 64;
    long long grid = (ntiles + kHufWaves - 1) / kHufWaves;
    const long long cap = (long long)num_cus * kHufGridPerCu;
    if (grid > cap) grid = cap;
    hipLaunchKernelGGL(huffman_bits_kernel, dim3((unsigned)grid), dim3(kHufThreads), 0, stream, coef, nblk, bits,
                       ntiles);
    return hipGetLastError();
}

// ============================================================================
// The reference pipeline's per-block size straight from pixels (SURVEY 8(f)4 fed
// by 8(a)): forward DCT + quantization (fdct8_core.h, ties resolved in place in
// the reference's order) -> tile_bits on the rows where the forward left them
// (copying them into the tile layout first was 2.8-4.5 % slower).  The
// coefficients never leave LDS: 64 B read and 4 B written per block, against
// 192 + 132 for dctq_forward_quant_planes followed by dctq_huffman_bits.
// Same grid, occupancy (3 waves/SIMD) and LDS as huffman_bits_kernel, plus the
// exact path's 1 KiB table copy.  The next batch's rows are loaded into `cur`
// as soon as the tie pass is done with them, so the loads fly through the size
// computation (-3.4 %).
template <bool ADAPTIVE>
__global__ __launch_bounds__(kHufThreads, kHufMinWaves) void huffman_from_pixels_kernel(EncodeSet es,
                                                                                              const DevTables *__restrict__ dev,
                                                                                              uint32_t *__restrict__ bits) {
    __shared__ uint4 lds[kHufWaves * kHufWaveLds / 16];
    __shared__ uint4 ctr_lds[kHufCtrBytes / 16];
    __shared__ ExactTables tab;
    static_assert(64 * kPitch2 + 128 <= kHufWaveLds, "forward stage + tie scratch fit the wave's region");
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    char *mine = reinterpret_cast<char *>(lds) + wv * kHufWaveLds;
    char *ctr = reinterpret_cast<char *>(ctr_lds);
    // the forward core addresses the stage as (wv * 64 + lane) * kPitch2 from its base
    uint4 *stage = reinterpret_cast<uint4 *>(mine - wv * 64 * kPitch2);
    uint16_t *scr = reinterpret_cast<uint16_t *>(mine + 64 * kPitch2);
    for (int i = threadIdx.x; i < kHufCtrBytes / 16; i += kHufThreads) ctr_lds[i] = make_uint4(0, 0, 0, 0);
    load_exact_tables(&tab, dev);  // ends with __syncthreads
    const PlaneSet &ps = es.ps;
    const uint32_t nbatch = ps.first[ps.n];
    const uint32_t step = gridDim.x * kHufWaves;
    uint2 cur[8];
    // global row loads here: the buffer-descriptor form (load_rows<true>) costs this
    // kernel one VGPR spill at its bound
    prefetch_batch<true, false>(ps, blockIdx.x * kHufWaves + wv, lane, cur);
    for (uint32_t g = blockIdx.x * kHufWaves + wv; g < nbatch; g += step) {
        const int k = plane_of(ps, g);
        const PlaneArgs &p = ps.pl[k];
        const uint32_t b = g - first_of(ps, k);
        const uint32_t n = b * 64 + lane;
        const bool valid = n < (uint32_t)p.nblk;
        const int nb = (uint32_t)p.nblk - b * 64 < 64u ? (int)((uint32_t)p.nblk - b * 64) : 64;
        // the rows are in, and the previous batch's bits store has left before
        // LDS reads land in VGPRs (the store-data hazard)
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
        uint32_t mlo, mhi;
        int32_t var_num;
        fdct8_compute<ADAPTIVE, false>(dev, cur, stage, lane, wv, mlo, mhi, var_num);
        flat_dc_fix(dev, cur, stage, lane, wv, mlo);
        if (!valid) mlo = mhi = 0;
        if (__builtin_amdgcn_ballot_w64((mlo | mhi) != 0))
            (void)resolve_ties_compact<ADAPTIVE, kHpGroup8, kHpWide>(&tab, cur, stage, scr, lane, wv, mlo, mhi);
        wave_sync();
        prefetch_batch<true, false>(ps, g + step, lane, cur);  // the rows are dead now; nothing past the last batch
        if (nb < 64) {  // blocks past the end are empty
            if (lane >= nb) {
#pragma unroll
                for (int q = 0; q < 16; ++q) *reinterpret_cast<uint2 *>(mine + lane * kPitch2 + 8 * q) = make_uint2(0, 0);
            }
            __builtin_amdgcn_s_waitcnt(0xC07F);
            wave_sync();
        }
        const uint32_t out = tile_bits<true>(mine, ctr, lane, wv, nb, [] {});
        // (pinning this destination in SGPRs at the top, as the forward kernels do, spilled 8 B here)
        const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
            bits + es.blk_first[k] + (size_t)b * 64, (short)0, nb * 4, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b32(out, rb, lane * 4, 0, kHufBitsAux);
        // tile_bits leaves the stage to the next batch's forward only after its own reads
        __builtin_amdgcn_s_waitcnt(0xC07F);
        wave_sync();
    }
}

hipError_t launch_huffman_from_pixels(const EncodeSet &es, const DevTables *dev, int adaptive, uint32_t *bits,
                                      hipStream_t stream, int num_cus) {
    const uint32_t nbatch = es.ps.first[es.ps.n];
    long long grid = ((long long)nbatch + kHufWaves - 1) / kHufWaves;
    const long long cap = (long long)num_cus * kHufGridPerCu;  // a persistent grid (3 per CU) is +11 %
    if (grid > cap) grid = cap;
    if (grid < 1) return hipSuccess;
    if (adaptive)
        hipLaunchKernelGGL(huffman_from_pixels_kernel<true>, dim3((unsigned)grid), dim3(kHufThreads), 0, stream, es, dev,
                           bits);
    else
        hipLaunchKernelGGL(huffman_from_pixels_kernel<false>, dim3((unsigned)grid), dim3(kHufThreads), 0, stream, es,
                           dev, bits);
    return hipGetLastError();
}

}  // namespace dctq
