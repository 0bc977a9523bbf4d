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
// Layout: one LANE per block (64 blocks per wave).  The wave stages its tile
// (8 KiB) in LDS with 1 KiB loads; each lane sorts its values with a Batcher
// odd-even merge network in registers (equal values become adjacent; zeros map
// to the top and are dropped) -- all 64, or, when every block of the tile has
// at most 16 / 32 nonzero coefficients (natural content), just those, compacted
// through LDS -- adds one count per run length into its column of an LDS
// histogram (16-bit counters, two lanes per dword, ds_add_u32), then runs the
// bucket merge.  Dense tiles whose every block's values span < 64 integers
// (q50 noise, most natural content) skip the sort: dense_counts below.  VALU-bound (~2000 instructions per 64 dense blocks).
// DCTQ_HUF_MIN_WAVES (launch bound, default 3 waves/SIMD: 168 VGPRs) is an A/B knob.
#include "dctq_internal.h"

namespace dctq {

constexpr int kHufWaves = 4;
constexpr int kHufThreads = 64 * kHufWaves;
constexpr int kHufPitch = 144;  // bytes per block in the tile stage (128 + 16: ds_read_b128 spread)
constexpr int kHufWaveLds = 12288;  // >= 64 * kHufPitch and 8 KiB histogram + 4 KiB counters

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

// Histogram column of `lane`: 16-bit counter of weight w (1..64) at byte
// (w-1)*128 + lane*2 (dword (w-1)*32 + lane/2: lanes 2q, 2q+1 share a dword,
// bank q -- conflict-free for any mix of weights across lanes).
__device__ __forceinline__ void hist_add(char *h, int w, int lane, uint32_t n) {
    __hip_atomic_fetch_add(reinterpret_cast<uint32_t *>(h + (w - 1) * 128 + (lane & ~1) * 2), n << (16 * (lane & 1)),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

// Occupancy of the lane's histogram: bit w-1 set while bucket w may hold nodes
// (the merge jumps from one occupied bucket to the next).
__device__ __forceinline__ void mark(uint64_t &occ, uint32_t w, uint32_t n) {
    occ |= n ? 1ull << (w - 1) : 0ull;
}

constexpr uint32_t kSent = 0xFFFFFFFFu;  // a zero coefficient (dropped)

// Sort key of coefficient i of a block held as 32 dwords (two int16 each):
// value*65536 - 1 as uint32 -- injective, and 0 -> kSent, which sorts last.
__device__ __forceinline__ uint32_t key_of(const uint32_t (&d)[32], int i) {
    return ((i & 1) ? (d[i >> 1] & 0xFFFF0000u) : (d[i >> 1] << 16)) - 1u;
}

// Runs of equal values in the sorted registers -> one histogram count per
// distinct value at its frequency; `nodes` += distinct values.
template <int N, bool kMax>
__device__ __forceinline__ void runs_to_hist(const uint32_t (&a)[N], char *mine, int lane, uint32_t &nodes,
                                             uint32_t &lmax) {
    // branch-free: every element adds (end ? 1 : 0) at its run length, so no
    // per-element exec mask is live (64 of them spilled to SGPR lanes)
    uint32_t run = 1;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const uint32_t nxt = i + 1 < N ? a[i + 1 < N ? i + 1 : N - 1] : kSent;
        const uint32_t end = a[i] != kSent && nxt != a[i] ? 1u : 0u;
        hist_add(mine, run, lane, end);
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
__device__ __forceinline__ void tile_row(const char *mine, int lane, uint32_t (&d)[32]) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint4 w = *reinterpret_cast<const uint4 *>(mine + lane * kHufPitch + k * 16);
        d[4 * k] = w.x;
        d[4 * k + 1] = w.y;
        d[4 * k + 2] = w.z;
        d[4 * k + 3] = w.w;
    }
}

// Each path re-reads the tile row itself, so nothing but scalars is live across
// the path choice and each path gets its own register allocation (a shared
// 32-register row made the compiler hold 188-336 VGPRs).
template <int N>
__device__ __forceinline__ void sparse_runs(char *mine, int lane, uint32_t &nodes, uint32_t &lmax) {
    uint32_t d[32];
    tile_row(mine, lane, d);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): every lane has its row before the columns overwrite the tile
    __builtin_amdgcn_wave_barrier();
    // branch-free compaction: every key is written at the next slot, which advances
    // only past a nonzero (a zero's write is overwritten or lies past `pos`)
    uint32_t pos = 0;
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        const uint32_t v = key_of(d, i);
        *reinterpret_cast<uint32_t *>(mine + (pos * 64 + lane) * 4) = v;
        pos += v != kSent ? 1u : 0u;
    }
    __builtin_amdgcn_wave_barrier();
    uint32_t b[N];
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const uint32_t v = *reinterpret_cast<const uint32_t *>(mine + (k * 64 + lane) * 4);
        b[k] = (uint32_t)k < pos ? v : kSent;
    }
    sort_net<N>(b);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): column reads done before the histogram overwrites them
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < 8; ++k) *reinterpret_cast<uint4 *>(mine + k * 1024 + lane * 16) = make_uint4(0, 0, 0, 0);
    __builtin_amdgcn_wave_barrier();
    runs_to_hist<N, false>(b, mine, lane, nodes, lmax);
}

__device__ __forceinline__ void dense_runs(char *mine, int lane, uint32_t &nodes, uint32_t &lmax) {
    uint32_t a[64];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint4 w = *reinterpret_cast<const uint4 *>(mine + lane * kHufPitch + k * 16);
        const uint32_t d[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            a[8 * k + 2 * h] = (d[h] << 16) - 1u;
            a[8 * k + 2 * h + 1] = (d[h] & 0xFFFF0000u) - 1u;
        }
    }
    sort_net<64>(a);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the tile reads are done before the histogram overwrites them
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < 8; ++k) *reinterpret_cast<uint4 *>(mine + k * 1024 + lane * 16) = make_uint4(0, 0, 0, 0);
    __builtin_amdgcn_wave_barrier();
    runs_to_hist<64, true>(a, mine, lane, nodes, lmax);
}

// Dense tiles whose every block's nonzero values span fewer than 64 integers
// (q50 natural or noise content): no sort.  Lane b counts its values in 64
// 8-bit counters (value - min) in its LDS column past the histogram (16 dwords,
// dword k*64 + lane: conflict-free, ds_add_u32), then each nonzero counter is
// one distinct value of that frequency.  ~850 VALU per 64 blocks against ~1 470
// for the 64-network and its run scan.
constexpr int kHufCnt = 8192;  // byte offset of the counters in the wave's LDS (after the histogram)

__device__ __forceinline__ int32_t coef_at(const uint32_t (&d)[32], int i) {
    return (i & 1) ? (int32_t)d[i >> 1] >> 16 : (int32_t)(int16_t)(d[i >> 1] & 0xFFFFu);
}

__device__ __forceinline__ void dense_counts(char *mine, int lane, int32_t vmin, uint32_t &nodes, uint32_t &lmax) {
    uint32_t d[32];
    tile_row(mine, lane, d);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the row is in registers before the tile is overwritten
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < 12; ++k) *reinterpret_cast<uint4 *>(mine + k * 1024 + lane * 16) = make_uint4(0, 0, 0, 0);
    __builtin_amdgcn_wave_barrier();
    char *cnt = mine + kHufCnt + lane * 4;
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        const int32_t v = coef_at(d, i);
        const uint32_t s = (uint32_t)(v - vmin) & 63u;
        __hip_atomic_fetch_add(reinterpret_cast<uint32_t *>(cnt + (s >> 2) * 256), (v != 0 ? 1u : 0u) << (8 * (s & 3)),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t w = *reinterpret_cast<const uint32_t *>(cnt + k * 256);
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint32_t f = (w >> (8 * b)) & 0xFFu;
            hist_add(mine, f ? f : 1u, lane, f ? 1u : 0u);  // branch-free (an add of 0 for an empty counter)
            lmax = f > lmax ? f : lmax;
            nodes += f ? 1u : 0u;
        }
    }
}

#ifndef DCTQ_HUF_MIN_WAVES
#define DCTQ_HUF_MIN_WAVES 3
#endif
__global__ __launch_bounds__(kHufThreads, DCTQ_HUF_MIN_WAVES) void huffman_bits_kernel(const int16_t *__restrict__ coef, long long nblk,
                                                                   uint32_t *__restrict__ bits, long long ntiles) {
    // per wave: the tile stage (9 KiB), then the histogram (8 KiB) and the dense counters (4 KiB)
    __shared__ uint4 lds[kHufWaves * kHufWaveLds / 16];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    char *mine = reinterpret_cast<char *>(lds) + wv * kHufWaveLds;
    const long long stride = (long long)gridDim.x * kHufWaves;
    for (long long t = (long long)blockIdx.x * kHufWaves + wv; t < ntiles; t += stride) {
        const long long left = nblk - t * 64;
        const int nb = left < 64 ? (int)left : 64;
        // ---- tile -> LDS: load k covers blocks 8k..8k+7 (16 B per lane, 1 KiB per load)
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<int16_t *>(coef) + t * 64 * 64, (short)0, nb * 128, 0x00020000);  // past the tail: zeros
        uint4 q[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, k * 1024, 2 /* nt */);
            q[k] = make_uint4(v[0], v[1], v[2], v[3]);
        }
        // the previous tile's histogram reads are done (lgkmcnt) and its bits store
        // retired with the loads above (one in-order vmcnt) before LDS is rewritten
        __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0)
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int k = 0; k < 8; ++k)
            *reinterpret_cast<uint4 *>(mine + (8 * k + (lane >> 3)) * kHufPitch + (lane & 7) * 16) = q[k];
        __builtin_amdgcn_wave_barrier();
        uint32_t nz = 0;
        bool last_zero;  // c[63] == 0: value 0 is a symbol once
        bool narrow = false;  // dense tile whose every block's values span < 64 integers
        int32_t vmin = 0;
        {
            uint32_t d[32];
            tile_row(mine, lane, d);
#pragma unroll
            for (int k = 0; k < 32; ++k) nz += ((d[k] & 0xFFFFu) != 0u) + ((d[k] >> 16) != 0u);
            last_zero = (d[31] >> 16) == 0u;
            if (__builtin_amdgcn_ballot_w64(nz > 32)) {
                // dense tile: the span of its values, zeros included (packed 16-bit min/max)
                typedef short s2 __attribute__((ext_vector_type(2)));
                s2 mn = __builtin_bit_cast(s2, d[0]), mx = mn;
#pragma unroll
                for (int k = 1; k < 32; ++k) {
                    const s2 x = __builtin_bit_cast(s2, d[k]);
                    mn = __builtin_elementwise_min(mn, x);
                    mx = __builtin_elementwise_max(mx, x);
                }
                vmin = mn.x < mn.y ? mn.x : mn.y;
                const int32_t vmax = mx.x > mx.y ? mx.x : mx.y;
                narrow = !__builtin_amdgcn_ballot_w64(lane < nb && vmax - vmin >= 64);
            }
        }
        // the paths re-read the row: a memory clobber keeps the compiler from reusing
        // (and holding) these 32 registers across the choice
        asm volatile("" ::: "memory");
        // ---- runs of equal values -> histogram of frequencies (the tile's LDS is reused)
        const uint32_t count = nz + (last_zero ? 1u : 0u);  // symbols: the nonzeros, plus a 0 once if c[63] == 0
        uint32_t nodes = last_zero ? 1u : 0u;
        uint32_t lmax = last_zero ? 1u : 0u;  // the largest leaf weight (dense paths)
#ifdef DCTQ_HUF_UNIFORM_MERGE
        const bool lane_merge = false;
#else
        const bool lane_merge = __builtin_amdgcn_ballot_w64(nz > 32) != 0;  // the dense paths mark occ
#endif
#ifdef DCTQ_HUF_ABLATE_FLOOR  // timing ablation only: the tile load and classification, no sizes
        if (true) {
        } else
#endif
        if (!__builtin_amdgcn_ballot_w64(nz > 16))
            sparse_runs<16>(mine, lane, nodes, lmax);
        else if (!__builtin_amdgcn_ballot_w64(nz > 32))
            sparse_runs<32>(mine, lane, nodes, lmax);
        else if (narrow)
            dense_counts(mine, lane, vmin, nodes, lmax);
        else
            dense_runs(mine, lane, nodes, lmax);
        if (last_zero) hist_add(mine, 1, lane, 1);
        // ---- bucket merge (see the header): wpl = sum of internal node weights.
        uint32_t wpl = 0, pending = 0;
        if (lane >= nb) nodes = 1;  // past the tail: nothing to do
        const uint16_t *bucket = reinterpret_cast<const uint16_t *>(mine + lane * 2);  // weight w at [(w-1)*64]
        uint64_t occ = 0;
        if (lane_merge) {
            // occupancy of the leaf buckets, read back up to the wave's largest leaf weight
            // (cheaper than marking every leaf; this wave's LDS atomics are already ordered)
#pragma unroll
            for (uint32_t w = 1; w <= 8; ++w)  // independent reads, in flight together
                occ |= bucket[(w - 1) * 64] ? 1ull << (w - 1) : 0ull;
            for (uint32_t w = 9; __builtin_amdgcn_ballot_w64(w <= lmax); ++w)
                occ |= bucket[(w - 1) * 64] ? 1ull << (w - 1) : 0ull;
        // Dense tiles: each lane jumps to its own next occupied bucket (lowest bit of occ), so the
        // loop runs as many steps as the busiest lane has occupied buckets, not up to
        // its largest weight.  New weights (pending + w, 2w) are above w, so the
        // scan order is the bucket order.  Every step merges at least one pair of a
        // consistent histogram; the step cap only bounds the loop.
        for (int step = 0; step < 130 && __builtin_amdgcn_ballot_w64(nodes > 1); ++step) {
            if (nodes > 1) {
                const uint32_t w = (uint32_t)__builtin_ctzll(occ) + 1u;
                occ &= occ - 1ull;  // bucket w is emptied by this step
                uint32_t c = w <= 64u ? bucket[(w - 1) * 64] : 0u;
                if (pending && c) {
                    const uint32_t nw = pending + w;
                    wpl += nw;
                    hist_add(mine, nw, lane, 1);
                    mark(occ, nw, 1);
                    --c;
                    --nodes;
                    pending = 0;
                }
                const uint32_t pairs = c >> 1;
                if (pairs) {
                    wpl += pairs * 2 * w;
                    nodes -= pairs;
                    hist_add(mine, 2 * w, lane, pairs);
                    mark(occ, 2 * w, 1);
                }
                if (c & 1) pending = w;
            }
        }
        } else {
        // Sparse tiles (few weights): every weight in turn; bucket w+1 is read at the top of iteration w, so its
        // LDS latency hides behind the iteration; the only merges of iteration w that
        // land on w+1 (pending 1 + w, and the pairs of w = 1) are carried in a register
        uint32_t cur = bucket[0];
        for (uint32_t w = 1; w <= 64 && __builtin_amdgcn_ballot_w64(nodes > 1); ++w) {
            const uint32_t nxt = w < 64 ? bucket[w * 64] : 0u;
            uint32_t c = cur, carry = 0;
            if (nodes > 1) {
                if (pending && c) {
                    const uint32_t nw = pending + w;
                    wpl += nw;
                    if (nw == w + 1)
                        carry = 1;
                    else
                        hist_add(mine, nw, lane, 1);
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
                        hist_add(mine, 2 * w, lane, pairs);
                }
                if (c & 1) pending = w;
            }
            cur = nxt + carry;
        }
        }
        const __amdgpu_buffer_rsrc_t rb =
            __builtin_amdgcn_make_buffer_rsrc(bits + t * 64, (short)0, nb * 4, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b32(8u * count + wpl, rb, lane * 4, 0, 0);
    }
}

hipError_t launch_huffman_bits(const int16_t *coef, long long nblk, uint32_t *bits, hipStream_t stream, int num_cus) {
    const long long ntiles = (nblk + 63) / 64;
    long long grid = (ntiles + kHufWaves - 1) / kHufWaves;
    const long long cap = (long long)num_cus * 8;
    if (grid > cap) grid = cap;
    hipLaunchKernelGGL(huffman_bits_kernel, dim3((unsigned)grid), dim3(kHufThreads), 0, stream, coef, nblk, bits,
                       ntiles);
    return hipGetLastError();
}
}  // namespace dctq
