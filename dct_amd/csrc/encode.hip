// dct_amd/csrc/encode.hip -- fused encoder: u8 planes -> zigzag run-length
// symbols ("shrink the coefficient planes before the xGMI
// gather"), i.e. dctq_forward_quant_planes followed by dctq_rle_count/emit over
// the concatenated planes, without the int16 coefficients ever reaching HBM.
//
// Two passes over the pixels, with the forward recomputed instead of stored:
//   1. encode_count: forward (fdct8_core.h, flagged coefficients resolved in
//      place -- a tie can decide zero vs nonzero) into the LDS stage; per-block
//      symbol counts by the DPP method of rle_count_kernel on the stage's 1 KiB
//      chunks -> tile-local offsets + one total per 64-block batch;
//   2. the segmented tile scan and a per-plane fix-up (rle.hip) -> offsets;
//   3. encode_emit: the same forward again, then every block's symbols from the
//      stage (lane i = zigzag element i, as rle_emit_kernel) to their offsets.
// HBM traffic: 64 + 4 (pass 1) + 8 (fix-up) + 64 + 4 + 4 x symbols (pass 2)
// bytes per block, against 192 + 140 + 132 + 4 x symbols for the three kernels
// of the unfused path.  Pass 1 and the forward half of pass 2 are VALU work the
// forward kernel hides under its memory time.
//
// Store-data hazard: every LDS read-back follows the prefetch fence,
// which retires the wave's stores of the previous batch; no LDS read follows a
// store within a batch.
#include "fdct8_core.h"
#include "scan_core.h"
#include "zigzag.h"

namespace dctq {

__device__ __forceinline__ void fence_rows(uint2 (&nxt)[8]) {
    asm volatile("" : "+v"(nxt[0]), "+v"(nxt[1]), "+v"(nxt[2]), "+v"(nxt[3]), "+v"(nxt[4]), "+v"(nxt[5]),
                 "+v"(nxt[6]), "+v"(nxt[7])::"memory");
}

__device__ __forceinline__ uint32_t nz16e(uint32_t w) { return ((w & 0xFFFFu) != 0u) + ((w >> 16) != 0u); }

template <bool ADAPTIVE>
__global__ __launch_bounds__(kThreads, 4) void encode_count_kernel(EncodeSet es, const DevTables *__restrict__ dev,
                                                                   uint32_t *__restrict__ offsets,
                                                                   uint32_t *__restrict__ tiles) {
    __shared__ uint4 stage[kThreads * kPitch2 / 16];
    const PlaneSet &ps = es.ps;
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t nbatch = ps.first[ps.n];
    const uint32_t step = gridDim.x * kWaves;
    uint32_t g = blockIdx.x * kWaves + wv;
    uint2 nxt[8];
    prefetch_batch(ps, g, lane, nxt);
    fence_rows(nxt);
    for (; g < nbatch; g += step) {
        const int k = plane_of(ps, g);
        const uint32_t b = g - ps.first[k];
        const int nblk = ps.pl[k].nblk;
        uint2 cur[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) cur[r] = nxt[r];
        prefetch_batch(ps, g + step, lane, nxt);
        int32_t vn;
        forward_exact_batch<ADAPTIVE, false>(dev, cur, stage, lane, wv, b * 64 + lane < (uint32_t)nblk, vn);
        fence_rows(nxt);  // the prefetch wait: retires the previous batch's stores too
        wave_sync();
        u4v q[8];
        stage_chunks(stage, wv, lane, q);
        const int nb = nblk - (int)(b * 64) < 64 ? nblk - (int)(b * 64) : 64;
        uint32_t *off = offsets + es.blk_first[k] + (size_t)b * 64;
        uint32_t run = 0;
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
            const int blk = 8 * kk + (lane >> 3);  // chunk 64kk + lane holds 16 B of this block
            uint32_t e = nz16e(q[kk][0]) + nz16e(q[kk][1]) + nz16e(q[kk][2]) + nz16e(q[kk][3]);
            if ((lane & 7) == 7) e += 1u - ((q[kk][3] >> 16) != 0u);  // +1 per block, c[63] excluded
            if (blk >= nb) e = 0u;
            const uint32_t inc = wave_inclusive_scan(e);
            const uint32_t before = __builtin_amdgcn_update_dpp(0u, inc - e, 0x117, 0xF, 0xF, false);  // row_shr:7
            if ((lane & 7) == 7 && blk < nb) off[blk] = run + before;
            run += __builtin_amdgcn_readlane(inc, 63);
        }
        if (lane == 0) tiles[g] = run;
    }
}

template <bool ADAPTIVE>
__global__ __launch_bounds__(kThreads, 4) void encode_emit_kernel(EncodeSet es, const DevTables *__restrict__ dev,
                                                                  const uint32_t *__restrict__ offsets,
                                                                  uint32_t *__restrict__ symbols,
                                                                  unsigned long long capacity) {
    __shared__ uint4 stage[kThreads * kPitch2 / 16];
    const PlaneSet &ps = es.ps;
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t nbatch = ps.first[ps.n];
    const uint32_t step = gridDim.x * kWaves;
    const uint32_t zoff = 2u * kZigzag[lane];
    const uint64_t upto = ~0ull >> (63 - lane);  // lanes 0..lane
    const uint32_t upto_lo = (uint32_t)upto, upto_hi = (uint32_t)(upto >> 32);
    const char *wst = reinterpret_cast<const char *>(stage) + wv * 64 * kPitch2;
    uint32_t g = blockIdx.x * kWaves + wv;
    uint2 nxt[8];
    prefetch_batch(ps, g, lane, nxt);
    fence_rows(nxt);
    for (; g < nbatch; g += step) {
        const int k = plane_of(ps, g);
        const uint32_t b = g - ps.first[k];
        const int nblk = ps.pl[k].nblk;
        const int nb = nblk - (int)(b * 64) < 64 ? nblk - (int)(b * 64) : 64;
        uint2 cur[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) cur[r] = nxt[r];
        prefetch_batch(ps, g + step, lane, nxt);
        const uint32_t offv = offsets[es.blk_first[k] + (size_t)b * 64 + (lane < nb ? lane : nb - 1)];
        int32_t vn;
        forward_exact_batch<ADAPTIVE, false>(dev, cur, stage, lane, wv, lane < nb, vn);
        fence_rows(nxt);  // the prefetch wait: retires the previous batch's symbol stores too
        wave_sync();
        uint32_t z[32];  // zigzag element `lane` of blocks 2u (low half) and 2u+1 (high half)
#pragma unroll
        for (int u = 0; u < 32; ++u)
            z[u] = (uint32_t)*reinterpret_cast<const uint16_t *>(wst + 2 * u * kPitch2 + zoff) |
                   ((uint32_t)*reinterpret_cast<const uint16_t *>(wst + (2 * u + 1) * kPitch2 + zoff) << 16);
        // symbols of this batch from offsets[first block] on; those at or past
        // `capacity` are dropped by num_records
        const uint32_t o0 = __builtin_amdgcn_readlane(offv, 0);
        const unsigned long long room = capacity > o0 ? capacity - o0 : 0ull;
        const __amdgpu_buffer_rsrc_t rsym = __builtin_amdgcn_make_buffer_rsrc(
            symbols + o0, (short)0, (int)((room < 4096ull ? room : 4096ull) * 4u), 0x00020000);
#pragma unroll
        for (int u = 0; u < 64; ++u) {
            const uint32_t val = (u & 1) ? z[u >> 1] >> 16 : z[u >> 1] & 0xFFFFu;
            const bool emit = val != 0u || lane == 63;
            const uint64_t E = __builtin_amdgcn_ballot_w64(emit);
            const uint64_t E2 = (E << 1) | 1ull;  // bit 0: "no earlier symbol"
            const uint64_t prev =
                (uint64_t)(upto_lo & (uint32_t)E2) | ((uint64_t)(upto_hi & (uint32_t)(E2 >> 32)) << 32);
            uint32_t runlen = (uint32_t)(lane - 63 + __builtin_clzll(prev));
            if (lane == 63 && val == 0u) runlen += 1u;  // the last symbol's run counts itself (src/entropy.c:231-233)
            const uint32_t idx =
                __builtin_amdgcn_mbcnt_hi((uint32_t)(E >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)E, 0u));
            const uint32_t o = __builtin_amdgcn_readlane(offv, u);
            const uint32_t addr = (emit && u < nb) ? (o - o0 + idx) * 4u : 0xFFFFFFF0u;
            __builtin_amdgcn_raw_buffer_store_b32(val | (runlen << 16), rsym, addr, 0, 0);
        }
    }
}

template <typename K, typename... A>
static hipError_t launch_enc(K kernel, uint32_t nbatch, int num_cus, hipStream_t stream, A... args) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kThreads, 0) != hipSuccess || per_cu < 1)
        per_cu = 1;
    const uint32_t want = (nbatch + kWaves - 1) / kWaves;
    const uint32_t cap = (uint32_t)(num_cus * per_cu);
    hipLaunchKernelGGL(kernel, dim3(want < cap ? want : cap), dim3(kThreads), 0, stream, args...);
    return hipGetLastError();
}

size_t encode_workspace_bytes(long long nbatch) { return rle_scan_workspace_bytes(nbatch); }

hipError_t launch_encode(const EncodeSet &es, const DevTables *dev, int adaptive, uint32_t *offsets,
                         uint32_t *symbols, unsigned long long capacity, void *ws, hipStream_t stream, int num_cus) {
    const uint32_t nbatch = es.ps.first[es.ps.n];
    uint32_t *tiles = (uint32_t *)ws;
    hipError_t e = adaptive ? launch_enc(encode_count_kernel<true>, nbatch, num_cus, stream, es, dev, offsets, tiles)
                            : launch_enc(encode_count_kernel<false>, nbatch, num_cus, stream, es, dev, offsets, tiles);
    if (e != hipSuccess) return e;
    if ((e = launch_rle_scan(ws, nbatch, stream)) != hipSuccess) return e;
    for (int k = 0; k < es.ps.n; ++k) {
        uint32_t *total = k == es.ps.n - 1 ? offsets + es.blk_first[es.ps.n] : nullptr;
        if ((e = launch_rle_fixup(offsets + es.blk_first[k], es.ps.pl[k].nblk, ws, nbatch, es.ps.first[k], total,
                                  stream)) != hipSuccess)
            return e;
    }
    if (!symbols || capacity == 0) return hipSuccess;  // offsets only
    return adaptive ? launch_enc(encode_emit_kernel<true>, nbatch, num_cus, stream, es, dev, (const uint32_t *)offsets,
                                 symbols, capacity)
                    : launch_enc(encode_emit_kernel<false>, nbatch, num_cus, stream, es, dev,
                                 (const uint32_t *)offsets, symbols, capacity);
}

}  // namespace dctq
