// dct_amd/csrc/encode.hip -- the encoder: u8 planes -> int16 coefficients AND
// zigzag run-length symbols ("shrink the coefficient planes before
// the xGMI gather") = dctq_forward_quant_planes + dctq_rle_count + dctq_rle_emit
// over the concatenated planes, with the count fused into the forward:
//   1. encode_count: the forward (fdct8_core.h) with flagged coefficients
//      resolved in place -- a tie can decide zero vs nonzero -- whose 1 KiB
//      stage chunks are stored AND counted (the DPP method of rle_count_kernel)
//      -> coefficients, tile-local offsets, one total per 64-block batch;
//   2. the segmented tile scan and a per-plane fix-up (rle.hip) -> offsets;
//   3. rle_emit per plane over the coefficients.
// The count costs the forward kernel VALU it has to spare (it is memory-bound)
// and saves the count pass's 128 B/block re-read.  A variant that never stored
// the coefficients and recomputed the forward for the emission instead (64 B
// instead of 256 B per block) measured slower: both of its passes were
// VALU-bound.
//
// Store-data hazard: every LDS read-back follows the prefetch fence,
// which retires the wave's stores of the previous batch; no LDS read follows a
// store within a batch.
#include "fdct8_core.h"
#include "scan_core.h"

namespace dctq {

__device__ __forceinline__ void fence_rows(uint2 (&nxt)[8]) {
    asm volatile("" : "+v"(nxt[0]), "+v"(nxt[1]), "+v"(nxt[2]), "+v"(nxt[3]), "+v"(nxt[4]), "+v"(nxt[5]),
                 "+v"(nxt[6]), "+v"(nxt[7])::"memory");
}

__device__ __forceinline__ uint32_t nz16e(uint32_t w) { return ((w & 0xFFFFu) != 0u) + ((w >> 16) != 0u); }

// Passes of <= 8 tie entries run 8 lanes per entry (exact_grouped<8>): -0.9 %; the wide
// rounds spill at this kernel's 128-VGPR bound.
constexpr bool kEncGroup8 = true;
constexpr int kEncWide = 0;
// encode_count launches 32 x its resident workgroups (about one and a half batches per wave on the
// bench step): -1.2..-1.5 % on the whole encode step against 8 x, 48 x and 64 x the same, 16 x half
// of it (round 6, profiles/r06/enc_count_packed_ab/enc_grid_ab*.log, tools/enc_ab.py).
constexpr int kEncGridMult = 32;

template <bool ADAPTIVE>
__global__ __launch_bounds__(kThreads, 4) void encode_count_kernel(EncodeSet es, const DevTables *__restrict__ dev,
                                                                   uint32_t *__restrict__ offsets,
                                                                   uint32_t *__restrict__ tiles) {
    __shared__ uint4 stage[kThreads * kPitch2 / 16];
    __shared__ ExactTables tab;
    __shared__ uint16_t scr[kWaves * 64];  // resolve_ties_compact's entries
    load_exact_tables(&tab, dev);
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
        const uint32_t b = g - first_of(ps, k);
        const int nblk = ps.pl[k].nblk;
        uint2 cur[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) cur[r] = nxt[r];
        prefetch_batch(ps, g + step, lane, nxt);
        const BatchOut out = batch_out(ps, k, b);  // resolved before the fence (fdct8_core.h)
        uint32_t *off = offsets + es.blk_first[k] + (size_t)b * 64;
        asm volatile("" : "+s"(off));
        int32_t vn;
        uint32_t mlo, mhi;
        forward_flags_batch<ADAPTIVE, false>(dev, cur, stage, lane, wv, b * 64 + lane < (uint32_t)nblk, vn, mlo, mhi);
        fence_rows(nxt);  // the prefetch wait: retires the previous batch's stores too
        resolve_ties_compact<ADAPTIVE, kEncGroup8, kEncWide>(&tab, cur, stage, scr + wv * 64, lane, wv, mlo, mhi);
        wave_sync();
        u4v q[8];
        stage_chunks(stage, wv, lane, q);
        const int nb = (int)out.nb;
        {
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out.base, (short)0, nb * 128, 0x00020000);
#pragma unroll
            for (int c = 0; c < 8; ++c) __builtin_amdgcn_raw_buffer_store_b128(q[c], rs, lane * 16, c * 1024, kNtAux);
        }
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

template <typename K, typename... A>
static hipError_t launch_enc(K kernel, uint32_t nbatch, int num_cus, hipStream_t stream, A... args) {
    const int per_cu = resident_per_cu(kernel, kThreads);
    const uint32_t want = (nbatch + kWaves - 1) / kWaves;
    const uint32_t cap = (uint32_t)(num_cus * per_cu * kEncGridMult);
    hipLaunchKernelGGL(kernel, dim3(want < cap ? want : cap), dim3(kThreads), 0, stream, args...);
    return hipGetLastError();
}

size_t encode_workspace_bytes(long long nbatch) { return rle_scan_workspace_bytes(nbatch); }

hipError_t launch_encode(const EncodeSet &es, const DevTables *dev, int adaptive, uint32_t *offsets, void *symbols,
                         int symbol_bytes, unsigned long long capacity, void *ws, hipStream_t stream, int num_cus) {
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
    if (!symbols || capacity == 0) return hipSuccess;  // coefficients and offsets only
    for (int k = 0; k < es.ps.n; ++k)
        if ((e = launch_rle_emit(es.ps.coef[k], es.ps.pl[k].nblk, offsets + es.blk_first[k], symbols, symbol_bytes,
                                 capacity, stream, num_cus)) != hipSuccess)
            return e;
    return hipSuccess;
}

}  // namespace dctq
