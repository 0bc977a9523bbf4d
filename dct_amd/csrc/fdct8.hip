// dct_amd/csrc/fdct8.hip -- the MI355X hot path: 8x8 forward DCT + quantization.
//
// Replaces the per-block loop of the reference pipeline (tests/test_entropy.c:300-316):
//   create_block_from_pixels (src/dct.c:109-120) -> dct_forward (src/dct.c:52-77)
//   -> calculate_block_variance (src/quantization.c:153-169)
//   -> quantize (src/quantization.c:113-131, adaptive :171-211)
// for every block of a stack of u8 planes, in ONE launch.
//
// Layout (DESIGN.md "Kernels"): one LANE owns one 8x8 block, a wave64 owns 64
// consecutive blocks in raster order.  Each lane loads its block as 8 x 8-byte
// rows (a wave-instruction reads 512 contiguous bytes of one pixel row), runs the
// separable AAN butterfly entirely in registers (no cross-lane traffic, all
// constants wave-uniform), quantizes, and the wave stages its 8 KiB of int16
// output through LDS so the global stores are 1 KiB contiguous per instruction.
//
// Exactness (DESIGN.md "Exactness"): the fp32 butterfly is ~1e-4 away from the
// reference's fp64 values, which matters only when c/Q lies near a rounding
// tie (x.5).  tools/guard_bound.py proves a per-coefficient error bound; a
// coefficient whose fractional part is within that band of 0.5 is recomputed
// in the reference's exact fp64 operation order (no FMA
// contraction: this file is compiled with -ffp-contract=off), with IEEE
// division and round-half-away-from-zero.  All other coefficients are provably
// rounded the same way the reference rounds them.
#include "fdct8_core.h"

namespace dctq {

// ============================================================================
// fdct8_quant_v3, the product kernel for every plan and size: a persistent
// grid-stride loop over 64-block batches (one lane per block), the next batch's
// rows prefetched, the forward core of fdct8_core.h into the wave's LDS stage, the
// flagged coefficients resolved IN PLACE after the prefetch fence
// (resolve_ties_compact: reference-order fp64 from the pixels still in registers,
// in grouped passes, tables from a 1 KiB LDS copy), then 8 x 1 KiB stores.  No
// stash, no drains, no patch stores: its HBM traffic is the algorithmic 192 B per
// block (PMC 1.0001x, profiles/traffic.json).  The round-1/2 queue kernel (v2) and
// the per-workgroup v1 live in the diagnostic library only (fdct8_diag.hip).
// Passes of <= 8 tie entries run 8 lanes per entry (exact_grouped<8>), and without the
// variance output or the fallback counter passes of 9..32 entries run one round of 2
// lanes per entry (round 4, profiles/r04/wide2_ab.log, three rotations with every build
// at every slot: q97 -7 %, extreme q10 -4 %, q100 -1 %, uniform q50 within the noise).
// The 4-lane rounds put a scratch reload in front of the stores, and with VAR or STATS
// the 2-lane rounds spill too, so those instantiations keep one entry per lane.
constexpr bool kV3Group8 = true;
constexpr int kV3Wide = 2;
// fdct8_quant_v3 launches 16 x its resident workgroups (round 4, profiles/r04/forward_grid_sweep.log,
// one box, interleaved, two passes: x8 424.6 / 424.0 us, x12 417.1 / 416.1, x16 413.3 / 412.1,
// x24 416.9 / 417.6, x32 424.0 / 421.0, x48 (one batch per wave) 428.4 / 427.4 on the bench step;
// x16 also -1.8 % extreme q10, -3.5 % smooth q90 adaptive, +0.5 % constant blocks).  With no stash
// (v3 resolves ties in place) the grid costs nothing but workgroup starts (kV3GridMult,
// fdct8_core.h, where the movement twin of the diagnostic library reads it too).
template <bool ADAPTIVE, bool VAR, bool STATS>
__global__ __launch_bounds__(kFThreads, 4) void fdct8_quant_v3(PlaneSet ps, const DevTables *__restrict__ dev,
                                                              unsigned long long *fallbacks) {
    __shared__ uint4 stage[kFThreads * kPitch2 / 16];
    __shared__ ExactTables tab;
    __shared__ uint16_t scr[kFWaves * 64];  // resolve_ties_compact's entries
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    load_exact_tables(&tab, dev);
    const uint32_t nbatch = ps.first[ps.n];
    const uint32_t step = gridDim.x * kFWaves;
    uint32_t g = blockIdx.x * kFWaves + wv;
    uint2 nxt[8];
    prefetch_batch(ps, g, lane, nxt);
    asm volatile("" : "+v"(nxt[0]), "+v"(nxt[1]), "+v"(nxt[2]), "+v"(nxt[3]), "+v"(nxt[4]), "+v"(nxt[5]),
                 "+v"(nxt[6]), "+v"(nxt[7])::"memory");
    uint32_t resolved = 0;
    for (; g < nbatch; g += step) {
        const uint32_t gnext = g + step;
        const int k = plane_of(ps, g);
        const PlaneArgs &p = ps.pl[k];
        const uint32_t b = g - first_of(ps, k);
        uint2 cur[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) cur[r] = nxt[r];
        prefetch_batch(ps, gnext, lane, nxt);
        const BatchOut out = batch_out(ps, k, b);
        int32_t var_num;
        uint32_t mlo, mhi;
        forward_flags_batch<ADAPTIVE, VAR>(dev, cur, stage, lane, wv, b * 64 + lane < (uint32_t)p.nblk, var_num, mlo,
                                           mhi);
        // the prefetch wait (retires the previous batch's stores too), then LDS reads
        asm volatile("" : "+v"(nxt[0]), "+v"(nxt[1]), "+v"(nxt[2]), "+v"(nxt[3]), "+v"(nxt[4]), "+v"(nxt[5]),
                     "+v"(nxt[6]), "+v"(nxt[7])::"memory");
        resolved += resolve_ties_compact<ADAPTIVE, kV3Group8, (VAR || STATS) ? 0 : kV3Wide>(
            &tab, cur, stage, scr + wv * 64, lane, wv, mlo, mhi);
        wave_sync();
        u4v val[8];
        stage_chunks(stage, wv, lane, val);
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(out.base, (short)0, (int)(out.nb * 128u), 0x00020000);
#pragma unroll
        for (int c = 0; c < 8; ++c) __builtin_amdgcn_raw_buffer_store_b128(val[c], rs, lane * 16, c * 1024, kStoreAux);
        if (VAR) {
            const __amdgpu_buffer_rsrc_t rv =
                __builtin_amdgcn_make_buffer_rsrc(out.var, (short)0, (int)(out.nb * 4u), 0x00020000);
            __builtin_amdgcn_raw_buffer_store_b32(var_num, rv, lane * 4, 0, kStoreAux);
        }
    }
    if (STATS && resolved) atomicAdd(fallbacks, (unsigned long long)resolved);
}

template <bool A, bool V, bool S>
static hipError_t launch_v3(const PlaneSet &ps, const DevTables *dev, unsigned long long *fb, hipStream_t stream,
                            int num_cus) {
    static const int per_cu = resident_per_cu(fdct8_quant_v3<A, V, S>, kFThreads);
    const uint32_t nbatch = ps.first[ps.n];
    const uint32_t want = (nbatch + kFWaves - 1) / kFWaves;
    const uint32_t cap = (uint32_t)(num_cus * per_cu * kV3GridMult);
    hipLaunchKernelGGL((fdct8_quant_v3<A, V, S>), dim3(want < cap ? want : cap), dim3(kFThreads), 0, stream, ps, dev, fb);
    return hipGetLastError();
}

hipError_t launch_fdct8_quant(const PlaneSet &ps, const DevTables *dev, int adaptive, unsigned long long *fallbacks,
                              hipStream_t stream, int num_cus) {
    const bool a = adaptive != 0, v = ps.var[0] != nullptr, s = fallbacks != nullptr;
    if (a) {
        if (v) return s ? launch_v3<true, true, true>(ps, dev, fallbacks, stream, num_cus)
                        : launch_v3<true, true, false>(ps, dev, fallbacks, stream, num_cus);
        return s ? launch_v3<true, false, true>(ps, dev, fallbacks, stream, num_cus)
                 : launch_v3<true, false, false>(ps, dev, fallbacks, stream, num_cus);
    }
    if (v) return s ? launch_v3<false, true, true>(ps, dev, fallbacks, stream, num_cus)
                    : launch_v3<false, true, false>(ps, dev, fallbacks, stream, num_cus);
    return s ? launch_v3<false, false, true>(ps, dev, fallbacks, stream, num_cus)
             : launch_v3<false, false, false>(ps, dev, fallbacks, stream, num_cus);
}

}  // namespace dctq
