// dct_amd/csrc/fdct8_diag.hip -- kernels and machinery of the DIAGNOSTIC library
// only (libdct_amd_diag.so; dct_amd/build.py DIAG_SOURCES).  libdct_amd.so, the
// product, carries none of it: its forward is fdct8_quant_v3 for every plan
// (fdct8.hip), its round trip roundtrip8 (roundtrip.hip).
//   * fdct8_quant_v1 (one workgroup per 256 blocks, divergent exact path) and
//     fdct8_quant_v2 (the round-1/2 tie-queue kernel with its per-stream pixel
//     stash), selected per plan by dctq_diag_plan_set_variant (1 / 4) for the
//     A/B harnesses and the forced-kernel parity tests;
//   * the lane-per-block fp64 float-forward and inverse kernels (variant 1 of
//     dctq_forward_float / dctq_inverse; the product runs the paired-lane ones,
//     f64_pair.hip);
//   * the no-arithmetic movement twins of the forward and round-trip kernels
//     (bench.py's same-box ceilings).
// The diagnostic entry points dctq_diag_forward_quant_planes / _forward_float / _inverse
// reach the variants (the product entry points never do),
// which this file fills when the diagnostic library loads.
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "aan_f64.h"
#include "dctq_diag.h"
#include "fdct8_core.h"
#include "pair_core.h"
#include "plan.h"

// Timing ablations of the retired kernels here (diagnostic builds only, -DDCTQ_ABLATE=m):
// 1 no tie flags, 8 flags but no queue, 16 queue without drains, 32 queue code never
// run, 128 no coefficient stores, 1024 no stash stores, 2048 no final drain, 4096
// drains compute but do not patch.  0 in every build this tree makes.
#ifndef DCTQ_ABLATE
#define DCTQ_ABLATE 0
#endif

namespace dctq {

// ---- the v2 queue kernel's constants
constexpr int kQCap = 128;     // per-wave tie queue: < 64 between rounds + one round of <= 64
static_assert(kQCap <= 128, "queue entries hold the stash slot in 7 bits");
#ifndef DCTQ_PATCH_COND
#define DCTQ_PATCH_COND 1  // drains store only coefficients whose exact value differs from the fast one
#endif
#ifndef DCTQ_STASH_DEDUP
#define DCTQ_STASH_DEDUP 1  // one pixel stash per flagged block and batch (its entries share it)
#endif
constexpr int kV2GridMult = kGridMult;  // fdct8_quant_v2's grid (its stash is sized to it: 8 KiB per wave)

// Where the v2 forward gets its tie-path pixel stash: get(ctx, bytes) returns
// device memory of at least `bytes` that no other in-flight launch uses, or
// nullptr (one stash per (device, stream), grown to the launched grid: below).
struct RingSource {
    void *(*get)(void *ctx, size_t bytes);
    void *ctx;
};
// bytes of the v2 tie-path pixel stash for a grid of `workgroups` (64 B per queue slot)
size_t fdct8_ring_bytes(int workgroups);

// Reference-order fp64 recomputation of ONE quantized coefficient c = 8i + j:
//   temp[k][j] = sum_l x[k][l] * D^T[l][j]      (src/dct.c:57-64, l ascending)
//   out[i][j]  = sum_k D[i][k] * temp[k][j]     (src/dct.c:67-74, k ascending)
//   q          = (int) round(out / M_ij)        (src/quantization.c:124)
// with x = (double)px - 128.0 (src/dct.c:115).  Separate multiply and add
// (file compiled with -ffp-contract=off), each accumulator starting at 0.0.
__device__ __forceinline__ int exact_quant(const uint8_t *__restrict__ px, long long stride, int c,
                                        const double *__restrict__ dct, double m) {
    const int i = c >> 3, j = c & 7;
    double out = 0.0;
    // rolled: one row (8 doubles) live at a time -- this path must not set the
    // register allocation of the streaming loop around it
#pragma unroll 1
    for (int k = 0; k < 8; ++k) {
        const uint2 row = *reinterpret_cast<const uint2 *>(px + k * stride);
        double t = 0.0;
#pragma unroll
        for (int l = 0; l < 8; ++l) {
            const uint32_t w = l < 4 ? row.x : row.y;
            const double x = (double)((w >> (8 * (l & 3))) & 0xFFu) - 128.0;
            t += x * dct[j * 8 + l];
        }
        out += dct[i * 8 + k] * t;
    }
    return (int)round(out / m);
}

template <bool ADAPTIVE, bool VAR, bool STATS>
__global__ __launch_bounds__(kThreads) void fdct8_quant_v1(PlaneArgs p, FastTables t,
                                                               const DevTables *__restrict__ dev,
                                                               int16_t *__restrict__ coef,
                                                               int32_t *__restrict__ var_out,
                                                               unsigned long long *fallbacks) {
    __shared__ uint4 stage[kThreads * kPitch];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t wave0 = blockIdx.x * kThreads + wv * 64;  // first block of this wave
    const uint32_t n = wave0 + lane;
    const bool valid = n < (uint32_t)p.nblk;

    // ---- load: 8 rows x 8 B per lane
    const uint8_t *px = block_ptr(p, valid ? n : 0);
    uint2 rows[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) rows[r] = *reinterpret_cast<const uint2 *>(px + r * p.stride);

    // ---- unpack u8 -> fp32 (exact); the -128 centring is applied to Y00 only (exact)
    float v[8][8];
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            v[r][k] = (float)((rows[r].x >> (8 * k)) & 0xFFu);
            v[r][k + 4] = (float)((rows[r].y >> (8 * k)) & 0xFFu);
        }

    // ---- block variance numerator 64*sum(x^2) - sum(x)^2, x = px - 128 (exact integers)
    int32_t var_num = 0;
    if (ADAPTIVE || VAR) {
        uint32_t s1 = 0, s2 = 0;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            s1 = __builtin_amdgcn_udot4(rows[r].x, 0x01010101u, s1, false);
            s1 = __builtin_amdgcn_udot4(rows[r].y, 0x01010101u, s1, false);
            s2 = __builtin_amdgcn_udot4(rows[r].x, rows[r].x, s2, false);
            s2 = __builtin_amdgcn_udot4(rows[r].y, rows[r].y, s2, false);
        }
        const int32_t sx = (int32_t)s1 - 8192;
        const int32_t sxx = (int32_t)s2 - 256 * (int32_t)s1 + 1048576;
        var_num = 64 * sxx - sx * sx;
        if (VAR && valid) var_out[n] = var_num;
    }

    // ---- 2-D butterfly
    aan8x8(v, DCTQ_C4, DCTQ_C6, DCTQ_C2MC6, DCTQ_C2PC6);
    v[0][0] -= 8192.0f;  // 64 * 128: exact (integer < 2^24)

    float inv_s = 1.0f;
    double s64 = 1.0;
    if (ADAPTIVE) {
        s64 = adaptive_scale(var_num);
        inv_s = (float)(1.0 / s64);
    }

    // ---- quantize: t = rint(Y*w) in the low bits of t; flag |frac| beyond the guard
    uint32_t packed[32];
    uint32_t mlo = 0, mhi = 0;  // bit (31 - c%32) set => coefficient c needs the exact path
#pragma unroll
    for (int c = 0; c < 64; c += 2) {
        uint32_t tb[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int cc = c + h;
            const float y = v[cc >> 3][cc & 7];
            const float w = (ADAPTIVE && cc != 0) ? t.w[cc] * inv_s : t.w[cc];
            const float tt = __builtin_fmaf(y, w, kMagic);
            const float r = tt - kMagic;
            const float f = __builtin_fmaf(y, w, -r);
            const uint32_t fl = fabsf(f) > t.thr[cc] ? 1u : 0u;
            if (cc < 32) mlo = mlo + mlo + fl;
            else mhi = mhi + mhi + fl;
            tb[h] = __float_as_uint(tt);
        }
        packed[c >> 1] = __builtin_amdgcn_perm(tb[1], tb[0], 0x05040100u);
    }

    // ---- stage the lane's 128 B block in LDS (pitch 144 B: conflict-free b128 writes)
    uint4 *mine = stage + (wv * 64 + lane) * kPitch;
#pragma unroll
    for (int s = 0; s < 8; ++s)
        mine[s] = make_uint4(packed[4 * s], packed[4 * s + 1], packed[4 * s + 2], packed[4 * s + 3]);

    // ---- rare path: exact fp64 reference-order recomputation of flagged coefficients
    if (!valid) mlo = mhi = 0;
    if (__builtin_amdgcn_ballot_w64((mlo | mhi) != 0)) {
        int16_t *mine16 = reinterpret_cast<int16_t *>(mine);
        int cnt = 0;
        while (mlo | mhi) {
            int c;
            if (mlo) {
                c = __clz(mlo);
                mlo &= ~(0x80000000u >> c);
            } else {
                const int k = __clz(mhi);
                mhi &= ~(0x80000000u >> k);
                c = 32 + k;
            }
            double m = dev->quant[c];
            if (ADAPTIVE && c != 0) {
                m = m * s64;
                if (m < 1.0) m = 1.0;
            }
            mine16[c] = (int16_t)exact_quant(px, p.stride, c, dev->dct, m);
            ++cnt;
        }
        if (STATS) {
            // wave-sum of cnt, one atomic per wave
            int tot = cnt;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
            if (lane == 0 && tot) atomicAdd(fallbacks, (unsigned long long)tot);
        }
    }

    // ---- wave-local LDS hand-off, then 1 KiB-contiguous global stores
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint4 *dst = reinterpret_cast<uint4 *>(coef) + (size_t)wave0 * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int m = k * 64 + lane;  // 16-byte chunk of the wave's 8 KiB output
        const int bl = m >> 3;
        if (wave0 + bl < (uint32_t)p.nblk) dst[m] = stage[(wv * 64 + bl) * kPitch + (m & 7)];
    }
}

// ============================================================================
// v2 (default): persistent grid-stride kernel, sized for the gfx950 VALU cost
// model measured in profiles/r01/valu_issue_rates.md.
//  * each wave walks 64-block batches b, b+W, b+2W, ... and prefetches the next
//    batch's 8 rows (non-temporal) while it computes the current one;
//  * u8 -> fp32 with v_cvt_f32_ubyteN (inline asm, so the compiler cannot turn
//    the first butterfly stage into half-rate SDWA integer adds + converts);
//  * the second butterfly pass runs two columns at a time, fused with the
//    quantization of those 16 coefficients, whose packed int16 pairs go straight
//    to the LDS stage (16 of the 64 second-pass values live at a time);
//  * quantization in packed fp32 (the per-plan tables are read through scalar
//    loads in processing order), tie flags as sign bits of thr^2 - f^2 shifted
//    into a per-lane 64-bit mask with v_alignbit;
//  * the LDS stage is written out as 1 KiB-contiguous buffer stores (num_records
//    clips the tail, so the stores are unconditional);
//  * flagged (block, coefficient) pairs go to a wave-local LDS queue and are
//    recomputed exactly 64 at a time (every lane busy), then patched in HBM
//    where the result changes; a full queue drains at the next batch, before
//    that batch's stores are issued (vmcnt is one in-order counter: behind
//    8 KiB of fresh stores, the drain's stash loads would wait for all of them);
//  * one launch covers up to 4 planes (PlaneSet): the grid-stride index runs
//    over the concatenated 64-block batches, each batch finding its plane by
//    wave-uniform compares against the planes' batch prefixes.
// The per-batch building blocks (block addressing, row loads, the arithmetic
// into the stage, the constant-block DC fix) are in fdct8_core.h.

// Exact reference-order quantization of coefficient c of the block at px (one
// queue entry): exact_from_rows() over the pixels stashed when it was queued.
// A drain runs 64 of these at once (one per lane), so latency matters: all 8
// pixel rows are requested before the fp64 chain.
template <bool ADAPTIVE>
__device__ int exact_entry(const uint4 *__restrict__ stash, int c, const DevTables *__restrict__ dev) {
    uint2 rows[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint4 w = stash[k];  // rows 2k, 2k+1 of the block
        rows[2 * k] = make_uint2(w.x, w.y);
        rows[2 * k + 1] = make_uint2(w.z, w.w);
    }
    return exact_from_rows<ADAPTIVE>(rows, c, dev);
}

// Exact recomputation of up to 64 queued (block, coefficient) entries, one per
// lane, patched into their planes' coefficient arrays where the exact value
// differs from the fast one already stored (the two differ by at most 1 inside
// the guard band, so the parity bit kept in the entry decides).  A 2-B patch
// into a line already written back costs a read-modify-write at the memory
// (~155 B of stream time, profiles/r02/forward_overheads.md), so skipping the
// ~half of them that would rewrite the same value is the cheapest patch.
template <bool ADAPTIVE, bool STATS>
__device__ __forceinline__ void drain_queue(const PlaneSet &ps, const DevTables *__restrict__ dev, const uint32_t *qb,
                                            const uint16_t *qc, const uint4 *ring, int &qn, int lane,
                                            unsigned long long *fallbacks) {
    // the wave's own coefficient stores (and its stash stores) must land first
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    const int take = qn < 64 ? qn : 64;
    // the planes' output pointers in SGPRs: selected per lane with v_cndmask (left
    // to itself the compiler indexes the kernel-argument array with a per-lane
    // global load, one more memory latency in front of every patch)
    int16_t *cp[kMaxPlanes];
#pragma unroll
    for (int i = 0; i < kMaxPlanes; ++i) {
        cp[i] = ps.coef[i];
        asm volatile("" : "+s"(cp[i]));
    }
    if (lane < take) {
        const int slot = qn - take + lane;
        const uint32_t n = qb[slot], e = qc[slot];
        const int c = (int)(e & 63u);
        const int val = exact_entry<ADAPTIVE>(ring + (e >> 9) * 4, c, dev);
        if (DCTQ_ABLATE & 4096) {
            asm volatile("" ::"v"(val));  // diagnostic: computed, not patched
        } else if (!DCTQ_PATCH_COND || (((uint32_t)val ^ (e >> 8)) & 1u)) {
            const uint32_t k = (e >> 6) & 3u;
            int16_t *dst = cp[0];
#pragma unroll
            for (int i = 1; i < kMaxPlanes; ++i) dst = k == (uint32_t)i ? cp[i] : dst;
            ((__attribute__((address_space(1))) int16_t *)dst)[(size_t)n * 64 + c] = (int16_t)val;
        }
    }
    qn -= take;
    if (STATS && lane == 0) atomicAdd(fallbacks, (unsigned long long)take);
}

#ifndef DCTQ_LAST_INPLACE
#define DCTQ_LAST_INPLACE 1  // a wave's last batch empties the queue before its stores and resolves in place
#endif
#ifndef DCTQ_V2_GROUP
#define DCTQ_V2_GROUP 0  // A/B: the in-stage passes of the queue kernel in grouped rounds (resolve_ties_compact GROUP8)
#endif
#ifndef DCTQ_V2_WIDE
#define DCTQ_V2_WIDE 3   // ... and with the 4- / 2-lane rounds when DCTQ_V2_GROUP
#endif
#ifndef DCTQ_INSTAGE_LANES
// A batch with at least this many flagged blocks resolves its ties in the stage,
// before its stores (resolve_in_stage); sparser batches queue them.  65 = never.
#define DCTQ_INSTAGE_LANES 8
#endif

// One 64-block batch of the v2 loop.  `nxt` holds this batch's rows on entry and
// the next batch's rows on exit.
template <bool ADAPTIVE, bool VAR, bool STATS>
__device__ __forceinline__ void fdct8_batch(const PlaneSet &ps, const DevTables *__restrict__ dev,
                                            const ExactTables *tab,
                                            unsigned long long *fallbacks, uint4 *stage, uint32_t *qb, uint16_t *qc,
                                            uint4 *ring, int &qn, uint2 (&nxt)[8], uint32_t g, uint32_t step, int lane,
                                            int wv) {
    // global batch g -> plane k, plane-local batch b (wave-uniform)
    const int k = plane_of(ps, g);
    const PlaneArgs &p = ps.pl[k];
    const uint32_t b = g - first_of(ps, k);
    uint2 cur[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) cur[r] = nxt[r];
    const uint32_t n = b * 64 + lane;
    const bool valid = n < (uint32_t)p.nblk;
    prefetch_batch(ps, g + step, lane, nxt);
    const BatchOut out = batch_out(ps, k, b);

    uint32_t mlo, mhi;
    int32_t var_num;
    fdct8_compute<ADAPTIVE, VAR>(dev, cur, stage, lane, wv, mlo, mhi, var_num);

    flat_dc_fix(dev, cur, stage, lane, wv, mlo);

    // Consume the prefetched rows HERE, before this batch's stores are issued:
    // the wait the compiler puts in front of this fence then covers loads issued
    // a whole compute phase ago and nothing younger.  Left to itself it waits at
    // the top of the next batch, where LLVM orders the youngest load against
    // younger loads only and emits vmcnt(0) -- which on gfx950 (one in-order
    // counter for loads and stores) also drains this batch's stores.
    asm volatile("" : "+v"(nxt[0]), "+v"(nxt[1]), "+v"(nxt[2]), "+v"(nxt[3]), "+v"(nxt[4]), "+v"(nxt[5]),
                 "+v"(nxt[6]), "+v"(nxt[7])::"memory");

    // A full round of entries from earlier batches drains HERE, before this
    // batch's stores are issued: vmcnt counts in issue order, so a drain after
    // them would wait for all 8 KiB of them before its first stash load returns.
    // The wave's LAST batch (DCTQ_LAST_INPLACE) drains every entry still queued
    // here -- behind the previous batch's long-issued stores, not behind its own
    // -- and resolves its own ties in the stage, so the wave ends with its last
    // stores: no final drain (vmcnt(0) behind 8 KiB of fresh stores, stash
    // loads, fp64, patches) in the kernel's tail.
    const bool last = DCTQ_LAST_INPLACE && g + step >= ps.first[ps.n];
    while (qn >= 64 || (last && qn > 0)) {
        if (DCTQ_ABLATE & 16) qn = 0;
        else drain_queue<ADAPTIVE, STATS>(ps, dev, qb, qc, ring, qn, lane, fallbacks);
    }

    if (!valid || (DCTQ_ABLATE & 8)) mlo = mhi = 0;
    const int nflag = __builtin_popcountll(__builtin_amdgcn_ballot_w64((mlo | mhi) != 0));
    if ((DCTQ_INSTAGE_LANES <= 64 && nflag >= DCTQ_INSTAGE_LANES) || (last && nflag > 0))
    {
        // tie-heavy batch: resolved in the stage before its stores (no stash, no patches)
        const uint32_t n = resolve_ties_compact<ADAPTIVE, DCTQ_V2_GROUP, DCTQ_V2_GROUP ? DCTQ_V2_WIDE : 0>(tab, cur, stage, qc + qn, lane, wv, mlo, mhi);
        if (STATS && n) atomicAdd(fallbacks, (unsigned long long)n);
    }

    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    {
        // Stores through a buffer descriptor whose num_records ends at the last
        // valid block: out-of-range lanes are dropped by the hardware, so the
        // stores are unconditional (predicated stores made the waitcnt pass give
        // up and wait vmcnt(0) at the loop latch).
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(out.base, (short)0, (int)(out.nb * 128u), 0x00020000);
        const uint2 *st64 = reinterpret_cast<const uint2 *>(stage) + wv * 64 * (kPitch2 / 8);
        // all 8 chunks into distinct registers first, one voffset register and
        // per-store soffsets: a store's VGPR operands must not be overwritten
        // while it is in flight (reuse would put vmcnt waits between the stores)
        u4v val[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int m = k * 64 + lane;
            const int bl = m >> 3;
            const uint2 lo = st64[bl * (kPitch2 / 8) + (m & 7) * 2], hi = st64[bl * (kPitch2 / 8) + (m & 7) * 2 + 1];
            val[k] = u4v{lo.x, lo.y, hi.x, hi.y};
        }
        if (DCTQ_ABLATE & 128) {  // diagnostic: consume the staged values, store nothing
#pragma unroll
            for (int k = 0; k < 8; ++k) asm volatile("" ::"v"(val[k]));
        } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) __builtin_amdgcn_raw_buffer_store_b128(val[k], rs, lane * 16, k * 1024, kStoreAux);
        }
        if (VAR) {
            const __amdgpu_buffer_rsrc_t rv =
                __builtin_amdgcn_make_buffer_rsrc(out.var, (short)0, (int)(out.nb * 4u), 0x00020000);
            __builtin_amdgcn_raw_buffer_store_b32(var_num, rv, lane * 4, 0, kStoreAux);
        }
    }

    // ---- defer flagged coefficients to the wave's queue (rare: ~1.5 per batch at q50)
    if (DCTQ_ABLATE & 32) asm volatile("" : "+v"(mlo), "+v"(mhi), "+s"(qn));  // keep code, never run (diagnostic)
    uint64_t has = __builtin_amdgcn_ballot_w64((DCTQ_ABLATE & 32) ? (mlo == 0x12345u && mhi == 0x6789u) : (mlo | mhi) != 0);
    const int16_t *mine16 = reinterpret_cast<const int16_t *>(stage) + (wv * 64 + lane) * (kPitch2 / 2);
    int sfirst = -1;  // ring slot holding this lane's pixels for this batch's entries
    while (has) {
        if (qn > kQCap - 64) {
            if (DCTQ_ABLATE & 16) qn = 0;
            else drain_queue<ADAPTIVE, STATS>(ps, dev, qb, qc, ring, qn, lane, fallbacks);
            sfirst = -1;  // the drained slots are reused from here on
        }
        if (mlo | mhi) {
            const int c = pop_flag(mlo, mhi);
            const uint32_t pos =
                qn + __builtin_amdgcn_mbcnt_hi((uint32_t)(has >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)has, 0u));
            const bool fresh = !DCTQ_STASH_DEDUP || sfirst < 0;
            const uint32_t s = fresh ? pos : (uint32_t)sfirst;
            qb[pos] = n;
            // entry: coefficient | plane << 6 | parity of the stored fast value << 8 | stash slot << 9
            qc[pos] = (uint16_t)((uint32_t)c | ((uint32_t)k << 6) | (((uint32_t)mine16[c] & 1u) << 8) | (s << 9));
            // stash the block's pixels while they are still in registers: the
            // drain must not go back to HBM for them (8 random 64-B bursts per entry)
            if (fresh) {
                uint4 *st = ring + pos * 4;
                sfirst = (int)pos;
                if (!(DCTQ_ABLATE & 1024))
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        st[k] = make_uint4(cur[2 * k].x, cur[2 * k].y, cur[2 * k + 1].x, cur[2 * k + 1].y);
            }
        }
        qn += __builtin_popcountll(has);
        has = __builtin_amdgcn_ballot_w64((mlo | mhi) != 0);
    }
}

// Waves per workgroup of the stream kernels (v2, v3, movement).  Every wave is
// independent (own stage slice, queue, stash slot); only the 1 KiB exact-table
// copy is shared per workgroup.

template <bool ADAPTIVE, bool VAR, bool STATS>
__global__ __launch_bounds__(kFThreads, 4) void fdct8_quant_v2(PlaneSet ps, FastTables t,
                                                              const DevTables *__restrict__ dev,
                                                              unsigned long long *fallbacks, uint4 *ring_all) {
    __shared__ uint4 stage[kFThreads * kPitch2 / 16];
    __shared__ uint32_t qblk[kFWaves * kQCap];
    __shared__ uint16_t qcoef[kFWaves * kQCap];
    __shared__ ExactTables tab;  // the in-stage resolution's D and Q (1 KiB; 4 workgroups still fit a CU)
    load_exact_tables(&tab, dev);
    // readfirstlane: the wave index is uniform, so batch pointers and buffer
    // descriptors live in SGPRs (no waterfall loops around the stores)
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t nbatch = ps.first[ps.n];
    const uint32_t step = gridDim.x * kFWaves;
    uint32_t *qb = qblk + wv * kQCap;
    uint16_t *qc = qcoef + wv * kQCap;
    uint4 *ring = ring_all + (size_t)(blockIdx.x * kFWaves + wv) * kQCap * 4;  // 64 B per queue slot
    int qn = 0;
    uint32_t g = blockIdx.x * kFWaves + wv;
    uint2 nxt[8];
    {
        const int k0 = plane_of(ps, g);
        load_rows(ps.pl[k0], (g - first_of(ps, k0)) * 64 + lane, nxt);
    }
    // same fence as at the end of a batch: the loop header then sees no load in
    // flight on either incoming edge and needs no wait at all
    asm volatile("" : "+v"(nxt[0]), "+v"(nxt[1]), "+v"(nxt[2]), "+v"(nxt[3]), "+v"(nxt[4]), "+v"(nxt[5]),
                 "+v"(nxt[6]), "+v"(nxt[7])::"memory");
    for (; g < nbatch; g += step)
        fdct8_batch<ADAPTIVE, VAR, STATS>(ps, dev, &tab, fallbacks, stage, qb, qc, ring, qn, nxt, g, step, lane, wv);
    if (DCTQ_ABLATE & 16) qn = 0;
    if (DCTQ_ABLATE & 2048) qn = 0;  // diagnostic: skip the final drain
    while (qn > 0) drain_queue<ADAPTIVE, STATS>(ps, dev, qb, qc, ring, qn, lane, fallbacks);
}


#define DCTQ_SELECT(KERN, A, V, S, ...)                                          \
    do {                                                                         \
        if (A) {                                                                 \
            if (V) { if (S) KERN<true, true, true> __VA_ARGS__; else KERN<true, true, false> __VA_ARGS__; } \
            else { if (S) KERN<true, false, true> __VA_ARGS__; else KERN<true, false, false> __VA_ARGS__; } \
        } else {                                                                 \
            if (V) { if (S) KERN<false, true, true> __VA_ARGS__; else KERN<false, true, false> __VA_ARGS__; } \
            else { if (S) KERN<false, false, true> __VA_ARGS__; else KERN<false, false, false> __VA_ARGS__; } \
        }                                                                        \
    } while (0)

template <bool A, bool V, bool S>
static hipError_t launch_v1(const PlaneSet &ps, const FastTables &t, const DevTables *dev, unsigned long long *fb,
                            hipStream_t stream) {
    for (int k = 0; k < ps.n; ++k)
        hipLaunchKernelGGL((fdct8_quant_v1<A, V, S>), dim3((ps.pl[k].nblk + kThreads - 1) / kThreads), dim3(kThreads),
                           0, stream, ps.pl[k], t, dev, ps.coef[k], ps.var[k], fb);
    return hipGetLastError();
}

template <bool A, bool V, bool S>
static hipError_t launch_v2(const PlaneSet &ps, const FastTables &t, const DevTables *dev, unsigned long long *fb,
                            hipStream_t stream, int num_cus, const RingSource &rs) {
    static const int per_cu = resident_per_cu(fdct8_quant_v2<A, V, S>, kFThreads);
    const uint32_t nbatch = ps.first[ps.n];
    const uint32_t want = (nbatch + kFWaves - 1) / kFWaves;
    const uint32_t cap = (uint32_t)(num_cus * per_cu * kV2GridMult);
    const uint32_t grid = want < cap ? want : cap;
    // the stash is sized to THIS grid (every workgroup owns its waves' slots) and
    // handed out by the caller per (device, stream): launches on one stream are
    // ordered, so they share it (api.hip stash_for)
    void *ring = rs.get(rs.ctx, fdct8_ring_bytes((int)grid));
    if (!ring) return hipErrorOutOfMemory;
    hipLaunchKernelGGL((fdct8_quant_v2<A, V, S>), dim3(grid), dim3(kFThreads), 0, stream, ps, t, dev, fb, (uint4 *)ring);
    return hipGetLastError();
}

size_t fdct8_ring_bytes(int workgroups) { return (size_t)workgroups * kFWaves * kQCap * 64; }


// The forward kernel (1, 2 or 3 = fdct8_quant_v1 / v2 / v3) a plan of `variant` runs:
// 1 -> v1, 4 -> v2 (the queue kernel at any size), anything else -> v3, the product's
// kernel for every plan and size (fdct8.hip).
int forward_kernel_for(int variant, uint32_t nbatch, int num_cus, bool tie_heavy) {
    (void)nbatch, (void)num_cus, (void)tie_heavy;
    return variant == 1 ? 1 : variant == 4 ? 2 : 3;
}

// ============================================================================
// Diagnostics: the forward kernels' data movement with no arithmetic (the
// memory ceiling of their exact access patterns, measured on the same box as
// the kernel -- bench.py reports kernel time / movement time).  Same grid,
// occupancy (LDS footprint), prefetch, LDS stage, fence and 1 KiB
// non-temporal stores as the kernel; the "coefficients" are the pixel rows
// twice over.
//  fdct8_movement     -- fdct8_quant_v3, the product kernel: its LDS (stage, 1 KiB
//                        exact tables loaded at start, 512 B of entries), its
//                        prefetch (nothing past the end), its 32 b32 stage writes
//                        per lane and its stage read-back;
//  fdct8_movement_v2  -- fdct8_quant_v2 (the tie-heavy plans' queue kernel): its
//                        queue arrays and first-batch load_rows.
#ifndef DCTQ_MV3_TAB
#define DCTQ_MV3_TAB 1  // A/B: the workgroup-start table copy of fdct8_quant_v3
#endif
#ifndef DCTQ_MV3_SLEEP
#define DCTQ_MV3_SLEEP 0  // A/B: s_sleep between the stage writes and the prefetch wait (64 clk units)
#endif
#ifndef DCTQ_MV3_B64
#define DCTQ_MV3_B64 0  // A/B: b64 stage writes instead of fdct8_compute's 32 b32
#endif
__global__ __launch_bounds__(kFThreads, 4) void fdct8_movement(PlaneSet ps, const DevTables *__restrict__ dev) {
    __shared__ uint4 stage[kFThreads * kPitch2 / 16];
    __shared__ ExactTables tab;
    __shared__ uint16_t scr[kFWaves * 64];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (DCTQ_MV3_TAB) load_exact_tables(&tab, dev);
    if (ps.n < 0) scr[threadIdx.x] = (uint16_t)tab.dct[lane];  // keep the footprint allocated
    const uint32_t nbatch = ps.first[ps.n];
    const uint32_t step = gridDim.x * kFWaves;
    uint32_t g = blockIdx.x * kFWaves + wv;
    uint2 nxt[8];
    prefetch_batch(ps, g, lane, nxt);
    asm volatile("" : "+v"(nxt[0]), "+v"(nxt[1]), "+v"(nxt[2]), "+v"(nxt[3]), "+v"(nxt[4]), "+v"(nxt[5]),
                 "+v"(nxt[6]), "+v"(nxt[7])::"memory");
    for (; g < nbatch; g += step) {
        const int k = plane_of(ps, g);
        const uint32_t b = g - first_of(ps, k);
        uint2 cur[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) cur[r] = nxt[r];
        prefetch_batch(ps, g + step, lane, nxt);
        const BatchOut out = batch_out(ps, k, b);
        // fdct8_compute's stage writes: dword i*4 + cp of the lane's 136-B slot
        uint32_t *st32 = reinterpret_cast<uint32_t *>(stage) + (wv * 64 + lane) * (kPitch2 / 4);
        if (DCTQ_MV3_B64) {  // A/B: 16 b64 writes (fdct8_movement_v2's)
            uint2 *mine = reinterpret_cast<uint2 *>(st32);
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                mine[2 * r] = cur[r];
                mine[2 * r + 1] = make_uint2(cur[r].y, cur[r].x);
            }
        } else {
#pragma unroll
            for (int cp = 0; cp < 4; ++cp)
#pragma unroll
                for (int i = 0; i < 8; ++i) st32[i * 4 + cp] = cp & 1 ? cur[i].y : cur[i].x ^ (uint32_t)cp;
        }
        if (DCTQ_MV3_SLEEP) __builtin_amdgcn_s_sleep(DCTQ_MV3_SLEEP);  // A/B: the arithmetic's latency slack
        asm volatile("" : "+v"(nxt[0]), "+v"(nxt[1]), "+v"(nxt[2]), "+v"(nxt[3]), "+v"(nxt[4]), "+v"(nxt[5]),
                     "+v"(nxt[6]), "+v"(nxt[7])::"memory");
        wave_sync();
        u4v val[8];
        stage_chunks(stage, wv, lane, val);
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(out.base, (short)0, (int)(out.nb * 128u), 0x00020000);
#pragma unroll
        for (int c = 0; c < 8; ++c) __builtin_amdgcn_raw_buffer_store_b128(val[c], rs, lane * 16, c * 1024, kStoreAux);
    }
}

__global__ __launch_bounds__(kFThreads, 4) void fdct8_movement_v2(PlaneSet ps) {
    __shared__ uint4 stage[kFThreads * kPitch2 / 16];
    __shared__ uint32_t qpad[kFWaves * kQCap];   // same LDS footprint as fdct8_quant_v2
    __shared__ uint16_t qpad2[kFWaves * kQCap];  // (occupancy is LDS-bound)
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (ps.n < 0) { qpad[threadIdx.x] = 0; qpad2[threadIdx.x] = 0; }  // keep the padding allocated
    const uint32_t nbatch = ps.first[ps.n];
    const uint32_t step = gridDim.x * kFWaves;
    uint32_t g = blockIdx.x * kFWaves + wv;
    uint2 nxt[8];
    {
        const int k0 = plane_of(ps, g);
        load_rows(ps.pl[k0], (g - first_of(ps, k0)) * 64 + lane, nxt);
    }
    asm volatile("" : "+v"(nxt[0]), "+v"(nxt[1]), "+v"(nxt[2]), "+v"(nxt[3]), "+v"(nxt[4]), "+v"(nxt[5]),
                 "+v"(nxt[6]), "+v"(nxt[7])::"memory");
    for (; g < nbatch; g += step) {
        const int k = plane_of(ps, g);
        const PlaneArgs &p = ps.pl[k];
        const uint32_t b = g - first_of(ps, k);
        uint2 cur[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) cur[r] = nxt[r];
        prefetch_batch(ps, g + step, lane, nxt);
        uint2 *mine = reinterpret_cast<uint2 *>(reinterpret_cast<char *>(stage) + (wv * 64 + lane) * kPitch2);
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            mine[2 * r] = cur[r];
            mine[2 * r + 1] = make_uint2(cur[r].y, cur[r].x);
        }
        asm volatile("" : "+v"(nxt[0]), "+v"(nxt[1]), "+v"(nxt[2]), "+v"(nxt[3]), "+v"(nxt[4]), "+v"(nxt[5]),
                     "+v"(nxt[6]), "+v"(nxt[7])::"memory");
        wave_sync();
        const uint32_t left = (uint32_t)p.nblk - b * 64;
        const uint32_t nb = left < 64u ? left : 64u;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            reinterpret_cast<char *>(coef_of(ps, k)) + (size_t)b * 64 * 128, (short)0, (int)(nb * 128u), 0x00020000);
        u4v val[8];
        stage_chunks(stage, wv, lane, val);
#pragma unroll
        for (int q = 0; q < 8; ++q) __builtin_amdgcn_raw_buffer_store_b128(val[q], rs, lane * 16, q * 1024, kStoreAux);
    }
}

hipError_t launch_fdct8_movement(const PlaneSet &ps, const DevTables *dev, hipStream_t stream, int num_cus, int shape,
                                 int grid_mult) {
    const uint32_t nbatch = ps.first[ps.n];
    const uint32_t want = (nbatch + kFWaves - 1) / kFWaves;
    if (shape == 2) {
        static const int per_cu = resident_per_cu(fdct8_movement_v2, kFThreads);
        const uint32_t cap = (uint32_t)(num_cus * per_cu * kV2GridMult);  // the same grid as launch_v2
        hipLaunchKernelGGL(fdct8_movement_v2, dim3(want < cap ? want : cap), dim3(kFThreads), 0, stream, ps);
    } else {
        static const int per_cu = resident_per_cu(fdct8_movement, kFThreads);
        const uint32_t cap = (uint32_t)(num_cus * per_cu * (grid_mult > 0 ? grid_mult : kV3GridMult));  // launch_v3's
        hipLaunchKernelGGL(fdct8_movement, dim3(want < cap ? want : cap), dim3(kFThreads), 0, stream, ps, dev);
    }
    return hipGetLastError();
}

// ============================================================================
// Lane-per-block fp64 kernels (variant 1 of dctq_forward_float / dctq_inverse):
//   * fdct8_float_kernel: forward DCT to float coefficients (dct_forward,
//     src/dct.c:52-77, without quantization), fp64 butterfly, one fp32 rounding.
//   * idct8_kernel: dequantize (src/quantization.c:133-151, incl. the
//     non-adaptive 1/Q multiplier) + dct_inverse (src/dct.c:80-105) + 128.
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


// ============================================================================
// Diagnostic: roundtrip8's data movement with no arithmetic (bench.py
// round_trip.movement_ceiling).  Same grid, occupancy bound, LDS footprint,
// prefetch, stage writes, LDS read-backs, stores and vmcnt(0) points as
// roundtrip8 (the product's fp32 and fp64 instantiations share them): per batch
// the pixel rows go into the stage as the "coefficients" (8 x 1 KiB stores), then
// twice 32 blocks of 256 B "recon" (the rows repeated) through the paired-inverse
// stage layout (8 x 1 KiB each), each half written to the stage, retired, stored.
// Round 5 (profiles/r05/rt_ab.log): this twin, one without any wait, ones
// with s_sleep where the arithmetic sits and ones writing product-like bytes all
// run 1.5-2 % SLOWER than the product on the same box -- the product's stores
// leave spaced by its compute phases, which this write-heavy mix takes better --
// so it is reported beside the flat 1:2:4 stream, not as a ceiling.
__global__ __launch_bounds__(kThreads, kRtOcc) void roundtrip_movement(RoundTripSet rt) {
    __shared__ uint4 stage[kThreads * kPitch2 / 16];
    __shared__ ExactTables tabpad;          // same LDS footprint as roundtrip8
    __shared__ uint16_t scrpad[kWaves * 64];
    const PlaneSet &ps = rt.ps;
    if (ps.n < 0) {  // keep the padding allocated
        scrpad[threadIdx.x] = 0;
        reinterpret_cast<volatile uint32_t *>(&tabpad)[threadIdx.x] = 0;
    }
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5, j = lane & 31;
    const uint32_t nbatch = ps.first[ps.n];
    const uint32_t step = gridDim.x * kWaves;
    uint32_t g = blockIdx.x * kWaves + wv;
    uint2 nxt[8];
    prefetch_batch(ps, g, lane, nxt);
    asm volatile("" : "+v"(nxt[0]), "+v"(nxt[1]), "+v"(nxt[2]), "+v"(nxt[3]), "+v"(nxt[4]), "+v"(nxt[5]),
                 "+v"(nxt[6]), "+v"(nxt[7])::"memory");
    char *wstage = reinterpret_cast<char *>(stage) + wv * 64 * kPitch2;
    for (; g < nbatch; g += step) {
        const int k = plane_of(ps, g);
        const uint32_t b = g - first_of(ps, k);
        uint2 cur[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) cur[r] = nxt[r];
        prefetch_batch<false>(ps, g + step, lane, nxt);
        const BatchOut out = batch_out(ps, k, b);
        char *recon = reinterpret_cast<char *>(rt.recon[k]) + (size_t)b * 64 * 256;
        asm volatile("" : "+s"(recon));
        uint2 *mine2 = reinterpret_cast<uint2 *>(wstage + lane * kPitch2);
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            mine2[2 * r] = cur[r];
            mine2[2 * r + 1] = make_uint2(cur[r].y, cur[r].x);
        }
        retire_stores();  // roundtrip8: after its forward, before the tie pass's LDS reads
        wave_sync();
        const uint32_t nb = out.nb;
        u4v val[8];
        stage_chunks(stage, wv, lane, val);
        {
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc(out.base, (short)0, (int)(nb * 128u), 0x00020000);
#pragma unroll
            for (int c = 0; c < 8; ++c) __builtin_amdgcn_raw_buffer_store_b128(val[c], rs, lane * 16, c * 1024, kNtAux);
        }
        char *mine = wstage + j * kPitchP + h * 128;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
#pragma unroll
            for (int r = 0; r < 8; ++r)
                *reinterpret_cast<uint4 *>(mine + r * 16) =
                    make_uint4(cur[r].x, cur[r].y, cur[r].x ^ (uint32_t)half, cur[r].y ^ (uint32_t)lane);
            retire_stores();  // roundtrip8: after each inverse half, before its read-back
            wave_sync();
            const uint32_t n32 = half ? (nb > 32u ? nb - 32u : 0u) : (nb < 32u ? nb : 32u);
            store_stage(stage, wv, lane, recon + half * 32 * 256, n32 * 256u);
        }
    }
}

hipError_t launch_roundtrip_movement(const RoundTripSet &rt, hipStream_t stream, int num_cus) {
    static const int per_cu = resident_per_cu(roundtrip_movement, kThreads);
    const uint32_t nbatch = rt.ps.first[rt.ps.n];
    const uint32_t want = (nbatch + kWaves - 1) / kWaves;
    const uint32_t cap = (uint32_t)(num_cus * per_cu * kRtGridMult);  // the same grid as launch_rt
    hipLaunchKernelGGL(roundtrip_movement, dim3(want < cap ? want : cap), dim3(kThreads), 0, stream, rt);
    return hipGetLastError();
}



}  // namespace dctq

// The v2 forward's tie-path pixel stash (above: 8 KiB per wave of the
// launched grid).  One per (device, stream), allocated on the first launch that
// needs it and grown to the largest grid launched there: launches on one stream
// run in order, so every plan used on that stream shares it, and a plan costs
// no stash at all until it runs a multi-batch-per-wave forward.  The mutex is
// held from the lookup to the kernel launch (stash_guard), so a grow -- which
// waits for the stream before freeing the smaller stash -- never frees memory a
// launch enqueued by another thread is about to use.
//  * The special handles name a different real stream per thread
//    (hipStreamPerThread always; the null stream under per-thread default-stream
//    semantics, which a caller may have compiled with): they are keyed by the
//    calling thread too, so two threads never share a stash through them.
//  * A launch captured into a graph gets a stash of its OWN, never shared with
//    direct launches or other captures and never freed by a grow: a replay may
//    run at any later time, on any stream.  It is allocated in relaxed capture
//    mode (no stream work) and released by dctq_diag_stream_release (destroying
//    the graph does not free it: a stream that re-captures keeps adding stashes
//    until it is released, and the per-thread entries of exited threads stay).
namespace {
struct Stash {
    void *ptr = nullptr;
    size_t bytes = 0;
};
struct StreamStash {
    Stash live;                   // direct launches on this stream
    std::vector<void *> captured;  // one per captured launch, kept until dctq_diag_stream_release
};
struct StashKey {
    int device;
    hipStream_t stream;
    std::thread::id thread;  // default-constructed (no thread) for ordinary streams
    bool operator<(const StashKey &o) const {
        if (device != o.device) return device < o.device;
        if (stream != o.stream) return std::less<hipStream_t>()(stream, o.stream);
        return thread < o.thread;
    }
};
std::mutex g_stash_mu;
std::map<StashKey, StreamStash> g_stash;
struct StashCtx {
    int device;
    hipStream_t stream;
    hipError_t err;
};

StashKey stash_key(int device, hipStream_t stream) {
    const bool per_thread = stream == nullptr || stream == hipStreamPerThread;
    return StashKey{device, stream, per_thread ? std::this_thread::get_id() : std::thread::id()};
}

void *stash_for(void *vctx, size_t bytes) {  // called with g_stash_mu held
    StashCtx &c = *static_cast<StashCtx *>(vctx);
    StreamStash &s = g_stash[stash_key(c.device, c.stream)];
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(c.stream, &cap) == hipSuccess && cap != hipStreamCaptureStatusNone) {
        hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
        (void)hipThreadExchangeStreamCaptureMode(&mode);
        void *p = nullptr;
        c.err = hipMalloc(&p, bytes);
        (void)hipThreadExchangeStreamCaptureMode(&mode);  // restore the caller's mode
        if (c.err != hipSuccess) return nullptr;
        s.captured.push_back(p);
        return p;
    }
    if (s.live.bytes >= bytes) return s.live.ptr;
    if (s.live.ptr) {
        if ((c.err = hipStreamSynchronize(c.stream)) != hipSuccess) return nullptr;
        (void)hipFree(s.live.ptr);
        s.live = Stash{};
    }
    if ((c.err = hipMalloc(&s.live.ptr, bytes)) != hipSuccess) {
        s.live = Stash{};
        return nullptr;
    }
    s.live.bytes = bytes;
    return s.live.ptr;
}
}  // namespace

extern "C" {

int dctq_diag_stream_release(void *stream) {
    DCTQ_ENTRY;
    int dev = -1;
    HIPCHK(hipGetDevice(&dev), "hipGetDevice");
    // a synchronize inside a capture would invalidate the caller's graph
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    HIPCHK(hipStreamIsCapturing((hipStream_t)stream, &cap), "hipStreamIsCapturing");
    if (cap != hipStreamCaptureStatusNone) return dctq::fail(DCTQ_EINVAL, "stream is being captured");
    StreamStash st;
    {  // take the entry out under the lock; wait and free outside it, so other threads' launches never wait on this
        std::lock_guard<std::mutex> stash_guard(g_stash_mu);
        auto it = g_stash.find(stash_key(dev, (hipStream_t)stream));
        if (it == g_stash.end()) return DCTQ_OK;
        st = std::move(it->second);
        g_stash.erase(it);
    }
    const hipError_t e = hipStreamSynchronize((hipStream_t)stream);
    (void)hipFree(st.live.ptr);
    for (void *p : st.captured) (void)hipFree(p);
    HIPCHK(e, "hipStreamSynchronize");
    return DCTQ_OK;
}

long long dctq_diag_stream_stash_bytes(void *stream) {
    DCTQ_ENTRY;
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    std::lock_guard<std::mutex> stash_guard(g_stash_mu);
    auto it = g_stash.find(stash_key(dev, (hipStream_t)stream));
    if (it == g_stash.end()) return 0;
    return (long long)it->second.live.bytes;
}

}  // extern "C"

namespace {
// The variant-1/4 forward of a diagnostic plan (dctq_forward_quant_planes).
int diag_forward_quant(const dctq_plan *plan, const dctq::PlaneSet &ps, hipStream_t stream) {
    DCTQ_ENTRY;  // the v2 path may hipMalloc its stash: isolated like every allocating entry point
    StashCtx sc{plan->device, stream, hipSuccess};
    hipError_t e;
    {
        const bool a = plan->adaptive != 0, v = ps.var[0] != nullptr, s = plan->fallbacks != nullptr;
        std::lock_guard<std::mutex> stash_guard(g_stash_mu);
        if (plan->variant == 1) {
            DCTQ_SELECT(e = dctq::launch_v1, a, v, s, (ps, plan->fast, plan->dev, plan->fallbacks, stream));
        } else {
            DCTQ_SELECT(e = dctq::launch_v2, a, v, s, (ps, plan->fast, plan->dev, plan->fallbacks, stream,
                                                       plan->num_cus, dctq::RingSource{stash_for, &sc}));
        }
    }
    if (sc.err != hipSuccess) return dctq::fail(DCTQ_ENOMEM, "tie-path stash", sc.err);
    HIPCHK(e, "fdct8_quant variant launch");
    return DCTQ_OK;
}

}  // namespace

extern "C" {

// The diagnostic library's own forward / float / inverse entry points: a plan's
// forced variant (dctq_diag_plan_set_variant) picks the retired kernel here, any
// other plan runs the product entry point.  The product entry points never look at
// the variant.
int dctq_diag_forward_quant_planes(const dctq_plan *plan, const dctq_plane *planes, int nplanes, int16_t *const *coef,
                                   int32_t *const *var_num, void *stream) {
    if (!plan || (plan->variant != 1 && plan->variant != 4))
        return dctq_forward_quant_planes(plan, planes, nplanes, coef, var_num, stream);
    if (int rc = dctq::check_plan(plan)) return rc;
    dctq::PlaneSet ps;
    if (int rc = dctq::plane_set(planes, nplanes, coef, var_num, &ps)) return rc;
    return diag_forward_quant(plan, ps, (hipStream_t)stream);
}

int dctq_diag_forward_float(const dctq_plan *plan, const dctq_plane *src, float *coef, void *stream) {
    if (!plan || plan->variant != 1) return dctq_forward_float(plan, src, coef, stream);
    DCTQ_LAUNCH(stream, 3);
    if (int rc = dctq::check_plan(plan)) return rc;
    if (!coef || ((uintptr_t)coef) % 16) return dctq::fail(DCTQ_EINVAL, "coef NULL or not 16-byte aligned");
    dctq::PlaneArgs a;
    if (int rc = dctq::plane_args(src, &a)) return rc;
    HIPCHK(dctq::launch_fdct8_float(a, plan->dev, coef, (hipStream_t)stream), "fdct8_float launch");
    return DCTQ_OK;
}

int dctq_diag_inverse(const dctq_plan *plan, const int16_t *coef, const int32_t *var_num, long long nblocks,
                      float *recon, void *stream) {
    if (!plan || plan->variant != 1) return dctq_inverse(plan, coef, var_num, nblocks, recon, stream);
    DCTQ_LAUNCH(stream, 4);
    if (int rc = dctq::check_plan(plan)) return rc;
    if (!coef || !recon) return dctq::fail(DCTQ_EINVAL, "coef/recon is NULL");
    if (plan->adaptive && !var_num) return dctq::fail(DCTQ_EINVAL, "adaptive inverse needs var_num");
    if (nblocks < 0 || nblocks >= (1ll << 40)) return dctq::fail(DCTQ_EINVAL, "bad nblocks");
    if (((uintptr_t)coef) % 16 || ((uintptr_t)recon) % 16)
        return dctq::fail(DCTQ_EINVAL, "coef/recon must be 16-byte aligned");
    if (nblocks == 0) return DCTQ_OK;
    HIPCHK(dctq::launch_idct8(plan->dev, plan->adaptive, coef, var_num, nblocks, recon, (hipStream_t)stream),
           "idct8 launch");
    return DCTQ_OK;
}

}  // extern "C"
