// dct_amd/csrc/roundtrip.hip -- the fused round trip (BASELINE configs[4],
// SURVEY 8(f) rank 1): for every block of up to 4 planes, in ONE launch,
//   coef  = quantize(dct_forward(px - 128))                 (bit-exact, as dctq_forward_quant)
//   recon = dct_inverse(dequantize(coef)) + 128              (fp32, |err| <= 1e-4, as dctq_inverse)
// i.e. the reference's per-block pipeline tests/test_entropy.c:300-330
// (create_block_from_pixels, dct_forward, calculate_block_variance, quantize,
// dequantize, dct_inverse) with the quantized ints handed to the inverse in LDS
// instead of through HBM: 64 B in, 128 + 256 B out per block (448 B) against
// 584 B for the two kernels back to back (coef and var_num written and re-read).
//
// One wave, one 64-block batch, three phases over the same 8.5 KiB LDS stage:
//  1. forward, lane per block (fdct8_core.h): fp32 AAN, quantization into the
//     stage, tie flags.  Flagged coefficients are recomputed in the reference's
//     exact fp64 order right here, by the lane that owns the block (its pixels
//     are still in registers), and patched into the stage -- the inverse must see
//     the final ints, so there is no deferral queue as in the forward kernel;
//  2. the stage is read back for the 1 KiB coefficient stores AND, per lane, the
//     two half blocks the paired inverse needs (lane (h, j): rows 4h..4h+3 of
//     blocks j and 32 + j); var_num follows by one v_permlane32_swap;
//  3. two paired-lane fp64 inverses (pair_core.h, as idct8_pair), 32 blocks
//     each, staged as fp32 rows and written as 1 KiB stores.
// Store-data hazard: every LDS read-back that lands in VGPRs comes
// after a wait that retires the wave's pending stores -- the prefetch fence for
// phase 2, an explicit vmcnt(0) before each recon read-back.
#include "fdct8_core.h"
#include "pair_core.h"

#ifndef DCTQ_RT_GRID_MULT
#define DCTQ_RT_GRID_MULT DCTQ_GRID_MULT  // grid multiplier of this file's streaming kernels (dctq_internal.h)
#endif

namespace dctq {

#ifndef DCTQ_RT_EARLY_PREFETCH
#define DCTQ_RT_EARLY_PREFETCH 1  // next batch's rows requested at the top of the batch (0: after inverse A)
#endif
#ifndef DCTQ_RT_OCC
#define DCTQ_RT_OCC 4  // waves per SIMD (launch bound)
#endif
#ifndef DCTQ_RT_GROUP8
#define DCTQ_RT_GROUP8 1  // passes of <= 8 entries run 8 lanes per entry (exact_grouped<8>): -4.9 % on the bench step
#endif
#ifndef DCTQ_RT_WIDE
#define DCTQ_RT_WIDE 0  // resolve_ties_compact WIDE: at this kernel's 128-VGPR bound the wide rounds spill (A/B knob)
#endif

static_assert(kThreads == kThreadsP && 64 * kPitch2 == 32 * kPitchP, "forward and inverse share the wave's stage");

// Dequantize + inverse DCT + 128 of one 32-block sub-batch, lane (h, j) holding
// rows 4h..4h+3 of block j (8 int16 per uint4) and the block's var_num; fp32
// rows into the wave's stage (layout of idct8_pair).
template <bool ADAPTIVE>
__device__ __forceinline__ void inverse_half(const DevTables *__restrict__ dev, const uint4 (&q)[4], int32_t vn,
                                             int h, char *mine) {
    double v[4][8];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint32_t w[4] = {q[r].x, q[r].y, q[r].z, q[r].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            v[r][2 * k] = (double)(int)(int16_t)(w[k] & 0xFFFFu);
            v[r][2 * k + 1] = (double)((int)w[k] >> 16);
        }
    }
    //   non-adaptive: q * (1/Q) S_u S_c      (src/quantization.c:139,144)
    //   adaptive:     q * Q S_u S_c * (2-nv), DC: q * Q S_0 S_0 (:137,144,193)
    ConstTables *tp = tables(dev);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        ConstDouble *tlo = ADAPTIVE ? &tp->qscale[8 * r] : &tp->iscale[8 * r];
        ConstDouble *thi = ADAPTIVE ? &tp->qscale[8 * (r + 4)] : &tp->iscale[8 * (r + 4)];
        half_wave_scale(v[r], tlo, thi);
    }
    if (ADAPTIVE) {
        const double var = (double)vn / 4096.0;
        const double sc = 2.0 - fmin(1.0, fmax(0.1, var / 1000.0));
        const double dc = v[0][0];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 8; ++c) v[r][c] *= sc;
        if (h == 0) v[0][0] = dc;  // the DC keeps Q (src/quantization.c:198-199)
    }
    // + 128 on every output pixel = + 128 on the scaled DC (row 0 of the AAN
    // transpose graph is all ones and S_0^2 = 1/8 is already applied)
    if (h == 0) v[0][0] += 128.0;
    transpose_halves(v);
#pragma unroll
    for (int k = 0; k < 4; ++k)
        aan8t_d(v[0][k], v[1][k], v[2][k], v[3][k], v[0][k + 4], v[1][k + 4], v[2][k + 4], v[3][k + 4]);
    transpose_halves(v);
#pragma unroll
    for (int r = 0; r < 4; ++r) aan8t_d(v[r][0], v[r][1], v[r][2], v[r][3], v[r][4], v[r][5], v[r][6], v[r][7]);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        *reinterpret_cast<float4 *>(mine + r * 32) = make_float4(
            (float)v[r][0], (float)v[r][1], (float)v[r][2], (float)v[r][3]);
        *reinterpret_cast<float4 *>(mine + r * 32 + 16) = make_float4(
            (float)v[r][4], (float)v[r][5], (float)v[r][6], (float)v[r][7]);
    }
}

template <bool ADAPTIVE, bool VAR, bool STATS>
__global__ __launch_bounds__(kThreads, DCTQ_RT_OCC) void roundtrip8(RoundTripSet rt, const DevTables *__restrict__ dev,
                                                          unsigned long long *fallbacks) {
    __shared__ uint4 stage[kThreads * kPitch2 / 16];
    __shared__ ExactTables tab;
    __shared__ uint16_t scr[kWaves * 64];  // resolve_ties_compact's entries
    load_exact_tables(&tab, dev);
    const PlaneSet &ps = rt.ps;
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5, j = lane & 31;
    const uint32_t nbatch = ps.first[ps.n];
    const uint32_t step = gridDim.x * kWaves;
    uint32_t g = blockIdx.x * kWaves + wv;
    uint2 nxt[8];
    prefetch_batch(ps, g, lane, nxt);
    asm volatile("" : "+v"(nxt[0]), "+v"(nxt[1]), "+v"(nxt[2]), "+v"(nxt[3]), "+v"(nxt[4]), "+v"(nxt[5]),
                 "+v"(nxt[6]), "+v"(nxt[7])::"memory");
    uint32_t exact_count = 0;
    char *wstage = reinterpret_cast<char *>(stage) + wv * 64 * kPitch2;
    for (; g < nbatch; g += step) {
        const int k = plane_of(ps, g);
        const PlaneArgs &p = ps.pl[k];
        const uint32_t b = g - first_of(ps, k);
        uint2 cur[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) cur[r] = nxt[r];
        const bool valid = b * 64 + lane < (uint32_t)p.nblk;
        if (DCTQ_RT_EARLY_PREFETCH) prefetch_batch<false>(ps, g + step, lane, nxt);
        const BatchOut out = batch_out(ps, k, b);  // resolved before the fences (fdct8_core.h)
        char *recon = reinterpret_cast<char *>(rt.recon[k]) + (size_t)b * 64 * 256;
        if (DCTQ_PIN_OUT) asm volatile("" : "+s"(recon));

        // ---- 1. forward into the stage; ties resolved in place
        int32_t var_num;
        uint32_t mlo, mhi;
        forward_flags_batch<ADAPTIVE, VAR>(dev, cur, stage, lane, wv, valid, var_num, mlo, mhi);
        retire_stores();  // the previous batch's recon stores (long issued) before any LDS read
        const uint32_t ne =
            resolve_ties_compact<ADAPTIVE, DCTQ_RT_GROUP8, DCTQ_RT_WIDE>(&tab, cur, stage, scr + wv * 64, lane, wv, mlo, mhi);
        if (STATS) exact_count += ne;
        wave_sync();

        // ---- 2. read-back: coefficient chunks + the inverse's half blocks
        const uint32_t nb = out.nb;
        u4v val[8];
        stage_chunks(stage, wv, lane, val);
        const uint2 *st64 = reinterpret_cast<const uint2 *>(wstage);
        uint4 qa[4], qb[4];
        {
            const uint2 *sa = st64 + j * (kPitch2 / 8) + h * 8;  // block j, rows 4h..4h+3 (64 B)
            const uint2 *sb = sa + 32 * (kPitch2 / 8);            // block 32 + j
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint2 a0 = sa[2 * r], a1 = sa[2 * r + 1], b0 = sb[2 * r], b1 = sb[2 * r + 1];
                qa[r] = make_uint4(a0.x, a0.y, a1.x, a1.y);
                qb[r] = make_uint4(b0.x, b0.y, b1.x, b1.y);
            }
        }
        // lanes j / 32+j: var of block j in x, of block 32+j in y
        const auto vv = __builtin_amdgcn_permlane32_swap((uint32_t)var_num, (uint32_t)var_num, false, false);
        {
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc(out.base, (short)0, (int)(nb * 128u), 0x00020000);
#pragma unroll
            for (int c = 0; c < 8; ++c) __builtin_amdgcn_raw_buffer_store_b128(val[c], rs, lane * 16, c * 1024, DCTQ_NT_AUX);
            if (VAR) {
                const __amdgpu_buffer_rsrc_t rv =
                    __builtin_amdgcn_make_buffer_rsrc(out.var, (short)0, (int)(nb * 4u), 0x00020000);
                __builtin_amdgcn_raw_buffer_store_b32(var_num, rv, lane * 4, 0, DCTQ_NT_AUX);
            }
        }

        // ---- 3. paired fp64 inverses, blocks 0-31 then 32-63 of the batch
        char *mine = wstage + j * kPitchP + h * 128;
        inverse_half<ADAPTIVE>(dev, qa, (int32_t)vv[0], h, mine);
        retire_stores();
        wave_sync();
        store_stage(stage, wv, lane, recon, (nb < 32u ? nb : 32u) * 256u);
        if (!DCTQ_RT_EARLY_PREFETCH) prefetch_batch<false>(ps, g + step, lane, nxt);
        // keep inverse B's inputs packed until here (converted early they are 64 more live VGPRs)
#pragma unroll
        for (int r = 0; r < 4; ++r) asm volatile("" : "+v"(qb[r].x), "+v"(qb[r].y), "+v"(qb[r].z), "+v"(qb[r].w));
        inverse_half<ADAPTIVE>(dev, qb, (int32_t)vv[1], h, mine);
        retire_stores();
        wave_sync();
        store_stage(stage, wv, lane, recon + 32 * 256, (nb > 32u ? nb - 32u : 0u) * 256u);
    }
    if (STATS) {
        uint32_t tot = exact_count;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
        if (lane == 0 && tot) atomicAdd(fallbacks, (unsigned long long)tot);
    }
}

template <bool A, bool V, bool S>
static hipError_t launch_rt(const RoundTripSet &rt, const DevTables *dev, unsigned long long *fb, hipStream_t stream,
                            int num_cus) {
    static const int per_cu = resident_per_cu(roundtrip8<A, V, S>, kThreads);
    const uint32_t nbatch = rt.ps.first[rt.ps.n];
    const uint32_t want = (nbatch + kWaves - 1) / kWaves;
    const uint32_t cap = (uint32_t)(num_cus * per_cu * DCTQ_RT_GRID_MULT);
    hipLaunchKernelGGL((roundtrip8<A, V, S>), dim3(want < cap ? want : cap), dim3(kThreads), 0, stream, rt, dev, fb);
    return hipGetLastError();
}

// ============================================================================
// Diagnostic: roundtrip8's data movement with no arithmetic -- the memory
// ceiling of this exact access pattern (bench.py round_trip.movement_ceiling).
// Same grid, occupancy bound, LDS footprint, prefetch, retire/sync points and
// stores as roundtrip8: per batch the pixel rows go into the stage as the
// "coefficients" (8 x 1 KiB stores), then twice 32 blocks of 256 B "recon"
// (the rows repeated) through the paired-inverse stage layout (8 x 1 KiB each).
__global__ __launch_bounds__(kThreads, DCTQ_RT_OCC) void roundtrip_movement(RoundTripSet rt) {
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
        if (DCTQ_PIN_OUT) asm volatile("" : "+s"(recon));
        uint2 *mine2 = reinterpret_cast<uint2 *>(wstage + lane * kPitch2);
        retire_stores();
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            mine2[2 * r] = cur[r];
            mine2[2 * r + 1] = make_uint2(cur[r].y, cur[r].x);
        }
        wave_sync();
        const uint32_t nb = out.nb;
        u4v val[8];
        stage_chunks(stage, wv, lane, val);
        {
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc(out.base, (short)0, (int)(nb * 128u), 0x00020000);
#pragma unroll
            for (int c = 0; c < 8; ++c) __builtin_amdgcn_raw_buffer_store_b128(val[c], rs, lane * 16, c * 1024, DCTQ_NT_AUX);
        }
        char *mine = wstage + j * kPitchP + h * 128;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            retire_stores();
            wave_sync();
#pragma unroll
            for (int r = 0; r < 8; ++r)
                *reinterpret_cast<uint4 *>(mine + r * 16) =
                    make_uint4(cur[r].x, cur[r].y, cur[r].x ^ (uint32_t)half, cur[r].y ^ (uint32_t)lane);
            retire_stores();
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
    const uint32_t cap = (uint32_t)(num_cus * per_cu * DCTQ_RT_GRID_MULT);  // the same grid as launch_rt
    hipLaunchKernelGGL(roundtrip_movement, dim3(want < cap ? want : cap), dim3(kThreads), 0, stream, rt);
    return hipGetLastError();
}

hipError_t launch_roundtrip(const RoundTripSet &rt, const DevTables *dev, int adaptive, unsigned long long *fallbacks,
                            hipStream_t stream, int num_cus) {
    const bool a = adaptive != 0, v = rt.ps.var[0] != nullptr, s = fallbacks != nullptr;
    if (a) {
        if (v) return s ? launch_rt<true, true, true>(rt, dev, fallbacks, stream, num_cus)
                        : launch_rt<true, true, false>(rt, dev, fallbacks, stream, num_cus);
        return s ? launch_rt<true, false, true>(rt, dev, fallbacks, stream, num_cus)
                 : launch_rt<true, false, false>(rt, dev, fallbacks, stream, num_cus);
    }
    if (v) return s ? launch_rt<false, true, true>(rt, dev, fallbacks, stream, num_cus)
                    : launch_rt<false, true, false>(rt, dev, fallbacks, stream, num_cus);
    return s ? launch_rt<false, false, true>(rt, dev, fallbacks, stream, num_cus)
             : launch_rt<false, false, false>(rt, dev, fallbacks, stream, num_cus);
}

}  // namespace dctq
