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

namespace dctq {

// Passes of <= 8 tie entries run 8 lanes per entry (exact_grouped<8>): -4.9 % on the bench
// step (round 3); the wide rounds spill at these kernels' 128-VGPR bound.
constexpr bool kRtGroup8 = true;
constexpr int kRtWide = 0;

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

// The 8-point transposed AAN graph in fp32, operation for operation
// tools/aan_model.py aan8t (the graph tools/inv_bound.py bounds; aan8t_d in fp64),
// with the fp32 constants of fdct8_bound.h.  Every op is a separately rounded fp32
// add / sub / mul or an explicit fma (-ffp-contract=off).
__device__ __forceinline__ void aan8t_f(float &v0, float &v1, float &v2, float &v3, float &v4, float &v5, float &v6,
                                        float &v7) {
    const float gz13 = v5 + v3, gz2 = v5 - v3, gz11 = v1 + v7, gz4 = v1 - v7;
    float gb0 = gz11 + gz13;
    const float gz3 = gz11 - gz13;
    const float go1 = gz3 * DCTQ_C4;
    const float gz5 = (gz2 + gz4) * DCTQ_C6;
    const float go0 = __builtin_fmaf(DCTQ_C2MC6, gz2, gz5);
    const float go2 = __builtin_fmaf(DCTQ_C2PC6, gz4, -gz5);
    const float gb3 = go0, gb2 = go0 + go1, gb1 = go1 + go2;
    gb0 = gb0 + go2;
    float ge3 = v2 + v6;
    const float gm = v2 - v6;
    const float gs = gm * DCTQ_C4;
    const float ge2 = gs;
    ge3 = ge3 + gs;
    const float ge0 = v0 + v4, ge1 = v0 - v4;
    const float ga0 = ge0 + ge3, ga3 = ge0 - ge3, ga1 = ge1 + ge2, ga2 = ge1 - ge2;
    v0 = ga0 + gb0;
    v1 = ga1 + gb1;
    v2 = ga2 + gb2;
    v3 = ga3 + gb3;
    v4 = ga3 - gb3;
    v5 = ga2 - gb2;
    v6 = ga1 - gb1;
    v7 = ga0 - gb0;
}

// Dequantize + inverse DCT + 128 of the lane's own block in fp32, for the plans
// api.hip admits (inverse_f32_bound: |recon - reference| <= 5e-5 for every input
// block; non-adaptive only, whose dequantisation is the reference's q * (1/Q),
// src/quantization.c:139,144): x_uv = fl32(q_uv * fl32(iscale_uv)) (one v_pk_mul per
// coefficient pair, the scale pair in SGPRs), the columns then the rows through
// aan8t_f (src/dct.c:80-105 as D^T X D), then + 128 (tools/inv_bound.py models
// exactly this sequence).  qw = the block's 64 int16 (row-major, two per dword).
__device__ __forceinline__ void inverse_block_f32(const DevTables *__restrict__ dev, const uint2 (&qw)[16],
                                                  float (&x)[64]) {
    ConstTables *tp = tables(dev);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const uint32_t w[2] = {qw[r].x, qw[r].y};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int c = 4 * r + 2 * h;
            const f2 q = {(float)(int)(int16_t)(w[h] & 0xFFFFu), (float)((int)w[h] >> 16)};
            const f2 sc = {tp->iscale32[c], tp->iscale32[c + 1]};
            const f2 v = q * sc;
            x[c] = v.x;
            x[c + 1] = v.y;
        }
    }
#pragma unroll
    for (int v = 0; v < 8; ++v)
        aan8t_f(x[v], x[8 + v], x[16 + v], x[24 + v], x[32 + v], x[40 + v], x[48 + v], x[56 + v]);
#pragma unroll
    for (int i = 0; i < 8; ++i)
        aan8t_f(x[8 * i], x[8 * i + 1], x[8 * i + 2], x[8 * i + 3], x[8 * i + 4], x[8 * i + 5], x[8 * i + 6],
                x[8 * i + 7]);
    const f2 k128 = {128.0f, 128.0f};
#pragma unroll
    for (int c = 0; c < 64; c += 2) {
        const f2 v = f2{x[c], x[c + 1]} + k128;
        x[c] = v.x;
        x[c + 1] = v.y;
    }
}

// The fused round trip with the fp32 inverse (non-adaptive plans admitted by
// api.hip inverse_f32_bound, e.g. q <= 71 of the standard table).  Phases 1-2 are
// roundtrip8's; phase 3 runs lane per block (no transposes, half the fp64 kernel's
// VALU issue: PMC profiles/r05/): every lane inverts its own block in registers,
// then the recon leaves through the stage in two 8 KiB halves (blocks 0-31, then
// 32-63).  The second half's read-back lands in registers disjoint from the first
// half's pending store data (kept live across it), so no vmcnt(0) sits between the
// two halves' stores; the only waits are the prefetch fence after the forward and
// one retire of the coefficient stores after the inverse, both behind a compute phase.
template <bool VAR, bool STATS>
__global__ __launch_bounds__(kThreads, kRtOcc) void roundtrip8_f32(RoundTripSet rt,
                                                                       const DevTables *__restrict__ dev,
                                                                       unsigned long long *fallbacks) {
    __shared__ uint4 stage[kThreads * kPitch2 / 16];
    __shared__ ExactTables tab;
    __shared__ uint16_t scr[kWaves * 64];  // resolve_ties_compact's entries
    load_exact_tables(&tab, dev);
    const PlaneSet &ps = rt.ps;
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
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
        prefetch_batch<false>(ps, g + step, lane, nxt);
        const BatchOut out = batch_out(ps, k, b);  // resolved before the fences (fdct8_core.h)
        char *recon = reinterpret_cast<char *>(rt.recon[k]) + (size_t)b * 64 * 256;
        if (DCTQ_PIN_OUT) asm volatile("" : "+s"(recon));

        // ---- 1. forward into the stage; ties resolved in place
        int32_t var_num;
        uint32_t mlo, mhi;
        forward_flags_batch<false, VAR>(dev, cur, stage, lane, wv, valid, var_num, mlo, mhi);
        retire_stores();  // the previous batch's recon stores (long issued) before any LDS read
        const uint32_t ne = resolve_ties_compact<false, true, 0>(&tab, cur, stage, scr + wv * 64, lane, wv, mlo, mhi);
        if (STATS) exact_count += ne;
        wave_sync();

        // ---- 2. read-back: the coefficient chunks and the lane's own block
        const uint32_t nb = out.nb;
        u4v val[8];
        stage_chunks(stage, wv, lane, val);
        uint2 qw[16];
        {
            const uint2 *row = reinterpret_cast<const uint2 *>(wstage + lane * kPitch2);
#pragma unroll
            for (int r = 0; r < 16; ++r) qw[r] = row[r];
        }
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

        // ---- 3. fp32 inverse, lane per block; recon out in two 8 KiB halves
        float x[64];
        inverse_block_f32(dev, qw, x);
        stage_recon_half<0>(wstage, lane, x);
        retire_stores();  // the coefficient stores have read their data (store-data hazard)
        wave_sync();
        u4p va[8], vb[8];
        stage_read_half(stage, wv, lane, va);
        store_half(va, lane, recon, (nb < 32u ? nb : 32u) * 256u);
        stage_recon_half<1>(wstage, lane, x);
        wave_sync();
        stage_read_half(stage, wv, lane, vb);
        // A's store data stays live until B's rows are in: B's LDS loads cannot land in it
#pragma unroll
        for (int c = 0; c < 8; ++c) asm volatile("" : "+v"(vb[c]) : "v"(va[c]));
        store_half(vb, lane, recon + 32 * 256, (nb > 32u ? nb - 32u : 0u) * 256u);
    }
    if (STATS) {
        uint32_t tot = exact_count;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
        if (lane == 0 && tot) atomicAdd(fallbacks, (unsigned long long)tot);
    }
}

template <bool ADAPTIVE, bool VAR, bool STATS>
__global__ __launch_bounds__(kThreads, kRtOcc) void roundtrip8(RoundTripSet rt, const DevTables *__restrict__ dev,
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
        prefetch_batch<false>(ps, g + step, lane, nxt);
        const BatchOut out = batch_out(ps, k, b);  // resolved before the fences (fdct8_core.h)
        char *recon = reinterpret_cast<char *>(rt.recon[k]) + (size_t)b * 64 * 256;
        if (DCTQ_PIN_OUT) asm volatile("" : "+s"(recon));

        // ---- 1. forward into the stage; ties resolved in place
        int32_t var_num;
        uint32_t mlo, mhi;
        forward_flags_batch<ADAPTIVE, VAR>(dev, cur, stage, lane, wv, valid, var_num, mlo, mhi);
        retire_stores();  // the previous batch's recon stores (long issued) before any LDS read
        const uint32_t ne =
            resolve_ties_compact<ADAPTIVE, kRtGroup8, kRtWide>(&tab, cur, stage, scr + wv * 64, lane, wv, mlo, mhi);
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
    const uint32_t cap = (uint32_t)(num_cus * per_cu * kRtGridMult);
    hipLaunchKernelGGL((roundtrip8<A, V, S>), dim3(want < cap ? want : cap), dim3(kThreads), 0, stream, rt, dev, fb);
    return hipGetLastError();
}

template <bool V, bool S>
static hipError_t launch_rt_f32(const RoundTripSet &rt, const DevTables *dev, unsigned long long *fb,
                                hipStream_t stream, int num_cus) {
    static const int per_cu = resident_per_cu(roundtrip8_f32<V, S>, kThreads);
    const uint32_t nbatch = rt.ps.first[rt.ps.n];
    const uint32_t want = (nbatch + kWaves - 1) / kWaves;
    const uint32_t cap = (uint32_t)(num_cus * per_cu * kRtGridMult);
    hipLaunchKernelGGL((roundtrip8_f32<V, S>), dim3(want < cap ? want : cap), dim3(kThreads), 0, stream, rt, dev, fb);
    return hipGetLastError();
}

hipError_t launch_roundtrip(const RoundTripSet &rt, const DevTables *dev, int adaptive, bool inv_f32,
                            unsigned long long *fallbacks, hipStream_t stream, int num_cus) {
    const bool a = adaptive != 0, v = rt.ps.var[0] != nullptr, s = fallbacks != nullptr;
    if (inv_f32 && !a) {
        if (v) return s ? launch_rt_f32<true, true>(rt, dev, fallbacks, stream, num_cus)
                        : launch_rt_f32<true, false>(rt, dev, fallbacks, stream, num_cus);
        return s ? launch_rt_f32<false, true>(rt, dev, fallbacks, stream, num_cus)
                 : launch_rt_f32<false, false>(rt, dev, fallbacks, stream, num_cus);
    }
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
