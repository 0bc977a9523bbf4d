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
//  3. two paired-lane inverses (pair_core.h, as idct8_pair), 32 blocks each,
//     staged as fp32 rows and written as 1 KiB stores: fp32 arithmetic for the
//     plans a rigorous error bound admits (inverse_half_f32), fp64 otherwise.
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
// Pixel rows through a plane-bounded buffer descriptor (load_rows<true>): a wrong row
// address reads zeros instead of faulting; within noise of global loads
// (profiles/r05/rt_ab_keep_late_rows.log).
constexpr bool kRtBufRows = true;

static_assert(kThreads == kThreadsP && 64 * kPitch2 == 32 * kPitchP, "forward and inverse share the wave's stage");

// Dequantize + inverse DCT + 128 of one 32-block sub-batch in fp64, lane (h, j)
// holding rows 4h..4h+3 of block j (8 int16 per uint4) and the block's var_num;
// fp32 rows into the wave's stage (layout of idct8_pair).  Adaptive plans and the
// non-adaptive plans the fp32 bound does not admit.
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

// The fp32 inverse (non-adaptive plans admitted by api.hip inverse_f32_bound:
// |recon - reference| <= 5e-5 for every input block, e.g. q <= 71 of the standard
// table; their dequantisation is the reference's q * (1/Q), src/quantization.c:139,
// 144), in inverse_half's paired-lane layout (lane (h, j): rows 4h..4h+3 of block j):
// x_uv = fl32(q_uv * fl32(iscale_uv)) (one v_pk_mul per coefficient pair, the scale
// pair of the lane's half-wave in SGPRs), the columns (after the exact lane-half
// transpose) then the rows through aan8t_f (src/dct.c:80-105 as D^T X D), then
// + 128 -- exactly the sequence tools/inv_bound.py bounds.  Half the fp64 kernel's
// VALU issue (profiles/r05/pmc_rt_*).  Lane per block (every lane inverting its own
// block in registers, no transposes, the 16 KiB of recon then leaving as two 8 KiB
// halves back to back) issued less still but ran 4.4-4.6 % slower on the bench step
// (profiles/r05/rt_ab.log): the paired layout's stores leave in three spaced
// groups (coefficients, half A after inverse A, half B after inverse B), which this
// write-heavy stream (64 B read : 384 B written per block) takes better than bursts.
__device__ __forceinline__ void swap_halves_f(float &x, float &y) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(y), false, false);
    x = __uint_as_float(r[0]);
    y = __uint_as_float(r[1]);
}
// v[k] (a row's pairs of coefficients) *= lo[k] in lanes 0-31 and *= hi[k] in lanes
// 32-63, both scale rows in SGPR pairs: two exec-masked v_pk_mul_f32 per pair (a
// per-lane select of the factor costs 2 v_mov + 1 v_cndmask per value, and spilled).
// The wave is fully active here; exec is saved and restored inside the block, and the
// block ends with the wait states a v_permlane read of its outputs needs (hipcc cannot
// see inside it).
typedef const __attribute__((address_space(4))) uint64_t ConstPair;
__device__ __forceinline__ void half_wave_scale_f32(f2 (&v)[4], ConstPair *lo, ConstPair *hi) {
    uint64_t save;
    asm volatile(
        "s_mov_b64 %[sv], exec\n\t"
        "s_mov_b32 exec_hi, 0\n\t"
        "v_pk_mul_f32 %0, %0, %5\n\tv_pk_mul_f32 %1, %1, %6\n\tv_pk_mul_f32 %2, %2, %7\n\tv_pk_mul_f32 %3, %3, %8\n\t"
        "s_mov_b64 exec, %[sv]\n\t"
        "s_mov_b32 exec_lo, 0\n\t"
        "v_pk_mul_f32 %0, %0, %9\n\tv_pk_mul_f32 %1, %1, %10\n\tv_pk_mul_f32 %2, %2, %11\n\tv_pk_mul_f32 %3, %3, %12\n\t"
        "s_mov_b64 exec, %[sv]\n\t"
        "s_nop 1"  // VALU write -> v_permlane32_swap read (swap_halves_f next): 2 wait states, ours to pad
        : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), [sv] "=&s"(save)
        : "s"(lo[0]), "s"(lo[1]), "s"(lo[2]), "s"(lo[3]), "s"(hi[0]), "s"(hi[1]), "s"(hi[2]), "s"(hi[3]));
}

__device__ __forceinline__ void inverse_half_f32(const DevTables *__restrict__ dev, const uint4 (&q)[4], int h,
                                                 char *mine) {
    float v[4][8];
    ConstTables *tp = tables(dev);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint32_t w[4] = {q[r].x, q[r].y, q[r].z, q[r].w};
        f2 x[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = f2{(float)(int)(int16_t)(w[k] & 0xFFFFu), (float)((int)w[k] >> 16)};
        // row r of the half-wave: row r (lanes 0-31) or r + 4 (lanes 32-63) of the block
        half_wave_scale_f32(x, reinterpret_cast<ConstPair *>(&tp->iscale32[8 * r]),
                            reinterpret_cast<ConstPair *>(&tp->iscale32[8 * (r + 4)]));
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            v[r][2 * k] = x[k].x;
            v[r][2 * k + 1] = x[k].y;
        }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int k = 0; k < 4; ++k) swap_halves_f(v[r][k], v[r][k + 4]);
#pragma unroll
    for (int k = 0; k < 4; ++k)
        aan8t_f(v[0][k], v[1][k], v[2][k], v[3][k], v[0][k + 4], v[1][k + 4], v[2][k + 4], v[3][k + 4]);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int k = 0; k < 4; ++k) swap_halves_f(v[r][k], v[r][k + 4]);
#pragma unroll
    for (int r = 0; r < 4; ++r) aan8t_f(v[r][0], v[r][1], v[r][2], v[r][3], v[r][4], v[r][5], v[r][6], v[r][7]);
    const f2 k128 = {128.0f, 128.0f};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        f2 o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = f2{v[r][2 * k], v[r][2 * k + 1]} + k128;
        *reinterpret_cast<float4 *>(mine + r * 32) = make_float4(o[0].x, o[0].y, o[1].x, o[1].y);
        *reinterpret_cast<float4 *>(mine + r * 32 + 16) = make_float4(o[2].x, o[2].y, o[3].x, o[3].y);
    }
}

template <bool ADAPTIVE, bool VAR, bool STATS, bool INV32 = false>
__global__ __launch_bounds__(kThreads, kRtOcc) void roundtrip8(RoundTripSet rt, const DevTables *__restrict__ dev,
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
    prefetch_batch<true, kRtBufRows>(ps, g, lane, nxt);
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
        prefetch_batch<false, kRtBufRows>(ps, g + step, lane, nxt);
        const BatchOut out = batch_out(ps, k, b);  // resolved before the fences (fdct8_core.h)
        char *recon = reinterpret_cast<char *>(rt.recon[k]) + (size_t)b * 64 * 256;
        asm volatile("" : "+s"(recon));

        // ---- 1. forward into the stage; ties resolved in place
        int32_t var_num;
        uint32_t mlo, mhi;
        forward_flags_batch<ADAPTIVE, VAR>(dev, cur, stage, lane, wv, valid, var_num, mlo, mhi);
        // vmcnt(0): the previous batch's recon stores (store-data hazard) and this
        // batch's prefetch before any LDS read.  Waiting later (the rows requested after the
        // forward, vmcnt(8)) or not at all before the recon read-backs (the pending stores' data
        // kept live instead) measured within noise (profiles/r05/rt_ab_keep_late_rows.log)
        retire_stores();
        const uint32_t ne =
            resolve_ties_compact<ADAPTIVE, kRtGroup8, kRtWide>(&tab, cur, stage, scr + wv * 64, lane, wv, mlo, mhi);
        if (STATS) exact_count += ne;
        wave_sync();

        // ---- 2. read-back: coefficient chunks + the inverse's half blocks
        const uint32_t nb = out.nb;
        // the inverse's lane roles from an opaque copy of the lane id: hoisted out of the
        // loop, these indices and the LDS addresses made of them sat in VGPRs across the
        // forward and pushed a prefetched row into scratch
        int ol = lane;
        asm volatile("" : "+v"(ol));
        const int h = ol >> 5, j = ol & 31;
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
            for (int c = 0; c < 8; ++c) __builtin_amdgcn_raw_buffer_store_b128(val[c], rs, lane * 16, c * 1024, kNtAux);
            if (VAR) {
                const __amdgpu_buffer_rsrc_t rv =
                    __builtin_amdgcn_make_buffer_rsrc(out.var, (short)0, (int)(nb * 4u), 0x00020000);
                __builtin_amdgcn_raw_buffer_store_b32(var_num, rv, lane * 4, 0, kNtAux);
            }
        }

        // ---- 3. paired inverses, blocks 0-31 then 32-63 of the batch
        char *mine = wstage + j * kPitchP + h * 128;
        if constexpr (INV32) inverse_half_f32(dev, qa, h, mine);
        else inverse_half<ADAPTIVE>(dev, qa, (int32_t)vv[0], h, mine);
        retire_stores();
        wave_sync();
        store_stage(stage, wv, lane, recon, (nb < 32u ? nb : 32u) * 256u);
        // keep inverse B's inputs packed until here (converted early they are 64 more live VGPRs)
#pragma unroll
        for (int r = 0; r < 4; ++r) asm volatile("" : "+v"(qb[r].x), "+v"(qb[r].y), "+v"(qb[r].z), "+v"(qb[r].w));
        if constexpr (INV32) inverse_half_f32(dev, qb, h, mine);
        else inverse_half<ADAPTIVE>(dev, qb, (int32_t)vv[1], h, mine);
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
    static const int per_cu = resident_per_cu(roundtrip8<false, V, S, true>, kThreads);
    const uint32_t nbatch = rt.ps.first[rt.ps.n];
    const uint32_t want = (nbatch + kWaves - 1) / kWaves;
    const uint32_t cap = (uint32_t)(num_cus * per_cu * kRtGridMult);
    hipLaunchKernelGGL((roundtrip8<false, V, S, true>), dim3(want < cap ? want : cap), dim3(kThreads), 0, stream, rt,
                       dev, fb);
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
