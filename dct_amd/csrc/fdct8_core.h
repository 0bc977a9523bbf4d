// dct_amd/csrc/fdct8_core.h -- the lane-per-block fp32 forward DCT + quantization
// core shared by the forward kernels (fdct8.hip) and the fused round trip
// (roundtrip.hip): block addressing, the AAN butterfly, the per-batch compute
// into the wave's LDS stage with tie flags, and the constant-block DC fix.
// Design notes: fdct8.hip header and DESIGN.md "Kernels".
#pragma once
#include "dctq_internal.h"
#include "fdct8_bound.h"

namespace dctq {

constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;
constexpr int kFWaves = 4;  // the streaming forward kernels' workgroup: 4 waves
constexpr int kFThreads = 64 * kFWaves;
constexpr int kV3GridMult = 16;  // fdct8_quant_v3's grid: 16 x its resident workgroups (fdct8.hip)
constexpr int kPitch = 9;  // uint4 per block in the LDS stage: 128 B + 16 B pad
constexpr float kMagic = 12582912.0f;  // 1.5 * 2^23: fma(y, w, kMagic) rounds y*w to an integer in its low bits

__device__ __forceinline__ float fma_t(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
__device__ __forceinline__ double fma_t(double a, double b, double c) { return __builtin_fma(a, b, c); }

// The 8-point AAN flow graph, operation for operation tools/aan_model.py::aan8
// (the model tools/guard_bound.py bounds).  Outputs y_k with X_k = kAanScale[k]*y_k.
template <typename T>
__device__ __forceinline__ void aan8(T &v0, T &v1, T &v2, T &v3, T &v4, T &v5, T &v6, T &v7, T c4, T c6,
                                     T c2mc6, T c2pc6) {
    T a0 = v0 + v7, b0 = v0 - v7;
    T a1 = v1 + v6, b1 = v1 - v6;
    T a2 = v2 + v5, b2 = v2 - v5;
    T a3 = v3 + v4, b3 = v3 - v4;
    T e0 = a0 + a3, e3 = a0 - a3;
    T e1 = a1 + a2, e2 = a1 - a2;
    T y0 = e0 + e1, y4 = e0 - e1;
    T m = (e2 + e3) * c4;
    T y2 = e3 + m, y6 = e3 - m;
    T o0 = b3 + b2;
    T o1 = b2 + b1;
    T o2 = b1 + b0;
    T z5 = (o0 - o2) * c6;
    T z2 = fma_t(c2mc6, o0, z5);
    T z4 = fma_t(c2pc6, o2, z5);
    T z3 = o1 * c4;
    T z11 = b0 + z3, z13 = b0 - z3;
    v0 = y0;
    v1 = z11 + z4;
    v2 = y2;
    v3 = z13 - z2;
    v4 = y4;
    v5 = z13 + z2;
    v6 = y6;
    v7 = z11 - z4;
}

template <typename T>
__device__ __forceinline__ void aan8x8(T (&v)[8][8], T c4, T c6, T c2mc6, T c2pc6) {
#pragma unroll
    for (int r = 0; r < 8; ++r) aan8(v[r][0], v[r][1], v[r][2], v[r][3], v[r][4], v[r][5], v[r][6], v[r][7], c4, c6, c2mc6, c2pc6);
#pragma unroll
    for (int c = 0; c < 8; ++c) aan8(v[0][c], v[1][c], v[2][c], v[3][c], v[4][c], v[5][c], v[6][c], v[7][c], c4, c6, c2mc6, c2pc6);
}

// Locate the lane's block: n -> (frame, by, bx) -> pointer to its top-left pixel.
__device__ __forceinline__ const uint8_t *block_ptr(const PlaneArgs &p, uint32_t n) {
    uint32_t f = fdiv(n, p.div_frame);
    uint32_t rem = n - f * (uint32_t)p.nblk_frame;
    uint32_t by = fdiv(rem, p.div_bw);
    uint32_t bx = rem - by * (uint32_t)p.bw;
    return p.src + (long long)f * p.frame_stride + (long long)(by * 8) * p.stride + (long long)bx * 8;
}

// src/quantization.c:171-211 for is_quantize=1, element c, given the block's
// exact variance (var_num / 4096): nv = fmin(1, fmax(0.1, var/1000)),
// M = Q*(2-nv) clamped to >= 1, DC keeps Q.
__device__ __forceinline__ double adaptive_scale(int32_t var_num) {
    const double var = (double)var_num / 4096.0;  // == (sum_sq/64) - mean*mean exactly
    const double nv = fmin(1.0, fmax(0.1, var / 1000.0));
    return 2.0 - nv;
}

// out / m for the exact paths: every divisor of a tie-heavy plan is 1 (q >= 97 without
// adaptation), and x / 1.0 == x exactly, so the fp64 division sequence (~11 VALU) runs
// only when some lane of the wave has a divisor other than 1.
__device__ __forceinline__ double exact_div(double out, double m) {
    if (!__builtin_amdgcn_ballot_w64(m != 1.0)) return out;
    return out / m;
}

// ============================================================================
// v2 building blocks (see fdct8.hip for the loop around them).
typedef float f2 __attribute__((ext_vector_type(2)));
typedef uint32_t u2v __attribute__((ext_vector_type(2)));
typedef uint32_t u4v __attribute__((ext_vector_type(4)));
constexpr int kPitch2 = 136;   // bytes per block in the stage: 2-way (free) conflicts for the b32 writes
// Cache policy of the bulk coefficient stores: non-temporal (kNtAux), -15 % kernel
// time on the 4K stream (profiles/r01/store_policy.md); the written lines are never
// re-read by this kernel except by tie patches, which come after a vmcnt(0).
constexpr int kStoreAux = kNtAux;

template <int K>
__device__ __forceinline__ float cvt_ubyte(uint32_t w) {
    float f;
    if constexpr (K == 0) asm("v_cvt_f32_ubyte0 %0, %1" : "=v"(f) : "v"(w));
    else if constexpr (K == 1) asm("v_cvt_f32_ubyte1 %0, %1" : "=v"(f) : "v"(w));
    else if constexpr (K == 2) asm("v_cvt_f32_ubyte2 %0, %1" : "=v"(f) : "v"(w));
    else asm("v_cvt_f32_ubyte3 %0, %1" : "=v"(f) : "v"(w));
    return f;
}

// Pixel rows are read exactly once: non-temporal loads (+8.7 % on the memory
// ceiling of this stream, profiles/r01/valu_issue_rates.md).
// BUF (every product kernel): through a buffer descriptor over the plane (p.span
// bytes from p.src) when the plane spans < 4 GiB: an address that went wrong then
// reads zeros -- and fails parity -- instead of faulting the device (round 5,
// profiles/r05/INDEX.md); within noise of global loads on the forward and the round
// trip (profiles/r05/forward_buf_rows_ab.log, rt_ab_keep_late_rows.log).
template <bool BUF = true>
__device__ __forceinline__ void load_rows(const PlaneArgs &p, uint32_t n, uint2 (&rows)[8]) {
    const uint8_t *px = block_ptr(p, n < (uint32_t)p.nblk ? n : 0);
    if constexpr (BUF) {
        if (p.span) {  // kernel argument: wave-uniform
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(p.src), (short)0, (int)p.span, 0x00020000);
            const uint32_t off = (uint32_t)(px - p.src), st = (uint32_t)p.stride;
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const u2v t = __builtin_amdgcn_raw_buffer_load_b64(rs, off + r * st, 0, 2 /* nt */);
                rows[r] = make_uint2(t.x, t.y);
            }
            return;
        }
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const u2v t = __builtin_nontemporal_load(reinterpret_cast<const u2v *>(px + r * p.stride));
        rows[r] = make_uint2(t.x, t.y);
    }
}

// Coefficient output of plane k (k wave-uniform or not: a select chain, no indexed kernarg loads).
__device__ __forceinline__ int16_t *coef_of(const PlaneSet &ps, uint32_t k) {
    int16_t *c = ps.coef[0];
#pragma unroll
    for (int i = 1; i < kMaxPlanes; ++i) c = k == (uint32_t)i ? ps.coef[i] : c;
    return c;
}

// First global batch of plane k (wave-uniform k): a select chain over the batch
// prefixes, which sit in SGPRs for the whole kernel -- an indexed kernel-argument
// load here was one more scalar-cache round trip in front of every prefetch.
__device__ __forceinline__ uint32_t first_of(const PlaneSet &ps, int k) {
    uint32_t f = 0u;
#pragma unroll
    for (int i = 1; i < kMaxPlanes; ++i) f = k == i ? ps.first[i] : f;
    return f;
}

// Plane of global batch g (wave-uniform).
__device__ __forceinline__ int plane_of(const PlaneSet &ps, uint32_t g) {
    int k = 0;
#pragma unroll
    for (int i = 1; i < kMaxPlanes; ++i) k += (i < ps.n && g >= ps.first[i]) ? 1 : 0;
    return k;
}

// The arithmetic of one 64-block batch (one block per lane): u8 rows -> fp32,
// exact variance numerator, AAN row pass, column pairs fused with quantization
// into the wave's LDS stage, tie masks (bit 31 - p%32 of mlo/mhi = processing
// slot p = 16*cp + 2*i + h needs the exact path).
template <bool ADAPTIVE, bool VAR>
__device__ __forceinline__ void fdct8_compute(const DevTables *__restrict__ dev, const uint2 (&cur)[8], uint4 *stage,
                                              int lane, int wv, uint32_t &mlo, uint32_t &mhi, int32_t &var_num) {
    const f2 M2 = {kMagic, kMagic};
    float v[8][8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        v[r][0] = cvt_ubyte<0>(cur[r].x);
        v[r][1] = cvt_ubyte<1>(cur[r].x);
        v[r][2] = cvt_ubyte<2>(cur[r].x);
        v[r][3] = cvt_ubyte<3>(cur[r].x);
        v[r][4] = cvt_ubyte<0>(cur[r].y);
        v[r][5] = cvt_ubyte<1>(cur[r].y);
        v[r][6] = cvt_ubyte<2>(cur[r].y);
        v[r][7] = cvt_ubyte<3>(cur[r].y);
    }
    var_num = 0;
    if (ADAPTIVE || VAR) {
        uint32_t s1 = 0, s2 = 0;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            s1 = __builtin_amdgcn_udot4(cur[r].x, 0x01010101u, s1, false);
            s1 = __builtin_amdgcn_udot4(cur[r].y, 0x01010101u, s1, false);
            s2 = __builtin_amdgcn_udot4(cur[r].x, cur[r].x, s2, false);
            s2 = __builtin_amdgcn_udot4(cur[r].y, cur[r].y, s2, false);
        }
        const int32_t sx = (int32_t)s1 - 8192;
        const int32_t sxx = (int32_t)s2 - 256 * (int32_t)s1 + 1048576;
        var_num = 64 * sxx - sx * sx;
    }

    // ---- row pass, then column pairs fused with quantization
#pragma unroll
    for (int r = 0; r < 8; ++r)
        aan8(v[r][0], v[r][1], v[r][2], v[r][3], v[r][4], v[r][5], v[r][6], v[r][7], DCTQ_C4, DCTQ_C6, DCTQ_C2MC6,
             DCTQ_C2PC6);

    f2 sc2 = {1.0f, 1.0f};
    if (ADAPTIVE) {
        // The fast path only needs 1/(2-nv) within its guard band (4.5u relative for
        // adaptive plans, api.hip fill_fast_tables): nv through a multiply by
        // fl(0.001) instead of the reference's division (relative error ~2^-52),
        // then fl32(2-nv) (0.5u) and v_rcp_f32 (1 ulp = 2u) -- two fp64 divisions
        // per lane per batch were ~8 % of the adaptive kernel's time.  The exact
        // path keeps the reference's arithmetic (adaptive_scale).
        const double nv = fmin(1.0, fmax(0.1, (double)var_num * (1.0 / 4096.0) * 0.001));
        const float inv = __builtin_amdgcn_rcpf((float)(2.0 - nv));
        sc2 = f2{inv, inv};
    }
    // Per-plan tables through an opaque per-batch pointer in the constant address
    // space: scalar loads stay inside the loop (hoisted, they would need 128 live
    // SGPRs) and stay scalar (a generic pointer becomes flat_load + vmcnt(0)).
    const FastTables *tg = &dev->fast;
    asm volatile("" : "+s"(tg));
    const __attribute__((address_space(4))) FastTables *tp = (const __attribute__((address_space(4))) FastTables *)tg;
    mlo = 0;
    mhi = 0;  // bit (31 - p%32): processing slot p = 16*cp + 2*i + h flagged
    uint32_t *st32 = reinterpret_cast<uint32_t *>(stage) + (wv * 64 + lane) * (kPitch2 / 4);
#pragma unroll
    for (int cp = 0; cp < 4; ++cp) {
        const int c0 = 2 * cp;
        aan8(v[0][c0], v[1][c0], v[2][c0], v[3][c0], v[4][c0], v[5][c0], v[6][c0], v[7][c0], DCTQ_C4, DCTQ_C6,
             DCTQ_C2MC6, DCTQ_C2PC6);
        aan8(v[0][c0 + 1], v[1][c0 + 1], v[2][c0 + 1], v[3][c0 + 1], v[4][c0 + 1], v[5][c0 + 1], v[6][c0 + 1],
             v[7][c0 + 1], DCTQ_C4, DCTQ_C6, DCTQ_C2MC6, DCTQ_C2PC6);
        if (cp == 0) v[0][0] -= 8192.0f;  // 64 * 128: exact (integer < 2^24)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int c = i * 8 + c0, slot = 16 * cp + 2 * i;
            const f2 y = {v[i][c0], v[i][c0 + 1]};
            f2 w = {tp->ws[slot], tp->ws[slot + 1]};
            if (ADAPTIVE) {
                if (c == 0) w.y *= sc2.y;  // the DC keeps Q (src/quantization.c:198-199)
                else w *= sc2;
            }
            const f2 tt = __builtin_elementwise_fma(y, w, M2);
            const f2 nr = M2 - tt;
            const f2 f = __builtin_elementwise_fma(y, w, nr);
            const f2 T = {tp->t2s[slot], tp->t2s[slot + 1]};
            const f2 d = __builtin_elementwise_fma(-f, f, T);  // < 0  <=>  |f| beyond the guard
            if (cp < 2) {
                mlo = __builtin_amdgcn_alignbit(mlo, __float_as_uint(d.x), 31);
                mlo = __builtin_amdgcn_alignbit(mlo, __float_as_uint(d.y), 31);
            } else {
                mhi = __builtin_amdgcn_alignbit(mhi, __float_as_uint(d.x), 31);
                mhi = __builtin_amdgcn_alignbit(mhi, __float_as_uint(d.y), 31);
            }
            st32[i * 4 + cp] = __builtin_amdgcn_perm(__float_as_uint(tt.y), __float_as_uint(tt.x), 0x05040100u);
        }
        // Pin the flag mask here: otherwise LLVM sinks the 32 residual tests of
        // this column pair to their only use (the queue phase, after the stores)
        // and keeps every residual live across the stores.
        asm volatile("" : "+v"(mlo), "+v"(mhi));
    }
}

// A flagged DC of a CONSTANT block (flat image areas: an exact .5 tie for half
// of all pixel values at q50) is resolved from the plan's table of
// reference-order DCs instead of the exact path.  Checked only when some lane's
// DC (processing slot 0 = bit 31 of mlo) is flagged.
__device__ __forceinline__ void flat_dc_fix(const DevTables *__restrict__ dev, const uint2 (&cur)[8], uint4 *stage,
                                            int lane, int wv, uint32_t &mlo) {
    if (__builtin_amdgcn_ballot_w64((mlo >> 31) != 0u)) {
        const uint32_t w = cur[0].x;
        bool flat = w == (w & 0xFFu) * 0x01010101u;
#pragma unroll
        for (int r = 0; r < 8; ++r) flat &= (cur[r].x == w) & (cur[r].y == w);  // bitwise: no short-circuit branches
        if ((mlo >> 31) && flat) {
            reinterpret_cast<int16_t *>(stage)[(wv * 64 + lane) * (kPitch2 / 2)] = dev->dc_const[w & 0xFFu];
            mlo &= 0x7FFFFFFFu;
        }
    }
}

// temp[k][j] = sum_l x[k][l] D^T[l][j], l ascending from 0.0 (src/dct.c:57-64), x = px - 128.
// The sum starts at the first product instead of 0.0 + it (and the callers start
// `out` at its first term): 0.0 + p == p for every p except p == -0.0, so the sums
// differ at most in the sign of a zero, which neither a later nonzero term nor
// round() / the int conversion can see -- the int16 result is the reference's
// (DESIGN.md 4).  9 fp64 adds fewer per evaluation.
__device__ __forceinline__ double row_sum(uint32_t wx, uint32_t wy, const double *dj) {
    double t = 0.0;
#pragma unroll
    for (int l = 0; l < 8; ++l) {
        const uint32_t w = l < 4 ? wx : wy;
        const double p = ((double)((w >> (8 * (l & 3))) & 0xFFu) - 128.0) * dj[l];
        t = l == 0 ? p : t + p;
    }
    return t;
}

// The arithmetic of exact_quant() (fdct8.hip) on a block held in registers plus,
// for adaptive plans, the block's exact variance and adjusted divisor
// (src/quantization.c:153-211):
//   temp[k][j] = sum_l x[k][l] D^T[l][j]; out = sum_k D[i][k] temp[k][j]  (src/dct.c:57-74)
//   q = (int) round(out / M_ij)                                         (src/quantization.c:124)
// The 16 table entries are requested before the fp64 chain.
template <bool ADAPTIVE>
__device__ __forceinline__ int exact_from_rows(const uint2 (&rows)[8], int c, const DevTables *__restrict__ dev) {
    const int i = c >> 3, j = c & 7;
    double dj[8], di[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        dj[k] = dev->dct[j * 8 + k];  // D^T[k][j]
        di[k] = dev->dct[i * 8 + k];  // D[i][k]
    }
    double m = dev->quant[c];
    if (ADAPTIVE && c != 0) {
        uint32_t s1 = 0, s2 = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            s1 = __builtin_amdgcn_udot4(rows[k].x, 0x01010101u, s1, false);
            s1 = __builtin_amdgcn_udot4(rows[k].y, 0x01010101u, s1, false);
            s2 = __builtin_amdgcn_udot4(rows[k].x, rows[k].x, s2, false);
            s2 = __builtin_amdgcn_udot4(rows[k].y, rows[k].y, s2, false);
        }
        const int32_t sx = (int32_t)s1 - 8192;
        const int32_t sxx = (int32_t)s2 - 256 * (int32_t)s1 + 1048576;
        m = m * adaptive_scale(64 * sxx - sx * sx);
        if (m < 1.0) m = 1.0;
    }
    double out = 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const double t = row_sum(rows[k].x, rows[k].y, dj);
        out = k == 0 ? di[0] * t : out + di[k] * t;
    }
    return (int)round(exact_div(out, m));
}

// Next flagged processing slot of (mlo, mhi) -> coefficient index, clearing it.
// slot = 16*cp + 2*i + h  ->  coefficient 8*i + 2*cp + h
__device__ __forceinline__ int pop_flag(uint32_t &mlo, uint32_t &mhi) {
    int slot;
    if (mlo) {
        slot = __clz(mlo);
        mlo &= ~(0x80000000u >> slot);
    } else {
        const int z = __clz(mhi);
        mhi &= ~(0x80000000u >> z);
        slot = 32 + z;
    }
    return (((slot >> 1) & 7) << 3) + ((slot >> 4) << 1) + (slot & 1);
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// In-place tie resolution, for consumers that read the final ints from the
// stage in the same launch (the fused round trip and the encoder).  The exact
// path's tables live in LDS (one 1 KiB copy per workgroup): per-lane global
// table loads at L2 latency made the first version of that path cost ~40 % of
// the encoder's count pass.  So the resolution runs AFTER the prefetch fence
// (its LDS reads must not land in the previous batch's pending store data).
struct ExactTables {
    double dct[64];
    double quant[64];
};

__device__ __forceinline__ void load_exact_tables(ExactTables *t, const DevTables *__restrict__ dev) {
    for (int i = threadIdx.x; i < 128; i += blockDim.x)
        reinterpret_cast<double *>(t)[i] = i < 64 ? dev->dct[i] : dev->quant[i - 64];
    __syncthreads();
}

// A wave's own copy of the exact tables, without a workgroup barrier: each lane
// requests entries lane and 64 + lane (D and Q) with the wave's first pixel rows
// (wave_tables_load: their latency overlaps), and writes them to the wave's LDS copy
// once those rows have arrived (wave_tables_store, then wave_sync).  The
// workgroup-wide copy (load_exact_tables) is a global load, a vmcnt(0) and an
// s_barrier in front of every workgroup's first prefetch.
__device__ __forceinline__ void wave_tables_load(const DevTables *__restrict__ dev, int lane, double (&t)[2]) {
    t[0] = dev->dct[lane];
    t[1] = dev->quant[lane];
}
__device__ __forceinline__ void wave_tables_store(ExactTables *mine, int lane, const double (&t)[2]) {
    mine->dct[lane] = t[0];
    mine->quant[lane] = t[1];
}

// exact_from_rows() with the tables from LDS.
template <bool ADAPTIVE>
__device__ __forceinline__ int exact_from_rows_lds(const uint2 (&rows)[8], int c, const ExactTables *tab) {
    const int i = c >> 3, j = c & 7;
    double dj[8], di[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        dj[k] = tab->dct[j * 8 + k];  // D^T[k][j]
        di[k] = tab->dct[i * 8 + k];  // D[i][k]
    }
    double m = tab->quant[c];
    if (ADAPTIVE && c != 0) {
        uint32_t s1 = 0, s2 = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            s1 = __builtin_amdgcn_udot4(rows[k].x, 0x01010101u, s1, false);
            s1 = __builtin_amdgcn_udot4(rows[k].y, 0x01010101u, s1, false);
            s2 = __builtin_amdgcn_udot4(rows[k].x, rows[k].x, s2, false);
            s2 = __builtin_amdgcn_udot4(rows[k].y, rows[k].y, s2, false);
        }
        const int32_t sx = (int32_t)s1 - 8192;
        const int32_t sxx = (int32_t)s2 - 256 * (int32_t)s1 + 1048576;
        m = m * adaptive_scale(64 * sxx - sx * sx);
        if (m < 1.0) m = 1.0;
    }
    double out = 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const double t = row_sum(rows[k].x, rows[k].y, dj);
        out = k == 0 ? di[0] * t : out + di[k] * t;
    }
    return (int)round(exact_div(out, m));
}

// exact_from_rows_lds() for e <= 64 / G entries of one round, G = 8, 4 or 2 lanes
// per entry (lane = G * entry + part): each lane pulls R = 8 / G rows of the entry's
// block (rows part * R ..) from the owning lane and sums each in the reference's
// order (temp[k][j], src/dct.c:57-66); the group's first lane holds rows 0 .. R - 1
// and fetches the others' sums (ds_swizzle within the group), adding them in row
// order (src/dct.c:67-74); it stores round(out / M) (src/quantization.c:124) and
// returns 1 (its entry resolved).  Per round, against ~290 VALU for a pass of one
// entry per lane: ~100 (G = 8), ~125 (G = 4), ~190 (G = 2), so a pass of e entries
// takes the narrowest group that fits it in one round (resolve_ties_compact).
// Adaptive plans sum the block's variance terms over the group (group_add).
// Sum of v over the lane's group of G (ds_swizzle xor 1 .. G / 2 within 32 lanes).
template <int G>
__device__ __forceinline__ uint32_t group_add(uint32_t v) {
    if constexpr (G >= 2) v += (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (1 << 10));
    if constexpr (G >= 4) v += (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (2 << 10));
    if constexpr (G >= 8) v += (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (4 << 10));
    return v;
}

// out += D[i][q] * temp[q][j] for q = Q .. 7 in order: rows below R are the group
// leader's own, row q >= R comes from lane (lane & ~(G - 1)) + q / R (ds_swizzle
// bit mode: and_mask 0x1F & ~(G - 1), or_mask q / R).
template <int G, int Q>
__device__ __forceinline__ void group_sum(const double (&t)[8 / G], const double *di, double &out) {
    if constexpr (Q < 8) {
        constexpr int R = 8 / G;
        double tq;
        if constexpr (Q < R) {
            tq = t[Q];
        } else {
            constexpr int pat = (0x1F & ~(G - 1)) | ((Q / R) << 5);
            const uint64_t tb = __builtin_bit_cast(uint64_t, t[Q % R]);
            const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_swizzle((int)(uint32_t)tb, pat);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_swizzle((int)(uint32_t)(tb >> 32), pat);
            tq = __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
        }
        const double p = di[Q] * tq;
        out = Q == 0 ? p : out + p;
        group_sum<G, Q + 1>(t, di, out);
    }
}

template <int G, bool ADAPTIVE>
__device__ __forceinline__ uint32_t exact_grouped(const ExactTables *tab, const uint2 (&cur)[8], int16_t *st16,
                                                  const uint16_t *scr, int lane, uint32_t e) {
    constexpr int R = 8 / G;
    const int grp = lane / G, part = lane % G;
    const uint32_t ent = (uint32_t)grp < e ? (uint32_t)scr[grp] : 0u;
    const int src = (int)(ent >> 6), c = (int)(ent & 63u);
    uint32_t rx[R], ry[R];  // rows part * R + i of the entry's block
#pragma unroll
    for (int i = 0; i < R; ++i) rx[i] = ry[i] = 0u;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const uint32_t x = (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)cur[q].x);
        const uint32_t y = (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)cur[q].y);
        rx[q % R] = part == q / R ? x : rx[q % R];
        ry[q % R] = part == q / R ? y : ry[q % R];
    }
    const double *dj = tab->dct + (c & 7) * 8;  // D^T[l][j]
    double t[R];
    if constexpr (R == 1) {
        t[0] = row_sum(rx[0], ry[0], dj);
    } else {
        // the R sums side by side, l ascending in each (row_sum's order): one D^T[l][j]
        // live at a time
#pragma unroll
        for (int l = 0; l < 8; ++l) {
            const double d = dj[l];
#pragma unroll
            for (int i = 0; i < R; ++i) {
                const uint32_t w = l < 4 ? rx[i] : ry[i];
                const double p = ((double)((w >> (8 * (l & 3))) & 0xFFu) - 128.0) * d;
                t[i] = l == 0 ? p : t[i] + p;
            }
        }
    }
    // D[i][k] read only now: loaded with dj at the top (the compiler's choice) its 16
    // VGPRs were live across the row sums and the wide groups spilled
    int irow = (c >> 3) * 8;
    asm volatile("" : "+v"(irow), "+v"(t[0]));
    const double *di = tab->dct + irow;  // D[i][k]
    double out = 0.0;
    group_sum<G, 0>(t, di, out);
    double m = tab->quant[c];
    if (ADAPTIVE) {  // the block's exact variance from the group's rows (exact_from_rows_lds)
        uint32_t s1 = 0u, s2 = 0u;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            s1 = __builtin_amdgcn_udot4(ry[i], 0x01010101u, __builtin_amdgcn_udot4(rx[i], 0x01010101u, s1, false), false);
            s2 = __builtin_amdgcn_udot4(ry[i], ry[i], __builtin_amdgcn_udot4(rx[i], rx[i], s2, false), false);
        }
        s1 = group_add<G>(s1);
        s2 = group_add<G>(s2);
        if (c != 0) {
            const int32_t sx = (int32_t)s1 - 8192;
            const int32_t sxx = (int32_t)s2 - 256 * (int32_t)s1 + 1048576;
            m = m * adaptive_scale(64 * sxx - sx * sx);
            if (m < 1.0) m = 1.0;
        }
    }
    const double r = exact_div(out, m);
    if (part == 0 && (uint32_t)grp < e) {
        st16[src * (kPitch2 / 2) + c] = (int16_t)(int)round(r);
        return 1u;
    }
    return 0u;
}

// Phase 1: the forward of one 64-block batch into the stage plus the constant-
// block DC table; returns the lane's remaining tie flags (none for invalid lanes).
template <bool ADAPTIVE, bool VAR>
__device__ __forceinline__ void forward_flags_batch(const DevTables *__restrict__ dev, const uint2 (&cur)[8],
                                                    uint4 *stage, int lane, int wv, bool valid, int32_t &var_num,
                                                    uint32_t &mlo, uint32_t &mhi) {
    fdct8_compute<ADAPTIVE, VAR>(dev, cur, stage, lane, wv, mlo, mhi, var_num);
    flat_dc_fix(dev, cur, stage, lane, wv, mlo);
    if (!valid) mlo = mhi = 0;
}

// Phase 2 (after the prefetch fence): the batch's flagged coefficients resolved
// in place, compacted: every flagged (block, coefficient) becomes one entry, up
// to 64 entries per pass, one per lane (every lane busy; a loop in which each
// lane recomputes its own flags ran as many divergent fp64 passes as the busiest
// lane had flags).  The entry's lane fetches the block's pixel rows from the owning
// lane's registers (ds_bpermute: no LDS storage), computes the reference-order
// value (tables in LDS) and writes it into the stage.  `scr` = 64 uint16 of the
// wave's LDS (entry = coefficient | block lane << 6).  Call after the prefetch
// fence.  Returns the entries this lane resolved.
constexpr uint32_t kGroup8Max = 8u;  // GROUP8 passes with up to this many entries run in rounds of 8 lanes per entry
// WIDE (with GROUP8): bit 0 / bit 1 -- passes of 9..16 / 17..32 entries run as one round of
// 4 / 2 lanes per entry (exact_grouped) instead of one entry per lane.  Per kernel: the
// register-bound kernels (128 VGPRs at 4 waves/SIMD) spill with them.
template <bool ADAPTIVE, bool GROUP8 = false, int WIDE = 0>
__device__ __forceinline__ uint32_t resolve_ties_compact(const ExactTables *tab, const uint2 (&cur)[8], uint4 *stage,
                                                         uint16_t *scr, int lane, int wv, uint32_t &mlo,
                                                         uint32_t &mhi) {
    int16_t *st16 = reinterpret_cast<int16_t *>(stage) + wv * 64 * (kPitch2 / 2);
    uint32_t mine = 0;
    uint64_t has = __builtin_amdgcn_ballot_w64((mlo | mhi) != 0);
    while (has) {
        uint32_t e = 0;  // entries of this pass
        while (has && e + (uint32_t)__builtin_popcountll(has) <= 64u) {
            if (mlo | mhi) {
                const int c = pop_flag(mlo, mhi);
                const uint32_t pos =
                    e + __builtin_amdgcn_mbcnt_hi((uint32_t)(has >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)has, 0u));
                scr[pos] = (uint16_t)((uint32_t)c | ((uint32_t)lane << 6));
            }
            e += (uint32_t)__builtin_popcountll(has);
            has = __builtin_amdgcn_ballot_w64((mlo | mhi) != 0);
        }
        wave_sync();
        if constexpr (GROUP8) {
            if (e <= kGroup8Max) {  // wave-uniform: rounds of 8 entries (~100 VALU each, against ~290 for a pass)
                for (uint32_t e0 = 0; e0 < e; e0 += 8u)
                    mine += exact_grouped<8, ADAPTIVE>(tab, cur, st16, scr + e0, lane, e - e0 < 8u ? e - e0 : 8u);
                wave_sync();
                continue;
            }
            if ((WIDE & 1) && e <= 16u) {  // one round of 4 lanes per entry (~125 VALU)
                mine += exact_grouped<4, ADAPTIVE>(tab, cur, st16, scr, lane, e);
                wave_sync();
                continue;
            }
            if ((WIDE & 2) && e <= 32u) {  // one round of 2 lanes per entry (~190 VALU)
                mine += exact_grouped<2, ADAPTIVE>(tab, cur, st16, scr, lane, e);
                wave_sync();
                continue;
            }
        }
        const uint32_t ent = (uint32_t)lane < e ? (uint32_t)scr[lane] : 0u;
        const int src = (int)(ent >> 6);
        uint2 rows[8];  // the block's rows, from its owning lane (every lane takes part)
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            rows[r].x = (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)cur[r].x);
            rows[r].y = (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)cur[r].y);
        }
        if ((uint32_t)lane < e) {
            const int c = (int)(ent & 63u);
            st16[src * (kPitch2 / 2) + c] = (int16_t)exact_from_rows_lds<ADAPTIVE>(rows, c, tab);
            ++mine;
        }
        wave_sync();  // the next pass rewrites scr
    }
    return mine;
}

// The wave's stage as the 8 chunks of 1 KiB stores: chunk c, lane l = 16 B at
// byte 16 (64c + l) of the batch's 8 KiB (block (64c + l) / 8).
__device__ __forceinline__ void stage_chunks(const uint4 *stage, int wv, int lane, u4v (&val)[8]) {
    const uint2 *st64 = reinterpret_cast<const uint2 *>(stage) + wv * 64 * (kPitch2 / 8);
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const int m = c * 64 + lane;
        const int bl = m >> 3;
        const uint2 lo = st64[bl * (kPitch2 / 8) + (m & 7) * 2], hi = st64[bl * (kPitch2 / 8) + (m & 7) * 2 + 1];
        val[c] = u4v{lo.x, lo.y, hi.x, hi.y};
    }
}

// A batch's coefficient destination (plane k's output + its 64-block batch b, and the
// blocks it holds), resolved where it is called.  pin_sgpr pins the values in
// SGPRs there: without it LLVM re-issues their kernel-argument loads after the
// prefetch fence (an asm with a "memory" clobber), so a scalar-cache round trip sits
// between the rows' arrival and the stores of every batch.
struct BatchOut {
    char *base;   // output of block 0 of the batch
    int32_t *var; // var_num of block 0 of the batch (if the plane set has var_num outputs)
    uint32_t nb;  // valid blocks in the batch
};
__device__ __forceinline__ BatchOut batch_out(const PlaneSet &ps, int k, uint32_t b) {
    const uint32_t left = (uint32_t)ps.pl[k].nblk - b * 64;
    BatchOut o;
    o.nb = left < 64u ? left : 64u;
    o.base = reinterpret_cast<char *>(ps.coef[k]) + (size_t)b * 64 * 128;
    o.var = ps.var[k] ? ps.var[k] + (size_t)b * 64 : nullptr;
    asm volatile("" : "+s"(o.nb), "+s"(o.base), "+s"(o.var));
    return o;
}

// vmcnt(0): the wave's stores have read their data VGPRs (and left the CU).
__device__ __forceinline__ void retire_stores() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// Rows of global batch gn.  Past the end (a wave's last batch), SKIP loads
// nothing: the rows would be unused, and with the grid 8x the resident one every
// wave pays that tail once (forward -0.3 to -7 %, q100 most; the fused round trip
// measured +1 % and keeps the load of the last plane's block 0:
// profiles/r02/grid_mult_ab.log).
template <bool SKIP = true, bool BUF = true>
__device__ __forceinline__ void prefetch_batch(const PlaneSet &ps, uint32_t gn, int lane, uint2 (&nxt)[8]) {
    if (SKIP && gn >= ps.first[ps.n]) return;  // wave-uniform
    const int kn = plane_of(ps, gn);
    load_rows<BUF>(ps.pl[kn], (gn - first_of(ps, kn)) * 64 + lane, nxt);
}

}  // namespace dctq
