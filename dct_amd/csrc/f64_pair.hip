// dct_amd/csrc/f64_pair.hip -- the fp64 kernels of the batched API, paired-lane layout:
//   * fdct8_float_pair: dctq_forward_float -- dct_forward (src/dct.c:52-77) of
//     every block, float out, |err| <= 1e-4 (fp64 AAN, one rounding to fp32).
//   * idct8_pair<ADAPTIVE>: dctq_inverse -- dequantize (src/quantization.c:133-151,
//     incl. the non-adaptive 1/Q multiplier) + dct_inverse (src/dct.c:80-105) + 128.
//
// Why paired lanes (DESIGN.md "Kernels"): a whole 8x8 block in fp64 is 128
// VGPRs, which leaves no room for a prefetch buffer, a 4-waves/SIMD
// occupancy or an LDS-staged store.  Here block j of a 32-block batch lives
// in lanes j and j+32, half each (32 doubles = 64 VGPRs).  The pass along the
// lane's own half runs locally; v_permlane32_swap_b32 then exchanges the 2x2
// (register x half-wave) tiles so each lane holds 4 complete lines in natural
// order for the other pass -- no lane-parity selects, the same code in every
// lane.  Per-slot AAN scales are wave-uniform (S_c before the swap, S_u after).
//
// Memory structure as in fdct8.hip v2: persistent grid-stride loop, next
// batch's inputs prefetched into registers, outputs staged through LDS and
// written as 1 KiB-contiguous non-temporal buffer stores.  The LDS read-back
// comes after the fence that retires the previous batch's stores (a store may
// still be reading its data VGPRs; LDS returns are not ordered after that).
#include "pair_core.h"


namespace dctq {

__device__ __forceinline__ const uint8_t *pixel_block(const PlaneArgs &p, uint32_t n) {
    uint32_t f = fdiv(n, p.div_frame);
    uint32_t rem = n - f * (uint32_t)p.nblk_frame;
    uint32_t by = fdiv(rem, p.div_bw);
    uint32_t bx = rem - by * (uint32_t)p.bw;
    return p.src + (long long)f * p.frame_stride + (long long)(by * 8) * p.stride + (long long)bx * 8;
}

// Rows 4h..4h+3 of block n (past the end: block 0), non-temporal.
__device__ __forceinline__ void load_half_rows(const PlaneArgs &p, uint32_t n, int h, uint2 (&rows)[4]) {
    const uint8_t *px = pixel_block(p, n < (uint32_t)p.nblk ? n : 0) + (long long)(4 * h) * p.stride;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const u2p t = __builtin_nontemporal_load(reinterpret_cast<const u2p *>(px + r * p.stride));
        rows[r] = make_uint2(t.x, t.y);
    }
}

__global__ __launch_bounds__(kThreadsP, 4) void fdct8_float_pair(PlaneArgs p, const DevTables *__restrict__ dev,
                                                                float *__restrict__ coef) {
    __shared__ uint4 stage[kWavesP * 32 * kPitchP / 16];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5, j = lane & 31;
    const uint32_t nbatch = ((uint32_t)p.nblk + 31u) >> 5;
    const uint32_t step = gridDim.x * kWavesP;
    uint32_t b = blockIdx.x * kWavesP + wv;
    uint2 nxt[4];
    load_half_rows(p, b * 32 + j, h, nxt);
    asm volatile("" : "+v"(nxt[0]), "+v"(nxt[1]), "+v"(nxt[2]), "+v"(nxt[3])::"memory");
    for (; b < nbatch; b += step) {
        uint2 cur[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) cur[r] = nxt[r];
        load_half_rows(p, (b + step) * 32 + j, h, nxt);

        // centred pixels, exactly: (byte ^ 0x80) as int8 == byte - 128
        double v[4][8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t w0 = cur[r].x ^ 0x80808080u, w1 = cur[r].y ^ 0x80808080u;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                v[r][k] = (double)(int)(int8_t)(w0 >> (8 * k));
                v[r][k + 4] = (double)(int)(int8_t)(w1 >> (8 * k));
            }
        }
        ConstTables *tp = tables(dev);
        // row pass (own rows), x S_c (slot c is column frequency c in every lane)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            aan8_d(v[r][0], v[r][1], v[r][2], v[r][3], v[r][4], v[r][5], v[r][6], v[r][7]);
#pragma unroll
            for (int c = 0; c < 8; ++c) v[r][c] *= tp->s1[c];
        }
        transpose_halves(v);
        // column pass (own columns 4h+k), x S_u (slot [u][k] = u, [u-4][k+4] = u)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            aan8_d(v[0][k], v[1][k], v[2][k], v[3][k], v[0][k + 4], v[1][k + 4], v[2][k + 4], v[3][k + 4]);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                v[u][k] *= tp->s1[u];
                v[u][k + 4] *= tp->s1[u + 4];
            }
        }
        // stage: row u of the block = 8 floats; this lane owns floats 4h..4h+3
        char *mine = reinterpret_cast<char *>(stage) + (wv * 32 + j) * kPitchP + h * 16;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int r = u & 3, o = (u >> 2) * 4;
            *reinterpret_cast<float4 *>(mine + u * 32) =
                make_float4((float)v[r][o], (float)v[r][o + 1], (float)v[r][o + 2], (float)v[r][o + 3]);
        }
        // retire the previous batch's stores (with this prefetch) before reading the stage back
        asm volatile("" : "+v"(nxt[0]), "+v"(nxt[1]), "+v"(nxt[2]), "+v"(nxt[3])::"memory");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t left = (uint32_t)p.nblk - b * 32;
        store_stage(stage, wv, lane, reinterpret_cast<char *>(coef) + (size_t)b * 32 * 256,
                    (left < 32u ? left : 32u) * 256u);
    }
}

// Consume prefetched rows (forces the wait for their loads -- and so for every
// older store -- at this point; see fdct8.hip v2).
__device__ __forceinline__ void fence_rows(uint4 (&r)[4], int32_t &vn) {
    asm volatile("" : "+v"(r[0].x), "+v"(r[0].y), "+v"(r[0].z), "+v"(r[0].w), "+v"(r[1].x), "+v"(r[1].y),
                 "+v"(r[1].z), "+v"(r[1].w), "+v"(r[2].x), "+v"(r[2].y), "+v"(r[2].z), "+v"(r[2].w), "+v"(r[3].x),
                 "+v"(r[3].y), "+v"(r[3].z), "+v"(r[3].w), "+v"(vn)::"memory");
}

// Coefficient rows 4h..4h+3 of block n (16 B each) + its variance numerator.
template <bool ADAPTIVE>
__device__ __forceinline__ void load_half_coefs(const int16_t *coef, const int32_t *var_num, long long nblk,
                                                uint32_t n, int h, uint4 (&rows)[4], int32_t &vn) {
    const uint32_t m = (long long)n < nblk ? n : 0;
    const uint4 *src = reinterpret_cast<const uint4 *>(coef + (size_t)m * 64) + 4 * h;
#pragma unroll
    for (int r = 0; r < 4; ++r) rows[r] = src[r];
    if (ADAPTIVE) vn = var_num[m];
}

template <bool ADAPTIVE>
__global__ __launch_bounds__(kThreadsP, 4) void idct8_pair(const DevTables *__restrict__ dev,
                                                          const int16_t *__restrict__ coef,
                                                          const int32_t *__restrict__ var_num, long long nblk,
                                                          float *__restrict__ recon) {
    __shared__ uint4 stage[kWavesP * 32 * kPitchP / 16];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5, j = lane & 31;
    const uint32_t nbatch = (uint32_t)((nblk + 31) >> 5);
    const uint32_t step = gridDim.x * kWavesP;
    uint32_t b = blockIdx.x * kWavesP + wv;
    uint4 nxt[4];
    int32_t nvn = 0;
    load_half_coefs<ADAPTIVE>(coef, var_num, nblk, b * 32 + j, h, nxt, nvn);
    fence_rows(nxt, nvn);
    for (; b < nbatch; b += step) {
        uint4 cur[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) cur[r] = nxt[r];
        const int32_t vn = nvn;
        load_half_coefs<ADAPTIVE>(coef, var_num, nblk, (b + step) * 32 + j, h, nxt, nvn);

        double v[4][8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t w[4] = {cur[r].x, cur[r].y, cur[r].z, cur[r].w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                v[r][2 * k] = (double)(int)(int16_t)(w[k] & 0xFFFFu);
                v[r][2 * k + 1] = (double)((int)w[k] >> 16);
            }
        }
        // dequantize, folded with the A^T input scale S_u S_c (DevTables iscale /
        // qscale): the table row is u = 4h + r, i.e. it differs between the two
        // half-waves -- see half_wave_scale
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
        // column pass over u (own columns), then rows
#pragma unroll
        for (int k = 0; k < 4; ++k)
            aan8t_d(v[0][k], v[1][k], v[2][k], v[3][k], v[0][k + 4], v[1][k + 4], v[2][k + 4], v[3][k + 4]);
        transpose_halves(v);
#pragma unroll
        for (int r = 0; r < 4; ++r) aan8t_d(v[r][0], v[r][1], v[r][2], v[r][3], v[r][4], v[r][5], v[r][6], v[r][7]);
        // stage: this lane owns rows 4h..4h+3 (32 B each) of block j
        char *mine = reinterpret_cast<char *>(stage) + (wv * 32 + j) * kPitchP + h * 128;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            *reinterpret_cast<float4 *>(mine + r * 32) = make_float4(
                (float)v[r][0], (float)v[r][1], (float)v[r][2], (float)v[r][3]);
            *reinterpret_cast<float4 *>(mine + r * 32 + 16) = make_float4(
                (float)v[r][4], (float)v[r][5], (float)v[r][6], (float)v[r][7]);
        }
        fence_rows(nxt, nvn);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const long long left = nblk - (long long)b * 32;
        store_stage(stage, wv, lane, reinterpret_cast<char *>(recon) + (size_t)b * 32 * 256,
                    (uint32_t)(left < 32 ? left : 32) * 256u);
    }
}

// Both paired kernels launch up to 64 x their resident workgroups (about one 32-block batch per
// wave on 4K-frame stacks): round 6, tools/pair_ab.py, three passes, 64 4K frames: dctq_inverse
// -1.2..-3.7 % and dctq_forward_float -4.2..-4.7 % against 8 x (32 x / 48 x in between; 16 x made
// the forward 4-5 % slower), profiles/r06/pair_grid_ab/.
constexpr int kPairGridMult = 64;

template <typename K, typename... A>
static hipError_t launch_persistent(K kernel, long long nblk, int num_cus, hipStream_t stream, A... args) {
    const int per_cu = resident_per_cu(kernel, kThreadsP);
    const long long nbatch = (nblk + 31) / 32;
    const long long want = (nbatch + kWavesP - 1) / kWavesP;
    const long long cap = (long long)num_cus * per_cu * kPairGridMult;
    hipLaunchKernelGGL(kernel, dim3((unsigned)(want < cap ? want : cap)), dim3(kThreadsP), 0, stream, args...);
    return hipGetLastError();
}

hipError_t launch_fdct8_float_pair(const PlaneArgs &p, const DevTables *dev, float *coef, hipStream_t stream,
                                   int num_cus) {
    return launch_persistent(fdct8_float_pair, p.nblk, num_cus, stream, p, dev, coef);
}

hipError_t launch_idct8_pair(const DevTables *dev, int adaptive, const int16_t *coef, const int32_t *var_num,
                             long long nblk, float *recon, hipStream_t stream, int num_cus) {
    if (adaptive) return launch_persistent(idct8_pair<true>, nblk, num_cus, stream, dev, coef, var_num, nblk, recon);
    return launch_persistent(idct8_pair<false>, nblk, num_cus, stream, dev, coef, var_num, nblk, recon);
}

}  // namespace dctq
