// dct_amd/csrc/pair_core.h -- paired-lane fp64 helpers (block j of a 32-block
// batch in lanes j and j+32, half each), shared by f64_pair.hip and the fused
// round trip (roundtrip.hip).  Layout rationale: f64_pair.hip header.
#pragma once
#include "aan_f64.h"
#include "dctq_internal.h"

namespace dctq {

constexpr int kWavesP = 4;
constexpr int kThreadsP = 64 * kWavesP;
constexpr int kPitchP = 272;          // bytes per block in the stage: 256 + 16 (b128 writes spread over the banks)
constexpr int kRtOcc = 4;             // the fused round trip's waves per SIMD (launch bound)
// ... and its grid multiplier: 32 x the resident workgroups (round 6, tools/rt_ab.py, interleaved,
// both orders: 8 x +3.0..+3.5 %, 16 x +2.2..+2.4 %, 24 x +1.3..+1.4 %, 48 x -0.6..-1.1 %, 64 x +1.2 %
// against 32 x; profiles/r06/rt_grid_ab/)
constexpr int kRtGridMult = 32;

typedef uint32_t u2p __attribute__((ext_vector_type(2)));
typedef uint32_t u4p __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(4))) DevTables ConstTables;
typedef const __attribute__((address_space(4))) double ConstDouble;

// Lanes 0-31 keep x and receive lane+32's x in y; lanes 32-63 receive lane-32's
// y in x and keep y (measured semantics, tools/ubench/permlane.hip).
__device__ __forceinline__ void swap_halves(double &x, double &y) {
    const uint64_t xb = (uint64_t)__double_as_longlong(x), yb = (uint64_t)__double_as_longlong(y);
    const auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)xb, (uint32_t)yb, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)(xb >> 32), (uint32_t)(yb >> 32), false, false);
    x = __longlong_as_double((long long)(((uint64_t)hi[0] << 32) | lo[0]));
    y = __longlong_as_double((long long)(((uint64_t)hi[1] << 32) | lo[1]));
}

// Row layout (lane holds rows 4h..4h+3, all columns) <-> column layout (lane
// holds columns 4h..4h+3, all rows): slot [r][k] / [r][k+4] = line k, entries r / r+4.
__device__ __forceinline__ void transpose_halves(double (&v)[4][8]) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int k = 0; k < 4; ++k) swap_halves(v[r][k], v[r][k + 4]);
}

// Opaque per-batch table pointer in the constant address space: scalar loads
// that stay in the loop (hoisted they would need >100 live SGPRs).
__device__ __forceinline__ ConstTables *tables(const DevTables *dev) {
    asm volatile("" : "+s"(dev));
    return (ConstTables *)dev;
}

// v[c] *= lo[c] in lanes 0-31 and *= hi[c] in lanes 32-63, with both tables in
// SGPRs: two exec-masked v_mul_f64 per value and no VGPR temporaries (selecting
// the factor per lane needs 4 VGPRs per value in flight, which spilled).  The
// wave is fully active here; exec is saved and restored inside the block.
// (Operand numbering: %0-%7 the values, %8 the exec save, %9-%16 lo, %17-%24 hi.)
__device__ __forceinline__ void half_wave_scale(double (&v)[8], ConstDouble *lo, ConstDouble *hi) {
    uint64_t save;
    asm volatile(
        "s_mov_b64 %[sv], exec\n\t"
        "s_mov_b32 exec_hi, 0\n\t"
        "v_mul_f64 %0, %0, %9\n\tv_mul_f64 %1, %1, %10\n\tv_mul_f64 %2, %2, %11\n\tv_mul_f64 %3, %3, %12\n\t"
        "v_mul_f64 %4, %4, %13\n\tv_mul_f64 %5, %5, %14\n\tv_mul_f64 %6, %6, %15\n\tv_mul_f64 %7, %7, %16\n\t"
        "s_mov_b64 exec, %[sv]\n\t"
        "s_mov_b32 exec_lo, 0\n\t"
        "v_mul_f64 %0, %0, %17\n\tv_mul_f64 %1, %1, %18\n\tv_mul_f64 %2, %2, %19\n\tv_mul_f64 %3, %3, %20\n\t"
        "v_mul_f64 %4, %4, %21\n\tv_mul_f64 %5, %5, %22\n\tv_mul_f64 %6, %6, %23\n\tv_mul_f64 %7, %7, %24\n\t"
        "s_mov_b64 exec, %[sv]\n\t"
        "s_nop 1"  // VALU write -> v_permlane32_swap read (transpose_halves): 2 wait states, ours to pad
        : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]),
          [sv] "=&s"(save)
        : "s"(lo[0]), "s"(lo[1]), "s"(lo[2]), "s"(lo[3]), "s"(lo[4]), "s"(lo[5]), "s"(lo[6]), "s"(lo[7]),
          "s"(hi[0]), "s"(hi[1]), "s"(hi[2]), "s"(hi[3]), "s"(hi[4]), "s"(hi[5]), "s"(hi[6]), "s"(hi[7]));
}

// Stage chunk k of the wave's 8 KiB (blocks 4k..4k+3, 16 B per lane) -> registers ...
__device__ __forceinline__ void stage_load(const uint4 *stage, int wv, int lane, u4p (&val)[8]) {
    const char *base = reinterpret_cast<const char *>(stage) + wv * 32 * kPitchP;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int bl = 4 * k + (lane >> 4);
        const uint4 t = *reinterpret_cast<const uint4 *>(base + bl * kPitchP + (lane & 15) * 16);
        val[k] = u4p{t.x, t.y, t.z, t.w};
    }
}
// ... -> HBM as 8 1 KiB stores.  dst and nbytes are wave-uniform; readfirstlane says so
// to the compiler, which otherwise may keep them in VGPRs under SGPR pressure and wrap
// every store in a waterfall loop (the fused round trip's second half did).
__device__ __forceinline__ void stage_store(const u4p (&val)[8], int lane, char *dst, uint32_t nbytes) {
    const uint64_t d = reinterpret_cast<uint64_t>(dst);
    // __builtin_amdgcn_readfirstlane returns int: each half goes back through uint32_t,
    // or the low half is sign-extended into the high one (an address with bit 31 set
    // became 0xFFFFFFFF'xxxxxxxx -- the round-5 device faults, profiles/r05/INDEX.md)
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(d >> 32));
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)d);
    dst = reinterpret_cast<char *>(((uint64_t)hi << 32) | (uint64_t)lo);
    nbytes = (uint32_t)__builtin_amdgcn_readfirstlane(nbytes);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, (short)0, (int)nbytes, 0x00020000);
#pragma unroll
    for (int k = 0; k < 8; ++k) __builtin_amdgcn_raw_buffer_store_b128(val[k], rs, lane * 16, k * 1024, kNtAux);
}
__device__ __forceinline__ void store_stage(const uint4 *stage, int wv, int lane, char *dst, uint32_t nbytes) {
    u4p val[8];
    stage_load(stage, wv, lane, val);
    stage_store(val, lane, dst, nbytes);
}

}  // namespace dctq
