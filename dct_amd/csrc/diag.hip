// dct_amd/csrc/diag.hip -- the diagnostic entry points of libdct_amd_diag.so
// (dctq_diag.h): kernel selection for tests, the forward kernel's movement
// ceiling, the hardware ceilings of its traffic mix, and host-only table
// introspection.  Linked into the diagnostic library only; libdct_amd.so (the
// product) neither contains nor exports any of it.
#include <string.h>

#include "dctq_diag.h"
#include "fdct8_bound.h"
#include "host_tables.h"
#include "plan.h"

namespace dctq {
namespace {

typedef unsigned int u4v __attribute__((ext_vector_type(4)));
typedef unsigned int u2v2 __attribute__((ext_vector_type(2)));

// Flat 1:2 stream (profiles/r02/hbm_ceilings.md "s12"): wave-batch b reads
// src[4 KiB * b, +4 KiB) with 4 x 16-B-per-lane loads and writes
// dst[8 KiB * b, +8 KiB) with 8 x 1 KiB stores.  AUX = store policy.
template <int AUX>
__global__ __launch_bounds__(256) void stream12(const u4v *__restrict__ src, char *__restrict__ dst, uint32_t nb) {
    const int lane = threadIdx.x & 63;
    for (uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6); b < nb; b += gridDim.x * 4) {
        u4v v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = __builtin_nontemporal_load(src + (size_t)b * 256 + k * 64 + lane);
        const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(dst + (size_t)b * 8192, 0, 8192, 0x00020000);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            __builtin_amdgcn_raw_buffer_store_b128(v[k], rc, lane * 16, k * 1024, AUX);
            __builtin_amdgcn_raw_buffer_store_b128(v[k] ^ u4v{1, 0, 0, 0}, rc, lane * 16, (k + 4) * 1024, AUX);
        }
    }
}

// Flat 1:2:4 stream (the fused round trip's 64 B in : 128 + 256 B out): wave-batch
// b reads src[4 KiB * b, +4 KiB) and writes dst[24 KiB * b, +24 KiB), nt stores.
__global__ __launch_bounds__(256) void stream124(const u4v *__restrict__ src, char *__restrict__ dst, uint32_t nb) {
    const int lane = threadIdx.x & 63;
    for (uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6); b < nb; b += gridDim.x * 4) {
        u4v v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = __builtin_nontemporal_load(src + (size_t)b * 256 + k * 64 + lane);
        const __amdgpu_buffer_rsrc_t rc =
            __builtin_amdgcn_make_buffer_rsrc(dst + (size_t)b * 24576, 0, 24576, 0x00020000);
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int m = 0; m < 6; ++m)
                __builtin_amdgcn_raw_buffer_store_b128(v[k] ^ u4v{(unsigned)m, 0, 0, 0}, rc, lane * 16,
                                                       (k * 6 + m) * 1024, 2);
    }
}

// The flat 1:2:4 stream in the fused round trip's OUTPUT layout (round 6): the 8 KiB of a batch's
// coefficients go to region A (dst[8 KiB * b]) and its 16 KiB of recon to region B (dst[8 KiB * nb
// + 16 KiB * b]), two separate arrays as the API has them.  GROUPS: the stores leave in the round
// trip's three 8 KiB groups with a vmcnt(0) drain before each of the last two (its LDS read-backs).
template <bool GROUPS>
__global__ __launch_bounds__(256) void stream124_split(const u4v *__restrict__ src, char *__restrict__ dst,
                                                       uint32_t nb) {
    const int lane = threadIdx.x & 63;
    for (uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6); b < nb; b += gridDim.x * 4) {
        u4v v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = __builtin_nontemporal_load(src + (size_t)b * 256 + k * 64 + lane);
        const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(dst + (size_t)b * 8192, 0, 8192, 0x00020000);
        const __amdgpu_buffer_rsrc_t rb =
            __builtin_amdgcn_make_buffer_rsrc(dst + (size_t)nb * 8192 + (size_t)b * 16384, 0, 16384, 0x00020000);
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int m = 0; m < 2; ++m)
                __builtin_amdgcn_raw_buffer_store_b128(v[k] ^ u4v{(unsigned)m, 0, 0, 0}, ra, lane * 16,
                                                       (k * 2 + m) * 1024, 2);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (GROUPS) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), as before the round trip's read-backs
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int m = 0; m < 2; ++m)
                    __builtin_amdgcn_raw_buffer_store_b128(v[k] ^ u4v{(unsigned)(2 + 2 * h + m), 0, 0, 0}, rb,
                                                           lane * 16, (h * 8 + k * 2 + m) * 1024, 2);
        }
    }
}

// stream124_split<true> with the round trip's READ shape: each lane loads its block's
// 8 pixel rows as 8-byte non-temporal buffer loads.  W = 0: the 64 blocks of a batch
// are contiguous 512-B row slices (lane-contiguous, only the load width differs from
// kind 9); W = 3840: blocks of a 3840-px-wide plane (480 blocks per block row, a batch
// may straddle two block rows), the luma plane's pattern.  Blocks past the last whole
// block row wrap to the start (same bytes moved).
// MAP: which batches a wave takes.  0: grid-stride (batch blockIdx * 4 + wave, then
// + grid * 4: the product kernels' order); 1: workgroup-contiguous (workgroup i
// sweeps batches [i K, (i + 1) K) with its 4 waves side by side); 2: wave-contiguous
// (each wave sweeps its own run of consecutive batches).
template <int W, int MAP = 0>
__global__ __launch_bounds__(256) void stream124_rows(const uint8_t *__restrict__ src, char *__restrict__ dst,
                                                      uint32_t nb) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(src), (short)0, (int)(nb * 4096u), 0x00020000);
    constexpr uint32_t kBpr = W ? W / 8 : 64;  // blocks per block row
    const uint32_t nfull = W ? nb * 64u / kBpr * kBpr : nb * 64u;
    const uint32_t nwg = gridDim.x, kwg = (nb + nwg - 1) / nwg, kw = (nb + nwg * 4 - 1) / (nwg * 4);
    const uint32_t b0 = MAP == 0 ? blockIdx.x * 4 + wv : MAP == 1 ? blockIdx.x * kwg + wv : (blockIdx.x * 4 + wv) * kw;
    const uint32_t b1 = MAP == 0 ? nb : MAP == 1 ? min(nb, (blockIdx.x + 1) * kwg) : min(nb, b0 + kw);
    const uint32_t bs = MAP == 0 ? nwg * 4 : MAP == 1 ? 4u : 1u;
    for (uint32_t b = b0; b < b1; b += bs) {
        const uint32_t n = (b * 64u + (uint32_t)lane) % nfull;
        const uint32_t off = W ? (n / kBpr) * 8u * W + (n % kBpr) * 8u : (n >> 6) * 4096u + (n & 63u) * 8u;
        const uint32_t st = W ? (uint32_t)W : 512u;
        u2v2 r[8];
#pragma unroll
        for (int y = 0; y < 8; ++y) r[y] = __builtin_amdgcn_raw_buffer_load_b64(rs, off + y * st, 0, 2);
        u4v v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = u4v{r[2 * k].x, r[2 * k].y, r[2 * k + 1].x, r[2 * k + 1].y};
        const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(dst + (size_t)b * 8192, 0, 8192, 0x00020000);
        const __amdgpu_buffer_rsrc_t rb =
            __builtin_amdgcn_make_buffer_rsrc(dst + (size_t)nb * 8192 + (size_t)b * 16384, 0, 16384, 0x00020000);
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int m = 0; m < 2; ++m)
                __builtin_amdgcn_raw_buffer_store_b128(v[k] ^ u4v{(unsigned)m, 0, 0, 0}, ra, lane * 16,
                                                       (k * 2 + m) * 1024, 2);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int m = 0; m < 2; ++m)
                    __builtin_amdgcn_raw_buffer_store_b128(v[k] ^ u4v{(unsigned)(2 + 2 * h + m), 0, 0, 0}, rb,
                                                           lane * 16, (h * 8 + k * 2 + m) * 1024, 2);
        }
    }
}

// Kind 11 with 16-byte loads: per instruction k the wave reads rows 2k (lanes 0-31) and
// 2k + 1 (lanes 32-63) of the batch's 64 blocks, two blocks' row slices per lane (4 loads
// per batch instead of 8; a lane-per-block kernel would need a cross-lane exchange after).
__global__ __launch_bounds__(256) void stream124_rows16(const uint8_t *__restrict__ src, char *__restrict__ dst,
                                                        uint32_t nb) {
    constexpr uint32_t kW = 3840, kBpr = kW / 8;
    const int lane = threadIdx.x & 63;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(src), (short)0, (int)(nb * 4096u), 0x00020000);
    const uint32_t nfull = nb * 64u / kBpr * kBpr;
    for (uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6); b < nb; b += gridDim.x * 4) {
        const uint32_t n = (b * 64u + 2u * (uint32_t)(lane & 31)) % nfull;
        const uint32_t off = (n / kBpr) * 8u * kW + (n % kBpr) * 8u + (uint32_t)(lane >> 5) * kW;
        u4v v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 2 * k * kW, 0, 2);
        const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(dst + (size_t)b * 8192, 0, 8192, 0x00020000);
        const __amdgpu_buffer_rsrc_t rb =
            __builtin_amdgcn_make_buffer_rsrc(dst + (size_t)nb * 8192 + (size_t)b * 16384, 0, 16384, 0x00020000);
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int m = 0; m < 2; ++m)
                __builtin_amdgcn_raw_buffer_store_b128(v[k] ^ u4v{(unsigned)m, 0, 0, 0}, ra, lane * 16,
                                                       (k * 2 + m) * 1024, 2);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int m = 0; m < 2; ++m)
                    __builtin_amdgcn_raw_buffer_store_b128(v[k] ^ u4v{(unsigned)(2 + 2 * h + m), 0, 0, 0}, rb,
                                                           lane * 16, (h * 8 + k * 2 + m) * 1024, 2);
        }
    }
}

// Kind 7 (the flat 1:2 stream on a 32x grid, one batch per wave) with the forward's READ
// shape: each lane loads its block's 8 rows as 8-byte non-temporal buffer loads from a
// 3840-px-wide plane (480 blocks per block row; blocks past the last whole block row wrap).
__global__ __launch_bounds__(256) void stream12_plane(const uint8_t *__restrict__ src, char *__restrict__ dst,
                                                      uint32_t nb) {
    constexpr uint32_t kW = 3840, kBpr = kW / 8;
    const int lane = threadIdx.x & 63;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(src), (short)0, (int)(nb * 4096u), 0x00020000);
    const uint32_t nfull = nb * 64u / kBpr * kBpr;
    for (uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6); b < nb; b += gridDim.x * 4) {
        const uint32_t n = (b * 64u + (uint32_t)lane) % nfull;
        const uint32_t off = (n / kBpr) * 8u * kW + (n % kBpr) * 8u;
        u2v2 r[8];
#pragma unroll
        for (int y = 0; y < 8; ++y) r[y] = __builtin_amdgcn_raw_buffer_load_b64(rs, off + y * kW, 0, 2);
        const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(dst + (size_t)b * 8192, 0, 8192, 0x00020000);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const u4v v = u4v{r[2 * k].x, r[2 * k].y, r[2 * k + 1].x, r[2 * k + 1].y};
            __builtin_amdgcn_raw_buffer_store_b128(v, rc, lane * 16, k * 1024, 2);
            __builtin_amdgcn_raw_buffer_store_b128(v ^ u4v{1, 0, 0, 0}, rc, lane * 16, (k + 4) * 1024, 2);
        }
    }
}

// read-only: 4 x 16 B per thread, xor-reduced (the store never happens)
__global__ __launch_bounds__(256) void stream_read(const u4v *__restrict__ src, u4v *__restrict__ sink, size_t n16) {
    const size_t base = (size_t)blockIdx.x * 1024 + threadIdx.x;
    u4v acc = {0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < 4; ++u)
        if (base + u * 256 < n16) acc ^= __builtin_nontemporal_load(src + base + u * 256);
    if (acc.x == 0x12345678u && acc.y == 0x9abcdef0u && acc.z == 0x0fedcba9u) sink[0] = acc;
}

template <bool NT>
__global__ __launch_bounds__(256) void stream_write(u4v *__restrict__ dst, size_t n16) {
    const size_t base = (size_t)blockIdx.x * 1024 + threadIdx.x;
#pragma unroll
    for (int u = 0; u < 4; ++u)
        if (base + u * 256 < n16) {
            const u4v v = u4v{(unsigned)base, (unsigned)u, 7u, 9u};
            if (NT) __builtin_nontemporal_store(v, dst + base + u * 256);
            else dst[base + u * 256] = v;
        }
}

int device_cus() {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1) return 256;
    return n;
}

}  // namespace
}  // namespace dctq

extern "C" {

int dctq_diag_plan_set_variant(dctq_plan *plan, int variant) {
    DCTQ_ENTRY;
    if (!plan) return dctq::fail(DCTQ_EINVAL, "plan is NULL");
    if (variant < 1 || variant > 4) return dctq::fail(DCTQ_EINVAL, "variant must be 1..4");
    plan->variant = variant;
    return DCTQ_OK;
}

int dctq_diag_plan_set_inverse(dctq_plan *plan, int mode) {
    DCTQ_ENTRY;
    if (!plan) return dctq::fail(DCTQ_EINVAL, "plan is NULL");
    if (mode != 0 && mode != 1) return dctq::fail(DCTQ_EINVAL, "mode must be 0 (fp64) or 1 (the plan's own choice)");
    plan->inv_f32 = mode == 1 && !plan->adaptive && plan->inv_bound <= kInvTolDiag;
    return DCTQ_OK;
}

double dctq_debug_inverse_bound(int quality, int adaptive, int *admitted) {
    dctq::DevTables t;
    dctq_host::dct_matrix(8, t.dct);
    dctq_host::quant_matrix(8, dctq_host::clamp_quality(quality), t.quant);
    for (int c = 0; c < 64; ++c) {
        t.dequant[c] = 1.0 / t.quant[c];
        t.s2[c] = kAanScale[c >> 3] * kAanScale[c & 7];
    }
    const double b = dctq::inverse_f32_bound(t);
    if (admitted) *admitted = !adaptive && b <= kInvTolDiag;
    return b;
}

int dctq_diag_legacy_lanes(int *made, int *pooled) {
    if (!made || !pooled) return dctq::fail(DCTQ_EINVAL, "NULL pointer");
    dctq::legacy_lane_counts(made, pooled);
    return DCTQ_OK;
}

int dctq_debug_symbol_bytes(int quality, int adaptive) {
    (void)adaptive;  // adaptive divisors Q (2 - nv) >= Q: the same bound
    dctq::DevTables t;
    dctq_host::dct_matrix(8, t.dct);
    dctq_host::quant_matrix(8, dctq_host::clamp_quality(quality), t.quant);
    return dctq::max_abs_quantized(t) <= 511 ? 2 : 4;
}

int dctq_diag_plan_set_num_cus(dctq_plan *plan, int num_cus) {
    DCTQ_ENTRY;
    if (!plan) return dctq::fail(DCTQ_EINVAL, "plan is NULL");
    if (num_cus < 1 || num_cus > 4096) return dctq::fail(DCTQ_EINVAL, "num_cus must be 1..4096");
    plan->num_cus = num_cus;
    return DCTQ_OK;
}

int dctq_diag_movement_planes(const dctq_plan *plan, const dctq_plane *planes, int nplanes, int16_t *const *coef,
                              void *stream) {
    DCTQ_ENTRY;
    if (int rc = dctq::check_plan(plan)) return rc;
    dctq::PlaneSet ps;
    if (int rc = dctq::plane_set(planes, nplanes, coef, nullptr, &ps)) return rc;
    HIPCHK(dctq::launch_fdct8_movement(ps, plan->dev, (hipStream_t)stream, plan->num_cus, 3), "fdct8_movement launch");
    return DCTQ_OK;
}

int dctq_diag_movement_grid_planes(const dctq_plan *plan, const dctq_plane *planes, int nplanes, int16_t *const *coef,
                                   int grid_mult, void *stream) {
    DCTQ_ENTRY;
    if (int rc = dctq::check_plan(plan)) return rc;
    if (grid_mult < 1 || grid_mult > 64) return dctq::fail(DCTQ_EINVAL, "grid_mult must be 1..64");
    dctq::PlaneSet ps;
    if (int rc = dctq::plane_set(planes, nplanes, coef, nullptr, &ps)) return rc;
    HIPCHK(dctq::launch_fdct8_movement(ps, plan->dev, (hipStream_t)stream, plan->num_cus, 3, grid_mult),
           "fdct8_movement launch");
    return DCTQ_OK;
}

int dctq_diag_movement_v2_planes(const dctq_plan *plan, const dctq_plane *planes, int nplanes, int16_t *const *coef,
                                 void *stream) {
    DCTQ_ENTRY;
    if (int rc = dctq::check_plan(plan)) return rc;
    dctq::PlaneSet ps;
    if (int rc = dctq::plane_set(planes, nplanes, coef, nullptr, &ps)) return rc;
    HIPCHK(dctq::launch_fdct8_movement(ps, plan->dev, (hipStream_t)stream, plan->num_cus, 2), "fdct8_movement_v2 launch");
    return DCTQ_OK;
}

int dctq_diag_rt_movement_planes(const dctq_plan *plan, const dctq_plane *planes, int nplanes, int16_t *const *coef,
                                 float *const *recon, void *stream) {
    DCTQ_ENTRY;
    if (int rc = dctq::check_plan(plan)) return rc;
    if (!recon) return dctq::fail(DCTQ_EINVAL, "recon is NULL");
    dctq::RoundTripSet rt = {};
    if (int rc = dctq::plane_set(planes, nplanes, coef, nullptr, &rt.ps)) return rc;
    for (int k = 0; k < nplanes; ++k) {
        if (!recon[k] || ((uintptr_t)recon[k]) % 16) return dctq::fail(DCTQ_EINVAL, "recon[k] NULL or misaligned");
        rt.recon[k] = recon[k];
    }
    HIPCHK(dctq::launch_roundtrip_movement(rt, (hipStream_t)stream, plan->num_cus), "roundtrip_movement launch");
    return DCTQ_OK;
}

int dctq_diag_stream(int kind, const void *src, void *dst, long long blocks, void *stream) {
    DCTQ_ENTRY;
    using namespace dctq;
    if (!src || !dst || ((uintptr_t)src) % 16 || ((uintptr_t)dst) % 16) return fail(DCTQ_EINVAL, "src/dst NULL or misaligned");
    if (blocks < 64 || blocks % 64 || blocks >= (1ll << 31)) return fail(DCTQ_EINVAL, "blocks must be a multiple of 64 in [64, 2^31)");
    const uint32_t nb = (uint32_t)(blocks / 64);
    const hipStream_t s = (hipStream_t)stream;
    const int grid = device_cus() * 4;
    switch (kind) {
    case 0: hipLaunchKernelGGL(stream12<2>, dim3(grid), dim3(256), 0, s, (const u4v *)src, (char *)dst, nb); break;
    case 1: hipLaunchKernelGGL(stream12<0>, dim3(grid), dim3(256), 0, s, (const u4v *)src, (char *)dst, nb); break;
    case 2: {
        const size_t n16 = (size_t)blocks * 4;
        hipLaunchKernelGGL(stream_read, dim3((unsigned)((n16 + 1023) / 1024)), dim3(256), 0, s, (const u4v *)src,
                           (u4v *)dst, n16);
        break;
    }
    case 3:
    case 4: {
        const size_t n16 = (size_t)blocks * 8;
        if (kind == 3)
            hipLaunchKernelGGL(stream_write<false>, dim3((unsigned)((n16 + 1023) / 1024)), dim3(256), 0, s, (u4v *)dst, n16);
        else
            hipLaunchKernelGGL(stream_write<true>, dim3((unsigned)((n16 + 1023) / 1024)), dim3(256), 0, s, (u4v *)dst, n16);
        break;
    }
    case 5: hipLaunchKernelGGL(stream124, dim3(grid), dim3(256), 0, s, (const u4v *)src, (char *)dst, nb); break;
    case 6:
    case 7: {
        // kind 0 on a 16x / 32x grid (round 4: the forward's grid; the movement ubench's best for the flat
        // stream too, profiles/r04/forward_grid_sweep.log), capped at one batch per wave
        const unsigned want = (nb + 3) / 4, g = (unsigned)grid * (kind == 6 ? 16u : 32u);
        hipLaunchKernelGGL(stream12<2>, dim3(g < want ? g : want), dim3(256), 0, s, (const u4v *)src, (char *)dst, nb);
        break;
    }
    case 8: hipLaunchKernelGGL(stream124_split<false>, dim3(grid), dim3(256), 0, s, (const u4v *)src, (char *)dst, nb); break;
    case 9: hipLaunchKernelGGL(stream124_split<true>, dim3(grid), dim3(256), 0, s, (const u4v *)src, (char *)dst, nb); break;
    case 10: hipLaunchKernelGGL(stream124_rows<0>, dim3(grid), dim3(256), 0, s, (const uint8_t *)src, (char *)dst, nb); break;
    case 11: hipLaunchKernelGGL(stream124_rows<3840>, dim3(grid), dim3(256), 0, s, (const uint8_t *)src, (char *)dst, nb); break;
    case 12: hipLaunchKernelGGL((stream124_rows<3840, 1>), dim3(grid), dim3(256), 0, s, (const uint8_t *)src, (char *)dst, nb); break;
    case 13: hipLaunchKernelGGL((stream124_rows<3840, 2>), dim3(grid), dim3(256), 0, s, (const uint8_t *)src, (char *)dst, nb); break;
    case 14: {
        const unsigned want = (nb + 3) / 4, g = (unsigned)grid * 32u;
        hipLaunchKernelGGL(stream12_plane, dim3(g < want ? g : want), dim3(256), 0, s, (const uint8_t *)src, (char *)dst, nb);
        break;
    }
    case 15: hipLaunchKernelGGL(stream124_rows16, dim3(grid), dim3(256), 0, s, (const uint8_t *)src, (char *)dst, nb); break;
    case 16:
    case 17: {
        // kinds 9 / 11 on 32 x the resident grid (the round trip's grid, round 6), capped at one
        // batch per wave
        const unsigned want = (nb + 3) / 4, g = (unsigned)grid * 32u;
        if (kind == 16)
            hipLaunchKernelGGL(stream124_split<true>, dim3(g < want ? g : want), dim3(256), 0, s, (const u4v *)src,
                               (char *)dst, nb);
        else
            hipLaunchKernelGGL(stream124_rows<3840>, dim3(g < want ? g : want), dim3(256), 0, s,
                               (const uint8_t *)src, (char *)dst, nb);
        break;
    }
    default: return fail(DCTQ_EINVAL, "kind must be 0..17");
    }
    HIPCHK(hipGetLastError(), "diag stream launch");
    return DCTQ_OK;
}

int dctq_debug_tables(int quality, int adaptive, float *w, float *thr, double *dct, double *quant) {
    double q[64];
    quality = dctq_host::clamp_quality(quality);
    dctq_host::quant_matrix(8, quality, q);
    dctq::FastTables t;
    dctq::fill_fast_tables(q, adaptive, &t);
    if (w) memcpy(w, t.w, sizeof t.w);
    if (thr) memcpy(thr, t.thr, sizeof t.thr);
    if (dct) dctq_host::dct_matrix(8, dct);
    if (quant) memcpy(quant, q, sizeof q);
    return DCTQ_OK;
}

int dctq_debug_forward_kernel(int quality, int adaptive, long long batches, int num_cus) {
    (void)adaptive;
    double q[64];
    dctq_host::quant_matrix(8, dctq_host::clamp_quality(quality), q);
    const uint32_t nb = batches < 0 ? 0u : batches > 0xFFFFFFFFll ? 0xFFFFFFFFu : (uint32_t)batches;
    return dctq::forward_kernel_for(2, nb, num_cus, q[0] <= 1.0);
}

int dctq_debug_dc_table(int quality, int16_t *out) {
    double d[64], q[64];
    dctq_host::dct_matrix(8, d);
    dctq_host::quant_matrix(8, dctq_host::clamp_quality(quality), q);
    dctq::dc_const_table(d, q, out);
    return DCTQ_OK;
}

int dctq_debug_fastdiv(uint32_t d, uint32_t n) {
    dctq::FastDiv f = dctq::make_fastdiv(d);
    return (int)((((uint64_t)n * f.m >> 32) + n) >> f.s);
}

}  // extern "C"
