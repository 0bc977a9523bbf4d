/* dct_amd/csrc/dctq_diag.h -- the C-ABI of libdct_amd_diag.so, the DIAGNOSTIC
 * build of this library: the same objects as libdct_amd.so plus diag.hip.  Not
 * a codec surface (no include/ header): measurement (bench.py's ceilings, the
 * A/B tools) and test-only controls.  Every product entry point of
 * include/dct_amd.h is exported by this library too, so a plan created here can
 * be used with any of them -- but a plan belongs to the library that created it. */
#ifndef DCTQ_DIAG_H
#define DCTQ_DIAG_H

#include "dct_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Force the forward kernel of a plan (test-only; libdct_amd.so picks by launch
 * size): 2 = the product dispatch, 1 = v1 (one workgroup per 256 blocks), 3 =
 * v3 (in-place ties) at any size, 4 = v2 (tie queue) at any size; honoured by
 * the dctq_diag_* entry points below (lane-per-block float / inverse when 1). */
int dctq_diag_plan_set_variant(dctq_plan *plan, int variant);
/* dctq_forward_quant_planes / dctq_forward_float / dctq_inverse that honour the
 * plan's forced variant (the product entry points ignore it): variant 1 / 4 runs
 * the retired kernel, any other plan the product entry point. */
int dctq_diag_forward_quant_planes(const dctq_plan *plan, const dctq_plane *planes, int nplanes, int16_t *const *coef,
                                   int32_t *const *var_num, void *stream);
int dctq_diag_forward_float(const dctq_plan *plan, const dctq_plane *src, float *coef, void *stream);
int dctq_diag_inverse(const dctq_plan *plan, const int16_t *coef, const int32_t *var_num, long long nblocks,
                      float *recon, void *stream);

/* The fused round trip's inverse (test-only): mode 0 forces the paired-lane fp64
 * inverse; 1 restores the plan's own choice (the fp32 inverse when the plan is
 * admitted by the rigorous bound of tools/inv_bound.py, see dctq_debug_inverse_bound). */
int dctq_diag_plan_set_inverse(dctq_plan *plan, int mode);

/* Launch every kernel of a plan as if the device had num_cus CUs (1..4096; the
 * grids are capped per CU), so a test-sized input gives each wave many batches
 * (test-only: on the full grid a wave of the fused Huffman kernel sees about one
 * batch of a 4K frame stack, so its row carry between batches runs only then). */
int dctq_diag_plan_set_num_cus(dctq_plan *plan, int num_cus);

/* Moves exactly the bytes dctq_forward_quant_planes moves, in the access pattern
 * of its product kernel fdct8_quant_v3 (same grid, LDS footprint, prefetch, LDS
 * stage and 1 KiB stores) with no arithmetic.  coef[k] receives pixel bytes,
 * NOT coefficients.  Its time is the memory ceiling of the forward kernel's own
 * access pattern. */
int dctq_diag_movement_planes(const dctq_plan *plan, const dctq_plane *planes, int nplanes, int16_t *const *coef,
                              void *stream);
/* The same on a grid of grid_mult (1..64) x the resident workgroups instead of the
 * product kernel's (bench.py: the pattern's ceiling at the round-3 grid, x8). */
int dctq_diag_movement_grid_planes(const dctq_plan *plan, const dctq_plane *planes, int nplanes, int16_t *const *coef,
                                   int grid_mult, void *stream);
/* The same in the access pattern of fdct8_quant_v2 (the tie-heavy plans' queue
 * kernel: its queue arrays in LDS, its first-batch loads). */
int dctq_diag_movement_v2_planes(const dctq_plan *plan, const dctq_plane *planes, int nplanes, int16_t *const *coef,
                                 void *stream);

/* The same for the fused round trip (dctq_round_trip_planes): its grid, stage
 * and stores with no arithmetic; coef[k] and recon[k] receive pixel bytes. */
int dctq_diag_rt_movement_planes(const dctq_plan *plan, const dctq_plane *planes, int nplanes, int16_t *const *coef,
                                 float *const *recon, void *stream);

/* Hardware ceilings of the forward kernel's traffic (64 B read : 128 B written
 * per block), independent of its access pattern (profiles/r02/hbm_ceilings.md):
 *   kind 0: flat 1:2 stream, per wave 4 x 1 KiB loads then 8 x 1 KiB stores per
 *           64-block batch, persistent grid, nt loads, nt stores;
 *   kind 1: the same with default-policy stores;
 *   kind 2: read-only stream of blocks * 64 bytes of src (nt);
 *   kind 3: write-only stream of blocks * 128 bytes of dst (default policy);
 *   kind 4: the same with non-temporal stores;
 *   kind 5: the round trip's mix, flat: 64 B read : 128 + 256 B written per
 *           block (per wave 4 x 1 KiB loads, 24 x 1 KiB nt stores), persistent;
 *   kind 6, 7: kind 0 on a grid of 16 x / 32 x the resident one (the forward's
 *           grid and twice it), capped at one 64-block batch per wave;
 *   kind 8: kind 5's bytes in the round trip's output layout: each batch's 8 KiB
 *           to region A (the first blocks * 128 bytes of dst: the coefficients)
 *           and 16 KiB to region B (the rest: the recon);
 *   kind 9: kind 8 with the stores in the round trip's three 8 KiB groups and a
 *           vmcnt(0) drain before each of the last two;
 *   kind 10: kind 9 with the round trip's load shape: each lane loads its block's
 *           8 rows as 8-byte nt buffer loads, the batch's 4 KiB contiguous;
 *   kind 11: kind 10 over a 3840-px-wide plane (480 blocks per block row: the
 *           luma plane's row pitch between a block's rows);
 *   kind 12, 13: kind 11 with workgroup-contiguous / wave-contiguous runs of
 *           batches instead of the grid-stride order;
 *   kind 14: kind 7 with the forward's load shape over a 3840-px-wide plane (each
 *           lane its block's 8 rows, 8 B each);
 *   kind 15: kind 11 with 16-byte loads (per instruction, rows 2k and 2k + 1 of the
 *           batch, two blocks' row slices per lane);
 *   kind 16, 17: kinds 9 / 11 on 32 x the resident grid (the round trip's), at
 *           most one batch per wave.
 * src >= blocks * 64 bytes, dst >= blocks * 128 bytes (kinds 5, 8-13, 15-17: blocks *
 * 384), both 16-byte aligned. */
int dctq_diag_stream(int kind, const void *src, void *dst, long long blocks, void *stream);

/* The v2 queue kernel (variant 4) keeps a tie-path pixel stash per (device,
 * stream[, thread for the NULL stream and hipStreamPerThread]), sized to its grid;
 * a launch captured into a graph gets one of its own.  Release waits for `stream`
 * and frees the calling thread's stashes on it (direct and captured: call it only
 * after the last replay of such a graph); DCTQ_EINVAL while `stream` is being
 * captured.  Bytes: the stash direct launches on `stream` use (0 if none). */
int dctq_diag_stream_release(void *stream);
long long dctq_diag_stream_stash_bytes(void *stream);

/* Host-only introspection for the CPU tests (no GPU needed). */
/* The forward kernel (1, 2, 3 = fdct8_quant_v1/v2/v3) dctq_forward_quant_planes runs
 * for a plan of this quality / adaptive mode over `batches` 64-block batches on a
 * device of num_cus CUs (bench.py names the kernel its roofline is measured on). */
int dctq_debug_forward_kernel(int quality, int adaptive, long long batches, int num_cus);
int dctq_debug_tables(int quality, int adaptive, float *w, float *thr, double *dct, double *quant);
int dctq_debug_dc_table(int quality, int16_t *out);
int dctq_debug_fastdiv(uint32_t d, uint32_t n);
/* The rigorous bound of |recon - reference| of the round trip's fp32 inverse for a
 * standard-table plan (api.hip inverse_f32_bound); *admitted = whether
 * dctq_round_trip_planes runs that inverse for it (non-adaptive, bound <= 5e-5). */
double dctq_debug_inverse_bound(int quality, int adaptive, int *admitted);
/* The encoder's symbol bytes (2 or 4) for a standard-table plan (dctq_plan_symbol_bytes). */
int dctq_debug_symbol_bytes(int quality, int adaptive);
/* The legacy per-block API's lanes (legacy.hip: a stream + staging buffer per host
 * thread and device): how many were ever created, and how many wait in the pool for
 * a new thread (their threads exited).  For calls made through this library. */
int dctq_diag_legacy_lanes(int *made, int *pooled);

#ifdef __cplusplus
}
#endif
#endif
