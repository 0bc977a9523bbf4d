/*
 * dct_amd.h -- batched (plane/frame-level) C-ABI of libdct_amd.so: the MI355X
 * hot path.  New surface added NEXT TO the reference's per-block API
 * (include/dct.h, include/quantization.h), which has no frame-level entry
 * point: the reference's only frame-level caller is the per-block pipeline of
 * tests/test_entropy.c:300-316 (create_block_from_pixels -> dct_forward ->
 * calculate_block_variance -> quantize) and its inverse :350-373
 * (dequantize -> dct_inverse).  Each entry point below replaces that loop over
 * every 8x8 block of a plane with one HIP launch.
 *
 * Conventions: plain pointers and sizes, no HIP/torch types.  Device pointers
 * are HIP device memory of the calling thread's current device; `stream` is a
 * hipStream_t passed as void* (NULL = default stream).  Every call is
 * asynchronous on `stream` and returns 0 or a negative DCTQ_E* code
 * (dctq_error_string).  Results are bit-identical to the reference
 * (src/dct.c + src/quantization.c) for the quantized path; see DESIGN.md.
 */
#ifndef DCT_AMD_H
#define DCT_AMD_H

#include <stddef.h>
#include <stdint.h>

#include "quantization.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ABI revision of this header.  6: dctq_encode_planes writes 4-byte symbols for
 * every plan again (round 5 had switched plans with |q| <= 511 to 2-byte symbols
 * under the same entry point); the 2-byte format is dctq_encode_planes16, opt-in;
 * dctq_abi_version() returns the library's revision so a host can check both. */
#define DCTQ_ABI_VERSION 6
int dctq_abi_version(void);

#define DCTQ_OK 0
#define DCTQ_EINVAL (-1)   /* bad argument (sizes not multiples of 8, misaligned, ...) */
#define DCTQ_EHIP (-2)     /* a HIP runtime call failed (dctq_error_string has the detail) */
#define DCTQ_ENOMEM (-3)
#define DCTQ_ENODEV (-4)   /* no gfx950 device visible */

/* Opaque per-configuration state: the host-computed tables (D of src/dct.c:17-30,
 * Q of src/quantization.c:51-99, fast-path scale and guard tables) uploaded to
 * the device that was current at creation.  A plan is read-only after
 * creation: one plan may serve several streams and threads at once, and the
 * library keeps no per-stream device state.  Threading: the batched calls do not
 * serialise -- after a thread's first call of an entry point on a stream (which
 * shields the host's rand() stream from the HIP runtime, as every plan and
 * memory call does) they take no lock and touch no global state. */
typedef struct dctq_plan dctq_plan;

/* quality is clamped to 1..100 exactly as quant_init does (src/quantization.c:26-31).
 * A plan holds only its ~4 KB of tables in device memory; it is reusable and
 * cheap to keep (one per quality is fine).  The forward resolves every plan's
 * rounding ties in place and allocates nothing per launch. */
int dctq_plan_create(int quality, int adaptive, dctq_plan **plan);
/* Bind an existing reference-style context (block_size must be 8); its
 * quant_matrix VALUES are used, so a caller-modified table is honoured. */
int dctq_plan_from_context(const QuantContext *qctx, dctq_plan **plan);
/* Frees the plan's device tables (hipFree, which waits for the device as cudaFree
 * does); launches that use the plan must have been issued before. */
void dctq_plan_destroy(dctq_plan *plan);

/* A stack of equally-shaped u8 planes in device memory. */
typedef struct {
    const uint8_t *pixels;   /* frame 0, row 0; 8-byte aligned */
    long long stride;        /* bytes between pixel rows; multiple of 8, >= width */
    long long frame_stride;  /* bytes between consecutive frames */
    int width, height;       /* multiples of 8 */
    int nframes;             /* >= 1 */
} dctq_plane;

/* Forward DCT + quantization of every 8x8 block:
 *   coef[f][by][bx][64] (int16, row-major within the block, blocks in raster
 *   order -- the order the reference emits them) = quantize(dct_forward(px-128)).
 * var_num (optional, may be NULL): per block 64*sum(x^2) - sum(x)^2 with
 * x = px-128; calculate_block_variance() == var_num / 4096.0 exactly.  Needed by
 * the adaptive inverse. */
int dctq_forward_quant(const dctq_plan *plan, const dctq_plane *src, int16_t *coef, int32_t *var_num,
                       void *stream);

/* The same for up to 4 planes of independent geometry (e.g. the Y, Cb, Cr planes
 * of a 4:2:0 frame stack) in ONE launch: plane k writes coef[k] (and var_num[k]
 * when var_num is non-NULL, in which case every var_num[k] must be set), exactly
 * as dctq_forward_quant(plan, &planes[k], coef[k], var_num[k]) would.  Saves a
 * launch gap and a grid tail per extra plane (the reference has no plane
 * notion: a caller coding Y/Cb/Cr runs its per-block loop once per plane). */
int dctq_forward_quant_planes(const dctq_plan *plan, const dctq_plane *planes, int nplanes, int16_t *const *coef,
                              int32_t *const *var_num, void *stream);

/* Fused round trip (BASELINE configs[4]) of up to 4 planes in ONE launch: for
 * plane k, coef[k] (and var_num[k] if var_num is non-NULL) exactly as
 * dctq_forward_quant_planes, and
 *   recon[k][b][64] = dct_inverse(dequantize(coef[k][b])) + 128
 * exactly as dctq_inverse(plan, coef[k], var_num[k], ...) would produce it
 * (float, unclamped, |err| <= 1e-4).  The quantized ints go from the forward to
 * the inverse through LDS: 448 B of HBM traffic per block instead of 584 B for
 * the two calls.  var_num is optional even for adaptive plans.  recon 16-byte
 * aligned. */
int dctq_round_trip_planes(const dctq_plan *plan, const dctq_plane *planes, int nplanes, int16_t *const *coef,
                           int32_t *const *var_num, float *const *recon, void *stream);

/* Encoder: forward DCT + quantization + zigzag run-length
 * symbols of up to 4 planes.  coef[k] exactly as dctq_forward_quant_planes;
 * blocks numbered plane 0 first, then plane 1, ... (N in total, N < 2^26):
 *   offsets[b]  = first symbol of block b, offsets[N] = total symbols
 *   symbols[..] = the reference's run_length_encode of every block, in order
 *                 (as dctq_rle_count + dctq_rle_emit over the concatenated
 *                 coefficient planes): uint32_t (uint16_t)value | run << 16.
 * The symbol count is fused into the forward launch.  Symbols at index >=
 * symbols_capacity are not written; offsets are always complete (compare
 * offsets[N] with the capacity).  symbols == NULL or capacity 0: coefficients
 * and offsets only.  Worst case 64 symbols per block.  symbols 4-byte aligned.
 * workspace: dctq_encode_workspace_bytes(N) bytes. */
size_t dctq_encode_workspace_bytes(long long total_blocks);
int dctq_encode_planes(const dctq_plan *plan, const dctq_plane *planes, int nplanes, int16_t *const *coef,
                       uint32_t *offsets, uint32_t *symbols, long long symbols_capacity, void *workspace,
                       void *stream);
/* The same stream in 2-byte symbols (opt-in, half the bytes):
 *   uint16_t (run & 63) << 10 | (value & 0x3FF), value in [-511, 511];
 * runs are 0..63 except the one symbol of an all-zero block, (value 0, run 64),
 * which is 0x0000 (no other symbol is: a zero value only ends a block, with
 * run >= 1).  dctq_rle_decode16 reads it.  Only for plans whose quantization
 * table bounds every quantized coefficient by 511 (dctq_plan_symbol_bytes == 2;
 * q <= 90 of the standard table); DCTQ_EINVAL for the others.  capacity in
 * symbols; symbols 4-byte aligned. */
int dctq_encode_planes16(const dctq_plan *plan, const dctq_plane *planes, int nplanes, int16_t *const *coef,
                         uint32_t *offsets, uint16_t *symbols, long long symbols_capacity, void *workspace,
                         void *stream);
/* The most compact symbol format the plan admits: 2 (dctq_encode_planes16 may be
 * used) or 4 (dctq_encode_planes only). */
int dctq_plan_symbol_bytes(const dctq_plan *plan);

/* Forward DCT only, float coefficients coef[f][by][bx][64]
 * (|coef - dct_forward()| <= 1e-4; computed in fp64, rounded once to fp32). */
int dctq_forward_float(const dctq_plan *plan, const dctq_plane *src, float *coef, void *stream);

/* Inverse: dequantize (reference semantics incl. the non-adaptive 1/Q
 * multiplier, src/quantization.c:139,144) + dct_inverse + 128, per block:
 *   recon[b][64] = dct_inverse(dequantize(coef[b], var_num[b]/4096)) + 128
 * (float, unclamped; |err| <= 1e-4).  var_num is required when adaptive. */
int dctq_inverse(const dctq_plan *plan, const int16_t *coef, const int32_t *var_num, long long nblocks,
                 float *recon, void *stream);

/* Zigzag + run-length symbols of quantized blocks (the reference's
 * run_length_encode, src/entropy.c:216-256 over block_to_zigzag :158-178, for
 * every block, blocks concatenated in order).  symbol = (uint16_t)value |
 * run << 16.  A block has 1 + (nonzeros among its first 63 zigzag elements)
 * symbols, so the stream is built in two steps:
 *   dctq_rle_count: offsets[b] = symbols before block b, offsets[nblocks] =
 *                   total (nblocks + 1 entries); `workspace` is device memory
 *                   of dctq_rle_workspace_bytes(nblocks) bytes;
 *   dctq_rle_emit:  symbols[offsets[b] .. offsets[b+1]) for every block
 *                   (the caller sizes `symbols` from offsets[nblocks], or
 *                   64 * nblocks for the worst case).
 * nblocks < 2^26 (offsets are 32-bit). */
size_t dctq_rle_workspace_bytes(long long nblocks);
int dctq_rle_count(const int16_t *coef, long long nblocks, uint32_t *offsets, void *workspace, void *stream);
int dctq_rle_emit(const int16_t *coef, long long nblocks, const uint32_t *offsets, uint32_t *symbols, void *stream);
/* The inverse, run_length_decode (src/entropy.c:327-351) + zigzag_to_block
 * (:183-210) of every block: coef[b][64] from symbols[offsets[b] ..).
 * dctq_rle_decode16: the same from 2-byte symbols ((run & 63) << 10 | (value &
 * 0x3FF), 0x0000 = (0, 64); dctq_encode_planes16's output);
 * symbols 4-byte aligned. */
int dctq_rle_decode16(const uint16_t *symbols, const uint32_t *offsets, long long nblocks, int16_t *coef,
                      void *stream);
int dctq_rle_decode(const uint32_t *symbols, const uint32_t *offsets, long long nblocks, int16_t *coef,
                    void *stream);

/* Per-block Huffman size: bits[b] = what the reference's pipeline
 * reports for block b coded on its own (tests/test_entropy.c:329-341):
 * run_length_encode -> build_huffman_codes -> get_encoded_size
 * (src/entropy.c:216-256, 261-328, 363-399), i.e. sum over the block's RLE
 * symbols of (Huffman code length + 8).  The code lengths of one symbol depend
 * on the reference heap's tie order, their sum does not (Huffman trees are
 * optimal); the codes themselves are not produced.  coef 16-byte aligned. */
int dctq_huffman_bits(const int16_t *coef, long long nblocks, uint32_t *bits, void *stream);
/* The same per-block size straight from pixels: the whole per-block loop of
 * tests/test_entropy.c:300-341 (create_block_from_pixels -> dct_forward ->
 * quantize -> run_length_encode -> build_huffman_codes -> get_encoded_size) for
 * every block of up to 4 planes, blocks numbered plane 0 first (as
 * dctq_encode_planes).  Equal to dctq_forward_quant_planes followed by
 * dctq_huffman_bits over the concatenated coefficients, but the coefficients
 * never leave the chip.  bits: 4-byte aligned, one entry per block. */
int dctq_huffman_bits_planes(const dctq_plan *plan, const dctq_plane *planes, int nplanes, uint32_t *bits,
                             void *stream);

/* The calling thread forgets `stream` (call it before hipStreamDestroy): the
 * library keeps no per-stream device memory, only each thread's list of the
 * streams it has launched on, and a stream later created at the same handle
 * then gets its first call isolated again (that list is also keyed by the
 * runtime's stream id, so hosts that skip this call stay correct wherever the
 * runtime tells the two streams apart).  Returns DCTQ_OK. */
int dctq_stream_release(void *stream);

/* Optional diagnostics: if non-NULL, *counter (device, uint64) is incremented
 * by the number of coefficients resolved by the exact fp64 tie path in later
 * dctq_forward_quant / _planes / dctq_round_trip_planes calls on this plan (costs one atomic per affected wave). */
int dctq_plan_set_fallback_counter(dctq_plan *plan, unsigned long long *counter);

/* Synthetic frames (counter-based splitmix64; identical to the oracle's
 * generator): kind 0 uniform, 1 smooth, 2 constant 8x8 blocks, 3 extremes.
 * Frame f uses seed + f. */
int dctq_synth(uint64_t seed, int kind, const dctq_plane *dst, void *stream);

/* Device helpers so a plain C host needs no HIP headers. */
int dctq_device_count(int *count);
int dctq_set_device(int device);
int dctq_malloc(void **ptr, size_t bytes);
int dctq_free(void *ptr);
int dctq_memcpy_htod(void *dst, const void *src, size_t bytes);
int dctq_memcpy_dtoh(void *dst, const void *src, size_t bytes);
int dctq_synchronize(void *stream);
const char *dctq_error_string(int code);

#ifdef __cplusplus
}
#endif
#endif
