// dct_amd/csrc/dctq_internal.h -- shared between the kernels and the C-ABI shim.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <optional>

namespace dctq {

// The HSA runtime calls srand()/rand() (libhsa-runtime64 imports both), which
// would reseed or advance the HOST APPLICATION's rand() stream; the reference's
// own tests draw their blocks from rand() (tests/test_quantization.c:127,134).
// The entry points that allocate or free device memory or set up devices (plan
// create / destroy, the device-memory helpers, the legacy per-block API, the
// diagnostic library) hold one of these while they may reach the HIP runtime:
// glibc's global random state is swapped to a private one for the duration
// (initstate/setstate keep the caller's state and position intact).  Those entry
// points are serialised by it (recursive, so nesting is fine); the batched launch
// entry points are not (LaunchIsolation below).
class RandIsolation {
  public:
    RandIsolation();
    ~RandIsolation();
    RandIsolation(const RandIsolation &) = delete;
    RandIsolation &operator=(const RandIsolation &) = delete;

  private:
    char *saved_;
};
#define DCTQ_ENTRY ::dctq::RandIsolation dctq_rand_isolation_

// The batched launch entry points (and dctq_synchronize) do NOT serialise: the
// runtime's one rand() user (srand(now); rand() inside libhsa-runtime64, reached
// when the runtime initialises or creates device resources -- a stream's first
// hardware queue, a module's first load) can only run on a thread's FIRST call of
// an entry point on a stream, so that call is isolated as above; every later call
// of the thread with the same (device, stream, entry point) takes no lock and
// touches no global state (the reference API is reentrant and keeps
// no mutable global state).  `entry` < 32 names the entry point.
class LaunchIsolation {
  public:
    LaunchIsolation(const void *stream, int entry);
    LaunchIsolation(const LaunchIsolation &) = delete;
    LaunchIsolation &operator=(const LaunchIsolation &) = delete;

  private:
    std::optional<RandIsolation> iso_;
};
#define DCTQ_LAUNCH(stream, entry) ::dctq::LaunchIsolation dctq_launch_isolation_((stream), (entry))

// Whether some entry point has already initialised the HIP runtime in this
// process: until then any HIP call (even hipGetDevice) may initialise it, and so
// must be isolated.  forget_stream: the calling thread drops `stream` from its
// launch-isolation list (dctq_stream_release).
bool runtime_started();
void note_runtime_started();
void forget_stream(const void *stream);
// legacy.hip: per-thread lanes of the per-block API created so far / pooled (diagnostics)
void legacy_lane_counts(int *made, int *pooled);


// Resident workgroups per CU of `kernel` at `threads` per workgroup (>= 1).  The
// launchers cache it in a function-local static (thread-safe initialisation):
// every device this library runs on is a gfx950.
template <typename K>
inline int resident_per_cu(K kernel, int threads) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, threads, 0) != hipSuccess || nb < 1) nb = 1;
    return nb;
}

// Persistent grid-stride kernels launch kGridMult times their resident
// workgroups; the extra ones queue and start as the first wave of workgroups
// retires, which evens out batches of unequal cost and the launch tail
// (profiles/r02/grid_mult_ab.log: x8 is 2.4-7 % faster than x1 on the forward,
// round trip, inverse and encoder, outputs identical; x16/x32 regress on
// uniform input).
constexpr int kGridMult = 8;
// Cache policy of the bulk 1 KiB output stores of every streaming kernel
// (buffer-store aux bits, gfx950: 1 sc0, 2 nt, 16 sc1).  Non-temporal: the
// written lines are never re-read by the kernel that writes them.
constexpr int kNtAux = 2;

// n / d and n % d by multiply-high, valid for 0 <= n < 2^31 (host-built magic).
struct FastDiv {
    uint32_t d, m, s;
};
FastDiv make_fastdiv(uint32_t d);
__device__ __forceinline__ uint32_t fdiv(uint32_t n, FastDiv f) { return (__umulhi(n, f.m) + n) >> f.s; }

// Wave-uniform per-plan constants of the fp32 fast path, passed by value in the
// kernel arguments so every access is a scalar load into SGPRs.
struct FastTables {
    float w[64];    // S_i S_j / Q_ij  (AAN output scale folded into 1/Q)
    float thr[64];  // |frac| above which the exact fp64 path decides (guard band)
    float thr2[64]; // thr^2 rounded down: flag iff thr2 - f*f < 0
    // v2 processing order: slot p = 16*cp + 2*i + h holds coefficient 8*i + 2*cp + h
    float ws[64], t2s[64];
};

// Per-plan device-resident tables (runtime-indexed: exact tie path, inverse).
struct DevTables {
    double dct[64];    // D of src/dct.c:17-30, bit-identical to the host expression
    double quant[64];  // Q of src/quantization.c:51-99
    double dequant[64];// 1/Q (src/quantization.c:101-111)
    double iscale[64]; // inverse path: 1/Q * S_i S_j (non-adaptive dequant folded with AAN^T scale)
    double qscale[64]; // inverse path (adaptive): Q * S_i S_j
    double s2[64];     // S_i S_j
    double s1[8];      // S_k: AAN output scale X_k = S_k y_k (per-slot factors of the paired fp64 kernels)
    float iscale32[64];// fl32(iscale): the fused round trip's fp32 inverse (plans admitted by idct8_bound.h)
    FastTables fast;   // device copy of the fast-path tables (v2 reads them per batch)
    // quantized DC of a CONSTANT block of centred value v-128, computed on the
    // host in the reference's order (src/dct.c:57-74, src/quantization.c:124):
    // resolves the DC ties of flat blocks without the exact path.  The DC is
    // never adjusted by adaptive plans (src/quantization.c:198-199).
    int16_t dc_const[256];
};

struct PlaneArgs {
    const uint8_t *src;
    long long stride, frame_stride;
    int bw;             // blocks per row
    int nblk_frame;     // blocks per frame
    int nblk;           // total blocks (all frames), < 2^31
    FastDiv div_bw, div_frame;  // by bw and by nblk_frame
    uint32_t span;      // bytes from src to one past the last pixel when < 2^32, else 0 (load_rows<true>)
};

// Up to kMaxPlanes planes (e.g. Y, Cb, Cr) processed by ONE forward launch.
constexpr int kMaxPlanes = 4;
struct PlaneSet {
    PlaneArgs pl[kMaxPlanes];
    int16_t *coef[kMaxPlanes];
    int32_t *var[kMaxPlanes];          // all NULL or all set
    uint32_t first[kMaxPlanes + 1];    // global index of each plane's first 64-block batch; first[n] = total
    int n;
};

// The encoder's planes: PlaneSet (coef/var unused) plus each plane's first block
// in the concatenated block numbering of the offsets array; blk_first[n] = total.
struct EncodeSet {
    PlaneSet ps;
    uint32_t blk_first[kMaxPlanes + 1];
};

// The fused round trip's planes: forward outputs as PlaneSet, plus fp32 recon per plane.
struct RoundTripSet {
    PlaneSet ps;
    float *recon[kMaxPlanes];
};

// The product forward (fdct8.hip): fdct8_quant_v3 over every plane of ps, every plan.
hipError_t launch_fdct8_quant(const PlaneSet &ps, const DevTables *dev, int adaptive, unsigned long long *fallbacks,
                              hipStream_t stream, int num_cus);
// diagnostic library (fdct8_diag.hip): the forward kernel (1, 2 or 3 = fdct8_quant_v1/v2/v3)
// a plan of `variant` runs (the product: 3 for every plan and size)
int forward_kernel_for(int variant, uint32_t nbatch, int num_cus, bool tie_heavy);
// diagnostic: the forward's data movement without arithmetic (fdct8_diag.hip): shape 3 =
// fdct8_quant_v3's (the product kernel), 2 = fdct8_quant_v2's (the queue kernel);
// grid_mult 0 = the product kernel's grid
hipError_t launch_fdct8_movement(const PlaneSet &ps, const DevTables *dev, hipStream_t stream, int num_cus, int shape,
                                 int grid_mult = 0);
hipError_t launch_roundtrip(const RoundTripSet &rt, const DevTables *dev, int adaptive, bool inv_f32,
                            unsigned long long *fallbacks, hipStream_t stream, int num_cus);
// diagnostic: roundtrip8_f32's data movement without arithmetic (fdct8_diag.hip)
hipError_t launch_roundtrip_movement(const RoundTripSet &rt, hipStream_t stream, int num_cus);
size_t encode_workspace_bytes(long long nbatch);
// symbol_bytes 4: (uint16)value | run << 16; 2: run << 10 | (value & 0x3FF), |value| <= 511 (rle.hip)
hipError_t launch_encode(const EncodeSet &es, const DevTables *dev, int adaptive, uint32_t *offsets, void *symbols,
                         int symbol_bytes, unsigned long long capacity, void *ws, hipStream_t stream, int num_cus);
hipError_t launch_fdct8_float_pair(const PlaneArgs &p, const DevTables *dev, float *coef, hipStream_t stream,
                                   int num_cus);
hipError_t launch_idct8_pair(const DevTables *dev, int adaptive, const int16_t *coef, const int32_t *var_num,
                             long long nblk, float *recon, hipStream_t stream, int num_cus);
size_t rle_workspace_bytes(long long nblk);
size_t rle_scan_workspace_bytes(long long ntiles);
hipError_t launch_rle_scan(void *ws, long long ntiles, hipStream_t stream);
hipError_t launch_rle_fixup(uint32_t *offsets, long long nblk, const void *ws, long long ntiles, long long tile0,
                            uint32_t *total_out, hipStream_t stream);
hipError_t launch_rle_count(const int16_t *coef, long long nblk, uint32_t *offsets, void *ws, hipStream_t stream,
                            int num_cus);
hipError_t launch_rle_emit(const int16_t *coef, long long nblk, const uint32_t *offsets, void *symbols,
                           int symbol_bytes, unsigned long long capacity, hipStream_t stream, int num_cus);
// per-block Huffman size estimate (huffman.hip)
hipError_t launch_huffman_bits(const int16_t *coef, long long nblk, uint32_t *bits, hipStream_t stream, int num_cus);
hipError_t launch_huffman_from_pixels(const EncodeSet &es, const DevTables *dev, int adaptive, uint32_t *bits,
                                      hipStream_t stream, int num_cus);
hipError_t launch_rle_decode(const void *symbols, int symbol_bytes, const uint32_t *offsets, long long nblk,
                             int16_t *coef, hipStream_t stream, int num_cus);
// diagnostic library (fdct8_diag.hip): the lane-per-block fp64 kernels (variant 1)
hipError_t launch_fdct8_float(const PlaneArgs &p, const DevTables *dev, float *coef, hipStream_t stream);
hipError_t launch_idct8(const DevTables *dev, int adaptive, const int16_t *coef, const int32_t *var_num,
                        long long nblk, float *recon, hipStream_t stream);
hipError_t launch_synth(uint64_t seed, int kind, uint8_t *dst, long long stride, long long frame_stride,
                        int width, int height, int nframes, hipStream_t stream);

}  // namespace dctq
