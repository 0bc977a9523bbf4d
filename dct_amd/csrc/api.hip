// dct_amd/csrc/api.hip -- the batched C-ABI of include/dct_amd.h.
//
// Host side of the hot path: builds the per-plan tables (D of src/dct.c:17-30 and
// Q of src/quantization.c:51-99 with the reference's own expressions, so the
// exact tie path sees bit-identical constants; the fast path's scale and guard
// tables from the proven bound in fdct8_bound.h), validates arguments, and
// launches the kernels of fdct8.hip / fdct8_aux.hip on the caller's stream.
#include <dlfcn.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "dct_amd.h"
#include "dctq_diag.h"
#include "dctq_internal.h"
#include "fdct8_bound.h"
#include "host_tables.h"
#include "idct8_bound.h"
#include "plan.h"

namespace {
thread_local std::string g_err;
}  // namespace

namespace dctq {
int fail(int code, const char *what, hipError_t e) {
    g_err = what;
    if (e != hipSuccess) {
        g_err += ": ";
        g_err += hipGetErrorString(e);
    }
    return code;
}
}  // namespace dctq
using dctq::fail;


namespace dctq {
FastDiv make_fastdiv(uint32_t d) {
    uint32_t s = 0;
    while ((1ull << s) < d) ++s;
    const uint64_t m = ((1ull << 32) * ((1ull << s) - d)) / d + 1;
    return FastDiv{d, (uint32_t)m, s};
}

// Guard band of the fast path (DESIGN.md "Exactness").  With Y~ the fp32
// butterfly output (|Y~ - Y| <= kErrY), w~ = fl32(S_i S_j / Q) and
// f~ = fl(Y~ w~ - r) for r = rint(Y~ w~), the reference's quotient V = fl(ref / M)
// satisfies |V - (r + f~)| <= B below; hence |f~| <= 0.5 - B  =>  round(V) == r.
void fill_fast_tables(const double *q, int adaptive, FastTables *t) {
    const double u = 0x1p-24;
    // scale-factor representation: fl32(w) (0.5u) and its product (0.5u); adaptive
    // plans also the kernel's 1/(2-nv) = v_rcp_f32(fl32(2-nv)) (0.5u + 2u, fdct8_core.h)
    const double rel = adaptive ? 4.5 * u + 0x1p-48 : u + 0x1p-48;
    for (int c = 0; c < 64; ++c) {
        const int i = c >> 3, j = c & 7;
        const double w = kAanScale[i] * kAanScale[j] / q[c];
        const float wf = (float)w;
        const double wt = (double)wf;
        const double B = 0x1p-25                        /* rounding of f~ */
                         + kErrY[c] * wt * (1.0 + 4.0 * u) /* butterfly error, scaled */
                         + kMaxY[c] * w * rel           /* scale-factor representation */
                         + 1e-9 / q[c]                  /* reference's own fp64 error (< 1e-11) */
                         + (kMaxY[c] * w + 1.0) * 0x1p-52; /* reference's division rounding */
        double thr = (0.5 - B) * (1.0 - 0x1p-20);
        float tf = (float)thr;
        if ((double)tf > thr) tf = nextafterf(tf, 0.0f);
        t->w[c] = wf;
        t->thr[c] = tf;
        const double tt = (double)tf * (double)tf;  // exact
        float t2 = (float)tt;
        if ((double)t2 > tt) t2 = nextafterf(t2, 0.0f);
        t->thr2[c] = t2;
    }
    for (int p = 0; p < 64; ++p) {
        const int c = (((p >> 1) & 7) << 3) + ((p >> 4) << 1) + (p & 1);
        t->ws[p] = t->w[c];
        t->t2s[p] = t->thr2[c];
    }
}
}  // namespace dctq

// Quantized DC of a constant block, exactly as the reference computes it:
// temp[k][0] = sum_l x * D[0][l] (the same for every row k, l ascending), then
// out = sum_k D[0][k] * temp[k][0], q = (int) round(out / Q[0]).  This file is
// compiled with -ffp-contract=off, so host arithmetic is the reference's.
void dctq::dc_const_table(const double *d, const double *q, int16_t *tab) {
    for (int v = 0; v < 256; ++v) {
        const double x = (double)v - 128.0;
        double t = 0.0;
        for (int l = 0; l < 8; ++l) t += x * d[l];
        double out = 0.0;
        for (int k = 0; k < 8; ++k) out += d[k] * t;
        tab[v] = (int16_t)(int)round(out / q[0]);
    }
}

// The fused round trip's fp32 inverse is admitted for a non-adaptive plan when the
// rigorous bound of tools/inv_bound.py (idct8_bound.h) keeps |recon - reference|
// within kInvTol (5e-5, half of north_star's 1e-4) for EVERY input block:
// |c_uv| <= 128 L1(D_u) L1(D_v) for centred pixels, so |q_uv| <= round(c_max / Q)
// and |x_uv| <= B_uv = |q|max * (1/Q) * S_u S_v (the reference's 1/Q dequantisation,
// src/quantization.c:139,144); per output pixel the bound is G.B (1 + u) + u (128 + |L|.B)
// (the final + 128 rounding) + 1e-9 (the reference's own fp64 error).
static_assert(kInvTol == kInvTolDiag, "plan.h's copy of the fp32 inverse's admission tolerance");
double dctq::inverse_f32_bound(const dctq::DevTables &t) {
    const double u = 1.0 / 16777216.0;
    double l1[8];
    for (int r = 0; r < 8; ++r) {
        l1[r] = 0.0;
        for (int c = 0; c < 8; ++c) l1[r] += fabs(t.dct[r * 8 + c]);
    }
    double B[64];
    for (int k = 0; k < 64; ++k) {
        const double cmax = 128.0 * l1[k >> 3] * l1[k & 7] * (1.0 + 1e-12);
        const double qmax = floor(cmax / t.quant[k] + 0.5 + 1e-9);
        B[k] = qmax * t.dequant[k] * t.s2[k] * (1.0 + 1e-12);
    }
    double worst = 0.0;
    for (int p = 0; p < 64; ++p) {
        double g = 0.0, a = 0.0;
        for (int k = 0; k < 64; ++k) {
            g += kInvErrG[p][k] * B[k];
            a += kInvAbsL[p][k] * B[k];
        }
        const double e = g * (1.0 + u) + u * (128.0 + a) + 1e-9;
        worst = e > worst ? e : worst;
    }
    return worst;
}

int dctq::max_abs_quantized(const dctq::DevTables &t) {
    double l1[8];
    for (int r = 0; r < 8; ++r) {
        l1[r] = 0.0;
        for (int c = 0; c < 8; ++c) l1[r] += fabs(t.dct[r * 8 + c]);
    }
    int m = 0;
    for (int k = 0; k < 64; ++k) {
        const double cmax = 128.0 * l1[k >> 3] * l1[k & 7] * (1.0 + 1e-12);
        const int q = (int)floor(cmax / t.quant[k] + 0.5 + 1e-9);
        m = q > m ? q : m;
    }
    return m;
}

static int build_plan(const double *q, int quality, int adaptive, dctq_plan **out) {
    if (!out) return fail(DCTQ_EINVAL, "plan pointer is NULL");
    for (int c = 0; c < 64; ++c)
        if (!(q[c] >= 1.0 && q[c] <= 65535.0)) return fail(DCTQ_EINVAL, "quant_matrix entries must lie in [1, 65535]");
    int dev = 0, arch_ok = 0;
    HIPCHK(hipGetDevice(&dev), "hipGetDevice");
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, dev), "hipGetDeviceProperties");
    arch_ok = strncmp(prop.gcnArchName, "gfx950", 6) == 0;
    if (!arch_ok) return fail(DCTQ_ENODEV, "libdct_amd is built for gfx950 (MI355X) only");
    dctq_plan *p = new dctq_plan();
    p->quality = quality;
    p->adaptive = adaptive ? 1 : 0;
    p->device = dev;
    p->num_cus = prop.multiProcessorCount;
    p->variant = 2;  // the product kernels; dctq_diag_* entry points (libdct_amd_diag.so) can force another
    p->fallbacks = nullptr;
    dctq_host::dct_matrix(8, p->host.dct);
    for (int c = 0; c < 64; ++c) {
        const double s2 = kAanScale[c >> 3] * kAanScale[c & 7];
        p->host.quant[c] = q[c];
        p->host.dequant[c] = 1.0 / q[c];
        p->host.s2[c] = s2;
        p->host.iscale[c] = p->host.dequant[c] * s2;
        p->host.qscale[c] = q[c] * s2;
    }
    dctq::fill_fast_tables(q, p->adaptive, &p->fast);
    dctq::dc_const_table(p->host.dct, p->host.quant, p->host.dc_const);
    for (int k = 0; k < 8; ++k) p->host.s1[k] = kAanScale[k];
    for (int c = 0; c < 64; ++c) p->host.iscale32[c] = (float)p->host.iscale[c];
    p->inv_bound = dctq::inverse_f32_bound(p->host);
    p->inv_f32 = !p->adaptive && p->inv_bound <= kInvTol;
    p->symbol_bytes = dctq::max_abs_quantized(p->host) <= 511 ? 2 : 4;
    p->host.fast = p->fast;
    hipError_t e = hipMalloc(&p->dev, sizeof(dctq::DevTables));
    if (e != hipSuccess) {
        delete p;
        return fail(DCTQ_ENOMEM, "hipMalloc(plan tables)", e);
    }
    e = hipMemcpy(p->dev, &p->host, sizeof(dctq::DevTables), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        (void)hipFree(p->dev);
        delete p;
        return fail(DCTQ_EHIP, "hipMemcpy(plan tables)", e);
    }
    *out = p;
    return DCTQ_OK;
}

int dctq::plane_args(const dctq_plane *s, dctq::PlaneArgs *a) {
    if (!s || !s->pixels) return fail(DCTQ_EINVAL, "plane/pixels is NULL");
    if (s->width <= 0 || s->height <= 0 || s->width % 8 || s->height % 8)
        return fail(DCTQ_EINVAL, "width and height must be positive multiples of 8");
    if (s->stride < s->width || s->stride % 8) return fail(DCTQ_EINVAL, "stride must be >= width and a multiple of 8");
    if (((uintptr_t)s->pixels) % 8 || s->frame_stride % 8) return fail(DCTQ_EINVAL, "pixels/frame_stride must be 8-byte aligned");
    if (s->nframes < 1) return fail(DCTQ_EINVAL, "nframes must be >= 1");
    if (s->nframes > 1 && s->frame_stride < s->stride * (long long)s->height)
        return fail(DCTQ_EINVAL, "frame_stride smaller than one frame");
    const long long bw = s->width / 8, bh = s->height / 8, per = bw * bh, tot = per * s->nframes;
    if (tot >= (1ll << 31) - 256) return fail(DCTQ_EINVAL, "more than 2^31 blocks in one call");
    a->src = s->pixels;
    a->stride = s->stride;
    a->frame_stride = s->frame_stride;
    a->bw = (int)bw;
    a->nblk_frame = (int)per;
    a->nblk = (int)tot;
    a->div_bw = dctq::make_fastdiv((uint32_t)bw);
    a->div_frame = dctq::make_fastdiv((uint32_t)per);
    const long long span = (s->nframes - 1) * s->frame_stride + (s->height - 1) * s->stride + s->width;
    a->span = span < 0xFFFFFFFFll ? (uint32_t)span : 0u;
    return DCTQ_OK;
}


namespace dctq {
namespace {
std::recursive_mutex g_rand_mu;
char g_rand_state[256];  // the runtime's private rand() state, persists across calls
int g_rand_depth = 0;
bool g_rand_init = false;
}  // namespace

RandIsolation::RandIsolation() : saved_(nullptr) {
    g_rand_mu.lock();
    if (g_rand_depth++ == 0) {
        if (!g_rand_init) {
            saved_ = initstate(1u, g_rand_state, sizeof g_rand_state);
            g_rand_init = true;
        } else {
            saved_ = setstate(g_rand_state);
        }
    }
}

RandIsolation::~RandIsolation() {
    if (--g_rand_depth == 0) setstate(saved_);
    g_rand_mu.unlock();
}

namespace {
std::atomic<bool> g_runtime_up{false};  // some entry point initialised the HIP runtime
struct SeenKey {
    int device;
    const void *stream;
    unsigned long long id;  // hipStreamGetId: a re-created stream at a reused handle has another id
    uint32_t entries;       // bit e: entry point e already called by this thread on (device, stream)
};
thread_local std::vector<SeenKey> t_seen;
constexpr unsigned long long kNoId = ~0ull;
}  // namespace

bool runtime_started() { return g_runtime_up.load(std::memory_order_acquire); }
void note_runtime_started() { g_runtime_up.store(true, std::memory_order_release); }

// The stream's identity: its handle AND its runtime id.  The HIP runtime hands a
// destroyed stream's handle out again to the next hipStreamCreate, so the handle
// alone would take a re-created stream's first call (the one that may create its
// hardware queue, and reach libhsa's rand()) for a steady-state call.
// hipStreamGetId is looked up at run time: a process may have loaded an older HIP
// runtime than the one this library was built against (PyTorch ships its own
// libamdhip64.so.7, without it), and a link-time reference would then keep the
// library from loading.  Without it every stream's id reads 0 (the handle alone;
// hosts then call dctq_stream_release before hipStreamDestroy).
using StreamGetIdFn = hipError_t (*)(hipStream_t, unsigned long long *);
static StreamGetIdFn stream_get_id_fn() {
    static const StreamGetIdFn fn = (StreamGetIdFn)dlsym(RTLD_DEFAULT, "hipStreamGetId");
    return fn;
}
static unsigned long long stream_id(const void *stream) {
    const StreamGetIdFn fn = stream_get_id_fn();
    if (!fn) return 0;
    unsigned long long id = 0;
    if (fn((hipStream_t)stream, &id) != hipSuccess) {  // e.g. a special handle: the handle alone
        (void)hipGetLastError();
        return 0;
    }
    return id;
}

LaunchIsolation::LaunchIsolation(const void *stream, int entry) {
    const uint32_t bit = 1u << (entry & 31);
    int dev = -1;
    unsigned long long id = kNoId;
    if (runtime_started() && hipGetDevice(&dev) == hipSuccess) {
        id = stream_id(stream);
        for (const SeenKey &k : t_seen)
            if (k.device == dev && k.stream == stream && k.id == id && (k.entries & bit))
                return;  // steady state: no lock
    }
    iso_.emplace();
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) return;  // the call itself reports the error
    note_runtime_started();
    if (id == kNoId) id = stream_id(stream);
    for (SeenKey &k : t_seen)
        if (k.device == dev && k.stream == stream) {
            if (k.id != id) k = SeenKey{dev, stream, id, 0u};  // the handle now names another stream
            k.entries |= bit;
            return;
        }
    // a host that creates streams without end: forget them all now and then (each stream's
    // next first call is isolated again, which only costs that call the lock)
    if (t_seen.size() >= 64) t_seen.clear();
    t_seen.push_back(SeenKey{dev, stream, id, bit});
}

// dctq_stream_release: this thread forgets the stream (a host about to destroy it).
void forget_stream(const void *stream) {
    for (size_t i = 0; i < t_seen.size();)
        if (t_seen[i].stream == stream) {
            t_seen[i] = t_seen.back();
            t_seen.pop_back();
        } else {
            ++i;
        }
}
}  // namespace dctq

extern "C" {

int dctq_plan_create(int quality, int adaptive, dctq_plan **plan) {
    DCTQ_ENTRY;
    double q[64];
    quality = dctq_host::clamp_quality(quality);
    dctq_host::quant_matrix(8, quality, q);
    return build_plan(q, quality, adaptive, plan);
}

int dctq_plan_from_context(const QuantContext *qctx, dctq_plan **plan) {
    DCTQ_ENTRY;
    if (!qctx || qctx->block_size != 8 || !qctx->quant_matrix) return fail(DCTQ_EINVAL, "QuantContext must be 8x8");
    double q[64];
    for (int i = 0; i < 8; ++i)
        for (int j = 0; j < 8; ++j) q[i * 8 + j] = qctx->quant_matrix[i][j];
    return build_plan(q, qctx->quality, qctx->adaptive, plan);
}

void dctq_plan_destroy(dctq_plan *plan) {
    DCTQ_ENTRY;
    if (!plan) return;
    (void)hipFree(plan->dev);
    delete plan;
}

int dctq_plan_set_fallback_counter(dctq_plan *plan, unsigned long long *counter) {
    DCTQ_ENTRY;
    if (!plan) return fail(DCTQ_EINVAL, "plan is NULL");
    plan->fallbacks = counter;
    return DCTQ_OK;
}

}  // extern "C"

// A plan's tables and stash live on the device that was current at its creation.
int dctq::check_plan(const dctq_plan *plan) {
    if (!plan) return fail(DCTQ_EINVAL, "plan is NULL");
    int dev = -1;
    HIPCHK(hipGetDevice(&dev), "hipGetDevice");
    if (dev != plan->device) return fail(DCTQ_EINVAL, "plan was created on another device than the current one");
    return DCTQ_OK;
}

int dctq::plane_inputs(const dctq_plane *planes, int nplanes, dctq::PlaneSet *ps_out) {
    if (!planes) return fail(DCTQ_EINVAL, "planes is NULL");
    if (nplanes < 1 || nplanes > dctq::kMaxPlanes) return fail(DCTQ_EINVAL, "nplanes must be in [1, 4]");
    dctq::PlaneSet &ps = *ps_out;
    ps = {};
    ps.n = nplanes;
    uint32_t first = 0;
    for (int k = 0; k < nplanes; ++k) {
        int rc = dctq::plane_args(&planes[k], &ps.pl[k]);
        if (rc) return rc;
        ps.first[k] = first;
        first += (uint32_t)((ps.pl[k].nblk + 63) / 64);  // < 4 * 2^25
    }
    ps.first[nplanes] = first;
    for (int k = nplanes + 1; k <= dctq::kMaxPlanes; ++k) ps.first[k] = first;
    return DCTQ_OK;
}

int dctq::plane_set(const dctq_plane *planes, int nplanes, int16_t *const *coef, int32_t *const *var_num,
                    dctq::PlaneSet *ps_out) {
    if (!planes || !coef) return fail(DCTQ_EINVAL, "planes/coef is NULL");
    if (int rc = dctq::plane_inputs(planes, nplanes, ps_out)) return rc;
    dctq::PlaneSet &ps = *ps_out;
    for (int k = 0; k < nplanes; ++k) {
        if (!coef[k]) return fail(DCTQ_EINVAL, "coef[k] is NULL");
        if (((uintptr_t)coef[k]) % 16) return fail(DCTQ_EINVAL, "coef must be 16-byte aligned");
        if (var_num && !var_num[k]) return fail(DCTQ_EINVAL, "var_num given but var_num[k] is NULL");
        ps.coef[k] = coef[k];
        ps.var[k] = var_num ? var_num[k] : nullptr;
    }
    return DCTQ_OK;
}

extern "C" {

// The library holds no per-stream memory (the tie-queue kernel and its pixel stash
// are the diagnostic library's, fdct8_diag.hip); the calling thread only forgets
// the stream in its launch-isolation list, so a stream later created at the same
// handle is isolated on its first call even where the runtime cannot tell the two
// apart by id.
int dctq_stream_release(void *stream) {
    dctq::forget_stream(stream);
    return DCTQ_OK;
}

}  // extern "C"

extern "C" {

int dctq_forward_quant_planes(const dctq_plan *plan, const dctq_plane *planes, int nplanes, int16_t *const *coef,
                              int32_t *const *var_num, void *stream) {
    DCTQ_LAUNCH(stream, 0);
    if (int rc = dctq::check_plan(plan)) return rc;
    dctq::PlaneSet ps;
    int rc = dctq::plane_set(planes, nplanes, coef, var_num, &ps);
    if (rc) return rc;
    HIPCHK(dctq::launch_fdct8_quant(ps, plan->dev, plan->adaptive, plan->fallbacks, (hipStream_t)stream,
                                    plan->num_cus),
           "fdct8_quant_v3 launch");
    return DCTQ_OK;
}

int dctq_round_trip_planes(const dctq_plan *plan, const dctq_plane *planes, int nplanes, int16_t *const *coef,
                           int32_t *const *var_num, float *const *recon, void *stream) {
    DCTQ_LAUNCH(stream, 1);
    if (int rc = dctq::check_plan(plan)) return rc;
    if (!recon) return fail(DCTQ_EINVAL, "recon is NULL");
    dctq::RoundTripSet rt = {};
    int rc = dctq::plane_set(planes, nplanes, coef, var_num, &rt.ps);
    if (rc) return rc;
    for (int k = 0; k < nplanes; ++k) {
        if (!recon[k] || ((uintptr_t)recon[k]) % 16) return fail(DCTQ_EINVAL, "recon[k] NULL or not 16-byte aligned");
        rt.recon[k] = recon[k];
    }
    HIPCHK(dctq::launch_roundtrip(rt, plan->dev, plan->adaptive, plan->inv_f32 != 0, plan->fallbacks,
                                  (hipStream_t)stream, plan->num_cus),
           "roundtrip launch");
    return DCTQ_OK;
}

size_t dctq_encode_workspace_bytes(long long total_blocks) {
    return dctq::encode_workspace_bytes((total_blocks < 1 ? 1 : total_blocks) / 64 + dctq::kMaxPlanes + 1);
}

int dctq_plan_symbol_bytes(const dctq_plan *plan) { return plan ? plan->symbol_bytes : DCTQ_EINVAL; }

int dctq_abi_version(void) { return DCTQ_ABI_VERSION; }

static int encode_planes(const dctq_plan *plan, const dctq_plane *planes, int nplanes, int16_t *const *coef,
                         uint32_t *offsets, void *symbols, long long symbols_capacity, void *workspace, void *stream,
                         int symbol_bytes) {
    if (int rc = dctq::check_plan(plan)) return rc;
    if (!offsets || !workspace) return fail(DCTQ_EINVAL, "offsets/workspace is NULL");
    if (symbols_capacity < 0) return fail(DCTQ_EINVAL, "symbols_capacity < 0");
    if (((uintptr_t)symbols) % 4) return fail(DCTQ_EINVAL, "symbols must be 4-byte aligned");
    if (symbol_bytes == 2 && plan->symbol_bytes != 2)
        return fail(DCTQ_EINVAL, "the plan's quantized coefficients can exceed 511: 2-byte symbols cannot hold them "
                                 "(dctq_plan_symbol_bytes == 4; use dctq_encode_planes)");
    dctq::EncodeSet es = {};
    int rc = dctq::plane_set(planes, nplanes, coef, nullptr, &es.ps);
    if (rc) return rc;
    long long blocks = 0;
    for (int k = 0; k < nplanes; ++k) {
        es.blk_first[k] = (uint32_t)blocks;
        blocks += es.ps.pl[k].nblk;
        if (blocks >= (1ll << 26)) return fail(DCTQ_EINVAL, "more than 2^26 - 1 blocks in one encode");
    }
    es.blk_first[nplanes] = (uint32_t)blocks;
    HIPCHK(dctq::launch_encode(es, plan->dev, plan->adaptive, offsets, symbols, symbol_bytes,
                               symbols ? (unsigned long long)symbols_capacity : 0ull, workspace, (hipStream_t)stream,
                               plan->num_cus),
           "encode launch");
    return DCTQ_OK;
}

int dctq_encode_planes(const dctq_plan *plan, const dctq_plane *planes, int nplanes, int16_t *const *coef,
                       uint32_t *offsets, uint32_t *symbols, long long symbols_capacity, void *workspace,
                       void *stream) {
    DCTQ_LAUNCH(stream, 2);
    return encode_planes(plan, planes, nplanes, coef, offsets, symbols, symbols_capacity, workspace, stream, 4);
}

int dctq_encode_planes16(const dctq_plan *plan, const dctq_plane *planes, int nplanes, int16_t *const *coef,
                         uint32_t *offsets, uint16_t *symbols, long long symbols_capacity, void *workspace,
                         void *stream) {
    DCTQ_LAUNCH(stream, 13);
    return encode_planes(plan, planes, nplanes, coef, offsets, symbols, symbols_capacity, workspace, stream, 2);
}

int dctq_forward_quant(const dctq_plan *plan, const dctq_plane *src, int16_t *coef, int32_t *var_num, void *stream) {
    if (!src) return fail(DCTQ_EINVAL, "plane is NULL");
    return dctq_forward_quant_planes(plan, src, 1, &coef, var_num ? &var_num : nullptr, stream);
}

int dctq_forward_float(const dctq_plan *plan, const dctq_plane *src, float *coef, void *stream) {
    DCTQ_LAUNCH(stream, 3);
    if (int rc = dctq::check_plan(plan)) return rc;
    if (!coef) return fail(DCTQ_EINVAL, "coef is NULL");
    if (((uintptr_t)coef) % 16) return fail(DCTQ_EINVAL, "coef must be 16-byte aligned");
    dctq::PlaneArgs a;
    int rc = dctq::plane_args(src, &a);
    if (rc) return rc;
    HIPCHK(dctq::launch_fdct8_float_pair(a, plan->dev, coef, (hipStream_t)stream, plan->num_cus),
           "fdct8_float_pair launch");
    return DCTQ_OK;
}

int dctq_inverse(const dctq_plan *plan, const int16_t *coef, const int32_t *var_num, long long nblocks, float *recon,
                 void *stream) {
    DCTQ_LAUNCH(stream, 4);
    if (int rc = dctq::check_plan(plan)) return rc;
    if (!coef || !recon) return fail(DCTQ_EINVAL, "coef/recon is NULL");
    if (plan->adaptive && !var_num) return fail(DCTQ_EINVAL, "adaptive inverse needs var_num");
    if (nblocks < 0 || nblocks >= (1ll << 40)) return fail(DCTQ_EINVAL, "bad nblocks");
    if (((uintptr_t)coef) % 16 || ((uintptr_t)recon) % 16) return fail(DCTQ_EINVAL, "coef/recon must be 16-byte aligned");
    if (nblocks == 0) return DCTQ_OK;
    HIPCHK(dctq::launch_idct8_pair(plan->dev, plan->adaptive, coef, var_num, nblocks, recon, (hipStream_t)stream,
                                   plan->num_cus),
           "idct8_pair launch");
    return DCTQ_OK;
}

int dctq_synth(uint64_t seed, int kind, const dctq_plane *dst, void *stream) {
    DCTQ_LAUNCH(stream, 5);
    if (!dst || !dst->pixels) return fail(DCTQ_EINVAL, "dst is NULL");
    if (dst->width <= 0 || dst->height <= 0 || dst->width % 4 || dst->stride < dst->width || dst->stride % 4 ||
        dst->nframes < 1 || ((uintptr_t)dst->pixels) % 4)
        return fail(DCTQ_EINVAL, "bad synth plane geometry");
    HIPCHK(dctq::launch_synth(seed, kind, (uint8_t *)dst->pixels, dst->stride, dst->frame_stride, dst->width,
                              dst->height, dst->nframes, (hipStream_t)stream),
           "synth launch");
    return DCTQ_OK;
}

static int device_cus() {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1) return 256;
    return n;
}

static int rle_args(const void *a, const void *b, long long nblocks) {
    if (!a || !b) return fail(DCTQ_EINVAL, "NULL pointer");
    if (nblocks < 1 || nblocks >= (1ll << 26)) return fail(DCTQ_EINVAL, "nblocks must be in [1, 2^26)");
    return DCTQ_OK;
}

size_t dctq_rle_workspace_bytes(long long nblocks) { return dctq::rle_workspace_bytes(nblocks < 1 ? 1 : nblocks); }

int dctq_rle_count(const int16_t *coef, long long nblocks, uint32_t *offsets, void *workspace, void *stream) {
    DCTQ_LAUNCH(stream, 6);
    if (int rc = rle_args(coef, offsets, nblocks)) return rc;
    if (!workspace) return fail(DCTQ_EINVAL, "workspace is NULL");
    HIPCHK(dctq::launch_rle_count(coef, nblocks, offsets, workspace, (hipStream_t)stream, device_cus()),
           "rle_count launch");
    return DCTQ_OK;
}

int dctq_rle_emit(const int16_t *coef, long long nblocks, const uint32_t *offsets, uint32_t *symbols, void *stream) {
    DCTQ_LAUNCH(stream, 7);
    if (int rc = rle_args(coef, offsets, nblocks)) return rc;
    if (!symbols) return fail(DCTQ_EINVAL, "symbols is NULL");
    HIPCHK(dctq::launch_rle_emit(coef, nblocks, offsets, symbols, 4, ~0ull, (hipStream_t)stream, device_cus()),
           "rle_emit launch");
    return DCTQ_OK;
}

int dctq_rle_decode(const uint32_t *symbols, const uint32_t *offsets, long long nblocks, int16_t *coef,
                    void *stream) {
    DCTQ_LAUNCH(stream, 8);
    if (int rc = rle_args(symbols, offsets, nblocks)) return rc;
    if (!coef) return fail(DCTQ_EINVAL, "coef is NULL");
    HIPCHK(dctq::launch_rle_decode(symbols, 4, offsets, nblocks, coef, (hipStream_t)stream, device_cus()),
           "rle_decode launch");
    return DCTQ_OK;
}

int dctq_rle_decode16(const uint16_t *symbols, const uint32_t *offsets, long long nblocks, int16_t *coef,
                      void *stream) {
    DCTQ_LAUNCH(stream, 12);
    if (int rc = rle_args(symbols, offsets, nblocks)) return rc;
    if (!coef) return fail(DCTQ_EINVAL, "coef is NULL");
    if (((uintptr_t)symbols) % 4) return fail(DCTQ_EINVAL, "symbols must be 4-byte aligned");
    HIPCHK(dctq::launch_rle_decode(symbols, 2, offsets, nblocks, coef, (hipStream_t)stream, device_cus()),
           "rle_decode16 launch");
    return DCTQ_OK;
}

int dctq_huffman_bits(const int16_t *coef, long long nblocks, uint32_t *bits, void *stream) {
    DCTQ_LAUNCH(stream, 9);
    if (!coef || !bits) return fail(DCTQ_EINVAL, "coef/bits is NULL");
    if (nblocks < 0) return fail(DCTQ_EINVAL, "nblocks < 0");
    if (((uintptr_t)coef) % 16 || ((uintptr_t)bits) % 4) return fail(DCTQ_EINVAL, "coef must be 16-byte, bits 4-byte aligned");
    if (nblocks == 0) return DCTQ_OK;
    HIPCHK(dctq::launch_huffman_bits(coef, nblocks, bits, (hipStream_t)stream, device_cus()), "huffman_bits launch");
    return DCTQ_OK;
}

int dctq_huffman_bits_planes(const dctq_plan *plan, const dctq_plane *planes, int nplanes, uint32_t *bits,
                             void *stream) {
    DCTQ_LAUNCH(stream, 10);
    if (int rc = dctq::check_plan(plan)) return rc;
    if (!bits || ((uintptr_t)bits) % 4) return fail(DCTQ_EINVAL, "bits is NULL or not 4-byte aligned");
    // pixel planes only: the coefficients stay on chip (es.ps.coef stays NULL)
    dctq::EncodeSet es = {};
    int rc = dctq::plane_inputs(planes, nplanes, &es.ps);
    if (rc) return rc;
    long long blocks = 0;
    for (int k = 0; k < nplanes; ++k) {
        es.blk_first[k] = (uint32_t)blocks;
        blocks += es.ps.pl[k].nblk;
        if (blocks >= (1ll << 31)) return fail(DCTQ_EINVAL, "2^31 blocks or more in one launch");
    }
    es.blk_first[nplanes] = (uint32_t)blocks;
    HIPCHK(dctq::launch_huffman_from_pixels(es, plan->dev, plan->adaptive, bits, (hipStream_t)stream, plan->num_cus),
           "huffman_from_pixels launch");
    return DCTQ_OK;
}

int dctq_device_count(int *count) {
    DCTQ_ENTRY;
    HIPCHK(hipGetDeviceCount(count), "hipGetDeviceCount");
    return DCTQ_OK;
}
int dctq_set_device(int device) {
    DCTQ_ENTRY;
    HIPCHK(hipSetDevice(device), "hipSetDevice");
    return DCTQ_OK;
}
int dctq_malloc(void **ptr, size_t bytes) {
    DCTQ_ENTRY;
    HIPCHK(hipMalloc(ptr, bytes), "hipMalloc");
    return DCTQ_OK;
}
int dctq_free(void *ptr) {
    DCTQ_ENTRY;
    HIPCHK(hipFree(ptr), "hipFree");
    return DCTQ_OK;
}
int dctq_memcpy_htod(void *dst, const void *src, size_t bytes) {
    DCTQ_ENTRY;
    HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice), "hipMemcpy H2D");
    return DCTQ_OK;
}
int dctq_memcpy_dtoh(void *dst, const void *src, size_t bytes) {
    DCTQ_ENTRY;
    HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost), "hipMemcpy D2H");
    return DCTQ_OK;
}
int dctq_synchronize(void *stream) {
    DCTQ_LAUNCH(stream, 11);
    HIPCHK(hipStreamSynchronize((hipStream_t)stream), "hipStreamSynchronize");
    return DCTQ_OK;
}

const char *dctq_error_string(int code) {
    if (code == DCTQ_OK) return "ok";
    if (!g_err.empty()) return g_err.c_str();
    switch (code) {
    case DCTQ_EINVAL: return "invalid argument";
    case DCTQ_EHIP: return "HIP runtime error";
    case DCTQ_ENOMEM: return "out of device memory";
    case DCTQ_ENODEV: return "no gfx950 device";
    default: return "unknown error";
    }
}

}  // extern "C"
