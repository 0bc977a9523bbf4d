"""Time the non-quantizing kernels (forward_float, inverse) on 64 x 4K luma
planes in steady state (the bench's method: a 30 ms pre-warm, then samples of 3 launches back to
back after one untimed launch, HIP events, medians); report % of 8 TB/s on algorithmic bytes.
Labels: v1 = plan variant 1 (the one-workgroup-per-256-blocks kernels), v2 = plan
variant 2 (the product dispatch: paired lane-per-block kernels; the forward with
var_num runs whichever quantizing kernel the dispatch picks, fdct8_quant_v3 at q50)."""
import os
import statistics
import time
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dct_amd  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 64
W, H = 3840, 2160
nblk = F * (W // 8) * (H // 8)
px = dct_amd.synth(7, "uniform", W, H, F)
res = {}
def steady(fn, reps=8, b2b=3, prewarm_s=0.03):
    """Median launch time in steady state, the bench's method (round 4): ~30 ms of the
    launch back to back untimed (an idle MI355X drops its clocks within milliseconds),
    then `reps` samples of `b2b` launches back to back, each after one untimed launch
    (a launch pays for the write-back its predecessor left in the caches)."""
    t = time.perf_counter()
    while time.perf_counter() - t < prewarm_s:
        for _ in range(4):
            fn()
        torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        e0.record()
        for _ in range(b2b):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e-3 / b2b)
    return statistics.median(ts)


for var, ad in [(v, a) for a in (0, 1) for v in ("1", "2")]:
    plan = dct_amd.Plan(50, ad, variant=int(var))
    vn = torch.empty(nblk, dtype=torch.int32, device="cuda")
    coef = plan.forward_quant(px, var_num=vn)
    ff = torch.empty((nblk, 64), dtype=torch.float32, device="cuda")
    rec = torch.empty((nblk, 64), dtype=torch.float32, device="cuda")
    jobs = {f"v{var} forward_float a{ad}": (lambda: plan.forward_float(px, out=ff), 64 + 256),
            f"v{var} inverse a{ad}": (lambda: plan.inverse(coef, var_num=vn, out=rec), 128 + 256 + (4 if ad else 0))}
    if var == "2":
        jobs[f"v{var} forward_quant+var a{ad}"] = (lambda: plan.forward_quant(px, out=coef, var_num=vn), 64 + 128 + 4)
    for name, (fn, bpb) in jobs.items():
        med = steady(fn)
        print(f"{name:27s} median {med*1e6:8.1f} us  {nblk/med/1e9:6.2f} Gblk/s  {nblk*bpb/med/1e9:6.0f} GB/s "
              f"({nblk*bpb/med/8e12*100:5.1f}% of 8 TB/s, {bpb} B/block)")


# ---- zigzag + RLE on the forward-quant output (q50): count+emit and decode
for kind in ("uniform", "smooth"):
    px2 = dct_amd.synth(9, kind, W, H, F)
    plan = dct_amd.Plan(50, 0)
    coef = plan.forward_quant(px2)
    off, sym = dct_amd.rle_encode(coef)
    total = sym.numel()
    back = torch.empty_like(coef)
    hb = torch.empty(nblk, dtype=torch.int32, device="cuda")
    ws = torch.empty(int(dct_amd.lib().dctq_rle_workspace_bytes(nblk)) // 4 + 1, dtype=torch.int32, device="cuda")
    L = dct_amd.lib()
    import ctypes as C
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    jobs = {
        "rle_count": (lambda: L.dctq_rle_count(C.c_void_p(coef.data_ptr()), nblk, C.c_void_p(off.data_ptr()),
                                               C.c_void_p(ws.data_ptr()), s), nblk * (128 + 4 + 8)),
        "rle_emit": (lambda: L.dctq_rle_emit(C.c_void_p(coef.data_ptr()), nblk, C.c_void_p(off.data_ptr()),
                                             C.c_void_p(sym.data_ptr()), s), nblk * (128 + 4) + 4 * total),
        "huffman_bits": (lambda: L.dctq_huffman_bits(C.c_void_p(coef.data_ptr()), nblk, C.c_void_p(hb.data_ptr()), s),
                         nblk * (128 + 4)),
        "rle_decode": (lambda: L.dctq_rle_decode(C.c_void_p(sym.data_ptr()), C.c_void_p(off.data_ptr()), nblk,
                                                 C.c_void_p(back.data_ptr()), s), nblk * (128 + 4) + 4 * total),
    }
    for name, (fn, nbytes) in jobs.items():
        med = steady(fn)
        print(f"{name + ' ' + kind:27s} median {med*1e6:8.1f} us  {nblk/med/1e9:6.2f} Gblk/s  {nbytes/med/1e9:6.0f} GB/s "
              f"({nbytes/med/8e12*100:5.1f}% of 8 TB/s, {nbytes/nblk:.0f} B/block, {total/nblk:.1f} symbols/block)")
    assert torch.equal(back, coef)
