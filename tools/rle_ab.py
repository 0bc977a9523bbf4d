"""Same-box A/B of the standalone RLE kernels (dctq_rle_count, dctq_rle_emit, dctq_rle_decode,
dctq_rle_decode16) between the product library and diagnostic builds
(tools/ubench/libvar_*.so): the quantized coefficients of 64 4K luma frames (q50), interleaved
rounds, each sample 3 launches back to back after one untimed launch; outputs compared with
the product's (libvar_no*.so: timing ablations, not compared).

    python tools/rle_ab.py [--rounds 10] [--kind uniform]
"""
import argparse
import ctypes as C
import glob
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import dct_amd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=10)
ap.add_argument("--frames", type=int, default=64)
ap.add_argument("--kind", default="uniform")
args = ap.parse_args()

nb = args.frames * 480 * 270
plan = dct_amd.Plan(50, 0)
coef = plan.forward_quant(dct_amd.synth(4242, args.kind, 3840, 2160, args.frames))
_, off_ref, sym4 = plan.encode_planes([dct_amd.synth(4242, args.kind, 3840, 2160, args.frames)], symbol_bytes=4)
_, _, sym2 = plan.encode_planes([dct_amd.synth(4242, args.kind, 3840, 2160, args.frames)], symbol_bytes=2)
total = sym4.numel()
off = torch.empty(nb + 1, dtype=torch.int32, device="cuda")
sym_out = torch.empty(total + 64, dtype=torch.int32, device="cuda")
dec = torch.empty((nb, 64), dtype=torch.int16, device="cuda")
stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
libs = {"default": dct_amd.LIB_PATH}
for p in sorted(glob.glob(os.path.join(ROOT, "tools", "ubench", "libvar_*.so"))):
    libs[os.path.basename(p)[7:-3]] = p
runs, outs = {}, {"count": off, "emit": sym_out, "decode": dec, "decode16": dec}
for k, path in libs.items():
    L = C.CDLL(path)
    L.dctq_rle_workspace_bytes.argtypes = [C.c_longlong]
    L.dctq_rle_workspace_bytes.restype = C.c_size_t
    ws = torch.empty(int(L.dctq_rle_workspace_bytes(nb)) // 4 + 1, dtype=torch.int32, device="cuda")
    for f in ("dctq_rle_count", "dctq_rle_emit", "dctq_rle_decode", "dctq_rle_decode16"):
        getattr(L, f).argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    L.dctq_rle_count.argtypes = [C.c_void_p, C.c_longlong, C.c_void_p, C.c_void_p, C.c_void_p]
    L.dctq_rle_emit.argtypes = [C.c_void_p, C.c_longlong, C.c_void_p, C.c_void_p, C.c_void_p]
    L.dctq_rle_decode.argtypes = L.dctq_rle_decode16.argtypes = [C.c_void_p, C.c_void_p, C.c_longlong, C.c_void_p,
                                                                 C.c_void_p]
    runs[(k, "count")] = (lambda L=L, ws=ws: L.dctq_rle_count(coef.data_ptr(), nb, off.data_ptr(), ws.data_ptr(), stream), ws)
    runs[(k, "emit")] = (lambda L=L: L.dctq_rle_emit(coef.data_ptr(), nb, off_ref.data_ptr(), sym_out.data_ptr(), stream), None)
    runs[(k, "decode")] = (lambda L=L: L.dctq_rle_decode(sym4.data_ptr(), off_ref.data_ptr(), nb, dec.data_ptr(), stream), None)
    runs[(k, "decode16")] = (lambda L=L: L.dctq_rle_decode16(sym2.data_ptr(), off_ref.data_ptr(), nb, dec.data_ptr(), stream), None)
times = {k: [] for k in runs}
for r in range(args.rounds + 1):
    for k, (fn, _) in runs.items():
        assert fn() == 0, k
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            fn()
        e1.record()
        torch.cuda.synchronize()
        if r:
            times[k].append(e0.elapsed_time(e1) / 3 * 1e-3)
ref = {}
for k, (fn, _) in runs.items():
    assert fn() == 0, k
    torch.cuda.synchronize()
    o = outs[k[1]][:total] if k[1] == "emit" else outs[k[1]]
    if k[1] not in ref:
        ref[k[1]] = o.clone()
    same = torch.equal(o, ref[k[1]])
    if not same and not k[0].startswith("no"):
        raise SystemExit(f"{k} output differs from default")
for k, v in times.items():
    m = statistics.median(v)
    base = statistics.median(times[("default", k[1])])
    print(f"{args.kind:8s} {k[0]:12s} {k[1]:9s} median {m * 1e6:8.1f} us  x{m / base:5.3f} of default", flush=True)
