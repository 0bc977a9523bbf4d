#!/usr/bin/env python3
"""Encoder with the count fused into the forward (dctq_encode_planes) vs the unfused pipeline (forward_quant +
rle_count + rle_emit) on 64 4K luma planes, uniform and smooth, HIP events;
bytes per block are each path's algorithmic HBM traffic."""
import ctypes as C
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dct_amd  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 64
W, H = 3840, 2160
nblk = F * (W // 8) * (H // 8)
L = dct_amd.lib()
for kind in ("uniform", "smooth"):
    px = dct_amd.synth(21, kind, W, H, F)
    plan = dct_amd.Plan(50, 0)
    coef = plan.forward_quant(px)
    off, sym = dct_amd.rle_encode(coef)
    total = sym.numel()
    sym_buf = torch.empty(total + 64, dtype=torch.int32, device="cuda")
    off2 = torch.empty_like(off)
    ws = torch.empty(int(L.dctq_rle_workspace_bytes(nblk)) // 4 + 1, dtype=torch.int32, device="cuda")
    wse = torch.empty(int(L.dctq_encode_workspace_bytes(nblk)) // 4 + 1, dtype=torch.int32, device="cuda")
    d = (dct_amd._Plane * 1)(dct_amd.plane_desc(px))
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)

    def unfused():
        plan.forward_quant(px, out=coef)
        assert L.dctq_rle_count(C.c_void_p(coef.data_ptr()), nblk, C.c_void_p(off2.data_ptr()),
                                C.c_void_p(ws.data_ptr()), s) == 0
        assert L.dctq_rle_emit(C.c_void_p(coef.data_ptr()), nblk, C.c_void_p(off2.data_ptr()),
                               C.c_void_p(sym_buf.data_ptr()), s) == 0

    def fused():
        cp = (C.c_void_p * 1)(coef.data_ptr())
        assert L.dctq_encode_planes(plan._h, d, 1, C.cast(cp, C.c_void_p), C.c_void_p(off2.data_ptr()),
                                    C.c_void_p(sym_buf.data_ptr()), total + 64, C.c_void_p(wse.data_ptr()), s) == 0

    spb = 4.0 * total / nblk
    jobs = {"unfused forward+count+emit": (unfused, 192 + 140 + 132 + spb),
            "encode (count fused)": (fused, 192 + 4 + 8 + 132 + spb)}
    for name, (fn, bpb) in jobs.items():
        fn()
        torch.cuda.synchronize()
        assert torch.equal(off2, off) and torch.equal(sym_buf[:total], sym), name
        ts = []
        for _ in range(8):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e-3)
        med = statistics.median(ts)
        print(f"{name:28s} {kind:8s} median {med*1e6:8.1f} us  {nblk/med/1e9:6.2f} Gblk/s  "
              f"{nblk*bpb/med/1e9:6.0f} GB/s ({bpb:.0f} B/block, {total/nblk:.1f} symbols/block)")
