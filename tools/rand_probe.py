"""Which HIP operations consume the host's glibc rand() stream (GPU box).

    python tools/rand_probe.py

For each step: srand(1), the operation, a device synchronize and a short sleep,
then one rand() -- its index in glibc's seed-1 sequence is how many draws the
operation (or a runtime thread it started) consumed.  The library's own calls
are shown with and without a fresh stream.  Evidence for LaunchIsolation
(dct_amd/csrc/api.hip) and for the stream tests of tests/test_gpu_parity.py.
"""
import ctypes as C
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dct_amd  # noqa: E402

libc = C.CDLL("libc.so.6")
libc.rand.restype = C.c_int
libc.srand(1)
seq = [libc.rand() for _ in range(4096)]
hip = C.CDLL("libamdhip64.so.7")
hip.hipStreamCreate.argtypes = [C.POINTER(C.c_void_p)]
hip.hipStreamDestroy.argtypes = [C.c_void_p]
print("hipStreamGetId in the loaded runtime:", hasattr(hip, "hipStreamGetId"))
plan = dct_amd.Plan(50, 0)
px = dct_amd.synth(1, "uniform", 64, 64, 1)
out = plan.forward_quant(px)
torch.cuda.synchronize()
L = dct_amd.lib()


class S:
    def __init__(self, h):
        self.cuda_stream = h


def probe(name, fn):
    libc.srand(1)
    r = fn()
    torch.cuda.synchronize()
    time.sleep(0.05)
    v = libc.rand()
    idx = seq.index(v) if v in seq else -1
    print(f"{name:60s} draws consumed: {idx}")
    return r


def create():
    h = C.c_void_p()
    assert hip.hipStreamCreate(C.byref(h)) == 0
    return h.value


for rep in range(3):
    h = probe("hipStreamCreate", create)
    probe("library forward, first call on the new stream", lambda: plan.forward_quant(px, out=out, stream=S(h)))
    probe("library forward, second call", lambda: plan.forward_quant(px, out=out, stream=S(h)))
    probe("dctq_stream_release", lambda: L.dctq_stream_release(C.c_void_p(h)))
    probe("hipStreamDestroy", lambda: hip.hipStreamDestroy(C.c_void_p(h)))
    h2 = probe("hipStreamCreate (again)", create)
    print("   handle reused:", h2 == h)
    probe("library forward, first call on the re-created stream", lambda: plan.forward_quant(px, out=out, stream=S(h2)))
    probe("hipStreamDestroy", lambda: hip.hipStreamDestroy(C.c_void_p(h2)))
print("done")
