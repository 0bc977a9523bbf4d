"""Per-block Huffman sizes of the bench's 64-frame 4K 4:2:0 stack two ways, interleaved,
steady state (clock pre-warm, 3 calls back to back per sample): dctq_forward_quant_planes +
dctq_huffman_bits (two launches, the coefficients through HBM) against dctq_huffman_bits_planes
(one launch, coefficients on chip).  Outputs compared.

    python tools/huf_pixels_bench.py [frames] [kind]"""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dct_amd  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 64
kind = sys.argv[2] if len(sys.argv) > 2 else "uniform"
planes = [dct_amd.synth(1, kind, 3840, 2160, F), dct_amd.synth(2, kind, 1920, 1080, 2 * F)]
nblk = F * 480 * 270 + 2 * F * 240 * 135
plan = dct_amd.Plan(50, 0)
coefs = plan.forward_quant_planes(planes)
flat = torch.empty((nblk, 64), dtype=torch.int16, device="cuda")
bits_a = torch.empty(nblk, dtype=torch.int32, device="cuda")
bits_b = torch.empty(nblk, dtype=torch.int32, device="cuda")


def two_launch():
    plan.forward_quant_planes(planes, outs=[flat[:F * 480 * 270], flat[F * 480 * 270:]])
    dct_amd.huffman_bits(flat, out=bits_a)


def fused():
    plan.huffman_bits_planes(planes, out=bits_b)


t_end = time.perf_counter() + 0.3
while time.perf_counter() < t_end:
    fused()
    torch.cuda.synchronize()
two_launch()
fused()
torch.cuda.synchronize()
assert torch.equal(bits_a, bits_b), "fused sizes differ"
times = {"forward_quant_planes + huffman_bits": [], "huffman_bits_planes (fused)": []}
for r in range(10):
    for name, fn in (("forward_quant_planes + huffman_bits", two_launch), ("huffman_bits_planes (fused)", fused)):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            fn()
        e1.record()
        torch.cuda.synchronize()
        times[name].append(e0.elapsed_time(e1) * 1e-3 / 3)
for name, ts in times.items():
    m = statistics.median(ts)
    print(f"{name:38s} {kind:8s} median {m * 1e6:8.1f} us  {nblk / m / 1e9:6.2f} G blocks/s", flush=True)
print(f"blocks {nblk}, outputs equal")
