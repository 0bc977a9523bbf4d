"""dctq_huffman_bits on one input kind (q50, 16 4K luma planes), 5 launches: a
target for rocprofv3 --pmc passes (tools/gpu_session.sh pmchuf)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dct_amd  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "uniform"
F = int(sys.argv[2]) if len(sys.argv) > 2 else 16
coef = dct_amd.Plan(50, 0).forward_quant(dct_amd.synth(9, kind, 3840, 2160, F))
for _ in range(5):
    dct_amd.huffman_bits(coef)
torch.cuda.synchronize()
