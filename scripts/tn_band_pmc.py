"""w13 weight-gradient TN GEMM (28672 x 4096, K 32768) with XCD band heights 1 and 8, alternating, 3 each:
run under rocprofv3 --pmc to compare L2 hit / miss and HBM read requests per band (dispatch order = the
printed order)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorhive_fixed_amd.ops import _lib  # noqa: E402
from tensorhive_fixed_amd.ops.gemm_tn import gemm_tn_  # noqa: E402

_lib.load()
T, M, N = 32768, 28672, 4096
a = torch.randn(T, M, device="cuda", dtype=torch.bfloat16)
b = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
order = []
for _ in range(3):
    for band in (1, 8):
        gemm_tn_(a, b, c, splitk=1, pingpong=10, band=band)
        order.append(band)
torch.cuda.synchronize()
print("band order:", order, flush=True)
