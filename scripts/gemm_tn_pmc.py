"""Workload for rocprofv3 --pmc passes on the TN weight-gradient GEMM: the wo shape (4096 x 4096,
K = 32768: one 256x256 tile per CU), ping-pong and lockstep schedules, 5 launches each."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tensorhive_fixed_amd.ops import _lib  # noqa: E402
from tensorhive_fixed_amd.ops.gemm_tn import gemm_tn_  # noqa: E402

_lib.load()
M, N, K = 4096, 4096, 32768
a = torch.randn(K, M, device="cuda", dtype=torch.bfloat16)
b = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
o = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for pp in (True, False):
    for _ in range(5):
        gemm_tn_(a, b, o, splitk=1, pingpong=pp)
torch.cuda.synchronize()
print("done")
