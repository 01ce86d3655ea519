"""Workload for rocprofv3 --pmc runs on the TN weight-grad kernel: the w13 wgrad shape (28672 x 4096,
K = 32768 tokens), 5 launches of ping-pong mode TN_PP (2: chunk ^ (r & 3) images, 6: chunk ^ ((r + r>>3) & 3))."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tensorhive_fixed_amd.ops import _lib  # noqa: E402
from tensorhive_fixed_amd.ops.gemm_tn import gemm_tn_  # noqa: E402

_lib.load()
T, M, N = 32768, 28672, 4096
a = torch.randn(T, M, device="cuda", dtype=torch.bfloat16)
b = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
o = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(5):
    gemm_tn_(a, b, o, splitk=1, pingpong=int(os.environ.get("TN_PP", "6")))
torch.cuda.synchronize()
print("done")
