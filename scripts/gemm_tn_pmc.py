"""Workload for rocprofv3 --pmc passes: the gfx950 TN GEMM on the wo weight-grad shape (4096 x 4096,
K = 32768: one 256x256 tile per CU) under each schedule, and hipBLASLt on the same FLOPs in the
K-contiguous (NT) form, 5 launches each."""
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
for pp in [int(x) for x in os.environ.get("TN_SCHEDULES", "9").split(",")]:
    for _ in range(5):
        gemm_tn_(a, b, o, splitk=1, pingpong=pp)
aT, bT = a.t().contiguous(), b.t().contiguous()  # [M, K], [N, K]: K-contiguous operands
for _ in range(5):
    torch.mm(aT, bT.t(), out=o)
torch.cuda.synchronize()
print("done")
