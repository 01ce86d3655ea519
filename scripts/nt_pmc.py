"""Workload for rocprofv3 --pmc passes on the NT GEMM vs hipBLASLt: the w13 forward shape
(32768 x 28672 x 4096), 5 launches of the gfx950 16x16x32 kernel (variant NT_VARIANT, default 4 =
LDS epilogue) then 5 launches of torch.mm (hipBLASLt), random operands."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tensorhive_fixed_amd.ops import _lib  # noqa: E402
from tensorhive_fixed_amd.ops.gemm_nt import gemm_nt_  # noqa: E402

_lib.load()
M, N, K = 32768, 28672, 4096
a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(5):
    gemm_nt_(a, b, c)
for _ in range(5):
    torch.mm(a, b.t(), out=c)
torch.cuda.synchronize()
print("done")
