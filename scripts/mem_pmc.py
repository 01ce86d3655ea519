"""Workload for rocprofv3 --pmc on the LDS-using streaming kernels: SwiGLU backward with the transposed
output and the bf16 transpose, at the Llama-3-8B MLP shapes (3 launches each)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tensorhive_fixed_amd.ops import _lib  # noqa: E402
from tensorhive_fixed_amd.ops.transpose import transpose  # noqa: E402

_lib.load()
T, F, D = 32768, 14336, 4096
dev = torch.device("cuda")
gu = torch.randn(T, 2 * F, device=dev, dtype=torch.bfloat16)
da = torch.randn(T, F, device=dev, dtype=torch.bfloat16)
dgu = torch.empty_like(gu)
dguT = torch.empty(2 * F, T, device=dev, dtype=torch.bfloat16)
h = torch.randn(T, D, device=dev, dtype=torch.bfloat16)
for _ in range(3):
    _lib.call("th_swiglu_bwd_t", da.data_ptr(), gu.data_ptr(), dgu.data_ptr(), dguT.data_ptr(), T, F,
              _lib.stream_ptr(dev))
    transpose(h)
torch.cuda.synchronize()
print("done")
