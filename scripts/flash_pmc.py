"""Workload for rocprofv3 --pmc runs on the flash kernels: fwd x5, bwd x3 at B4 S4096 32/8 heads."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tensorhive_fixed_amd.ops import _lib  # noqa: E402
from tensorhive_fixed_amd.ops.attention import flash_bwd, flash_fwd  # noqa: E402

_lib.load()
B, S, Hq, Hkv, D = 4, 4096, 32, 8, 128
qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
var = os.environ.get("FA_VARIANT")
for _ in range(5):
    o, lse = flash_fwd(qkv, B, S, Hq, Hkv, D, variant=None if var is None else int(var))
do = torch.randn_like(o)
for _ in range(3):
    flash_bwd(do, qkv, o, lse, B, S, Hq, Hkv, D, flags=int(os.environ.get("FA_BWD_FLAGS", "0")))
torch.cuda.synchronize()
print("done")
