"""Achieved HBM bandwidth of the HIP bf16 transpose vs torch's ``.t().contiguous()`` on the
training-step shapes (read + write bytes / time)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tensorhive_fixed_amd.ops import _lib
from tensorhive_fixed_amd.ops.transpose import transpose

_lib.load(build_if_missing=True)


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


for R, C in ((32768, 28672), (32768, 4096), (28672, 4096), (4096, 14336), (4096, 6144), (128256, 4096)):
    x = torch.randn(R, C, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(C, R, device="cuda", dtype=torch.bfloat16)
    ms_k = t(lambda: transpose(x, out))
    ms_t = t(lambda: out.copy_(x.t()))
    gb = 2 * x.numel() * 2 / 1e9
    print(json.dumps({"R": R, "C": C, "hip_ms": round(ms_k, 4), "hip_TBps": round(gb / ms_k, 2),
                      "torch_ms": round(ms_t, 4), "torch_TBps": round(gb / ms_t, 2)}), flush=True)
    del x, out
    torch.cuda.empty_cache()
