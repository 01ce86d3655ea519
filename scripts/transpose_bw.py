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


# the step's weight transposes are [out, in] -> [in, out]: wqkv 6144x4096, wo 4096x4096, w13 28672x4096,
# w2 4096x14336, LM head 128256x4096
for R, C in ((32768, 28672), (32768, 4096), (28672, 4096), (4096, 14336), (4096, 6144), (6144, 4096), (4096, 4096),
             (128256, 4096)):
    x = torch.randn(R, C, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(C, R, device="cuda", dtype=torch.bfloat16)
    gb = 2 * x.numel() * 2 / 1e9
    res = {"R": R, "C": C}
    for tile in (0, 1, 2, 3):
        ms_k = t(lambda: transpose(x, out, tile=tile))
        assert torch.equal(out, x.t())
        res[f"tile{tile}_TBps"] = round(gb / ms_k, 2)
    ms_t = t(lambda: out.copy_(x.t()))
    res["torch_TBps"] = round(gb / ms_t, 2)
    print(json.dumps(res), flush=True)
    del x, out
    torch.cuda.empty_cache()
