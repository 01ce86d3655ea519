"""The gate|up (w13) weight gradient, two ways, at the training shape (T 32768, F 14336, D 4096), one box:
  NT (default): swiglu_bwd_t (dGU and dGU^T), transpose(H), hipBLASLt dGU^T @ (H^T)^T
  TN          : swiglu_bwd (dGU only), the gfx950 TN kernel on dGU and H as they are
Interleaved rounds of 10-launch medians; prints the per-layer cost of each path's kernels."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorhive_fixed_amd.ops import _lib  # noqa: E402
from tensorhive_fixed_amd.ops.gemm_tn import gemm_tn_  # noqa: E402
from tensorhive_fixed_amd.ops.transpose import transpose  # noqa: E402

T, F, D = 32768, 14336, 4096


def timed(fn, iters=10):
    ts = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    return statistics.median(ts)


def main():
    _lib.load()
    g = torch.Generator(device="cuda").manual_seed(0)
    gu = torch.randn(T, 2 * F, device="cuda", dtype=torch.bfloat16, generator=g)
    da = torch.randn(T, F, device="cuda", dtype=torch.bfloat16, generator=g) * 0.01
    h = torch.randn(T, D, device="cuda", dtype=torch.bfloat16, generator=g)
    dgu = torch.empty_like(gu)
    dguT = torch.empty(2 * F, T, device="cuda", dtype=torch.bfloat16)
    gw = torch.empty(2 * F, D, device="cuda", dtype=torch.bfloat16)
    st = _lib.stream_ptr(gu.device)
    parts = {
        "swiglu_bwd_t": lambda: _lib.call("th_swiglu_bwd_t", da.data_ptr(), gu.data_ptr(), dgu.data_ptr(), dguT.data_ptr(), T, F, st),
        "transpose_h": lambda: transpose(h),
        "hipblaslt_nt": lambda: torch.mm(dguT, transpose_cache["hT"].t(), out=gw),
        "swiglu_bwd": lambda: _lib.call("th_swiglu_bwd", da.data_ptr(), gu.data_ptr(), dgu.data_ptr(), T, F, st),
        "tn_hb": lambda: gemm_tn_(dgu, h, gw),
    }
    transpose_cache = {"hT": transpose(h)}
    parts["swiglu_bwd_t"]()
    ref = torch.mm(dguT, transpose_cache["hT"].t())
    parts["swiglu_bwd"]()
    gemm_tn_(dgu, h, gw)
    rel = ((gw.float() - ref.float()).norm() / ref.float().norm()).item()
    res = {k: [] for k in parts}
    for _ in range(3):
        for k, fn in parts.items():
            res[k].append(timed(fn))
    best = {k: round(min(v), 4) for k, v in res.items()}
    nt = best["swiglu_bwd_t"] + best["transpose_h"] + best["hipblaslt_nt"]
    tn = best["swiglu_bwd"] + best["tn_hb"]
    print(json.dumps({"ms": best, "nt_path_ms": round(nt, 4), "tn_path_ms": round(tn, 4),
                      "tn_vs_nt_rel_diff": rel}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
