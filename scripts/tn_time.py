"""TN weight-gradient GEMM timing on the Llama-3-8B shapes (K = 32768 tokens) with whatever kernel library
TH_KERNEL_LIB selects: fp32 check on wo, then 3 rounds x 10-launch medians per shape (best round)."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorhive_fixed_amd.ops import _lib  # noqa: E402
from tensorhive_fixed_amd.ops.gemm_tn import gemm_tn_, tn_plan  # noqa: E402

T = 32768
SHAPES = [("wqkv", 6144, 4096), ("wo", 4096, 4096), ("w2", 4096, 14336), ("w13", 28672, 4096)]


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
    torch.manual_seed(0)
    a = torch.randn(2048, 512, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(2048, 768, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(512, 768, device="cuda", dtype=torch.bfloat16)
    gemm_tn_(a, b, out)
    ref = a.float().t() @ b.float()
    err = ((out.float() - ref).norm() / ref.norm()).item()
    assert err < 1e-2, err
    lib = os.environ.get("TH_KERNEL_LIB", "prod")
    for name, n_out, k_in in SHAPES:
        dy = torch.randn(T, n_out, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(T, k_in, device="cuda", dtype=torch.bfloat16)
        c = torch.empty(n_out, k_in, device="cuda", dtype=torch.bfloat16)
        best = min(timed(lambda: gemm_tn_(dy, x, c)) for _ in range(3))
        flops = 2.0 * T * n_out * k_in
        print(json.dumps({"lib": os.path.basename(lib), "shape": name, "plan": list(tn_plan(n_out, k_in, T)),
                          "ms": round(best, 4), "tflops": round(flops / best / 1e9, 1), "check_rel_err": round(err, 5)}),
              flush=True)
        del dy, x, c


if __name__ == "__main__":
    main()
