"""NT GEMM K sweep at N = 4096 (round 5): where the one-k-tile schedule ("hb", flags 32) loses to the
round-4 default (variant 8) as K grows.  TFLOP/s per K for v8, hb and hipBLASLt; with PMC=1 runs each
kernel once on the K = 28672 shape (for rocprofv3 --pmc)."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorhive_fixed_amd.ops import _lib  # noqa: E402
from tensorhive_fixed_amd.ops.gemm_nt import gemm_nt_  # noqa: E402


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
    dev = torch.device("cuda:0")
    M, N = 32768, 4096
    if os.environ.get("PMC") == "1":
        K = 28672
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        b = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        for v in (8, 32):
            gemm_nt_(a, b, c, variant=v)
        torch.mm(a, b.t(), out=c)
        torch.cuda.synchronize()
        return 0
    for K in (4096, 8192, 16384, 28672):
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        b = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        out = {"M": M, "N": N, "K": K}
        fl = 2.0 * M * N * K
        res = {"v8": [], "hb": [], "hipblaslt": []}
        for _ in range(3):
            res["v8"].append(timed(lambda: gemm_nt_(a, b, c, variant=8)))
            res["hb"].append(timed(lambda: gemm_nt_(a, b, c, variant=32)))
            res["hipblaslt"].append(timed(lambda: torch.mm(a, b.t(), out=c)))
        for k, ts in res.items():
            out[k] = round(fl / min(ts) / 1e9)
        print(json.dumps(out), flush=True)
        del a, b, c
    return 0


if __name__ == "__main__":
    sys.exit(main())
