"""TN hb kernel (mode 10): XCD band height (output-tile rows per band) per wgrad shape, K = 32768 (the LM head:
one 4096-token chunk)."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorhive_fixed_amd.ops import _lib  # noqa: E402
from tensorhive_fixed_amd.ops.gemm_tn import default_splitk, gemm_tn_  # noqa: E402


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


BANDS = tuple(int(v) for v in os.environ.get("TN_BANDS", "1,2,4,8,15").split(","))


def main():
    _lib.load()
    for name, M, N, T in (("wqkv", 6144, 4096, 32768), ("wo", 4096, 4096, 32768), ("w2", 4096, 14336, 32768),
                          ("w13", 28672, 4096, 32768), ("head", 128256, 4096, 4096)):
        a = torch.randn(T, M, device="cuda", dtype=torch.bfloat16)
        b = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        sk = default_splitk(M, N, T)
        ref = torch.empty_like(c)
        gemm_tn_(a, b, ref, splitk=sk, pingpong=10, band=0)
        res = {}
        for band in BANDS:
            gemm_tn_(a, b, c, splitk=sk, pingpong=10, band=band)
            assert ((c.float() - ref.float()).norm() / ref.float().norm()).item() < 1e-3, band  # split order differs
        for _ in range(5):
            for band in BANDS:
                res.setdefault(band, []).append(timed(lambda: gemm_tn_(a, b, c, splitk=sk, pingpong=10, band=band)))
        fl = 2.0 * M * N * T
        print(json.dumps({"gemm": name, "K": T, "splitk": sk, **{f"band{k}_ms": round(min(v), 4) for k, v in res.items()},
                          **{f"band{k}_tflops": round(fl / min(v) / 1e9) for k, v in res.items()}}), flush=True)
        del a, b, c, ref
    return 0


if __name__ == "__main__":
    sys.exit(main())
