#!/usr/bin/env python3
"""A/B the gfx950 TN weight-gradient GEMM against hipBLASLt on the Llama-3-8B wgrad shapes (MB8),
interleaved rounds in one process (guide §5.4 rule 24), random operands."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tensorhive_fixed_amd.ops import _lib  # noqa: E402
from tensorhive_fixed_amd.ops.gemm_tn import default_splitk, gemm_tn_  # noqa: E402

T = int(os.environ.get("TH_TOKENS", "32768"))
SHAPES = [("wqkv", 6144, 4096), ("wo", 4096, 4096), ("w13", 28672, 4096), ("w2", 4096, 14336)]


def timed(fn, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    _lib.load()
    for name, M, N in SHAPES:
        a = torch.randn(T, M, device="cuda", dtype=torch.bfloat16)
        b = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        o1 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        o2 = torch.empty_like(o1)
        variants = {"hipblaslt": lambda: torch.mm(a.t(), b, out=o1)}
        pps = [int(x) for x in os.environ.get("TN_PP", "9,10").split(",")]
        sks = sorted({1, 2, default_splitk(M, N, T)}) if os.environ.get("TN_ALL_SPLITK", "1") == "1" \
            else [default_splitk(M, N, T)]
        for sk in sks:
            for pp in pps:
                variants[f"tn_s{pp}_sk{sk}"] = (lambda sk=sk, pp=pp: gemm_tn_(a, b, o2, splitk=sk, pingpong=pp))
        res = {k: [] for k in variants}
        for _ in range(3):
            for k, fn in variants.items():
                res[k].append(timed(fn))
        torch.mm(a.t(), b, out=o1)
        errs = {}
        for pp in pps:
            gemm_tn_(a, b, o2, splitk=1, pingpong=pp)
            errs[pp] = round(((o1.float() - o2.float()).abs().max() / o1.float().abs().max()).item(), 5)
        err = max(errs.values())
        fl = 2.0 * M * N * T
        print(json.dumps({"gemm": name, "M": M, "N": N, "K": T, "rel_err_vs_hipblaslt": round(err, 5),
                          "default_splitk": default_splitk(M, N, T),
                          **{k: {"ms": round(min(v), 4), "tflops": round(fl / min(v) / 1e9, 1)} for k, v in res.items()}}),
              flush=True)
        del a, b, o1, o2
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
