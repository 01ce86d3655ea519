"""gfx950 NT GEMM (ops/csrc/gemm_nt.hip) vs hipBLASLt (torch.mm) on the Llama-3-8B forward and
input-gradient shapes (MB 8 x 4096 tokens): fp32 check first, then interleaved timing on random
operands (median of 15 launches per arm, 3 rounds, best round).  One JSON line per shape.

    python scripts/bench_gemm_nt.py [SHAPE ...]
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, ".")
from tensorhive_fixed_amd.ops import _lib  # noqa: E402
from tensorhive_fixed_amd.ops.gemm_nt import gemm_nt_, usable  # noqa: E402

T, D, F, V = 32768, 4096, 14336, 128256
SHAPES = [("wqkv.fwd", T, 6144, D), ("wo.fwd", T, D, D), ("w13.fwd", T, 2 * F, D), ("w2.fwd", T, D, F),
          ("wqkv.dgrad", T, D, 6144), ("wo.dgrad", T, D, D), ("w13.dgrad", T, D, 2 * F), ("w2.dgrad", T, F, D),
          ("w13.wgrad", 2 * F, D, T), ("head.fwd", 4096, V, D), ("head.dgrad", 4096, D, V)]


VARIANTS = [int(v) for v in os.environ.get("GEMM_VARIANTS", "0").split(",")]


def timed(fn, iters=15):
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
    want = set(sys.argv[1:])
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    for (M, N, K) in ((512, 512, 64), (256, 768, 4096), (1024, 256, 14336)):
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
        b = torch.randn(N, K, device=dev, dtype=torch.bfloat16, generator=g)
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        gemm_nt_(a, b, c)
        ref = a.float() @ b.float().t()
        rel = ((c.float() - ref).norm() / ref.norm()).item()
        print(json.dumps({"check": [M, N, K], "rel_err": rel}), flush=True)
        assert rel < 1e-2, rel
    for name, M, N, K in SHAPES:
        if want and name not in want:
            continue
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
        b = torch.randn(N, K, device=dev, dtype=torch.bfloat16, generator=g)
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        c2 = torch.empty_like(c)
        assert usable(a, b, c)
        gemm_nt_(a, b, c)
        torch.mm(a, b.t(), out=c2)
        diff = ((c.float() - c2.float()).norm() / c2.float().norm()).item()
        res = {f"v{v}": [] for v in VARIANTS}
        res["hipblaslt"] = []
        for _ in range(3):
            for v in VARIANTS:
                res[f"v{v}"].append(timed(lambda: gemm_nt_(a, b, c, variant=v)))
            res["hipblaslt"].append(timed(lambda: torch.mm(a, b.t(), out=c2)))
        vdiff = {}
        for v in VARIANTS:  # every variant's output against hipBLASLt's (same operands)
            c.zero_()
            gemm_nt_(a, b, c, variant=v)
            vdiff[f"v{v}"] = ((c.float() - c2.float()).norm() / c2.float().norm()).item()
        fl = 2.0 * M * N * K
        hb = min(res["hipblaslt"])
        tf = {k: round(fl / min(v) / 1e9) for k, v in res.items()}
        best = max((k for k in tf if k != "hipblaslt"), key=lambda k: tf[k])
        print(json.dumps({"gemm": name, "M": M, "N": N, "K": K, "tflops": tf, "best": best,
                          "best_vs_hipblaslt": round(tf[best] / tf["hipblaslt"], 3), "hipblaslt_ms": round(hb, 4),
                          "rel_diff_vs_hipblaslt": diff, "variant_rel_diff": vdiff}), flush=True)
        del a, b, c, c2
    return 0


if __name__ == "__main__":
    sys.exit(main())
