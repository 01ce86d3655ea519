"""Round-5 NT GEMM parity probe (verdict r04 item 4): the one-k-tile-per-iteration schedule with
per-operand barriers and counted DMA waits (flags 32 / 96, ``gemm_nt_hb_kernel``) against the
round-4 default (variant 8) and hipBLASLt on the Llama-3-8B forward / input-gradient shapes.
fp32 check first, then interleaved timing (3 rounds x 10-launch medians, best round)."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorhive_fixed_amd.ops import _lib  # noqa: E402
from tensorhive_fixed_amd.ops.gemm_nt import gemm_nt_  # noqa: E402

T, D, F = 32768, 4096, 14336
SHAPES = [("w13.fwd", T, 2 * F, D), ("w2.fwd", T, D, F), ("wqkv.fwd", T, 6144, D), ("wo.fwd", T, D, D),
          ("w13.dgrad", T, D, 2 * F), ("w2.dgrad", T, F, D)]
VARIANTS = [int(v) for v in os.environ.get("NT_VARIANTS", "8,32,96,160,224").split(",")]


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
    g = torch.Generator(device=dev).manual_seed(0)
    for (M, N, K) in ((256, 256, 64), (512, 512, 128), (256, 768, 4096), (1024, 256, 14336), (768, 512, 192)):
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
        b = torch.randn(N, K, device=dev, dtype=torch.bfloat16, generator=g)
        ref = a.float() @ b.float().t()
        for v in VARIANTS:
            c = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
            gemm_nt_(a, b, c, variant=v)
            rel = ((c.float() - ref).norm() / ref.norm()).item()
            print(json.dumps({"check": [M, N, K], "variant": v, "rel_err": rel}), flush=True)
            assert rel < 1e-2, (v, rel)
    for name, M, N, K in SHAPES:
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
        b = torch.randn(N, K, device=dev, dtype=torch.bfloat16, generator=g)
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ref = torch.mm(a, b.t())
        res = {f"v{v}": [] for v in VARIANTS}
        res["hipblaslt"] = []
        diff = {}
        for v in VARIANTS:
            gemm_nt_(a, b, c, variant=v)
            diff[f"v{v}"] = ((c.float() - ref.float()).norm() / ref.float().norm()).item()
        for _ in range(3):
            for v in VARIANTS:
                res[f"v{v}"].append(timed(lambda: gemm_nt_(a, b, c, variant=v)))
            res["hipblaslt"].append(timed(lambda: torch.mm(a, b.t(), out=c)))
        fl = 2.0 * M * N * K
        out = {"gemm": name, "M": M, "N": N, "K": K, "rel_diff_vs_hipblaslt": diff}
        for k, ts in res.items():
            out[k + "_tflops"] = round(fl / min(ts) / 1e9)
        hb = out["hipblaslt_tflops"]
        out["ratio"] = {k: round(out[k + "_tflops"] / hb, 3) for k in res if k != "hipblaslt"}
        print(json.dumps(out), flush=True)
        del a, b, c, ref
    return 0


if __name__ == "__main__":
    sys.exit(main())
