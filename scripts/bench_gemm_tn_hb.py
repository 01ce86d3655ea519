"""Round-5 TN weight-gradient GEMM probe (verdict r04 item 3): the one-wave-per-SIMD "hb" schedule
(pingpong mode 9, ``gemm_tn_hb_kernel``) against the round-4 default (mode 6, 8-wave ping-pong) and
hipBLASLt on the Llama-3-8B wgrad shapes (K = 32768 tokens), at the default split-K.  fp32 check first
(split 1 / 2, beta 0 / 1), then interleaved timing (3 rounds x 10-launch medians, best round)."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorhive_fixed_amd.ops import _lib  # noqa: E402
from tensorhive_fixed_amd.ops.gemm_tn import default_splitk, gemm_tn_  # noqa: E402

T = 32768
SHAPES = [("wqkv", 6144, 4096), ("wo", 4096, 4096), ("w2", 4096, 14336), ("w13", 28672, 4096)]
MODES = [int(x) for x in os.environ.get("TN_MODES", "9,10").split(",")]


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
    for (K, M, N) in ((64, 256, 256), (128, 512, 256), (4096, 256, 768), (2048, 768, 512), (256, 4096, 4352)):
        a = torch.randn(K, M, device=dev, dtype=torch.bfloat16, generator=g)
        b = torch.randn(K, N, device=dev, dtype=torch.bfloat16, generator=g)
        ref = a.float().t() @ b.float()
        c0 = torch.randn(M, N, device=dev, dtype=torch.bfloat16, generator=g)
        for mode in MODES:
            for sk in (1, 2):
                if K % (64 * sk):
                    continue
                c = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
                gemm_tn_(a, b, c, splitk=sk, pingpong=mode)
                rel = ((c.float() - ref).norm() / ref.norm()).item()
                cb = c0.clone()
                gemm_tn_(a, b, cb, accumulate=True, splitk=sk, pingpong=mode)
                rel2 = ((cb.float() - (c0.float() + ref)).norm() / (c0.float() + ref).norm()).item()
                print(json.dumps({"check": [K, M, N], "mode": mode, "splitk": sk, "rel_err": rel, "rel_err_beta": rel2}),
                      flush=True)
                assert rel < 1e-2 and rel2 < 1e-2, (mode, sk, rel, rel2)
    for name, M, N in SHAPES:
        a = torch.randn(T, M, device=dev, dtype=torch.bfloat16, generator=g)
        b = torch.randn(T, N, device=dev, dtype=torch.bfloat16, generator=g)
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        sk = default_splitk(M, N, T)
        ref = torch.mm(a.t(), b)
        diff = {}
        for mode in MODES:
            gemm_tn_(a, b, c, splitk=sk, pingpong=mode)
            diff[f"m{mode}"] = ((c.float() - ref.float()).norm() / ref.float().norm()).item()
        res = {f"m{mode}": [] for mode in MODES}
        res["hipblaslt"] = []
        for _ in range(3):
            for mode in MODES:
                res[f"m{mode}"].append(timed(lambda: gemm_tn_(a, b, c, splitk=sk, pingpong=mode)))
            res["hipblaslt"].append(timed(lambda: torch.mm(a.t(), b, out=c)))
        fl = 2.0 * M * N * T
        out = {"gemm": name, "M": M, "N": N, "K": T, "splitk": sk, "rel_diff_vs_hipblaslt": diff}
        for k, ts in res.items():
            out[k + "_ms"] = round(min(ts), 4)
            out[k + "_tflops"] = round(fl / min(ts) / 1e9)
        print(json.dumps(out), flush=True)
        del a, b, c, ref
    return 0


if __name__ == "__main__":
    sys.exit(main())
