"""Round-3 hipBLASLt-parity probe of the gfx950 NT GEMM (ops/csrc/gemm_nt.hip): the 16x16x32
kernel and its variants (deep DMA ring, setprio, LDS epilogue) against hipBLASLt on the Llama-3-8B
forward / input-gradient shapes.  Exactness vs fp32 first (every variant, beta 0 and 1), then
interleaved timing: 3 rounds x 10-launch medians per arm, best round reported, random operands."""
import json
import statistics
import sys

import torch

sys.path.insert(0, ".")
from tensorhive_fixed_amd.ops import _lib  # noqa: E402
from tensorhive_fixed_amd.ops.gemm_nt import gemm_nt_  # noqa: E402

T, D, F = 32768, 4096, 14336
SHAPES = [("w13.fwd", T, 2 * F, D), ("w2.dgrad", T, F, D), ("w2.fwd", T, D, F), ("wqkv.fwd", T, 6144, D),
          ("wo.fwd", T, D, D), ("w13.dgrad", T, D, 2 * F)]
VARIANTS = [0, 1, 2, 4, 5, 7]


def run(a, b, c, v, accumulate=False):
    return gemm_nt_(a, b, c, accumulate=accumulate, mfma16=True, variant=v)


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
    for (M, N, K) in ((512, 512, 64), (256, 768, 4096), (1024, 256, 14336), (512, 512, 128)):
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
        b = torch.randn(N, K, device=dev, dtype=torch.bfloat16, generator=g)
        ref = a.float() @ b.float().t()
        c0 = torch.randn(M, N, device=dev, dtype=torch.bfloat16, generator=g)
        for v in VARIANTS:
            c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            run(a, b, c, v)
            rel = ((c.float() - ref).norm() / ref.norm()).item()
            cb = c0.clone()
            run(a, b, cb, v, accumulate=True)
            rel2 = ((cb.float() - (c0.float() + ref)).norm() / (c0.float() + ref).norm()).item()
            print(json.dumps({"check": [M, N, K], "variant": v, "rel_err": rel, "rel_err_beta": rel2}), flush=True)
            assert rel < 1e-2 and rel2 < 1e-2, (v, rel, rel2)
    for name, M, N, K in SHAPES:
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
        b = torch.randn(N, K, device=dev, dtype=torch.bfloat16, generator=g)
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        res = {f"v{v}": [] for v in VARIANTS}
        res["hipblaslt"] = []
        for _ in range(3):
            for v in VARIANTS:
                res[f"v{v}"].append(timed(lambda: run(a, b, c, v)))
            res["hipblaslt"].append(timed(lambda: torch.mm(a, b.t(), out=c)))
        fl = 2.0 * M * N * K
        out = {"gemm": name, "M": M, "N": N, "K": K}
        for k, ts in res.items():
            out[k + "_tflops"] = round(fl / min(ts) / 1e9)
        hb = out["hipblaslt_tflops"]
        out["best_ratio"] = round(max(v for k, v in out.items() if k.startswith("v") and k.endswith("_tflops")) / hb, 3)
        print(json.dumps(out), flush=True)
        del a, b, c
    return 0


if __name__ == "__main__":
    sys.exit(main())
