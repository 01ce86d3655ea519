"""Which operand layout does hipBLASLt run fastest for each GEMM of the Llama-3-8B step?

For a linear layer ``y = x W^T`` the three GEMMs of a training step can be issued against the
weight stored as ``[out, in]`` (what ``ops/linear.py`` does) or as ``[in, out]``; the weight
gradient can also be produced transposed and copied.  This script times every formulation
(and rocBLAS vs hipBLASLt) on the exact shapes of the MB8 step and prints one JSON line each:

    python scripts/gemm_layouts.py [tokens]        # default 32768 = micro-batch 8 x 4096
"""
from __future__ import annotations

import json
import sys

import torch

D, HQKV, FF, V = 4096, 6144, 14336, 128256


def timeit(fn, iters=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def r(*shape):
    return torch.randn(*shape, device="cuda", dtype=torch.bfloat16)


def linear_variants(T, n_out, k_in):
    x, dy = r(T, k_in), r(T, n_out)
    w_nk, w_kn = r(n_out, k_in), r(k_in, n_out)
    g_nk, g_kn = torch.empty(n_out, k_in, device="cuda", dtype=torch.bfloat16), \
        torch.empty(k_in, n_out, device="cuda", dtype=torch.bfloat16)
    return {
        "fwd[out,in]": lambda: torch.mm(x, w_nk.t()),
        "fwd[in,out]": lambda: torch.mm(x, w_kn),
        "dgrad[out,in]": lambda: torch.mm(dy, w_nk),
        "dgrad[in,out]": lambda: torch.mm(dy, w_kn.t()),
        "wgrad[out,in]": lambda: torch.mm(dy.t(), x, out=g_nk),
        "wgrad[in,out]": lambda: torch.mm(x.t(), dy, out=g_kn),
        "wgrad[out,in]via_T": lambda: g_nk.copy_(torch.mm(x.t(), dy).t()),
        # dgrad in the K-contiguous (NT) form: transpose W first (cost included)
        "dgrad[out,in]via_WT": lambda: torch.mm(dy, w_nk.t().contiguous().t()),
        # wgrad with both operands pre-transposed (token dim contiguous, NT form); transposes excluded
        "wgrad_NT_pre": (lambda dyT, xT: lambda: torch.mm(dyT, xT.t(), out=g_nk))(dy.t().contiguous(),
                                                                                x.t().contiguous()),
        "transpose_dy": lambda: dy.t().contiguous(),
        "transpose_x": lambda: x.t().contiguous(),
    }


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
    torch.backends.cuda.matmul.allow_tf32 = False
    layers = (("wqkv", HQKV, D), ("wo", D, D), ("w13", 2 * FF, D), ("w2", D, FF))
    libs = sys.argv[2].split(",") if len(sys.argv) > 2 else ["hipblaslt", "rocblas"]
    for lib in libs:
        try:
            torch.backends.cuda.preferred_blas_library("cublaslt" if lib == "hipblaslt" else "cublas")
        except Exception as e:  # noqa: BLE001
            print(json.dumps({"lib": lib, "error": str(e)}), flush=True)
            continue
        tot = {"[out,in]": 0.0, "[in,out]": 0.0}
        for name, n_out, k_in in layers:
            for var, fn in linear_variants(T, n_out, k_in).items():
                ms = timeit(fn)
                flops = 2.0 * T * n_out * k_in
                print(json.dumps({"lib": lib, "gemm": name, "variant": var, "ms": round(ms, 4),
                                  "tflops": round(flops / ms / 1e9, 1)}), flush=True)
                for k in tot:
                    if var.endswith(k):
                        tot[k] += ms
            torch.cuda.empty_cache()
        print(json.dumps({"lib": lib, "per_layer_ms": {k: round(v, 3) for k, v in tot.items()}}), flush=True)
        # LM head per CE chunk size (fwd + dgrad + accumulated wgrad), per token count T
        for ch in (4096, 8192, 16384):
            h, w, lg = r(ch, D), r(V, D), r(ch, V)
            acc = torch.zeros(V, D, device="cuda", dtype=torch.float32)
            accb = torch.zeros(V, D, device="cuda", dtype=torch.bfloat16)
            f = timeit(lambda: torch.mm(h, w.t()), iters=10)
            dg = timeit(lambda: torch.mm(lg, w), iters=10)
            wg = timeit(lambda: accb.addmm_(lg.t(), h), iters=10)
            wg_t = timeit(lambda: torch.mm(h.t(), lg), iters=10)
            print(json.dumps({"lib": lib, "gemm": "head", "chunk": ch, "fwd_ms": round(f, 3), "dgrad_ms": round(dg, 3),
                              "wgrad_acc_ms": round(wg, 3), "wgrad_T_ms": round(wg_t, 3),
                              "step_ms": round((f + dg + wg) * T / ch, 2)}), flush=True)
            del h, w, lg, acc, accb
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
