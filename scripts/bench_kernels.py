#!/usr/bin/env python3
"""Micro-benchmarks of the gfx950 kernels at Llama-3-8B training shapes (one process, interleaved
rounds, median of N).  Prints one JSON line per kernel with time and achieved TFLOP/s or TB/s."""
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tensorhive_fixed_amd.ops import _lib  # noqa: E402
from tensorhive_fixed_amd.ops.attention import flash_bwd, flash_fwd, qkv_attention  # noqa: E402


def timeit(fn, iters=10):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * iters)]
    fn()
    torch.cuda.synchronize()
    ts = []
    for i in range(iters):
        ev[2 * i].record()
        fn()
        ev[2 * i + 1].record()
    torch.cuda.synchronize()
    ts = sorted(ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(iters))
    return ts[len(ts) // 2]


def main():
    _lib.load(build_if_missing=True)
    B, S, Hq, Hkv, D = int(os.environ.get("B", 4)), int(os.environ.get("S", 4096)), 32, 8, 128
    qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    flops_fwd = 4 * B * Hq * S * S * D / 2
    o, lse = flash_fwd(qkv, B, S, Hq, Hkv, D)
    do = torch.randn_like(o)
    t = timeit(lambda: flash_fwd(qkv, B, S, Hq, Hkv, D))
    print(json.dumps({"kernel": "flash_fwd", "ms": t, "tflops": flops_fwd / t / 1e9}))
    t = timeit(lambda: flash_bwd(do, qkv, o, lse, B, S, Hq, Hkv, D))
    print(json.dumps({"kernel": "flash_bwd", "ms": t, "tflops": 2.5 * flops_fwd / t / 1e9}))
    q = qkv[:, :Hq * D].view(B, S, Hq, D).transpose(1, 2)
    k = qkv[:, Hq * D:(Hq + Hkv) * D].view(B, S, Hkv, D).transpose(1, 2)
    v = qkv[:, (Hq + Hkv) * D:].view(B, S, Hkv, D).transpose(1, 2)
    sd = lambda: torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=True)
    t = timeit(sd)
    print(json.dumps({"kernel": "sdpa_fwd(reference point)", "ms": t, "tflops": flops_fwd / t / 1e9}))
    x = torch.randn(B * S, 4096, device="cuda", dtype=torch.bfloat16)
    w = torch.ones(4096, device="cuda", dtype=torch.bfloat16)
    from tensorhive_fixed_amd.ops.rmsnorm import rmsnorm
    t = timeit(lambda: rmsnorm(x, w))
    print(json.dumps({"kernel": "rmsnorm_fwd", "ms": t, "TBps": 2 * x.numel() * 2 / t / 1e9}))
    gu = torch.randn(B * S, 2 * 14336, device="cuda", dtype=torch.bfloat16)
    from tensorhive_fixed_amd.ops.swiglu import swiglu
    t = timeit(lambda: swiglu(gu))
    print(json.dumps({"kernel": "swiglu_fwd", "ms": t, "TBps": 1.5 * gu.numel() * 2 / t / 1e9}))
    n = 1 << 28
    p = torch.zeros(n, device="cuda", dtype=torch.bfloat16)
    g = torch.zeros(n, device="cuda", dtype=torch.bfloat16)
    m = torch.zeros(n, device="cuda")
    from tensorhive_fixed_amd.ops.adamw import adamw_flat_
    t = timeit(lambda: adamw_flat_(p, m, m, m, g, lr=1e-3, beta1=0.9, beta2=0.95, eps=1e-8,
                                   weight_decay=0.1, step=1))
    print(json.dumps({"kernel": "adamw_flat(2^28)", "ms": t, "TBps": 28 * n / t / 1e9}))
    a = torch.randn(B * S, 4096, device="cuda", dtype=torch.bfloat16)
    wt = torch.randn(14336 * 2, 4096, device="cuda", dtype=torch.bfloat16)
    t = timeit(lambda: torch.mm(a, wt.t()))
    print(json.dumps({"kernel": "hipblaslt gate_up gemm", "ms": t, "tflops": 2 * a.shape[0] * 4096 * 28672 / t / 1e9}))


if __name__ == "__main__":
    main()
