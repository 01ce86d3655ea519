#!/usr/bin/env python3
"""Bandwidth of the streaming kernels of the step against a plain device copy (MB8 shapes)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tensorhive_fixed_amd.ops import _lib  # noqa: E402


def timeit(fn, iters=10):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * iters)]
    fn()
    torch.cuda.synchronize()
    for i in range(iters):
        ev[2 * i].record()
        fn()
        ev[2 * i + 1].record()
    torch.cuda.synchronize()
    ts = sorted(ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(iters))
    return ts[len(ts) // 2]


def main():
    _lib.load()
    dev = "cuda"
    out = {}
    src = torch.empty(1 << 30, device=dev, dtype=torch.bfloat16)  # 2 GB
    dst = torch.empty_like(src)
    t = timeit(lambda: dst.copy_(src))
    out["copy_2GB"] = {"ms": t, "TBps": 2 * src.numel() * 2 / t / 1e9}
    del src, dst
    n = 1 << 30  # 1.07e9 params: 30 GB of AdamW traffic
    p = torch.zeros(n, device=dev, dtype=torch.bfloat16)
    g = torch.randn(n, device=dev, dtype=torch.bfloat16)
    ms, m1, v1 = (torch.zeros(n, device=dev) for _ in range(3))
    from tensorhive_fixed_amd.ops.adamw import adamw_flat_
    t = timeit(lambda: adamw_flat_(p, ms, m1, v1, g, lr=1e-3, beta1=0.9, beta2=0.95, eps=1e-8, weight_decay=0.1,
                                   step=1))
    out["adamw_1G"] = {"ms": t, "TBps": 28 * n / t / 1e9}
    del p, g, ms, m1, v1
    T, F = 32768, 14336
    gu = torch.randn(T, 2 * F, device=dev, dtype=torch.bfloat16)
    d = torch.randn(T, F, device=dev, dtype=torch.bfloat16)
    dgu = torch.empty_like(gu)
    dguT = torch.empty(2 * F, T, device=dev, dtype=torch.bfloat16)
    st = _lib.stream_ptr(gu.device)
    t = timeit(lambda: _lib.call("th_swiglu_bwd_t", d.data_ptr(), gu.data_ptr(), dgu.data_ptr(), dguT.data_ptr(), T,
                                 F, st))
    out["swiglu_bwd_t"] = {"ms": t, "TBps": (3 * T * F + 2 * 2 * T * F + 2 * T * F) * 2 / t / 1e9}
    t = timeit(lambda: _lib.call("th_swiglu_bwd", d.data_ptr(), gu.data_ptr(), dgu.data_ptr(), T, F, st))
    out["swiglu_bwd"] = {"ms": t, "TBps": (3 * T * F + 2 * T * F) * 2 / t / 1e9}
    t = timeit(lambda: _lib.call("th_swiglu_fwd", gu.data_ptr(), d.data_ptr(), T, F, st))
    out["swiglu_fwd"] = {"ms": t, "TBps": 3 * T * F * 2 / t / 1e9}
    for k, v in out.items():
        print(json.dumps({"kernel": k, **{a: round(b, 3) for a, b in v.items()}}), flush=True)


if __name__ == "__main__":
    main()
