#!/usr/bin/env python3
"""Per-kernel cost of CUs held by an emulated RCCL channel kernel (parallel/comm_emu.py), one shape at a time.

For k in KS (channel workgroups, one per CU, idle: copy=1 GB/s so only the CUs are taken), the step's weight-
gradient TN GEMMs are timed with the 256-CU launch plan and with the plan for 256 - k CUs, the hipBLASLt
input-gradient GEMMs with the process's settings (run again with TENSILE_STREAMK_MAX_CUS set to compare),
and the flash backward.  One JSON line per (k, kernel).  profiles/r06_comm/.
"""
from __future__ import annotations

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tensorhive_fixed_amd.ops import _lib  # noqa: E402
from tensorhive_fixed_amd.ops.gemm_tn import cu_budget, gemm_tn_, tn_plan  # noqa: E402
from tensorhive_fixed_amd.parallel.comm_emu import CommEmulator, parse  # noqa: E402

T = 32768
WGRAD = {"wqkv": (6144, 4096), "wo": (4096, 4096), "w13": (28672, 4096), "w2": (4096, 14336)}
DGRAD = {"wqkv": (4096, 6144), "wo": (4096, 4096), "w13": (4096, 28672), "w2": (14336, 4096)}  # (N out, K)


def timed(fn, reps=5):
    # current-stream syncs only: a device-wide synchronize would also wait for the channel kernel on its side
    # stream (until its time slice ends), and the GEMMs would then run on an idle chip
    fn()
    torch.cuda.current_stream().synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = []
    for _ in range(reps):
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        best.append(e0.elapsed_time(e1))
    best.sort()
    return best[len(best) // 2]


def main():
    _lib.load()
    from tensorhive_fixed_amd.ops.tuned import load_gemm_table

    load_gemm_table()  # the step's measured hipBLASLt / rocBLAS choices
    dev = torch.device("cuda")
    ks = [int(x) for x in os.environ.get("KS", "0,8,16,32").split(",")]
    what = os.environ.get("WHAT", "tn,blas,flash").split(",")
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s: torch.randn(*s, device=dev, dtype=torch.bfloat16, generator=g)  # noqa: E731
    tag = os.environ.get("TAG", "")
    for k in ks:
        emu = CommEmulator(parse(f"cus={k},copy=1,slice_ms=9000,buffer_mb=64"), dev) if k else None
        if emu is not None:
            emu.bucket_ready(1)  # resident until stop() (or 9 s)
            time.sleep(0.05)  # the channel workgroups are on their CUs before the first GEMM

        rows = []
        if "tn" in what:
            for name, (m, n) in WGRAD.items():
                a, b, c = r(T, m), r(T, n), torch.empty(m, n, device=dev, dtype=torch.bfloat16)
                for plan_cus in sorted({256, 256 - k}, reverse=True):
                    with cu_budget(plan_cus):
                        ms = timed(lambda: gemm_tn_(a, b, c))
                        rows.append({"k": k, "kernel": f"tn.{name}", "plan_cus": plan_cus,
                                     "plan": list(tn_plan(m, n, T)), "ms": round(ms, 4)})
                del a, b, c
        if "blas" in what:
            for name, (n, kk) in DGRAD.items():
                dy, wT = r(T, kk), r(n, kk)
                ms = timed(lambda: torch.mm(dy, wT.t()))
                rows.append({"k": k, "kernel": f"blas.{name}.dgrad", "ms": round(ms, 4),
                             "streamk_max_cus": os.environ.get("TENSILE_STREAMK_MAX_CUS")})
                del dy, wT
        if "flash" in what:
            from tensorhive_fixed_amd.ops.attention import flash_bwd, flash_fwd

            B, S, H, HK, D = 8, 4096, 32, 8, 128
            qkv = r(B * S, (H + 2 * HK) * D)
            o, lse = flash_fwd(qkv, B, S, H, HK, D)
            do = r(*o.shape)
            ms = timed(lambda: flash_bwd(do, qkv, o, lse, B, S, H, HK, D))
            rows.append({"k": k, "kernel": "flash.bwd", "ms": round(ms, 4)})
            ms = timed(lambda: flash_fwd(qkv, B, S, H, HK, D))
            rows.append({"k": k, "kernel": "flash.fwd", "ms": round(ms, 4)})
            del qkv, o, lse, do
        if emu is not None:
            emu.stop()
            torch.cuda.synchronize()
            emu.side.synchronize()
        for row in rows:
            row["tag"] = tag
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
