"""MFMA loads of known kernel-level behaviour for validating the probe's MFMA metric
(round-3 verdict item 3): ``python scripts/mfma_load.py KIND SECONDS``.

KIND ``gemm``: 8192^3 bf16 ``torch.mm`` (hipBLASLt, one wave per SIMD); ``flash_bwd``: the
payload's flash-attention backward (B 8, S 4096, 32/8 heads, d 128; the dK|dV kernel runs two
workgroups per CU); ``idle``: nothing.  Prints ``{"ready": true}`` when the loop starts and one
JSON line at the end with iterations, wall seconds and the GPU-busy share of the wall time
(events around every burst)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    kind = sys.argv[1]
    secs = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
    dev = torch.device("cuda")
    if kind == "gemm":
        a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
        b = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)

        def burst():
            for _ in range(8):
                torch.mm(a, b)
            return 8
    elif kind == "flash_bwd":
        from tensorhive_fixed_amd.ops import _lib
        from tensorhive_fixed_amd.ops.attention import flash_bwd, flash_fwd

        _lib.load(build_if_missing=False)
        B, S, Hq, Hkv, D = 8, 4096, 32, 8, 128
        qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16)
        o, lse = flash_fwd(qkv, B, S, Hq, Hkv, D)
        do = torch.randn_like(o)

        def burst():
            for _ in range(4):
                flash_bwd(do, qkv, o, lse, B, S, Hq, Hkv, D)
            return 4
    elif kind == "idle":
        def burst():
            time.sleep(0.05)
            return 0
    else:
        raise SystemExit(f"unknown load {kind}")
    burst()
    torch.cuda.synchronize()
    print(json.dumps({"ready": True}), flush=True)
    t0 = time.perf_counter()
    iters, gpu_ms = 0, 0.0
    while time.perf_counter() - t0 < secs:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        iters += burst()
        e1.record()
        e1.synchronize()
        gpu_ms += e0.elapsed_time(e1)
    wall = time.perf_counter() - t0
    print(json.dumps({"kind": kind, "iters": iters, "seconds": round(wall, 3),
                      "gpu_share": round(gpu_ms / 1000.0 / wall, 4) if kind != "idle" else 0.0}), flush=True)


if __name__ == "__main__":
    main()
