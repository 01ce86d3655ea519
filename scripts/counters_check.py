"""Validate th-counters' derived metrics on an MI355X against work of known size.

Phase A: bf16 GEMM loop (known FLOPs / time)  -> compare with mfma_tflops.
Phase B: large device copy (known bytes / time) -> compare with hbm_read / hbm_write.
Prints one JSON line per phase with the torch-measured rate and the counter-derived rate.
"""
import json
import subprocess
import sys
import time

import torch

sys.path.insert(0, ".")
from tensorhive_fixed_amd.core.counters import derive  # noqa: E402
from tensorhive_fixed_amd.native.build import build_all, path_of  # noqa: E402


def sample_during(fn, seconds=2.0, window_ms=500):
    build_all(strict=False)
    p = subprocess.Popen([str(path_of("th-counters")), "--count", "3", "--period", str(window_ms + 100),
                          "--window", str(window_ms)], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    t0 = time.time()
    work = 0
    torch.cuda.synchronize()
    tt = time.perf_counter()
    while time.time() - t0 < seconds:
        work += fn()
    torch.cuda.synchronize()
    rate = work / (time.perf_counter() - tt)
    out, err = p.communicate(timeout=60)
    lines = [json.loads(l) for l in out.splitlines() if l.startswith("{")]
    return rate, lines, err


def main():
    if "--list" in sys.argv:
        build_all(strict=False)
        print(subprocess.run([str(path_of("th-counters")), "--list"], capture_output=True, text=True).stdout)
        return
    dev = torch.device("cuda")
    n = 8192
    a = torch.randn(n, n, device=dev, dtype=torch.bfloat16)
    b = torch.randn(n, n, device=dev, dtype=torch.bfloat16)

    def gemm():
        for _ in range(10):
            torch.mm(a, b)
        return 10 * 2.0 * n ** 3

    rate, lines, err = sample_during(gemm)
    derived = [derive(g, l["window_ms"]) for l in lines for g in l["gpus"]]
    print(json.dumps({"phase": "gemm", "torch_tflops": round(rate / 1e12, 1), "counters": derived,
                      "raw_last": lines[-1] if lines else None, "stderr": err[-500:]}), flush=True)

    x = torch.empty(1 << 30, device=dev, dtype=torch.uint8)  # 1 GiB
    y = torch.empty_like(x)

    def copy():
        for _ in range(10):
            y.copy_(x)
        return 10 * 2.0 * x.numel()  # read + write bytes

    rate, lines, err = sample_during(copy)
    derived = [derive(g, l["window_ms"]) for l in lines for g in l["gpus"]]
    print(json.dumps({"phase": "copy", "torch_GBps_rw": round(rate / 1e9, 1), "counters": derived,
                      "raw_last": lines[-1] if lines else None, "stderr": err[-500:]}), flush=True)


if __name__ == "__main__":
    main()
