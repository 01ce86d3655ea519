"""Known-byte HBM load for counter calibration: ``python scripts/hbm_stream.py SECONDS KIND [half]``.

KIND ``add`` runs ``y += x`` over 1 GiB fp32 tensors (a shader kernel: 2 reads + 1 write per
element), ``copy`` runs ``y.copy_(x)`` (the runtime's blit kernel).  Prints one JSON line with
the bytes moved and the rate torch measured, so a counter sampler running beside it can be
checked against a number that does not come from counters.  ``HBM_STREAM_START_AT`` (unix
seconds) delays the start, so concurrent streams cover the same window."""
import json
import os
import sys
import time

import torch


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
    kind = sys.argv[2] if len(sys.argv) > 2 else "add"
    half = len(sys.argv) > 3 and sys.argv[3] == "half"  # idle as long as each burst ran: ~half the rate
    n = 1 << 28  # 1 GiB of fp32
    x = torch.ones(n, device="cuda", dtype=torch.float32)
    y = torch.zeros_like(x)
    per = {"add": 3 * 4 * n, "copy": 2 * 4 * n}[kind]
    torch.cuda.synchronize()
    print(json.dumps({"ready": True}), flush=True)  # a sampler beside it starts from here
    start_at = float(os.environ.get("HBM_STREAM_START_AT", "0"))  # several streams over one window
    while time.time() < start_at:
        time.sleep(0.001)
    t0 = time.perf_counter()
    done = 0
    while time.perf_counter() - t0 < secs:
        tb = time.perf_counter()
        for _ in range(8):
            if kind == "add":
                y.add_(x)
            else:
                y.copy_(x)
        torch.cuda.synchronize()
        done += 8
        if half:
            time.sleep(time.perf_counter() - tb)
    dt = time.perf_counter() - t0
    print(json.dumps({"kind": kind, "iters": done, "bytes": done * per, "seconds": round(dt, 3),
                      "GBps": round(done * per / dt / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
