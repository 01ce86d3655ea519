"""The training step's GEMM + SwiGLU mix as a known, repeatable HBM load for counter validation:
``python scripts/hbm_mix.py SECONDS``.  Each iteration = the gate|up projection of 8192 tokens
(x[8192,4096] @ W13[28672,4096]^T, hipBLASLt) followed by the gfx950 SwiGLU forward on its
[8192, 28672] output.  Prints iterations and wall time: bytes per iteration is the invariant to
compare between a counter run (rate x seconds / iterations) and a rocprofv3 dispatch-PMC run."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorhive_fixed_amd.ops.swiglu import swiglu  # noqa: E402


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
    x = torch.randn(8192, 4096, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(28672, 4096, device="cuda", dtype=torch.bfloat16) * 0.02
    h = swiglu(x @ w.t())  # warm-up: hipBLASLt algorithm choice, kernel loads
    del h
    torch.cuda.synchronize()
    print(json.dumps({"ready": True}), flush=True)  # a sampler beside it starts from here
    t0 = time.perf_counter()
    it = 0
    while time.perf_counter() - t0 < secs:
        for _ in range(4):
            h = swiglu(x @ w.t())
            del h
        torch.cuda.synchronize()
        it += 4
    dt = time.perf_counter() - t0
    print(json.dumps({"kind": "gemm_swiglu", "iters": it, "seconds": round(dt, 3)}), flush=True)


if __name__ == "__main__":
    main()
