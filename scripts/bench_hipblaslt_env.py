"""hipBLASLt on the training step's GEMMs (torch.mm in the step's K-contiguous "NT" layout), for an
A/B of library environment settings: run once per setting (the library reads its environment at
load), compare the printed per-shape TFLOP/s and the FLOP-weighted total."""
import json
import os
import statistics
import sys

import torch

T = 32768
SHAPES = [  # name, M, N, K  (C[M,N] = A[M,K] B[N,K]^T); calls per step
    ("wqkv.fwd", T, 6144, 4096, 32), ("wo.fwd", T, 4096, 4096, 32), ("w13.fwd", T, 28672, 4096, 32),
    ("w2.fwd", T, 4096, 14336, 32), ("wqkv.dgrad", T, 4096, 6144, 32), ("wo.dgrad", T, 4096, 4096, 32),
    ("w13.dgrad", T, 4096, 28672, 32), ("w2.dgrad", T, 14336, 4096, 32), ("w13.wgrad", 28672, 4096, T, 32),
    ("head.fwd", 4096, 128256, 4096, 8), ("head.dgrad", 4096, 4096, 128256, 8), ("head.wgrad", 128256, 4096, 4096, 8),
]
tag = os.environ.get("AB_TAG", "default")
torch.manual_seed(0)
tot_ms, tot_fl = 0.0, 0.0
rows = []
for name, M, N, K, calls in SHAPES:
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        torch.mm(a, b.t(), out=c)
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            torch.mm(a, b.t(), out=c)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 5)
    ms = statistics.median(ts)
    fl = 2.0 * M * N * K
    rows.append({"gemm": name, "ms": round(ms, 4), "tflops": round(fl / ms / 1e9)})
    tot_ms += ms * calls
    tot_fl += fl * calls
    del a, b, c
print(json.dumps({"env": tag, "per_step_ms": round(tot_ms, 2), "avg_tflops": round(tot_fl / tot_ms / 1e9),
                  "shapes": rows}), flush=True)
