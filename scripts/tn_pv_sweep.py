"""TN hb kernel: LDS-DMA piece placement variants on the step's weight-gradient shapes, mode 10, interleaved timing
(3 rounds x 10-launch medians, best round).  Placement only moves instructions, so every variant's output must
equal variant 0's bit for bit.  Round 5 used it for the placement sweep (launch flags bits 13-15) and the per-wave
staggered pieces (bit 13): profiles/r05_gemm/tn_pv_sweep*.jsonl, tn_stagger.jsonl.  Both variants are retired, so
today every "variant" runs the one built-in placement (a timing-noise check)."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorhive_fixed_amd.ops import _lib  # noqa: E402
from tensorhive_fixed_amd.ops.gemm_tn import gemm_tn_  # noqa: E402

PVS = [int(x) for x in os.environ.get("TN_PVS", "0,1").split(",")]  # labels only (see the docstring)
SHAPES = [("wqkv", 6144, 4096, 32768), ("wo", 4096, 4096, 32768), ("w2", 4096, 14336, 32768),
          ("head_chunk", 128256 // 256 * 256, 4096, 4096)]


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
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, M, N, T in SHAPES:
        a = torch.randn(T, M, device="cuda", dtype=torch.bfloat16, generator=g)
        b = torch.randn(T, N, device="cuda", dtype=torch.bfloat16, generator=g)
        acc = name == "head_chunk"
        c0 = torch.randn(M, N, device="cuda", dtype=torch.bfloat16, generator=g)
        outs = {}
        for pv in PVS:
            c = c0.clone()
            gemm_tn_(a, b, c, accumulate=acc)
            outs[pv] = c
        same = {pv: bool(torch.equal(outs[pv], outs[PVS[0]])) for pv in PVS}
        assert all(same.values()), same
        c = c0.clone()
        res = {pv: [] for pv in PVS}
        for _ in range(3):
            for pv in PVS:
                res[pv].append(timed(lambda: gemm_tn_(a, b, c, accumulate=acc)))
        fl = 2.0 * M * N * T
        out = {"gemm": name, "M": M, "N": N, "K": T, "beta": acc}
        for pv, ts in res.items():
            out[f"pv{pv}_ms"] = round(min(ts), 4)
            out[f"pv{pv}_tflops"] = round(fl / min(ts) / 1e9)
        print(json.dumps(out), flush=True)
        del a, b, c, c0, outs
    return 0


if __name__ == "__main__":
    sys.exit(main())
