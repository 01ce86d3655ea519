"""Interleaved A/B of flash-backward launch flags at B4 S4096 32/8 heads d128 (causal):
median ms of the whole backward (delta + dQ + dK/dV) per flag set over 9 rounds, then the forward's median."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tensorhive_fixed_amd.ops import _lib  # noqa: E402
from tensorhive_fixed_amd.ops.attention import flash_bwd, flash_fwd  # noqa: E402

_lib.load()
B, S, Hq, Hkv, D = int(os.environ.get("FA_B", "4")), 4096, 32, 8, 128
flag_sets = [int(f) for f in os.environ.get("FA_FLAGS", "0,8").split(",")]
qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
o, lse = flash_fwd(qkv, B, S, Hq, Hkv, D)
do = torch.randn_like(o)
times = {f: [] for f in flag_sets}
for f in flag_sets:
    flash_bwd(do, qkv, o, lse, B, S, Hq, Hkv, D, flags=f)
for _ in range(9):
    for f in flag_sets:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            flash_bwd(do, qkv, o, lse, B, S, Hq, Hkv, D, flags=f)
        e1.record()
        torch.cuda.synchronize()
        times[f].append(e0.elapsed_time(e1) / 3)
# forward variants (FA_FWD_VARIANTS, comma list; "d" = the built-in default), interleaved
fwd_vars = [None if v == "d" else int(v) for v in os.environ.get("FA_FWD_VARIANTS", "d").split(",")]
fwd_t = {v: [] for v in fwd_vars}
for _ in range(9):
    for v in fwd_vars:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            flash_fwd(qkv, B, S, Hq, Hkv, D, variant=v)
        e1.record()
        torch.cuda.synchronize()
        fwd_t[v].append(e0.elapsed_time(e1) / 3)
for v in fwd_vars:
    med = statistics.median(fwd_t[v])
    print(json.dumps({"fwd_variant": v, "fwd_ms_median": round(med, 4),
                      "fwd_tflops": round(4 * B * Hq * S * S * D / 2 / med / 1e9, 1)}), flush=True)
flops = 2.5 * 4 * B * Hq * S * S * D / 2
for f in flag_sets:
    med = statistics.median(times[f])
    print(json.dumps({"flags": f, "bwd_ms_median": round(med, 4), "min": round(min(times[f]), 4),
                      "tflops": round(flops / med / 1e9, 1)}), flush=True)
