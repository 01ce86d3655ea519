"""Forward flash-attention variant sweep at the Llama-3-8B training shape (B=4, S=4096, 32/8 heads,
d=128): time (median of interleaved rounds) and error vs an fp32 reference on a slice."""
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tensorhive_fixed_amd.ops import _lib  # noqa: E402
from tensorhive_fixed_amd.ops.attention import attention_reference, flash_bwd, flash_fwd  # noqa: E402


def main():
    _lib.load()
    B, S, Hq, Hkv, D = int(os.environ.get("B", "4")), 4096, 32, 8, 128
    torch.manual_seed(0)
    qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    flops = 4 * B * Hq * S * S * D / 2
    if os.environ.get("NO_BWD"):
        globals()["bwd_time"] = lambda *a: None
    variants = [int(v) for v in os.environ.get("VARIANTS", "11").split(",")]
    # reference on batch 0, first 1024 queries
    Sr = 1024
    q = qkv[:S, : Hq * D].view(1, S, Hq, D)[:, :Sr]
    k = qkv[:S, Hq * D:(Hq + Hkv) * D].view(1, S, Hkv, D)[:, :Sr]
    v = qkv[:S, (Hq + Hkv) * D:].view(1, S, Hkv, D)[:, :Sr]
    ref = attention_reference(q, k, v).float().reshape(Sr, Hq * D)
    times = {v: [] for v in variants}
    outs = {}
    for v in variants:
        outs[v] = flash_fwd(qkv, B, S, Hq, Hkv, D, variant=v)
    for rnd in range(7):
        for v in variants:
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s0.record()
            for _ in range(3):
                flash_fwd(qkv, B, S, Hq, Hkv, D, variant=v)
            s1.record()
            torch.cuda.synchronize()
            times[v].append(s0.elapsed_time(s1) / 3)
    base_o = outs[variants[0]][0].float()
    for v in variants:
        o, lse = outs[v]
        t = sorted(times[v])[len(times[v]) // 2]
        err = (o[:Sr].float() - ref).abs().max().item()
        dv = (o.float() - base_o).abs().max().item()
        print(json.dumps({"variant": v, "ms": round(t, 4), "tflops": round(flops / t / 1e9, 1),
                          "max_err_vs_fp32": round(err, 5), "max_diff_vs_v0": round(dv, 5)}), flush=True)
    bwd_time(qkv, B, S, Hq, Hkv, D, flops)


def bwd_time(qkv, B, S, Hq, Hkv, D, flops):
    o, lse = flash_fwd(qkv, B, S, Hq, Hkv, D)
    do = torch.randn_like(o)
    ref = None
    for flags in [int(f) for f in os.environ.get("BWD_FLAGS", "0,8,0,8").split(",")]:
        ts = []
        for _ in range(5):
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s0.record()
            g = flash_bwd(do, qkv, o, lse, B, S, Hq, Hkv, D, flags=flags)
            s1.record()
            torch.cuda.synchronize()
            ts.append(s0.elapsed_time(s1))
        ref = g if ref is None else ref
        t = sorted(ts)[2]
        print(json.dumps({"kernel": "flash_bwd", "flags": flags, "ms": round(t, 4),
                          "tflops": round(2.5 * flops / t / 1e9, 1),
                          "max_diff_vs_first": round((g.float() - ref.float()).abs().max().item(), 5)}), flush=True)


if __name__ == "__main__":
    main()
