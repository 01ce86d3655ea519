#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats CSV of `bench.py --steps S --warmup W` into per-step
time by category (the run covers S + W steps; pass their sum as --steps)."""
import argparse
import csv
from collections import defaultdict

CATS = [("gemm (hipBLASLt)", ("Cijk_", "Custom_Cijk")), ("gemm TN (gfx950)", ("gemm_tn",)),
        ("attention fwd", ("fa_fwd",)), ("attention dQ", ("fa_bwd_dq",)), ("attention dK/dV", ("fa_bwd_dkv", "fa_bwd_kc", "fa_bwd_kh", "fa_bwd_kf")),
        ("attention delta", ("fa_delta",)), ("transpose", ("transpose",)), ("adamw+grad-norm", ("adamw", "sumsq", "final_sum")),
        ("swiglu", ("swiglu",)), ("rmsnorm", ("rmsnorm", "slab_reduce")), ("rope", ("rope",)),
        ("cross-entropy", ("ce_fwd",)), ("embedding", ("emb_",)), ("split-K reduce", ("splitk_reduce",)),
        ("comm emulation", ("comm_channel", "comm_stop"))]
SIDE = {"comm emulation"}  # concurrent side-stream kernels (TH_COMM_EMU): listed, not added to the step total


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, required=True)
    a = ap.parse_args()
    per = defaultdict(float)
    rows = []
    for r in csv.DictReader(open(a.csv)):
        name, tot, calls = r["Name"], float(r["TotalDurationNs"]) / 1e6, int(r["Calls"])
        cat = next((c for c, keys in CATS if any(k in name for k in keys)), "other")
        per[cat] += tot
        rows.append((tot, calls, name))
    total = sum(t for c, t in per.items() if c not in SIDE)
    print(f"per step (total / {a.steps}), kernel time {total / a.steps:.1f} ms")
    for c, t in sorted(per.items(), key=lambda x: -x[1]):
        if c in SIDE:
            print(f"  {c:22s} {t / a.steps:8.1f} ms  (side stream, concurrent; not in the total)")
        else:
            print(f"  {c:22s} {t / a.steps:8.1f} ms  {100 * t / total:5.1f} %")
    print()
    for tot, calls, name in sorted(rows, reverse=True)[:25]:
        print(f"{name[:80]:80s} calls={calls:5d} total={tot:9.1f} ms avg={1e3 * tot / calls:9.1f} us")


if __name__ == "__main__":
    main()
