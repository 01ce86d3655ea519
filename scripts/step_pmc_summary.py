"""MFMA busy per kernel category inside the training step, from a rocprofv3 --pmc run of bench.py:
busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs), summed over each category's
dispatches (MI355X: 8 XCDs, 256 CUs x 4 SIMDs), plus the effective clock GRBM / 8 / kernel time.

    python scripts/step_pmc_summary.py PMC_DIR
"""
from __future__ import annotations

import csv
import glob
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from step_summary import CATS  # noqa: E402


def cat_of(name: str) -> str:
    return next((c for c, keys in CATS if any(k in name for k in keys)), "other")


def main() -> int:
    d = sys.argv[1]
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        print("no counter_collection.csv under", d)
        return 1
    per = defaultdict(lambda: defaultdict(float))
    seen = set()
    for r in csv.DictReader(open(f[0])):
        c = cat_of(r.get("Kernel_Name", ""))
        per[c][r["Counter_Name"]] += float(r["Counter_Value"])
        key = (r.get("Dispatch_Id"), r.get("Kernel_Name"))
        if key not in seen:
            seen.add(key)
            per[c]["dispatches"] += 1
            try:
                per[c]["ns"] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
            except (KeyError, ValueError):
                pass
    print(f"{'category':22s} {'dispatches':>10s} {'MFMA busy':>10s} {'clock GHz':>10s}")
    for c, v in sorted(per.items(), key=lambda x: -x[1].get("SQ_VALU_MFMA_BUSY_CYCLES", 0)):
        g = v.get("GRBM_GUI_ACTIVE", 0.0)
        busy = 100 * v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (g / 8 * 1024) if g else 0.0
        clk = g / 8 / v["ns"] if v.get("ns") else 0.0
        print(f"{c:22s} {int(v['dispatches']):10d} {busy:9.1f}% {clk:10.2f}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
