#!/usr/bin/env python3
"""Per-step timeline of a rocprofv3 --kernel-trace run of bench.py: wall time of the last step, the
union of busy intervals (all streams), the idle gaps between kernels, and the time per kernel
category inside that step.

    python scripts/step_timeline.py PROF_DIR [--step-marker NAME]

Steps are cut at the launches of the step's first kernel (the synthetic token draw, torch's
``distribution_elementwise`` kernel, by default); the last complete step (between the last two
markers) is reported.
"""
from __future__ import annotations

import argparse
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
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("--step-marker", default="distribution_elementwise")
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.prof_dir, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        print("no kernel_trace.csv under", a.prof_dir)
        return 1
    ks = []
    for f in files:
        for r in csv.DictReader(open(f)):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    ks.sort()
    marks = [s for s, e, n in ks if a.step_marker in n]
    if len(marks) < 2:
        print(f"fewer than two '{a.step_marker}' launches; kernels seen:", len(ks))
        return 1
    t0, t1 = marks[-2], marks[-1]
    step = [(max(s, t0), min(e, t1), n) for s, e, n in ks if e > t0 and s < t1]
    busy, gaps, cur_s, cur_e = 0, [], None, None
    for s, e, _ in sorted(step):
        if cur_e is None:
            cur_s, cur_e = s, e
        elif s > cur_e:
            busy += cur_e - cur_s
            gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    per = defaultdict(float)
    for s, e, n in step:
        per[cat_of(n)] += e - s
    wall = t1 - t0
    print(f"last step: wall {wall / 1e6:.1f} ms, GPU busy (union) {busy / 1e6:.1f} ms, idle {(wall - busy) / 1e6:.1f} ms "
          f"in {len(gaps)} gaps (largest {max(gaps, default=0) / 1e3:.0f} us), {len(step)} kernels")
    tot = sum(per.values())
    for c, t in sorted(per.items(), key=lambda x: -x[1]):
        print(f"  {c:22s} {t / 1e6:8.1f} ms  {100 * t / tot:5.1f} % of kernel time")
    return 0


if __name__ == "__main__":
    sys.exit(main())
