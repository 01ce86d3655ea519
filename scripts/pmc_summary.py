"""Summarise rocprofv3 --pmc counter_collection CSVs: per kernel (short name), mean of each counter
over dispatches."""
import csv
import glob
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(d.rstrip("/") + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "?")
            short = name.replace("(anonymous namespace)::", "").split("(")[0][:60]
            acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(acc.items()):
    if not any(x in k for x in ("fa_", "flash", "Cijk", "rmsnorm", "swiglu", "gemm_tn", "gemm_nt")):
        continue
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:32s} {sum(v) / len(v):16.0f}  (n={len(v)})")
