"""Per-kernel clock and MFMA busy from a rocprofv3 --pmc + --kernel-trace run: clock = GRBM_GUI_ACTIVE / 8 XCDs
over the dispatch's wall time; MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)."""
import csv
import glob
import sys
from collections import defaultdict

for d in sys.argv[1:]:
    dur, cnt = defaultdict(list), defaultdict(lambda: defaultdict(list))
    for f in glob.glob(d.rstrip("/") + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:40]
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    for f in glob.glob(d.rstrip("/") + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:40]
            cnt[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(d)
    for k in sorted(cnt):
        if not k.startswith("fa_"):
            continue
        c = {n: sum(v) / len(v) for n, v in cnt[k].items()}
        t = sum(dur[k]) / max(1, len(dur[k])) if dur.get(k) else float("nan")
        g = c.get("GRBM_GUI_ACTIVE", float("nan")) / 8
        line = f"  {k:32s} {t * 1e3:8.3f} ms  clock {g / t / 1e9:5.3f} GHz"
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            line += f"  mfma_busy {c['SQ_VALU_MFMA_BUSY_CYCLES'] / (g * 1024):.3f}"
        if "SQ_WAIT_ANY" in c and "SQ_WAVE_CYCLES" in c:
            line += f"  wait_any {c['SQ_WAIT_ANY'] / c['SQ_WAVE_CYCLES']:.3f}"
        print(line)
