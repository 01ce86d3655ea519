# round 5: NT hb schedule vs K, plus L2 counters of v8 / hb / hipBLASLt at K = 28672
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; mkdir -p gpurun_out/r05/gemm
run_step r05/gemm/nt_ksweep 300 python -u scripts/nt_ksweep.py
cat gpurun_out/r05/gemm/nt_ksweep.log
cd /tmp && export TMPDIR=/tmp
PMC=1 timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_WAVES --kernel-trace --output-format csv -d $R/gpurun_out/r05/gemm/pmc_k -o run -- python3 $R/scripts/nt_ksweep.py > $R/gpurun_out/r05/gemm/pmc_k.log 2>&1 || exit 1
cd $R && python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r05/gemm/pmc_k/*counter_collection.csv")
rows = list(csv.DictReader(open(f[0]))) if f else []
agg = {}
for r in rows:
    k = r.get("Kernel_Name", "")[:60]
    if "gemm" not in k.lower() and "Cijk" not in k:
        continue
    agg.setdefault((r.get("Dispatch_Id"), k), {})[r["Counter_Name"]] = float(r["Counter_Value"])
for (d, k), v in agg.items():
    print(d, k, {c: round(x / 1e6, 2) for c, x in v.items()}, "hit%", round(100 * v.get("TCC_HIT_sum", 0) / max(1, v.get("TCC_HIT_sum", 0) + v.get("TCC_MISS_sum", 0)), 1))
PY
