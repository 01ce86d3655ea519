# round 5: L2 / HBM counters of the w13 TN GEMM at XCD band heights 1 and 8 (one PMC pass)
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/r05/bandpmc; cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/r05/bandpmc/pmc -o run -- python3 $R/scripts/tn_band_pmc.py > $R/gpurun_out/r05/bandpmc/run.log 2>&1 || exit 1
cd $R && python3 - <<'PY'
import csv, glob
rows = [r for r in csv.DictReader(open(glob.glob("gpurun_out/r05/bandpmc/pmc/**/*counter_collection.csv", recursive=True)[0])) if "gemm_tn" in r["Kernel_Name"]]
by = {}
for r in rows:
    by.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
order = [1, 8] * 3
with open("gpurun_out/r05/bandpmc/summary.txt", "w") as f:
    for band, (d, cs) in zip(order, sorted(by.items())):
        hit, miss = cs.get("TCC_HIT_sum", 0), cs.get("TCC_MISS_sum", 0)
        line = (f"band {band}: dispatch {d} L2 hit rate {hit / max(1, hit + miss):.3f} hits {hit:.3e} misses {miss:.3e} "
                f"EA0 rdreq {cs.get('TCC_EA0_RDREQ_sum', 0):.3e} GRBM {cs.get('GRBM_GUI_ACTIVE', 0):.3e}")
        print(line); f.write(line + "\n")
PY
