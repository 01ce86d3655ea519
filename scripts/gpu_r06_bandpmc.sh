# round 6 (round-5 verdict weak #9): why the w13 TN gradient runs faster in one-row XCD bands despite twice the
# fabric reads -- the fabric reads' average latency (Little: RDREQ_LEVEL / RDREQ) and DRAM credit stalls
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06/bandpmc; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc -o run -- python3 $R/scripts/tn_band_pmc.py > $O/run.log 2>&1 || exit 1
cd $R && python3 - <<'PY'
import csv, glob
rows = [r for r in csv.DictReader(open(glob.glob("gpurun_out/r06/bandpmc/pmc/**/*counter_collection.csv", recursive=True)[0])) if "gemm_tn" in r["Kernel_Name"]]
by = {}
for r in rows:
    by.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
order = [1, 8] * 3
with open("gpurun_out/r06/bandpmc/summary.txt", "w") as f:
    for band, (d, cs) in zip(order, sorted(by.items())):
        rq, lv = cs.get("TCC_EA0_RDREQ_sum", 0), cs.get("TCC_EA0_RDREQ_LEVEL_sum", 0)
        line = (f"band {band}: dispatch {d} EA rdreq {rq:.3e} level {lv:.3e} avg outstanding-cycles/req {lv / max(1, rq):.1f} "
                f"DRAM credit stall {cs.get('TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum', 0):.3e} GRBM {cs.get('GRBM_GUI_ACTIVE', 0):.3e}")
        print(line); f.write(line + "\n")
PY
