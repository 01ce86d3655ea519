"""MFMA metrics of the monitor vs dispatch-mode hardware counters (round-3 verdict item 3).

    python scripts/probe_vs_pmc.py OUTDIR

For each load (idle, 8192^3 hipBLASLt GEMM, flash-attention backward) in a child process that
carries the in-task HBM tool, the monitor (AmdSmiBackend with the probe agent and th-counters)
samples the GPU every 0.25 s:
  * ``mfma_contention`` -- the probe's estimate;
  * ``mfma_busy``       -- th-counters' device-wide SQ_VALU_MFMA_BUSY_CYCLES share;
then a rocprofv3 dispatch-PMC run of the same load gives the reference:
  MFMA busy (kernel) = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs),
  MFMA busy (wall)   = kernel value x the load's GPU-busy share of wall time.
The GEMM's PMC pass is repeated with th-counters sampling at the same time (can a user's
``rocprofv3 --pmc`` run beside the monitor's counting session?).
Writes OUTDIR/probe_vs_pmc.json and prints a table.
"""
import csv
import json
import os
import statistics
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

LOADS = ("idle", "gemm", "flash_bwd")
PMC = ["SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"]


def monitored(load: str, secs: float = 6.0) -> dict:
    """The monitor's view of ``load``: probe ``mfma_contention`` and the device counters'
    ``mfma_busy`` / ``gpu_busy`` / ``mfma_tflops`` (th-counters beside the load), with the load
    process carrying the in-task HBM tool (two counting sessions on one GPU)."""
    from tensorhive_fixed_amd.core import hbm
    from tensorhive_fixed_amd.core.telemetry import AmdSmiBackend

    be = AmdSmiBackend(probe=True, probe_period=0.25, counters=True, counters_period_ms=500, task_hbm=True)
    be.probe.wait_first(30)
    be.counters.wait_first(15)
    for _ in range(8):  # idle reference samples before the load starts
        be.sample("local")
        time.sleep(0.25)
    env = {**os.environ, "TENSORHIVE_TASK_ID": "1"}
    tool = hbm.tool_path()
    if tool and load != "idle":
        env["ROCP_TOOL_LIBRARIES"] = tool
    p = subprocess.Popen([sys.executable, str(ROOT / "scripts" / "mfma_load.py"), load, str(secs)],
                         stdout=subprocess.PIPE, text=True, env=env, cwd=str(ROOT))
    assert json.loads(p.stdout.readline()) == {"ready": True}
    time.sleep(1.0)
    rows = []
    t_end = time.time() + secs - 2.0
    while time.time() < t_end:
        e = be.sample("local")
        g = sorted(e["GPU"].values(), key=lambda g: g["index"])[0]
        m = g["metrics"]
        rows.append({k: (m.get(k) or {}).get("value") for k in
                     ("mfma_contention", "mfma_busy", "gpu_busy", "mfma_tflops", "hbm_bw_source")})
        time.sleep(0.25)
    out, _ = p.communicate(timeout=120)
    run = json.loads(out.strip().splitlines()[-1])
    counters_err = be.counters.error
    be.close()

    def med(k):
        v = [r[k] for r in rows if r[k] is not None]
        return statistics.median(v) if v else None

    return {"load": load, "run": run, "probe_mfma_contention": med("mfma_contention"),
            "counters_mfma_busy": med("mfma_busy"), "counters_gpu_busy": med("gpu_busy"),
            "counters_mfma_tflops": med("mfma_tflops"),
            "hbm_sources": sorted({r["hbm_bw_source"] for r in rows if r["hbm_bw_source"]}),
            "counters_error": counters_err, "samples": rows}


def pmc(load: str, outdir: Path, beside_counters: bool = False) -> dict:
    """Dispatch-mode PMC of ``load`` (MFMA busy per kernel); ``beside_counters``: with the
    monitor's device-wide th-counters session running at the same time (coexistence)."""
    if load == "idle":
        return {"kernel_busy_pct": 0.0}
    cs = None
    if beside_counters:
        from tensorhive_fixed_amd.core.counters import CounterStream

        cs = CounterStream(period_ms=500, window_ms=200)
        cs.wait_first(15)
    d = (outdir / f"pmc_{load}{'_coexist' if beside_counters else ''}").resolve()  # rocprofv3 runs from /tmp
    r = subprocess.run(["rocprofv3", "--pmc", *PMC, "--output-format", "csv", "-d", str(d), "-o", "run", "--",
                        sys.executable, str(ROOT / "scripts" / "mfma_load.py"), load, "2"],
                       capture_output=True, text=True, timeout=300, cwd="/tmp", env={**os.environ, "TMPDIR": "/tmp"})
    counters_alive = None
    if cs is not None:
        counters_alive = bool(cs.latest()) and cs.error is None and cs._proc is not None and cs._proc.poll() is None
        cs.close()
    if r.returncode != 0:
        return {"error": r.stderr[-1500:], "counters_alive": counters_alive}
    per: dict = {}
    for f in d.rglob("*counter_collection.csv"):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = (row.get("Dispatch_Id") or row.get("Correlation_Id"), row["Kernel_Name"])
                per.setdefault(k, {})[row["Counter_Name"]] = per.get(k, {}).get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    busy = sum(v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) for v in per.values())
    grbm = sum(v.get("GRBM_GUI_ACTIVE", 0.0) for v in per.values())
    names = sorted({k[1][:60] for k in per})
    return {"kernel_busy_pct": 100.0 * busy / (grbm / 8 * 1024) if grbm else None, "dispatches": len(per),
            "kernels": names[:6], "counters_alive": counters_alive}


def main():
    outdir = Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/probe_vs_pmc")
    outdir.mkdir(parents=True, exist_ok=True)
    res = []
    for load in LOADS:
        m = monitored(load)
        m["pmc"] = pmc(load, outdir)
        if load == "gemm":  # can a user's rocprofv3 --pmc run while th-counters samples the device?
            m["pmc_beside_th_counters"] = pmc(load, outdir, beside_counters=True)
        kb = m["pmc"].get("kernel_busy_pct")
        m["pmc_wall_busy_pct"] = None if kb is None else kb * (m["run"].get("gpu_share") or 0.0)
        res.append(m)
        print(json.dumps({k: v for k, v in m.items() if k != "samples"}), flush=True)
    (outdir / "probe_vs_pmc.json").write_text(json.dumps(res, indent=1))
    print(f"{'load':10} {'probe':>7} {'pmc wall':>9} {'pmc kern':>9} {'ctr busy':>8} {'gpu_busy':>8} {'TFLOP/s':>8}")
    for m in res:
        f = lambda v: "-" if v is None else f"{v:.1f}"  # noqa: E731
        print(f"{m['load']:10} {f(m['probe_mfma_contention']):>7} {f(m['pmc_wall_busy_pct']):>9} "
              f"{f(m['pmc'].get('kernel_busy_pct')):>9} {f(m['counters_mfma_busy']):>8} "
              f"{f(m['counters_gpu_busy']):>8} {f(m['counters_mfma_tflops']):>8}")


if __name__ == "__main__":
    main()
