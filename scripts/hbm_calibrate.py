"""Calibrate amdsmi memory-activity readings against known HBM traffic (SURVEY N03, round-2
verdict item 4).  Device-counting TCC counters do not see other processes on this driver
(profiles/r02_counters/), so the daemon's HBM bandwidth comes from amdsmi: this script checks
which amdsmi field tracks bytes/s.

For each load (idle, ``y += x`` stream, copy stream, and a half-duty stream) it samples, every
100 ms: ``get_gpu_activity().umc_activity``, gpu_metrics ``average_umc_activity`` and the
``mem_activity_acc`` accumulator, plus ``vram_max_bandwidth``; the stream prints the GB/s torch
measured.  Output: one JSON line per load."""
import json
import subprocess
import sys
import time

import amdsmi


def main():
    amdsmi.amdsmi_init()
    h = amdsmi.amdsmi_get_processor_handles()[0]
    try:
        vram = amdsmi.amdsmi_get_gpu_vram_info(h)
    except Exception as e:  # noqa: BLE001
        vram = {"error": str(e)}
    print(json.dumps({"vram_info": {k: str(v) for k, v in vram.items()}}), flush=True)
    loads = [("idle", None), ("add", ["4", "add"]), ("copy", ["4", "copy"]), ("add_half", ["4", "add", "half"])]
    for name, args in loads:
        p = None
        if args:
            p = subprocess.Popen([sys.executable, "scripts/hbm_stream.py", *args], stdout=subprocess.PIPE, text=True)
            time.sleep(1.5)
        samples = []
        t_end = time.time() + 2.0
        while time.time() < t_end:
            act = amdsmi.amdsmi_get_gpu_activity(h)
            gm = amdsmi.amdsmi_get_gpu_metrics_info(h)
            samples.append({"t": time.time(), "umc": act.get("umc_activity"), "gfx": act.get("gfx_activity"),
                            "avg_umc": gm.get("average_umc_activity"), "mem_acc": gm.get("mem_activity_acc"),
                            "mem_clk": gm.get("current_uclk")})
            time.sleep(0.1)
        stream = None
        if p is not None:
            out, _ = p.communicate(timeout=60)
            stream = json.loads(out.strip().splitlines()[-1])
        accs = [s["mem_acc"] for s in samples if isinstance(s["mem_acc"], int)]
        acc_rate = (accs[-1] - accs[0]) / (samples[-1]["t"] - samples[0]["t"]) if len(accs) > 1 else None
        umc = [s["umc"] for s in samples if isinstance(s["umc"], (int, float))]
        avg_umc = [s["avg_umc"] for s in samples if isinstance(s["avg_umc"], (int, float))]
        print(json.dumps({"load": name, "stream": stream, "umc_mean": sum(umc) / len(umc) if umc else None,
                          "avg_umc_mean": sum(avg_umc) / len(avg_umc) if avg_umc else None,
                          "mem_activity_acc_per_s": acc_rate, "samples": samples[:3]}), flush=True)
    amdsmi.amdsmi_shut_down()


if __name__ == "__main__":
    main()
