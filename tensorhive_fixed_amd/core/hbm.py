"""HBM bytes from hardware counters, per GPU (round-2 verdict item 3).

Tasks started by th-run carry the in-task counter tool (``native/th_hbm_tool.cpp`` ->
``lib/libthhbm.so``, loaded through ``ROCP_TOOL_LIBRARIES``): every process of the task writes
``/dev/shm/th-hbm-<pid>.json`` once per period with the L2's memory-side read/write request
counts of the GPU it drives, turned into bytes.  Counting from the monitor's own process cannot
do this -- on this stack the TCC request counters only count the counting process's traffic
(``profiles/r03_counters/``) -- so the task counts itself and the monitor sums the files per GPU.

:func:`read_rates` returns ``{bdf: {"hbm_read": GB/s, "hbm_write": GB/s, "pids": [...]}}`` over
the live, fresh files; files of dead processes are removed.  GPUs without a counting task keep
libthsmi's ``mem_activity_acc``-based ``hbm_bw`` estimate (``hbm_bw_source`` says which).
"""
from __future__ import annotations

import glob
import json
import os
import time
from pathlib import Path

SHM_GLOB = "/dev/shm/th-hbm-*.json"


def tool_path() -> str | None:
    from ..native.build import path_of

    p = path_of("libthhbm")
    return str(p) if p.exists() else None


def task_env() -> dict[str, str]:
    """Environment that makes a task count its own HBM traffic (empty when the tool is missing)."""
    p = tool_path()
    return {"ROCP_TOOL_LIBRARIES": p} if p else {}


def _alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
        return True
    except ProcessLookupError:
        return False
    except PermissionError:
        return True


def read_rates(pattern: str = SHM_GLOB, max_age_s: float = 5.0, now: float | None = None,
               cleanup: bool = True) -> dict[str, dict]:
    now = time.time() if now is None else now
    out: dict[str, dict] = {}
    for f in glob.glob(pattern):
        try:
            doc = json.loads(Path(f).read_text())
        except (OSError, ValueError):
            continue
        pid = int(doc.get("pid") or 0)
        if pid and not _alive(pid):
            if cleanup:
                try:
                    os.unlink(f)
                except OSError:
                    pass
            continue
        if now - int(doc.get("ts_ns", 0)) / 1e9 > max_age_s:
            continue
        win = max(float(doc.get("window_ms") or 0.0), 1e-3) / 1000.0
        for g in doc.get("gpus", []):
            r = out.setdefault(g.get("bdf"), {"hbm_read": 0.0, "hbm_write": 0.0, "pids": []})
            r["hbm_read"] += float(g.get("rd_bytes") or 0.0) / win / 1e9
            r["hbm_write"] += float(g.get("wr_bytes") or 0.0) / win / 1e9
            r["pids"].append(pid)
    return out


def metrics_for(gpus: list[dict], rates: dict[str, dict]) -> dict[int, dict]:
    """``{index: metrics}`` for the GPUs that have counted traffic: hbm_read / hbm_write and an
    ``hbm_bw`` that replaces the activity-based estimate, with ``hbm_bw_source = counters``."""
    out = {}
    for g in gpus:
        r = rates.get(g.get("bdf"))
        if r is None:
            continue
        rd, wr = round(r["hbm_read"], 1), round(r["hbm_write"], 1)
        out[g["index"]] = {"hbm_read": {"value": rd, "unit": "GB/s"}, "hbm_write": {"value": wr, "unit": "GB/s"},
                           "hbm_bw": {"value": round(rd + wr, 1), "unit": "GB/s"},
                           "hbm_bw_source": {"value": "counters", "unit": ""}}
    return out
