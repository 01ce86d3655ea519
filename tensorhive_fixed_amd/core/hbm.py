"""HBM bytes from hardware counters, per GPU (round-2 verdict item 3).

Tasks started by th-run carry the in-task counter tool (``native/th_hbm_tool.cpp`` ->
``lib/libthhbm.so``, loaded through ``ROCP_TOOL_LIBRARIES``): every process of the task writes
``/dev/shm/th-hbm-<pid>.json`` once per period with the L2's memory-side read/write request
counts of the GPU it drives, turned into bytes.  Counting from the monitor's own process cannot
do this -- on this stack the TCC request counters only count the counting process's traffic
(``profiles/r03_counters/``) -- so the task counts itself and the monitor sums the files per GPU.

:func:`read_rates` returns ``{bdf: {"hbm_read": GB/s, "hbm_write": GB/s, "pids": [...]}}`` over
the live, fresh files whose owner owns the pid; files of dead processes are removed.
:func:`metrics_for` keeps only pids libthsmi lists on that GPU as th-run task processes.  On a
node, the task ids are the processes' own claims; the daemon re-derives the metrics after
``core/attribution.py`` has attested every claim (:func:`finalize_entry`), so a process that
forges a task id cannot get its counts -- or its silence -- accepted.  GPUs
without a counting task keep libthsmi's ``mem_activity_acc``-based ``hbm_bw`` estimate; GPUs
where only some processes are counted say ``partial`` (``hbm_bw_source`` says which).
"""
from __future__ import annotations

import glob
import json
import logging
import os
import stat
import time

log = logging.getLogger(__name__)

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


def _proc_uid(pid: int) -> int | None:
    try:
        return os.stat(f"/proc/{pid}").st_uid
    except OSError:
        return None


MAX_FILE_BYTES = 64 << 10


def _read_small_regular(path: str) -> tuple[os.stat_result, bytes]:
    """Read a counter file that any local user could have planted: never follow a symlink, never
    block on a FIFO, only a regular file of at most ``MAX_FILE_BYTES``; the stat (owner) is the
    one of the file actually read."""
    fd = os.open(path, os.O_RDONLY | os.O_NOFOLLOW | os.O_NONBLOCK | getattr(os, "O_CLOEXEC", 0))
    try:
        st = os.fstat(fd)
        if not stat.S_ISREG(st.st_mode):
            raise OSError(f"{path}: not a regular file")
        if st.st_size > MAX_FILE_BYTES:
            raise OSError(f"{path}: {st.st_size} bytes")
        chunks, left = [], MAX_FILE_BYTES + 1
        while left > 0:
            b = os.read(fd, left)
            if not b:
                break
            chunks.append(b)
            left -= len(b)
        data = b"".join(chunks)
        if len(data) > MAX_FILE_BYTES:
            raise OSError(f"{path}: grew past the cap")
        return st, data
    finally:
        os.close(fd)


def read_rates(pattern: str = SHM_GLOB, max_age_s: float = 5.0, now: float | None = None,
               cleanup: bool = True) -> dict[str, dict]:
    """``{bdf: {"hbm_read", "hbm_write", "pids", "by_pid": {pid: (rd GB/s, wr GB/s)}}}`` over the
    fresh files of live processes. A file is taken only when its owner is the owner of the pid it
    names (``/dev/shm`` is world-writable: anyone could otherwise write a file naming pid 1 or a
    victim's training process); :func:`metrics_for` then checks the pid against the GPU's own
    process list."""
    now = time.time() if now is None else now
    out: dict[str, dict] = {}
    for f in glob.glob(pattern):
        try:
            st, raw = _read_small_regular(f)
            doc = json.loads(raw)
            pid = int(doc.get("pid") or 0)
        except (OSError, ValueError, TypeError, AttributeError):
            continue
        if pid <= 0:
            continue
        if not _alive(pid):
            if cleanup:
                try:
                    os.unlink(f)
                except OSError:
                    pass
            continue
        if _proc_uid(pid) != st.st_uid:
            log.warning("hbm: ignoring %s: file owner uid %d is not the owner of pid %d", f, st.st_uid, pid)
            continue
        if now - int(doc.get("ts_ns", 0)) / 1e9 > max_age_s:
            continue
        win = max(float(doc.get("window_ms") or 0.0), 1e-3) / 1000.0
        for g in doc.get("gpus", []):
            rd = float(g.get("rd_bytes") or 0.0) / win / 1e9
            wr = float(g.get("wr_bytes") or 0.0) / win / 1e9
            r = out.setdefault(g.get("bdf"), {"hbm_read": 0.0, "hbm_write": 0.0, "pids": [], "by_pid": {}})
            r["hbm_read"] += rd
            r["hbm_write"] += wr
            r["pids"].append(pid)
            prd, pwr = r["by_pid"].get(pid, (0.0, 0.0))
            r["by_pid"][pid] = (prd + rd, pwr + wr)
    return out


def metrics_for(gpus: list[dict], rates: dict[str, dict]) -> dict[int, dict]:
    """``{index: metrics}`` for the GPUs with counted traffic.

    A counted pid is kept only if libthsmi lists it on that very GPU with a ``TENSORHIVE_TASK_ID``
    (a th-run task's process); any other file is ignored and logged.  Then:

    * every process on the GPU is counted -> ``hbm_bw`` = counted read + write,
      ``hbm_bw_source = counters``;
    * some process on the GPU is not counted (a foreign tenant, a task without the tool) ->
      ``hbm_bw_source = partial``: ``hbm_bw`` keeps the device-wide activity estimate (raised to
      the counted sum if that is larger), ``hbm_counted`` carries the counted part.  An uncounted
      tenant never reads as 0 GB/s behind a ``counters`` label.

    GPU records without a ``processes`` key (callers that have no process list) keep the old
    behaviour: every file that names the GPU counts."""
    out = {}
    for g in gpus:
        r = rates.get(g.get("bdf"))
        if r is None:
            continue
        procs = g.get("processes")
        by_pid = r.get("by_pid") or {p: (r["hbm_read"] / max(1, len(r["pids"])),
                                         r["hbm_write"] / max(1, len(r["pids"]))) for p in r.get("pids", [])}
        if procs is None:
            valid = dict(by_pid)
            uncounted = []
        else:
            tasks = {int(p["pid"]): p.get("task_id") for p in procs if p.get("pid") is not None}
            valid = {}
            for pid, v in by_pid.items():
                if pid in tasks and tasks[pid] not in (None, ""):
                    valid[pid] = v
                else:
                    log.warning("hbm: ignoring counts of pid %d on %s: %s", pid, g.get("bdf"),
                                "not a th-run task process" if pid in tasks else "not a process of this GPU")
            uncounted = [p for p in tasks if p not in valid]
        if not valid:
            continue
        rd = round(sum(v[0] for v in valid.values()), 1)
        wr = round(sum(v[1] for v in valid.values()), 1)
        m = {"hbm_read": {"value": rd, "unit": "GB/s"}, "hbm_write": {"value": wr, "unit": "GB/s"},
             "hbm_counted": {"value": round(rd + wr, 1), "unit": "GB/s"}}
        if uncounted:
            est = ((g.get("metrics") or {}).get("hbm_bw") or {}).get("value")
            total = max(float(est or 0.0), rd + wr)
            m["hbm_bw"] = {"value": round(total, 1), "unit": "GB/s"}
            m["hbm_bw_source"] = {"value": "partial", "unit": ""}
            m["hbm_uncounted_pids"] = {"value": len(uncounted), "unit": ""}
        else:
            m["hbm_bw"] = {"value": round(rd + wr, 1), "unit": "GB/s"}
            m["hbm_bw_source"] = {"value": "counters", "unit": ""}
        out[g["index"]] = m
    return out


_DERIVED = ("hbm_read", "hbm_write", "hbm_counted", "hbm_bw_source", "hbm_uncounted_pids")


def raw_counts(rates: dict[str, dict], bdf) -> dict | None:
    """The per-pid counted rates of one GPU in wire form (``{"<pid>": [rd, wr]}``), or None."""
    r = rates.get(bdf)
    if not r:
        return None
    by_pid = r.get("by_pid") or {}
    return {str(pid): [round(v[0], 3), round(v[1], 3)] for pid, v in by_pid.items()}


def finalize_entry(entry: dict) -> dict:
    """Re-derive the counter-based HBM metrics of an infrastructure entry from its raw per-pid
    counts (``_hbm``, attached by ``telemetry.apply_task_hbm``) and the CURRENT -- attested -- task
    ids of its processes, then drop the raw counts.  GPUs without raw counts are left alone."""
    for g in ((entry or {}).get("GPU") or {}).values():
        if not g or "_hbm" not in g:
            continue
        raw = g.pop("_hbm") or {}
        m = g.setdefault("metrics", {})
        for k in _DERIVED:
            m.pop(k, None)
        if raw.get("est") is not None or "hbm_bw" in m:
            m["hbm_bw"] = {"value": raw.get("est"), "unit": "GB/s"}
        counts = raw.get("counts") or {}
        rates = {g.get("bdf"): {"by_pid": {int(p): (float(v[0]), float(v[1])) for p, v in counts.items()},
                                "pids": [int(p) for p in counts]}} if counts else {}
        got = metrics_for([g], rates).get(g.get("index")) if rates else None
        m.update(got or {"hbm_bw_source": {"value": "umc_activity", "unit": ""}})
    return entry
