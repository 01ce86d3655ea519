"""Self-diagnosis of a multi-GPU run (round-3 verdict item 7): what RCCL built at init, and how
much of each step the compute stream spent waiting on communication.

* :func:`prepare_rccl_log` (called by ``init_distributed`` before the communicator exists) sends
  RCCL's INIT-subsystem log of this rank to a private file (``NCCL_DEBUG=INFO``,
  ``NCCL_DEBUG_SUBSYS=INIT``, ``NCCL_DEBUG_FILE``) -- only for bench.py (``TH_RCCL_INIT_LOG=1``),
  whose :func:`comm_report` echoes the warnings found in it, and never over the user's own
  RCCL debug settings.
* :func:`parse_rccl_init` reads that log: library version, ranks, channels (the ``Channel xx/NN``
  rings and the ``N coll channels`` summary), trees, the transports each channel connected through
  (``via P2P/IPC`` = xGMI peer access), chunk size and thread thresholds.
* :func:`comm_report` all-gathers every rank's wait spans (``parallel/flat.py:WaitTimer``) and
  its RCCL summary into the block bench.py prints: ``exposed_comm_ms_per_step`` (gradient
  bucket waits + parameter all-gather waits), ``allgather_wait_ms``, ``opt_wait_ms`` (max over
  ranks, per step), plus the per-rank rows.

The reference has no data plane; this is the MI355X-side observability of
the one the payload brings.
"""
from __future__ import annotations

import os
import re
import sys
import tempfile

import torch
import torch.distributed as dist

_LOG_ENV = "TH_RCCL_INIT_LOG"


def prepare_rccl_log(rank: int) -> str | None:
    """Point RCCL's INIT log at a per-rank file; returns its path.  Opt-in: only when
    ``TH_RCCL_INIT_LOG=1`` (bench.py sets it, and then echoes the log's warnings), and never over
    the user's own debugging (a ``NCCL_DEBUG_FILE``, a level above INFO, another subsystem).  A
    training job (no opt-in) keeps RCCL's warnings and its requested debug output on stderr."""
    if os.environ.get(_LOG_ENV, "0") != "1" or os.environ.get("NCCL_DEBUG_FILE"):
        return None
    level = os.environ.get("NCCL_DEBUG", "").upper()
    if level not in ("", "WARN", "VERSION", "INFO"):
        return None  # TRACE or something custom: leave it alone
    if os.environ.get("NCCL_DEBUG_SUBSYS") not in (None, "", "INIT"):
        return None
    path = os.path.join(tempfile.gettempdir(), f"th-rccl-init-{os.getpid()}-r{rank}.log")
    os.environ["NCCL_DEBUG"] = "INFO"
    os.environ["NCCL_DEBUG_SUBSYS"] = "INIT"
    os.environ["NCCL_DEBUG_FILE"] = path
    os.environ[_LOG_ENV + "_PATH"] = path
    return path


_VERSION = re.compile(r"\b(RCCL|NCCL) version[ :]+(\S+)")
_NRANKS = re.compile(r"\bnRanks (\d+)")
_CHANNEL = re.compile(r"\bChannel (\d+)/(\d+)\s*:")
_COLL = re.compile(r"(\d+) coll channels(?:, (\d+) collnet channels)?(?:, (\d+) nvls channels)?(?:, (\d+) p2p channels)?")
_VIA = re.compile(r"\bvia (\S+)")
_TREES = re.compile(r"\bTrees\b")
_CHUNK = re.compile(r"P2P Chunksize set to (\d+)")
_THRESH = re.compile(r"threadThresholds (.+)$")
_KEEP = re.compile(r"coll channels|threadThresholds|Chunksize|Connected all|MSCCL|algo|Algo|proto|Proto|"
                   r"version|nRanks|Using network|XGMI|xGMI|P2P level")


def parse_rccl_init(text: str) -> dict:
    out: dict = {"version": None, "library": None, "nranks": None, "channels": None, "coll_channels": None,
                 "p2p_channels": None, "trees": 0, "transports": {}, "p2p_chunksize": None,
                 "thread_thresholds": None, "warnings": [], "lines": []}
    seen = set()
    for raw in text.splitlines():
        line = raw.strip()
        if not line:
            continue
        m = _VERSION.search(line)
        if m and out["version"] is None:
            out["library"], out["version"] = m.group(1), m.group(2)
        m = _NRANKS.search(line)
        if m:
            out["nranks"] = int(m.group(1))
        m = _CHANNEL.search(line)
        if m:
            out["channels"] = max(out["channels"] or 0, int(m.group(2)))
        m = _COLL.search(line)
        if m:
            out["coll_channels"] = int(m.group(1))
            if m.group(4):
                out["p2p_channels"] = int(m.group(4))
        for t in _VIA.findall(line):
            out["transports"][t] = out["transports"].get(t, 0) + 1
        if _TREES.search(line):
            out["trees"] += 1
        m = _CHUNK.search(line)
        if m:
            out["p2p_chunksize"] = int(m.group(1))
        m = _THRESH.search(line)
        if m:
            out["thread_thresholds"] = m.group(1).strip()
        if " WARN " in f" {line} ":
            msg = line.split(" WARN ", 1)[1].strip()[:200]
            if msg not in out["warnings"] and len(out["warnings"]) < 8:  # unique messages only
                out["warnings"].append(msg)
        # one example of each informative line, without the per-rank prefix
        body = line.split(" INFO ", 1)[-1]
        if _KEEP.search(body) and body not in seen and len(out["lines"]) < 24:
            seen.add(body)
            out["lines"].append(body[:240])
    return out


def rccl_summary() -> dict | None:
    """This rank's RCCL init summary (None when no RCCL communicator exists)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_backend() != "nccl":
        return None
    info: dict = {}
    try:
        v = torch.cuda.nccl.version()
        info["torch_reported_version"] = ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    except Exception:  # noqa: BLE001
        pass
    path = os.environ.get(_LOG_ENV + "_PATH")
    if path and os.path.exists(path):
        with open(path, errors="replace") as f:
            parsed = parse_rccl_init(f.read())
        for w in parsed["warnings"]:
            print(f"[rccl] {w}", file=sys.stderr)
        info.update(parsed)
        info["log"] = path
    return info


def comm_report(waits: dict, info) -> dict:
    """All ranks' wait spans (+ RCCL summary) -> the bench JSON block. Collective when a process
    group exists: every rank must call it."""
    mine = {"rank": info.rank, **waits}
    rccl = rccl_summary()
    if dist.is_available() and dist.is_initialized():
        rows: list = [None] * dist.get_world_size()
        dist.all_gather_object(rows, mine)
    else:
        rows = [mine]

    def worst(key: str) -> float:
        return round(max(float(r.get(key) or 0.0) for r in rows), 3)

    exposed = max(float(r.get("grad_sync_ms_per_step") or 0.0) + float(r.get("allgather_ms_per_step") or 0.0)
                  for r in rows)
    return {"exposed_comm_ms_per_step": round(exposed, 3),
            "grad_sync_wait_ms": worst("grad_sync_ms_per_step"),
            "allgather_wait_ms": worst("allgather_ms_per_step"),
            "opt_wait_ms": worst("opt_wait_ms_per_step"),
            "per_rank": rows, "rccl": rccl}
