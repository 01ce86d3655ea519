"""Runner and output contract of the native RCCL/xGMI microbenchmark (SURVEY N06,
``native/rccl_bench.hip``).

Two modes, as SURVEY N06 specifies:
  * ``single_process`` -- one process drives every GPU (``ncclCommInitAll``), plus the optional
    one-shot direct peer all-reduce kernel (16-byte xGMI loads/stores) for comparison;
  * ``per_rank`` -- one process per GPU under torchrun (``ncclCommInitRank``), exactly how the
    training job communicates; the reported time is the max over ranks.

Every run's stdout is JSON lines: a header ``{"rccl_bench": 1, "mode", "world", "rccl_version",
"env"}`` then one result per (op, message size).  :func:`parse` validates every line against
:data:`HEADER` / :data:`RESULT`, so a silently changed binary fails the tests, and the header
records the RCCL environment (``NCCL_*``) each number was taken under.
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

HEADER = {"rccl_bench": int, "mode": str, "world": int, "rccl_version": int, "env": dict}
RESULT = {"op": str, "mode": str, "gpus": int, "bytes": int, "time_us": (int, float), "algbw_GBps": (int, float),
          "busbw_GBps": (int, float)}
OPS = {"allreduce", "reducescatter", "allgather", "direct_allreduce"}
MODES = {"single_process", "per_rank"}


class SchemaError(ValueError):
    pass


def _check(doc: dict, schema: dict, what: str) -> None:
    missing = set(schema) - set(doc)
    if missing:
        raise SchemaError(f"{what}: missing {sorted(missing)} in {doc}")
    for k, t in schema.items():
        if not isinstance(doc[k], t) or isinstance(doc[k], bool):
            raise SchemaError(f"{what}: {k}={doc[k]!r} is not {t}")


def parse(stdout: str) -> dict:
    """Validate rccl-bench output; returns ``{"header": {...}, "results": [...]}``."""
    lines = [json.loads(ln) for ln in stdout.splitlines() if ln.startswith("{")]
    if not lines:
        raise SchemaError("no JSON output")
    header, results = lines[0], lines[1:]
    _check(header, HEADER, "header")
    if header["mode"] not in MODES:
        raise SchemaError(f"header: unknown mode {header['mode']}")
    for r in results:
        _check(r, RESULT, "result")
        if r["op"] not in OPS or r["mode"] != header["mode"] or r["gpus"] != header["world"]:
            raise SchemaError(f"result does not match its header: {r}")
        if r["bytes"] <= 0 or r["time_us"] <= 0 or r["algbw_GBps"] < 0:
            raise SchemaError(f"result out of range: {r}")
        n = r["gpus"]
        factor = 2.0 * (n - 1) / n if "allreduce" in r["op"] else (n - 1) / n
        if abs(r["busbw_GBps"] - r["algbw_GBps"] * factor) > 0.02 + 1e-3 * r["algbw_GBps"]:
            raise SchemaError(f"bus bandwidth inconsistent with algorithm bandwidth: {r}")
    return {"header": header, "results": results}


def _binary() -> str:
    from ..native.build import build_all, path_of

    p = path_of("rccl-bench")
    if not p.exists():
        build_all(strict=False)
    return str(p)


def run_single(gpus: int = 0, min_bytes: int = 8 << 20, max_bytes: int = 1 << 30, iters: int = 20,
               op: str = "all", direct: bool = False, env: dict | None = None, timeout: float = 600) -> dict:
    cmd = [_binary(), "--gpus", str(gpus), "--min", str(min_bytes), "--max", str(max_bytes), "--iters", str(iters),
           "--op", op] + (["--direct"] if direct else [])
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env={**os.environ, **(env or {})})
    if r.returncode != 0:
        raise RuntimeError(f"rccl-bench failed ({r.returncode}): {r.stderr[-2000:]}")
    return parse(r.stdout)


def run_per_rank(gpus: int, min_bytes: int = 8 << 20, max_bytes: int = 1 << 30, iters: int = 20, op: str = "all",
                 env: dict | None = None, timeout: float = 600) -> dict:
    """``TH_RCCL_PER_RANK=1 torchrun --no-python --nproc-per-node GPUS rccl-bench`` (one rank per
    GPU; the options travel in the environment, torchrun's parser would claim ``--min``/``--max``)."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "--no-python", _binary()]
    e = {**os.environ, "HSA_ENABLE_IPC_MODE_LEGACY": "0", "TH_RCCL_PER_RANK": "1", "TH_RCCL_MIN": str(min_bytes),
         "TH_RCCL_MAX": str(max_bytes), "TH_RCCL_ITERS": str(iters), "TH_RCCL_OP": op, **(env or {})}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=e)
    if r.returncode != 0:
        raise RuntimeError(f"rccl-bench --per-rank failed ({r.returncode}): {r.stderr[-2000:]}")
    return parse(r.stdout)
