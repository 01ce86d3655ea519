"""Measured GEMM algorithm choices for the step's hipBLASLt / rocBLAS GEMMs (PyTorch TunableOp tables).

``scripts/gemm_tune.py tune`` benchmarks every hipBLASLt and rocBLAS solution of each forward and
input-gradient GEMM of the Llama-3-8B step (32768 tokens per rank) and writes the fastest per shape.
:func:`load_gemm_table` makes a process use that table with tuning OFF: a GEMM whose shape is in the
table runs the recorded solution, any other shape keeps the library's default heuristic.  The
validators at the top of the table (PyTorch / HIP / hipBLASLt / rocBLAS versions, gfx arch) are
checked by TunableOp itself; a mismatch leaves the defaults in place.
"""
from __future__ import annotations

import logging
import os
from pathlib import Path

log = logging.getLogger(__name__)

HERE = Path(__file__).resolve().parent
TABLE = HERE / "gemm_gfx950_t32768.csv"


def table_path(path: str | os.PathLike | None = None) -> Path:
    """The table :func:`load_gemm_table` reads: ``path``, else ``TH_GEMM_TUNED_FILE``, else the shipped one."""
    return Path(path or os.environ.get("TH_GEMM_TUNED_FILE", TABLE))


def load_gemm_table(path: str | os.PathLike | None = None) -> bool:
    """Enable TunableOp in lookup-only mode with the tuned table (``TH_GEMM_TUNED=0`` disables).

    Multi-rank steps use the same table.  A table tuned while an emulated RCCL channel kernel held 16 CUs
    (replacing hipBLASLt's stream-K defaults, whose one-workgroup-per-CU grids double when CUs are held) measured
    worse in the step on an idle chip (w13 input gradient 5.09 -> 5.89 ms) and no better under held CUs with
    the channels' HBM traffic (10.6 ms for its MT192x256 kernel against 5.8 for stream-K): profiles/r06_comm/.

    On the round-5 table: -5.1 ms per step (three interleaved pairs: -3.8 / -4.5 / -7.1 ms), mostly the
    gate|up forward GEMM on a rocBLAS solution (5.11 -> 5.00 ms); the w13 input-gradient entry is pinned to
    the default, which its tuned choice was 1 % slower than (profiles/r05_gemm/tunableop_*.txt)."""
    if os.environ.get("TH_GEMM_TUNED", "1") != "1":
        return False
    import torch

    p = table_path(path)
    if not torch.cuda.is_available() or not p.exists():
        return False
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(False)
    if hasattr(tun, "record_untuned_enable"):
        tun.record_untuned_enable(False)
    ok = bool(tun.read_file(str(p)))
    log.info("GEMM table %s loaded: %s", p, ok)
    return ok
