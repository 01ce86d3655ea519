"""Device-wide hardware counters for the dashboard, from the native ``th-counters``
sampler (rocprofiler-sdk device counting service, ``native/th_counters.cpp``).

:class:`CounterStream` keeps one ``th-counters --count 0`` child per node (local) streaming a JSON
line per period; :func:`derive` turns raw counter sums of one window into the metrics the
monitoring entry carries (``{value, unit}`` like every other metric):

* ``gpu_busy``    -- GRBM_GUI_ACTIVE / GRBM_COUNT  (% of cycles the graphics engine was busy)
* ``mfma_busy``   -- SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_COUNT / XCDs x SIMDs): the share of every
  SIMD's cycles its matrix core was busy (the device-wide counterpart of the dispatch-PMC
  "MFMA busy" of ``profiles/r03_gemm``; 8 XCDs x 1024 SIMDs on MI355X)
* ``mfma_tflops`` -- SQ_INSTS_VALU_MFMA_MOPS_{BF16,F8,...} x 512 FLOP / window
* ``hbm_read`` / ``hbm_write`` -- TCC EA request counts x request size / window (GB/s), only when
  the requested counters include them (they read ~0 in device-counting mode on gfx950).

The MOPS scale is checked on hardware by ``scripts/counters_check.py`` against a GEMM of known
FLOPs (1400 vs 1342 TFLOP/s measured by torch, same window).
"""
from __future__ import annotations

import json
import logging
import subprocess
import threading
import time

from ..utils.proc import StderrTail

log = logging.getLogger(__name__)

MOPS_FLOP = 512.0
MFMA_MOPS = ("SQ_INSTS_VALU_MFMA_MOPS_BF16", "SQ_INSTS_VALU_MFMA_MOPS_F16", "SQ_INSTS_VALU_MFMA_MOPS_F8",
             "SQ_INSTS_VALU_MFMA_MOPS_F32", "SQ_INSTS_VALU_MFMA_MOPS_F64", "SQ_INSTS_VALU_MFMA_MOPS_I8")
# Validated on MI355X (scripts/counters_check.py, profiles/r01_counters/): GRBM busy and the MFMA
# MOPS counters (x512 FLOP) track a bf16 GEMM within 5 % of torch's own timing.  In device-counting
# mode the TCC/EA request counters and SQ_WAVES read ~0 under a 5 TB/s copy, so HBM traffic is not
# taken from counters (libthsmi's amdsmi memory activity is used instead).
DEFAULT_COUNTERS = ("GRBM_GUI_ACTIVE", "GRBM_COUNT", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VALU_MFMA_MOPS_BF16",
                    "SQ_INSTS_VALU_MFMA_MOPS_F16", "SQ_INSTS_VALU_MFMA_MOPS_F8", "SQ_INSTS_VALU_MFMA_MOPS_F32")
# SQ_VALU_MFMA_BUSY_CYCLES sums over every SIMD; GRBM counters sum over the XCDs (gfx950: 8 XCDs,
# 32 CUs x 4 SIMDs each).  Read device-wide from th-counters' own process it matches the probe
# validation loads (profiles/r04_probe/): the device counting service sees every tenant's SQ work.
XCDS, SIMDS = 8, 1024


def _m(value, unit):
    return {"value": value, "unit": unit}


def derive(gpu: dict, window_ms: float, xcds: int = XCDS, simds: int = SIMDS) -> dict:
    """One GPU's raw counter sums (``{"counters": {...}}``) -> dashboard metrics."""
    c = gpu.get("counters") or {}
    s = max(window_ms, 1e-3) / 1000.0
    out = {}
    if c.get("GRBM_COUNT"):
        out["gpu_busy"] = _m(round(100.0 * c.get("GRBM_GUI_ACTIVE", 0) / c["GRBM_COUNT"], 1), "%")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            cycles = c["GRBM_COUNT"] / xcds  # elapsed shader-clock cycles of the window
            busy = 100.0 * c["SQ_VALU_MFMA_BUSY_CYCLES"] / (cycles * simds)
            out["mfma_busy"] = _m(round(min(100.0, max(0.0, busy)), 1), "%")
    mops = [c[k] for k in MFMA_MOPS if k in c]
    if mops:
        out["mfma_tflops"] = _m(round(sum(mops) * MOPS_FLOP / s / 1e12, 1), "TFLOP/s")
    if "TCC_EA0_RDREQ_sum" in c:
        r32 = c.get("TCC_EA0_RDREQ_32B_sum", 0)
        rd = (c["TCC_EA0_RDREQ_sum"] - r32) * 64 + r32 * 32
        out["hbm_read"] = _m(round(rd / s / 1e9, 1), "GB/s")
    if "TCC_EA0_WRREQ_sum" in c:
        w64 = c.get("TCC_EA0_WRREQ_64B_sum", 0)
        wr = w64 * 64 + (c["TCC_EA0_WRREQ_sum"] - w64) * 32
        out["hbm_write"] = _m(round(wr / s / 1e9, 1), "GB/s")
    return out


class CounterStream:
    """Background reader of ``th-counters --count 0 --period P``; ``latest()`` returns
    ``{kfd_id: metrics}`` of the newest window (or ``{}`` when the sampler is unavailable)."""

    def __init__(self, period_ms: int = 1000, window_ms: int = 100, counters=DEFAULT_COUNTERS,
                 binary: str | None = None):
        from ..native.build import build_all, path_of

        if binary is None:
            if not path_of("th-counters").exists():
                build_all(strict=False)
            binary = str(path_of("th-counters"))
        self.cmd = [binary, "--count", "0", "--period", str(period_ms), "--window", str(window_ms),
                    "--counters", ",".join(counters)]
        self._latest: dict = {}
        self._raw: dict = {}
        self._lock = threading.Lock()
        self._proc: subprocess.Popen | None = None
        self._thread = threading.Thread(target=self._run, name="th-counters", daemon=True)
        self._stop = threading.Event()
        self.error: str | None = None
        self._thread.start()

    def _run(self) -> None:
        try:
            self._proc = subprocess.Popen(self.cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        except OSError as e:
            self.error = str(e)
            return
        err = StderrTail(self._proc.stderr, name="th-counters")
        for line in self._proc.stdout:  # type: ignore[union-attr]
            if self._stop.is_set():
                break
            try:
                doc = json.loads(line)
            except json.JSONDecodeError:
                continue
            if "error" in doc:
                self.error = doc["error"]
                continue
            metrics = {g.get("kfd_id"): derive(g, doc.get("window_ms", 100)) for g in doc.get("gpus", [])}
            with self._lock:
                self._latest = metrics
                self._raw = doc
        if self._proc.wait() != 0 and self.error is None and not self._stop.is_set():
            self.error = err.text() or f"th-counters exited ({self._proc.returncode})"

    @property
    def pid(self) -> int | None:
        """The sampler's pid (the monitor keeps it off every GPU's process list)."""
        return self._proc.pid if self._proc is not None else None

    def latest(self) -> dict:
        with self._lock:
            return dict(self._latest)

    def raw(self) -> dict:
        with self._lock:
            return dict(self._raw)

    def wait_first(self, timeout: float = 10.0) -> bool:
        t0 = time.time()
        while time.time() - t0 < timeout:
            if self._latest or self.error:
                return bool(self._latest)
            time.sleep(0.05)
        return False

    def close(self) -> None:
        self._stop.set()
        if self._proc is not None and self._proc.poll() is None:
            self._proc.terminate()
            try:
                self._proc.wait(5)
            except subprocess.TimeoutExpired:
                self._proc.kill()
