"""Telemetry backends (reference monitors ``core/monitors/{Monitor,CPUMonitor,GPUMonitor}.py``).

Every backend returns, per host, one complete infrastructure entry (see
:mod:`.infrastructure`) -- GPU metrics, processes with owners/task ids, CPU metrics -- in ONE
call.  Backends:

* :class:`AmdSmiBackend` -- the local node through ``native/lib/libthsmi.so`` (C++, amdsmi +
  /proc + KFD sysfs), optionally augmented by the gfx950 probe kernel (``mfma_busy``,
  ``hbm_contention``) from ``libthk.so``; ``hbm_bw`` (GB/s) comes from libthsmi's calibrated
  ``mem_activity_acc`` rate.
* :class:`RemoteBackend` -- other nodes: ``th-smi`` over the node transport, either one-shot or
  as a persistent ``th-smi --stream MS`` over one multiplexed SSH channel (sub-second cadence
  without a round trip per poll).
* :class:`StubBackend` -- deterministic fake MI355X nodes (CPU-only hosts, tests, demos), with
  process injection and fault injection (host down / stalled).
"""
from __future__ import annotations

import ctypes
import json
import logging
import math
import os
import subprocess
import threading
import time
import uuid as uuidlib
from pathlib import Path

log = logging.getLogger(__name__)

NATIVE_LIB = Path(__file__).resolve().parent.parent / "native" / "lib" / "libthsmi.so"


def _metric(v, unit):
    return {"value": v, "unit": unit}


def entry_from_thsmi(host: str, doc: dict, extra_gpu_metrics: dict | None = None) -> dict:
    """libthsmi JSON document -> infrastructure entry for ``host``."""
    gpus = {}
    for g in sorted(doc.get("gpus", []), key=lambda g: g.get("index", 0)):
        metrics = dict(g.get("metrics", {}))
        if extra_gpu_metrics and g.get("index") in extra_gpu_metrics:
            metrics.update(extra_gpu_metrics[g["index"]])
        procs = [{"pid": p["pid"], "command": p.get("command", ""), "owner": p.get("owner"),
                  "task_id": p.get("task_id"), "vram": p.get("vram")} for p in g.get("processes", [])]
        gpus[g["uuid"]] = {"name": g.get("name"), "index": g.get("index"), "bdf": g.get("bdf"),
                           "numa_node": g.get("numa_node"), "metrics": metrics, "processes": procs}
    cpu = doc.get("cpu")
    return {"CPU": {f"CPU_{host}": {"name": f"CPU_{host}", "index": 0, "metrics": cpu}} if cpu else None,
            "GPU": gpus}


class TelemetryBackend:
    name = "base"

    def sample(self, host: str) -> dict | None:
        raise NotImplementedError

    def topology(self, host: str) -> dict | None:
        return None

    def close(self) -> None:
        pass


class AmdSmiBackend(TelemetryBackend):
    """Local node through libthsmi (ctypes)."""

    name = "amdsmi"

    def __init__(self, probe: bool = False, probe_period: float = 1.0, counters: bool = False,
                 counters_period_ms: int = 1000):
        if not NATIVE_LIB.exists():
            from ..native.build import build_all

            build_all(strict=False)
        self.lib = ctypes.CDLL(str(NATIVE_LIB))
        self.lib.thsmi_sample_json.argtypes = [ctypes.c_char_p, ctypes.c_int]
        self.lib.thsmi_topology_json.argtypes = [ctypes.c_char_p, ctypes.c_int]
        n = self.lib.thsmi_init()
        if n < 0:
            raise RuntimeError(f"amdsmi initialisation failed ({n})")
        self.n_gpus = n
        self._buf = ctypes.create_string_buffer(1 << 20)
        self._lock = threading.Lock()
        self.probe = GpuProbe(probe_period) if probe else None
        self.counters = None
        if counters:
            from .counters import CounterStream

            self.counters = CounterStream(period_ms=counters_period_ms)

    def _call(self, fn) -> dict:
        with self._lock:
            n = fn(self._buf, len(self._buf))
            if n < 0:
                self._buf = ctypes.create_string_buffer(-n + 4096)
                n = fn(self._buf, len(self._buf))
            return json.loads(self._buf.value[:n].decode("utf-8", "replace"))

    def sample(self, host: str) -> dict | None:
        doc = self._call(self.lib.thsmi_sample_json)
        extra = {k: dict(v) for k, v in (self.probe.maybe_sample() or {}).items()} if self.probe else {}
        if self.counters is not None:
            by_kfd = self.counters.latest()
            for g in doc.get("gpus", []):
                m = by_kfd.get(g.get("kfd_id"))
                if m:
                    extra.setdefault(g["index"], {}).update(m)
        return entry_from_thsmi(host, doc, extra or None)

    def topology(self, host: str) -> dict | None:
        return self._call(self.lib.thsmi_topology_json)

    def close(self) -> None:
        if self.counters is not None:
            self.counters.close()
        self.lib.thsmi_shutdown()


class GpuProbe:
    """Runs the gfx950 th-probe kernel (libthk.so) at a low duty cycle and derives
    ``mfma_busy`` / ``hbm_contention`` per device from the slowdown against the best (idle) sample."""

    def __init__(self, period: float = 1.0, device: int = 0, n_wg: int = 8, mfma_iters: int = 512):
        from ..ops import _lib

        self.lib = _lib.load()
        self.lib.th_probe_init.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
        self.lib.th_probe_sample.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
        self.lib.th_probe_last_latency_us.restype = ctypes.c_double
        rc = self.lib.th_probe_init(device, n_wg, 1024)
        if rc != 0:
            raise RuntimeError(f"th_probe_init failed ({rc})")
        self.period, self.device, self.n_wg, self.iters = period, device, n_wg, mfma_iters
        self.best_mfma = math.inf
        self.best_lat = math.inf
        self.best_bw = 0.0
        self._last = 0.0
        self._cached: dict | None = None

    def sample_raw(self) -> list[dict]:
        out = (ctypes.c_double * (5 * self.n_wg))()
        n = self.lib.th_probe_sample(self.n_wg, self.iters, out)
        if n <= 0:
            raise RuntimeError(f"th_probe_sample failed ({n})")
        lat = float(self.lib.th_probe_last_latency_us())
        return [{"xcc": int(out[5 * i]), "mfma_us": out[5 * i + 1], "hbm_us": out[5 * i + 2],
                 "hbm_GBps": out[5 * i + 3], "latency_us": lat} for i in range(n)]

    def maybe_sample(self) -> dict | None:
        now = time.time()
        if now - self._last < self.period and self._cached is not None:
            return self._cached
        self._last = now
        rows = self.sample_raw()
        mfma = sum(r["mfma_us"] for r in rows) / len(rows)
        bw = sum(r["hbm_GBps"] for r in rows)
        lat = rows[0]["latency_us"]
        self.best_mfma = min(self.best_mfma, mfma)
        self.best_lat = min(self.best_lat, lat) if lat > 0 else self.best_lat
        self.best_bw = max(self.best_bw, bw)
        # Two ways a tenant shows up: it shares SIMDs with the probe (the MFMA chain slows down), or it
        # holds every CU's register file (the probe waits for a CU; the in-kernel time is unchanged).
        # mfma_busy is the larger of the two slowdowns.
        busy_chain = max(0.0, 1.0 - self.best_mfma / mfma) if mfma > 0 else 0.0
        busy_wait = max(0.0, 1.0 - self.best_lat / lat) if lat > 0 and math.isfinite(self.best_lat) else 0.0
        busy = max(busy_chain, busy_wait) * 100 if mfma > 0 else None
        share = max(0.0, 1.0 - bw / self.best_bw) * 100 if self.best_bw > 0 else None
        self._cached = {self.device: {"mfma_busy": _metric(busy, "%"), "hbm_contention": _metric(share, "%"),
                                      "probe_xcds": _metric(len({r["xcc"] for r in rows}), "")}}
        return self._cached


class RemoteBackend(TelemetryBackend):
    """th-smi on other nodes via their transport (one-shot or persistent stream)."""

    name = "remote"

    def __init__(self, transports, th_smi: str = "th-smi", stream_ms: int | None = None):
        self.transports = transports
        self.th_smi = th_smi
        self.stream_ms = stream_ms
        self._latest: dict[str, tuple[float, dict]] = {}
        self._procs: dict[str, subprocess.Popen] = {}
        self._lock = threading.Lock()

    def _start_stream(self, host: str) -> None:
        t = self.transports.get(host)
        argv = t.base_argv() + [f"{self.th_smi} --stream {int(self.stream_ms)}"] if hasattr(t, "base_argv") else \
            ["bash", "-c", f"{self.th_smi} --stream {int(self.stream_ms)}"]
        p = subprocess.Popen(argv, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True, bufsize=1)
        self._procs[host] = p

        def reader():
            for line in p.stdout:
                try:
                    doc = json.loads(line)
                except json.JSONDecodeError:
                    continue
                with self._lock:
                    self._latest[host] = (time.time(), doc)

        threading.Thread(target=reader, name=f"th-smi-stream-{host}", daemon=True).start()

    def sample(self, host: str) -> dict | None:
        if self.stream_ms:
            p = self._procs.get(host)
            if p is None or p.poll() is not None:
                self._start_stream(host)
            with self._lock:
                got = self._latest.get(host)
            return entry_from_thsmi(host, got[1]) if got else None
        r = self.transports.run(host, f"{self.th_smi} --json", timeout=15)
        if not r.ok:
            return None
        try:
            return entry_from_thsmi(host, json.loads(r.stdout.strip().splitlines()[-1]))
        except (json.JSONDecodeError, IndexError):
            return None

    def close(self) -> None:
        for p in self._procs.values():
            p.terminate()


class StubBackend(TelemetryBackend):
    """Fake MI355X nodes (8 GPUs each by default) with injectable processes and faults."""

    name = "stub"

    def __init__(self, gpus_per_host: int = 8, seed: int = 0):
        self.gpus_per_host = gpus_per_host
        self.seed = seed
        self.processes: dict[tuple[str, int], list[dict]] = {}
        self.down: set[str] = set()
        self.util_override: dict[tuple[str, int], float] = {}
        self._t0 = time.time()
        self._lock = threading.Lock()

    @staticmethod
    def gpu_uuid(host: str, index: int) -> str:
        return "GPU-" + str(uuidlib.uuid5(uuidlib.NAMESPACE_DNS, f"{host}/gpu{index}"))

    def add_process(self, host: str, gpu_index: int, pid: int, owner: str, command: str = "python train.py",
                    task_id: str | None = None) -> None:
        with self._lock:
            self.processes.setdefault((host, gpu_index), []).append(
                {"pid": pid, "command": command, "owner": owner, "task_id": task_id, "vram": 1 << 30})

    def clear_processes(self, host: str | None = None) -> None:
        with self._lock:
            for k in list(self.processes):
                if host is None or k[0] == host:
                    del self.processes[k]

    def sample(self, host: str) -> dict | None:
        if host in self.down:
            return None
        t = time.time() - self._t0
        gpus = {}
        with self._lock:
            for i in range(self.gpus_per_host):
                procs = [dict(p) for p in self.processes.get((host, i), [])]
                busy = bool(procs)
                util = self.util_override.get((host, i), (90.0 if busy else 0.0) + 5 * math.sin(t + i) * busy)
                used = (sum(p["vram"] for p in procs) >> 20) + 282
                gpus[self.gpu_uuid(host, i)] = {
                    "name": "AMD Instinct MI355X", "index": i, "bdf": f"0000:{0x05 + 0x10 * i:02x}:00.0",
                    "numa_node": 0 if i < 4 else 1,
                    "metrics": {
                        "fan_speed": _metric(None, "%"), "mem_free": _metric(294896 - used, "MiB"),
                        "mem_used": _metric(used, "MiB"), "mem_total": _metric(294896, "MiB"),
                        "utilization": _metric(round(util, 1), "%"),
                        "mem_util": _metric(round(util * 0.6, 1), "%"),
                        "temp": _metric(38 + util * 0.3, "C"), "power": _metric(180 + util * 8, "W"),
                        "hotspot_temp": _metric(45 + util * 0.4, "C"), "mem_temp": _metric(40 + util * 0.2, "C"),
                        "gfx_clock": _metric(2400 if busy else 150, "MHz"), "mem_clock": _metric(2000, "MHz"),
                        "xgmi_read": _metric(0.0, "GB/s"), "xgmi_write": _metric(0.0, "GB/s"),
                        "energy": _metric(180 + util * 8, "W"),  # accumulator-derived power, as libthsmi
                        "hbm_bw": _metric(round(util * 0.6 * 102.0, 1), "GB/s"),  # umc % x calibrated GB/s
                    },
                    "processes": procs,
                }
        cpu = {"utilization": _metric(3.0, "%"), "mem_total": _metric(1548000, "MiB"),
               "mem_free": _metric(1400000, "MiB"), "mem_used": _metric(148000, "MiB")}
        return {"CPU": {f"CPU_{host}": {"name": f"CPU_{host}", "index": 0, "metrics": cpu}}, "GPU": gpus}

    def topology(self, host: str) -> dict | None:
        n = self.gpus_per_host
        return {"gpus": [{"index": i, "uuid": self.gpu_uuid(host, i), "bdf": f"0000:{0x05 + 0x10 * i:02x}:00.0",
                          "numa_node": 0 if i < 4 else 1,
                          "links": [{"peer": j, "type": "self" if i == j else "xgmi", "hops": 0 if i == j else 1}
                                    for j in range(n)]} for i in range(n)]}


def make_backend(kind: str, host: str, transports=None, stub_gpus: int = 8, probe: bool = False,
                 probe_period: float = 1.0, stream_ms: int | None = None, counters: bool = False,
                 counters_period_ms: int = 1000) -> TelemetryBackend:
    """Pick a backend for ``host``: ``auto`` = amdsmi for the local node when /dev/kfd exists,
    remote th-smi for ssh nodes, stub otherwise."""
    spec_local = transports is None or getattr(transports.transports.get(host), "__class__", None).__name__ == "LocalTransport"
    if kind == "stub":
        return StubBackend(stub_gpus)
    if kind == "amdsmi" or (kind == "auto" and spec_local and os.path.exists("/dev/kfd")):
        return AmdSmiBackend(probe=probe, probe_period=probe_period, counters=counters,
                             counters_period_ms=counters_period_ms)
    if kind == "remote" or (kind == "auto" and not spec_local):
        return RemoteBackend(transports, stream_ms=stream_ms)
    return StubBackend(stub_gpus)
