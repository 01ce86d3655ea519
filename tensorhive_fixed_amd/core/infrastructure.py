"""In-memory infrastructure state: immutable snapshots published atomically (RCU style).

Reference: ``core/managers/InfrastructureManager.py`` holds one mutable dict that monitor
threads edit in place while API greenlets deep-copy it with no lock (SURVEY §5 race note).
Here monitors build a complete per-host entry and :meth:`publish` swaps in a NEW top-level
snapshot object (copy-on-write of one host); readers take a reference to the current snapshot
with no lock and never see a half-written host.  Every snapshot carries a version and per-host
sample timestamps so the API can report staleness.

Shape (the wire contract of ``/nodes/*``)::

    {host: {"CPU": {"CPU_<host>": {"metrics": {...}}},
            "GPU": {uuid: {"name", "index", "metrics": {key: {"value", "unit"}},
                           "processes": [{"pid", "command", "owner", ...}] | None}} | None}}
"""
from __future__ import annotations

import copy
import logging
import threading
import time
from dataclasses import dataclass, field

log = logging.getLogger(__name__)

IGNORED_PROCESSES = ("Xorg", "/usr/lib/xorg/Xorg", "/usr/bin/X", "X", "gnome-shell", "-")


@dataclass(frozen=True)
class Snapshot:
    version: int
    data: dict
    sampled_at: dict = field(default_factory=dict)  # host -> unix time of its last sample

    def age(self, host: str, now: float | None = None) -> float | None:
        t = self.sampled_at.get(host)
        return None if t is None else (now or time.time()) - t


class InfrastructureStore:
    """``attest(host, entry)`` (the daemon's ``core/attribution.Attestor``) runs on every entry
    before it is published: consumers only ever see attested task ids."""

    def __init__(self, hosts, attest=None):
        self._lock = threading.Lock()  # serialises writers only
        self._snap = Snapshot(0, {h: {} for h in hosts}, {})
        self._listeners: list = []
        self.attest = attest

    # ------------------------------------------------------------------ writers
    def publish(self, host: str, entry: dict, sampled_at: float | None = None) -> Snapshot:
        if self.attest is not None and entry:
            try:
                self.attest(host, entry)
            except Exception:  # noqa: BLE001 -- never publish unattested claims
                log.exception("attestation of %s failed; dropping its task claims", host)
                for g in (entry.get("GPU") or {}).values():
                    for p in (g or {}).get("processes") or []:
                        if p.get("task_id") not in (None, ""):
                            p["claimed_task_id"], p["task_id"] = str(p["task_id"]), None
        with self._lock:
            old = self._snap
            data = dict(old.data)
            data[host] = entry
            ts = dict(old.sampled_at)
            ts[host] = sampled_at or time.time()
            self._snap = Snapshot(old.version + 1, data, ts)
            snap = self._snap
        for fn in list(self._listeners):
            try:
                fn(host, snap)
            except Exception:  # noqa: BLE001
                pass
        return snap

    def on_publish(self, fn) -> None:
        self._listeners.append(fn)

    # ------------------------------------------------------------------ readers
    def snapshot(self) -> Snapshot:
        return self._snap

    @property
    def infrastructure(self) -> dict:
        """Deep copy (safe to mutate, e.g. for permission filtering)."""
        return copy.deepcopy(self._snap.data)

    def hosts(self) -> list[str]:
        return list(self._snap.data)

    def node_gpu_processes(self, hostname: str, snap: Snapshot | None = None) -> dict:
        gpus = (snap or self._snap).data.get(hostname, {}).get("GPU")
        if gpus is None:
            return {}
        out = {}
        for uuid, g in gpus.items():
            procs = g.get("processes")
            out[uuid] = [p for p in procs if p.get("command") not in IGNORED_PROCESSES] if procs else []
        return out

    def all_nodes_with_gpu_processes(self) -> dict[str, dict]:
        snap = self._snap
        return {h: self.node_gpu_processes(h, snap) for h in snap.data}

    def gpu_uuids(self, hostname: str) -> list[str]:
        """UUIDs in HIP index order."""
        gpus = self._snap.data.get(hostname, {}).get("GPU") or {}
        return [u for u, _ in sorted(gpus.items(), key=lambda kv: kv[1].get("index", 0))]

    def get_gpu_uid(self, hostname: str, gpu_id: int) -> str:
        return self.gpu_uuids(hostname)[gpu_id]
