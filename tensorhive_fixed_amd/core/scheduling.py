"""Queued-job scheduler (reference ``core/scheduling.py:10-62``), gang-aware.

Inputs of :meth:`Scheduler.schedule_jobs`:
  * ``jobs_to_hardware`` -- queued jobs (in queue order) -> eligible hosts/GPUs for their owner;
  * ``hardware_to_slots`` -- ``{host: {gpu_uuid: minutes_until_next_foreign_reservation}}`` with
    ``0`` = busy now, ``None`` = free for the foreseeable future.  The per-host dicts are ordered
    by HIP device index (the telemetry emits them that way).

A job is scheduled iff EVERY GPU of EVERY task (a task may own several GPUs through
``HIP_VISIBLE_DEVICES=0,1,2,3``) is (a) not taken by an earlier job of this round and (b) free
for at least ``schedule_queued_jobs_when_free_mins`` -- the owner's own upcoming reservations
count as free.  All-or-nothing per job (gang semantics), first-fit in queue order.
"""
from __future__ import annotations

import re
from abc import ABC, abstractmethod
from datetime import timedelta

_DEVICES_RE = re.compile(r"^\s*(?:HIP_VISIBLE_DEVICES|ROCR_VISIBLE_DEVICES)=([0-9,\s]+)")


def parse_device_list(value: str | None) -> list[int]:
    """'0,1, 3' -> [0, 1, 3]; empty/None -> []."""
    if not value:
        return []
    out = []
    for tok in value.replace(" ", "").split(","):
        if tok.isdigit():
            out.append(int(tok))
    return out


def task_gpu_indices(task) -> list[int]:
    """GPU indices of a task: its HIP_VISIBLE_DEVICES env segment, else the legacy ``gpu_id``."""
    for name, value in task.envs():
        if name in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES"):
            idx = parse_device_list(value)
            if idx:
                return idx
    m = _DEVICES_RE.match(task.command or "")
    if m:
        return parse_device_list(m.group(1))
    return [] if task.gpu_id is None else [task.gpu_id]


def assigned_gpu_uuids(task, hardware_map: dict) -> list[str | None]:
    """Map a task's GPU indices to UUIDs via the (index-ordered) per-host GPU dict."""
    host_gpus = list((hardware_map.get(task.hostname) or {}).keys())
    return [host_gpus[i] if 0 <= i < len(host_gpus) else None for i in task_gpu_indices(task)]


class Scheduler(ABC):
    @abstractmethod
    def schedule_jobs(self, jobs_to_hardware: dict, hardware_to_slots: dict) -> list:
        """Return the jobs (subset of ``jobs_to_hardware``) to start now."""

    @staticmethod
    def get_assigned_gpu_uid(task, hardware_map: dict) -> str | None:
        uuids = assigned_gpu_uuids(task, hardware_map)
        return uuids[0] if uuids else None


class GreedyScheduler(Scheduler):
    def __init__(self, free_window_mins: int = 30, own_reservations=None):
        """``own_reservations(uuid, job, window) -> bool`` tells whether the job owner holds an
        upcoming reservation on the GPU (defaults to a DB lookup)."""
        self.free_window_mins = free_window_mins
        self._own = own_reservations or self._owner_has_upcoming_reservation

    @staticmethod
    def _owner_has_upcoming_reservation(uuid: str, job, window: timedelta) -> bool:
        from ..models.orm import Reservation

        return any(r.user_id == job.user_id for r in Reservation.upcoming_events_for_resource(uuid, window))

    def schedule_jobs(self, jobs_to_hardware: dict, hardware_to_slots: dict) -> list:
        window = timedelta(minutes=self.free_window_mins)
        taken: set[tuple[str, str]] = set()
        scheduled = []
        for job in jobs_to_hardware:
            wanted: list[tuple[str, str]] = []
            ok = bool(job.tasks)
            for task in job.tasks:
                uuids = assigned_gpu_uuids(task, hardware_to_slots)
                if not uuids or any(u is None for u in uuids):
                    ok = False  # a task must name GPUs that exist on its host
                    break
                eligible = (jobs_to_hardware.get(job) or {}).get(task.hostname)
                for u in uuids:
                    key = (task.hostname, u)
                    if key in taken or key in wanted or (eligible is not None and u not in eligible):
                        ok = False
                        break
                    slot = hardware_to_slots[task.hostname][u]
                    if slot is not None and self._own(u, job, window):
                        slot = None
                    if not (slot is None or slot >= self.free_window_mins):
                        ok = False
                        break
                    wanted.append(key)
                if not ok:
                    break
            if ok:
                scheduled.append(job)
                taken.update(wanted)
        return scheduled
