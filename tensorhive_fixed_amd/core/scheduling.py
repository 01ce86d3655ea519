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

A task may also ask for a COUNT (``HIP_VISIBLE_DEVICES=auto:N``): the scheduler then picks N
GPUs itself -- free long enough, allowed for the owner, not taken this round -- preferring the
owner's own reservations and keeping the gang on as few NUMA nodes as possible
(:func:`.allocation.pick`).  The reference could only run jobs whose tasks named their device.
The choices are handed to ``business_execute``, which re-checks and claims them atomically.
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
    """GPU indices of a task: the devices it holds right now (``gpu_allocations``), else its
    pinned ``HIP_VISIBLE_DEVICES`` list; ``auto:N`` tasks that hold nothing yet have none."""
    from .allocation import device_request, devices_of

    tid = getattr(task, "id", None)
    held = devices_of(tid) if tid is not None else []
    if held:
        return held
    req = device_request(task)
    return list(req.pinned) if req is not None and not req.auto else []


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
        self.placements: dict[int, dict[int, list[str]]] = {}  # job id -> task id -> uuids (auto tasks)

    @staticmethod
    def _owner_has_upcoming_reservation(uuid: str, job, window: timedelta) -> bool:
        from ..models.orm import Reservation

        return any(r.user_id == job.user_id for r in Reservation.upcoming_events_for_resource(uuid, window))

    def _usable(self, host, u, job, slots, window) -> tuple[bool, int]:
        """(free long enough, preference tier) of one GPU for ``job``."""
        slot = slots[host][u]
        own = slot is not None and self._own(u, job, window)
        if own:
            return True, 0
        if slot is None:
            return True, 1
        return slot >= self.free_window_mins, 2

    def schedule_jobs(self, jobs_to_hardware: dict, hardware_to_slots: dict, gpu_info: dict | None = None) -> list:
        """``gpu_info`` = ``{host: {uuid: {"index": i, "numa_node": n}}}`` for placing ``auto:N``
        tasks (defaults: dict order, one NUMA node).  Chosen devices land in :attr:`placements`."""
        from .allocation import Candidate, device_request, pick

        window = timedelta(minutes=self.free_window_mins)
        taken: set[tuple[str, str]] = set()
        scheduled = []
        self.placements = {}
        for job in jobs_to_hardware:
            wanted: list[tuple[str, str]] = []
            chosen: dict[int, list[str]] = {}
            ok = bool(job.tasks)
            for task in job.tasks:
                host = task.hostname
                slots = hardware_to_slots.get(host) or {}
                eligible = (jobs_to_hardware.get(job) or {}).get(host)
                req = device_request(task)
                if req is not None and req.auto:
                    info = (gpu_info or {}).get(host) or {}
                    cands = []
                    for pos, u in enumerate(slots):
                        if (host, u) in taken or (host, u) in wanted or (eligible is not None and u not in eligible):
                            continue
                        usable, tier = self._usable(host, u, job, hardware_to_slots, window)
                        if usable:
                            g = info.get(u) or {}
                            numa = g.get("numa_node")
                            cands.append(Candidate(int(g.get("index", pos)), u,
                                                   numa if isinstance(numa, int) and numa >= 0 else 0, tier))
                    got = pick(cands, req.count)
                    if got is None:
                        ok = False
                        break
                    chosen[task.id] = [c.uuid for c in got]
                    wanted += [(host, c.uuid) for c in got]
                    continue
                uuids = assigned_gpu_uuids(task, hardware_to_slots)
                if not uuids or any(u is None for u in uuids):
                    ok = False  # a task must name GPUs that exist on its host
                    break
                for u in uuids:
                    key = (host, u)
                    if key in taken or key in wanted or (eligible is not None and u not in eligible):
                        ok = False
                        break
                    if not self._usable(host, u, job, hardware_to_slots, window)[0]:
                        ok = False
                        break
                    wanted.append(key)
                if not ok:
                    break
            if ok:
                scheduled.append(job)
                taken.update(wanted)
                if chosen:
                    self.placements[job.id] = chosen
        return scheduled
