"""Gang GPU allocation: which devices a task gets, claimed atomically.

The reference never chose GPUs.  A task named one device through ``CUDA_VISIBLE_DEVICES=<n>``,
the scheduler mapped that index to a UUID by list order (``tensorhive/core/scheduling.py:21-26``)
and deduplicated devices within one scheduling round only
(``tensorhive/core/services/JobSchedulingService.py:140-168``).  Nothing serialised a manual
``GET /jobs/{id}/execute`` against a scheduler tick, so two launches could land on one GPU.

Here:

* A task asks for devices through its ``HIP_VISIBLE_DEVICES`` env segment: a pinned list
  (``0,1``) or a count (``auto:4``, or ``auto`` = the ``--nproc_per_node=`` value).  The launch
  renders the chosen list into the command and sets ``--nproc_per_node=`` to match.
* :func:`plan_job` picks devices for ``auto`` tasks from the telemetry snapshot.  Eligible: no
  process on the device, not held by another task, allowed by the owner's restrictions, not
  inside someone else's current reservation.  Preference tiers: the owner's own current
  reservation, then free devices, then devices with a foreign reservation coming up.  Inside a
  tier the picker keeps a gang on as few NUMA nodes as possible (best fit).  An MI355X node's
  eight GPUs are all one xGMI hop apart, so the socket is the only topology level that matters
  for rank placement (host staging buffers, CPU affinity).
* :func:`claim` inserts one ``gpu_allocations`` row per device.  A UNIQUE (hostname, gpu_index)
  constraint makes a double allocation impossible at the database level.  The whole
  check-and-claim runs under :data:`ALLOC_LOCK`, which manual execute and the scheduler tick
  share.  A job id in :data:`launching` marks a launch in flight, so a double execute is
  rejected with 409 before any process starts.
* Rows are released when a task is seen not running (:func:`release_task`, called by task
  synchronisation), when its spawn fails, or by :func:`reap` for rows whose task is gone.
"""
from __future__ import annotations

import logging
import re
import threading
from dataclasses import dataclass
from datetime import timedelta

from ..utils import dates

log = logging.getLogger(__name__)

DEVICE_ENVS = ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES")
NPROC_PARAMS = ("--nproc_per_node=", "--nproc-per-node=", "--nproc_per_node", "--nproc-per-node")
_AUTO = re.compile(r"^\s*auto(?::(\d+))?\s*$")
_PREFIX = re.compile(r"^\s*(?:HIP_VISIBLE_DEVICES|ROCR_VISIBLE_DEVICES)=(\S+)")

ALLOC_LOCK = threading.RLock()
launching: set[int] = set()  # job ids whose launch holds claims but has not finished spawning
launched_at: dict[int, float] = {}  # job id -> time.monotonic() when its last launch finished


class AllocationError(Exception):
    def __init__(self, reason: str, status: int = 409):
        super().__init__(reason)
        self.reason = reason
        self.status = status


@dataclass(frozen=True)
class DeviceRequest:
    pinned: tuple[int, ...] | None  # explicit HIP indices, or None for "auto"
    count: int

    @property
    def auto(self) -> bool:
        return self.pinned is None


def parse_devices(value: str | None) -> list[int]:
    out = []
    for tok in (value or "").replace(" ", "").split(","):
        if tok.isdigit():
            out.append(int(tok))
    return out


def _nproc(task) -> int | None:
    for name, value in task.params():
        if name in NPROC_PARAMS and str(value).strip().isdigit():
            return int(value)
    return None


def device_request(task) -> DeviceRequest | None:
    """What a task asks for; ``None`` = no GPU (CPU-only task)."""
    for name, value in task.envs():
        if name in DEVICE_ENVS:
            m = _AUTO.match(value or "")
            if m:
                n = int(m.group(1)) if m.group(1) else (_nproc(task) or 1)
                if n < 1:
                    raise AllocationError("a GPU request must ask for at least one device", 422)
                return DeviceRequest(None, n)
            idx = parse_devices(value)
            if idx:
                return DeviceRequest(tuple(idx), len(idx))
    m = _PREFIX.match(task.command or "")
    if m:
        idx = parse_devices(m.group(1))
        if idx:
            return DeviceRequest(tuple(idx), len(idx))
    if task.gpu_id is not None:
        return DeviceRequest((task.gpu_id,), 1)
    return None


def render_command(task, devices: list[int] | None) -> str:
    """The task's full command with the device list substituted (``auto`` requests) and
    ``--nproc_per_node=`` matched to it.  Pinned tasks render unchanged."""
    req = device_request(task)
    if devices is None or req is None or not req.auto:
        return task.full_command
    dev = ",".join(str(i) for i in devices)
    envs = [(n, dev if n in DEVICE_ENVS else v) for n, v in task.envs()]
    params = [(n, str(len(devices)) if n in NPROC_PARAMS else v) for n, v in task.params()]
    return task.render(envs, params)


# ---------------------------------------------------------------------------------- picking
@dataclass(frozen=True)
class Candidate:
    index: int
    uuid: str | None
    numa: int
    tier: int  # 0 = owner's current reservation, 1 = free, 2 = foreign reservation upcoming


def pick(cands: list[Candidate], n: int) -> list[Candidate] | None:
    """Choose ``n`` devices: whole better tiers first, then NUMA best fit inside the last tier."""
    if n <= 0:
        return []
    if len(cands) < n:
        return None
    chosen: list[Candidate] = []
    for tier in sorted({c.tier for c in cands}):
        group = sorted((c for c in cands if c.tier == tier), key=lambda c: c.index)
        need = n - len(chosen)
        if len(group) <= need:
            chosen += group
        else:
            chosen += _numa_fit(group, need, {c.numa for c in chosen})
        if len(chosen) == n:
            break
    return sorted(chosen, key=lambda c: (c.numa, c.index))


def _numa_fit(group: list[Candidate], need: int, prefer: set[int]) -> list[Candidate]:
    """Take ``need`` devices from ``group`` spanning as few NUMA nodes as possible: nodes the
    gang already uses first, else the smallest node that holds the rest (best fit keeps whole
    sockets free for larger gangs), else the largest node, repeated until satisfied."""
    by_numa: dict[int, list[Candidate]] = {}
    for c in group:
        by_numa.setdefault(c.numa, []).append(c)
    out: list[Candidate] = []
    while len(out) < need:
        rem = need - len(out)
        nodes = [k for k in sorted(by_numa) if by_numa[k]]
        used = [k for k in nodes if k in prefer or any(c.numa == k for c in out)]
        fits = [k for k in nodes if len(by_numa[k]) >= rem]
        if used:
            k = max(used, key=lambda k: (len(by_numa[k]), -k))
        elif fits:
            k = min(fits, key=lambda k: (len(by_numa[k]), k))
        else:
            k = max(nodes, key=lambda k: (len(by_numa[k]), -k))
        out += by_numa[k][:rem]
        by_numa[k] = by_numa[k][rem:]
    return out


def candidates(task, job, snapshot: dict, held: set[tuple[str, int]], taken: set[tuple[str, int]],
               window: timedelta) -> list[Candidate]:
    """Free devices on the task's host for the job's owner, with preference tiers."""
    from ..models.orm import Reservation

    host = task.hostname
    gpus = ((snapshot.get(host) or {}).get("GPU")) or {}
    if job.user is not None:
        allowed = job.user.allowed_gpu_uuids()
        allowed_uuids = set(gpus) if allowed is None else allowed
    else:
        allowed_uuids = set()
    out = []
    for uuid, g in gpus.items():
        idx = int(g.get("index", -1))
        if idx < 0 or uuid not in allowed_uuids or (host, idx) in held or (host, idx) in taken:
            continue
        if g.get("processes"):
            continue
        events = Reservation.upcoming_events_for_resource(uuid, window)
        now = dates.utcnow()
        current = [r for r in events if r.start <= now <= r.end]
        if any(r.user_id != job.user_id for r in current):
            continue
        if any(r.user_id == job.user_id for r in current):
            tier = 0
        elif any(r.user_id != job.user_id for r in events):
            tier = 2
        else:
            tier = 1
        numa = g.get("numa_node")
        out.append(Candidate(idx, uuid, int(numa) if isinstance(numa, int) and numa >= 0 else 0, tier))
    return out


# ---------------------------------------------------------------------------------- planning
def plan_job(job, snapshot: dict, placements: dict | None = None, window: timedelta = timedelta(minutes=30),
             held: set[tuple[str, int]] | None = None) -> dict[int, list[tuple[int, str | None]]]:
    """task id -> [(HIP index, uuid)] for every task of ``job``; raises :class:`AllocationError`.

    ``placements`` (task id -> [uuid]) are the scheduler's choices for ``auto`` tasks; they are
    re-checked here, under the lock, against claims made since the scheduler looked."""
    from ..models.orm import GpuAllocation

    held = GpuAllocation.held() if held is None else held
    taken: set[tuple[str, int]] = set()
    plan: dict[int, list[tuple[int, str | None]]] = {}
    for task in job.tasks:
        req = device_request(task)
        if req is None:
            plan[task.id] = []
            continue
        host = task.hostname
        gpus = ((snapshot.get(host) or {}).get("GPU")) or {}
        uuid_of = {int(g.get("index", -1)): u for u, g in gpus.items()}
        if req.pinned is not None:
            chosen = [(i, uuid_of.get(i)) for i in req.pinned]
        elif placements and task.id in placements:
            chosen = []
            for u in placements[task.id]:
                g = gpus.get(u)
                if g is None:
                    raise AllocationError(f"GPU {u} is no longer reported by {host}")
                chosen.append((int(g["index"]), u))
        else:
            if not gpus:
                raise AllocationError(f"no telemetry for {host}: cannot place an auto:{req.count} request")
            got = pick(candidates(task, job, snapshot, held, taken, window), req.count)
            if got is None:
                free = len(candidates(task, job, snapshot, held, taken, window))
                raise AllocationError(f"{req.count} GPUs requested on {host}, {free} free")
            chosen = [(c.index, c.uuid) for c in got]
        for i, _u in chosen:
            if (host, i) in held:
                raise AllocationError(f"GPU {host}:{i} is held by another task")
            if (host, i) in taken:
                raise AllocationError(f"GPU {host}:{i} is requested twice by this job")
            taken.add((host, i))
        plan[task.id] = chosen
    return plan


def claim(job, plan: dict[int, list[tuple[int, str | None]]]) -> None:
    """Insert the plan's rows in one transaction (UNIQUE (hostname, gpu_index) backs the lock)."""
    from sqlalchemy.exc import IntegrityError

    from ..database import db_session
    from ..models.orm import GpuAllocation, Task

    rows = []
    for task_id, devs in plan.items():
        host = Task.get(task_id).hostname
        rows += [GpuAllocation(task_id=task_id, job_id=job.id, hostname=host, gpu_index=i, gpu_uuid=u)
                 for i, u in devs]
    if not rows:
        return
    try:
        db_session.add_all(rows)
        db_session.commit()
    except IntegrityError:
        db_session.rollback()
        raise AllocationError("a requested GPU was claimed concurrently")


def release_task(task_id: int) -> int:
    from ..database import db_session
    from ..models.orm import GpuAllocation

    n = GpuAllocation.query.filter(GpuAllocation.task_id == task_id).delete()
    # commit even when nothing matched: the DELETE opened a write transaction, and leaving it
    # open would keep SQLite's write lock on this thread's connection after ALLOC_LOCK is gone
    db_session.commit()
    return n


def devices_of(task_id: int) -> list[int]:
    from ..models.orm import GpuAllocation

    return [a.gpu_index for a in GpuAllocation.for_task(task_id)]


def reap(grace: timedelta = timedelta(minutes=2)) -> int:
    """Drop rows whose task is not running and whose launch finished over ``grace`` ago."""
    from ..database import db_session
    from ..models.orm import GpuAllocation, Task, TaskStatus

    cutoff = dates.utcnow() - grace
    n = 0
    with ALLOC_LOCK:
        for a in GpuAllocation.query.filter(GpuAllocation.created_at < cutoff).all():
            if a.job_id in launching:
                continue
            t = Task.query.filter(Task.id == a.task_id).first()
            if t is None or t.status is not TaskStatus.running:
                db_session.delete(a)
                n += 1
        db_session.commit()
    return n


def held_uuids(snapshot: dict) -> set[tuple[str, str]]:
    """(host, uuid) of every held device that the snapshot knows."""
    from ..models.orm import GpuAllocation

    out = set()
    for a in GpuAllocation.query.all():
        u = a.gpu_uuid
        if u is None:
            for uu, g in (((snapshot.get(a.hostname) or {}).get("GPU")) or {}).items():
                if int(g.get("index", -1)) == a.gpu_index:
                    u = uu
        if u:
            out.add((a.hostname, u))
    return out
