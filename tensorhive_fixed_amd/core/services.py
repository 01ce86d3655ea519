"""Background services (reference ``core/services/*.py``, ``core/utils/StoppableThread.py``).

All services are threads with an ``Event``-based stop (prompt shutdown) and per-loop timing
statistics (p50/p99 exposed at ``/api/metrics/internal``).

* :class:`MonitoringService` -- samples every host's telemetry backend (in parallel) at
  ``update_interval`` (sub-second for the native sampler) and publishes immutable snapshots.
* :class:`ProtectionService` -- foreign processes on reserved GPUs (level 1) or on any
  GPU without the owner's reservation (level 2, strict) -> violation handlers.  Processes of a
  TensorHive task of the reservation owner are never violations -- a task id counts only after
  ``core/attribution.py`` attested it (the process is in that task's th-run session and runs as
  its uid; the infrastructure store attests every sample it publishes).
* :class:`UsageLoggingService` -- per-reservation JSON time series; on expiry stores rounded
  averages on the reservation (+ extra MI355X metric averages in the JSON summary).
* :class:`JobSchedulingService` -- scheduled start/stop, queued gang scheduling and eviction of
  queued jobs, woken immediately by events (enqueue, reservation change, job stop) in
  addition to its period, so a queued job starts within milliseconds when GPUs are free.
"""
from __future__ import annotations

import collections
import concurrent.futures as cf
import json
import logging
import threading
import time
from datetime import timedelta
from pathlib import Path

from ..database import db_session
from ..utils import dates

log = logging.getLogger(__name__)


class LoopStats:
    def __init__(self, cap: int = 2048):
        self.d = collections.deque(maxlen=cap)
        self.lock = threading.Lock()

    def add(self, s: float) -> None:
        with self.lock:
            self.d.append(s)

    def summary(self) -> dict:
        with self.lock:
            xs = sorted(self.d)
        if not xs:
            return {"n": 0}
        return {"n": len(xs), "p50_ms": 1000 * xs[len(xs) // 2], "p99_ms": 1000 * xs[min(len(xs) - 1, int(.99 * len(xs)))],
                "max_ms": 1000 * xs[-1]}


class Service(threading.Thread):
    interval: float = 1.0

    def __init__(self, name: str, interval: float):
        super().__init__(name=name, daemon=True)
        self.interval = interval
        self._stop_ev = threading.Event()
        self._wake_ev = threading.Event()
        self.stats = LoopStats()
        self.ticks = 0

    def inject(self, daemon) -> None:
        self.d = daemon

    def stop(self) -> None:
        self._stop_ev.set()
        self._wake_ev.set()

    @property
    def stopped(self) -> bool:
        return self._stop_ev.is_set()

    def wake(self) -> None:
        self._wake_ev.set()

    def do_run(self) -> None:
        raise NotImplementedError

    def next_wait(self, dt: float) -> float:
        """Seconds to sleep after a tick that took ``dt`` (a wake-up cuts it short)."""
        return max(0.0, self.interval - dt)

    def run(self) -> None:
        while not self._stop_ev.is_set():
            t0 = time.perf_counter()
            try:
                self.do_run()
            except Exception:  # noqa: BLE001 -- a failing tick must never kill the service
                log.exception("%s tick failed", self.name)
            finally:
                db_session.remove()
            dt = time.perf_counter() - t0
            self.stats.add(dt)
            self.ticks += 1
            self._wake_ev.wait(self.next_wait(dt))
            self._wake_ev.clear()


# --------------------------------------------------------------------------- monitoring
class MonitoringService(Service):
    def __init__(self, interval: float, backends: dict):
        super().__init__("MonitoringService", interval)
        self.backends = backends  # host -> TelemetryBackend
        self._pool = cf.ThreadPoolExecutor(max_workers=max(1, min(32, len(backends))),
                                           thread_name_prefix="th-sample")
        self._busy: dict[str, set] = {}  # host -> UUIDs that held a process in the last sample

    def sample_host(self, host: str) -> None:
        try:
            entry = self.backends[host].sample(host)
        except Exception as e:  # noqa: BLE001 -- host isolation (stop_on_errors=False)
            log.debug("sampling %s failed: %s", host, e)
            entry = None
        if entry is None:
            entry = {"CPU": None, "GPU": None}
        busy = {u for u, g in ((entry.get("GPU") or {}).items()) if g and g.get("processes")}
        prev = self._busy.get(host)
        self._busy[host] = busy
        self.d.infrastructure.publish(host, entry)
        # A device whose last process exited is free for the queue NOW: wake the job scheduler
        # instead of leaving the next queued job to its periodic tick (30 s by default, the
        # reference's only trigger -- core/services/JobSchedulingService.py:44).
        if prev is not None and entry.get("GPU") is not None and prev - busy:
            self.d.wake("gpu_freed")

    def do_run(self) -> None:
        list(self._pool.map(self.sample_host, list(self.backends)))


# --------------------------------------------------------------------------- protection
class ProtectionService(Service):
    def __init__(self, interval: float, handlers: list, level: int = 1):
        super().__init__("ProtectionService", interval)
        self.handlers = handlers
        self.strict = level >= 2
        self.enabled = level > 0
        self.last_violations: dict = {}

    @staticmethod
    def _task_owner(task_id) -> str | None:
        from ..models.orm import Task

        try:
            t = Task.query.filter(Task.id == int(task_id)).first()
            return t.job.user.username if t is not None and t.job is not None and t.job.user else None
        except (ValueError, TypeError):
            return None

    def find_violations(self) -> dict:
        from ..models.orm import Reservation

        snap = self.d.infrastructure.snapshot()
        violations: dict = {}
        for host, entry in snap.data.items():
            gpus = (entry or {}).get("GPU") or {}
            procs_by_gpu = self.d.infrastructure.node_gpu_processes(host, snap)
            for uuid, procs in procs_by_gpu.items():
                if not procs:
                    continue
                current = Reservation.current_events(uuid)
                res = current[0] if current else None
                if res is None and not self.strict:
                    continue
                owner = res.user.username if res is not None and res.user is not None else None
                for p in procs:
                    if owner is not None and p.get("owner") == owner:
                        continue
                    if owner is not None and p.get("task_id") and self._task_owner(p["task_id"]) == owner:
                        continue
                    g = gpus.get(uuid, {})
                    rec = {"OWNER_USERNAME": owner, "OWNER_EMAIL": res.user.email if res is not None else None,
                           "END": dates.utc2local(res.end) if res is not None else None, "GPU_UUID": uuid,
                           "GPU_NAME": g.get("name", "<not available>"), "GPU_ID": g.get("index", "<not available>"),
                           "HOSTNAME": host}
                    v = violations.setdefault(p.get("owner"), {"INTRUDER_USERNAME": p.get("owner"),
                                                               "RESERVATIONS": [], "VIOLATION_PIDS": {}})
                    v["RESERVATIONS"].append(rec)
                    v["VIOLATION_PIDS"].setdefault(host, set()).add(p["pid"])
        for v in violations.values():
            rs = v["RESERVATIONS"]
            v["HOSTNAMES"] = sorted({r["HOSTNAME"] for r in rs})
            v["GPUS"] = ",\n".join(f"{r['HOSTNAME']} - GPU{r['GPU_ID']}: {r['GPU_NAME']}" for r in rs)
            v["OWNERS"] = ", ".join(f"{r['OWNER_USERNAME']} ({r['OWNER_EMAIL']})" for r in rs)
        return violations

    def do_run(self) -> None:
        if not self.enabled:
            return
        violations = self.find_violations()
        self.last_violations = violations
        for data in violations.values():
            for h in self.handlers:
                try:
                    h.trigger_action(data)
                except Exception:  # noqa: BLE001
                    log.exception("violation handler %s failed", type(h).__name__)


# ------------------------------------------------------------------------- usage logging
class UsageLoggingService(Service):
    """Per-reservation JSON logs, format of the reference (``UsageLoggingService.py:38-121``) plus
    extra MI355X metrics.  Cleanup action: 0 remove, 1 hide, 2 rename ``old_``."""

    EXTRA = ("power", "hbm_bw", "mfma_busy", "mfma_contention", "xgmi_read", "xgmi_write")

    def __init__(self, interval: float, log_dir: str, cleanup_action: int = 1):
        super().__init__("UsageLoggingService", interval)
        self.log_dir = Path(log_dir).expanduser()
        self.log_dir.mkdir(parents=True, exist_ok=True)
        self.cleanup_action = cleanup_action

    @staticmethod
    def avg(values) -> int:
        vals = [v for v in values if v is not None]
        return int(round(sum(vals) / len(vals))) if vals else -1

    def _gpu(self, uuid: str, snap) -> dict | None:
        for entry in snap.data.values():
            g = ((entry or {}).get("GPU") or {}).get(uuid)
            if g:
                return g
        return None

    def log_current_usage(self) -> None:
        from ..models.orm import Reservation

        snap = self.d.infrastructure.snapshot()
        for res in Reservation.current_events():
            g = self._gpu(res.resource_id, snap)
            if g is None:
                continue
            path = self.log_dir / f"{res.id}.json"
            doc = json.loads(path.read_text()) if path.exists() else {
                "name": "", "index": 0, "messages": [], "timestamps": [],
                "metrics": {"utilization": {"values": [], "unit": "%"}, "mem_util": {"values": [], "unit": "%"}}}
            doc["name"], doc["index"] = g.get("name"), g.get("index")
            m = g.get("metrics") or {}
            gu, mu = (m.get("utilization") or {}).get("value"), (m.get("mem_util") or {}).get("value")
            if gu is None or mu is None:
                msg = "`mem_util` or `utilization` is not supported by this GPU"
                if msg not in doc["messages"]:
                    doc["messages"].append(msg)
            else:
                doc["timestamps"].append(str(dates.utcnow()))
                doc["metrics"]["utilization"]["values"].append(gu)
                doc["metrics"]["mem_util"]["values"].append(mu)
                for k in self.EXTRA:
                    if k in m and (m[k] or {}).get("value") is not None:
                        doc["metrics"].setdefault(k, {"values": [], "unit": m[k].get("unit")})["values"].append(m[k]["value"])
            tmp = path.with_suffix(".json.tmp")
            tmp.write_text(json.dumps(doc))
            tmp.replace(path)

    def _cleanup(self, path: Path) -> None:
        if self.cleanup_action == 0:
            path.unlink()
        elif self.cleanup_action == 1:
            path.rename(path.parent / ("." + path.name))
        else:
            path.rename(path.parent / ("old_" + path.name))

    def handle_expired_logs(self) -> None:
        from sqlalchemy.exc import NoResultFound

        from ..models.orm import Reservation

        now = dates.utcnow()
        for item in self.log_dir.glob("[0-9]*.json"):
            try:
                res = Reservation.get(int(item.stem))
            except NoResultFound:
                self._cleanup(item)
                continue
            except ValueError:
                continue
            if res.end < now:
                doc = json.loads(item.read_text())
                res.gpu_util_avg = self.avg(doc["metrics"]["utilization"]["values"])
                res.mem_util_avg = self.avg(doc["metrics"]["mem_util"]["values"])
                res.save()
                summary = {k: self.avg(v.get("values", [])) for k, v in doc["metrics"].items()}
                (self.log_dir / f"{item.stem}.summary.json").write_text(json.dumps(summary))
                self._cleanup(item)

    def do_run(self) -> None:
        self.log_current_usage()
        self.handle_expired_logs()


# ------------------------------------------------------------------------ job scheduling
class JobSchedulingService(Service):
    def __init__(self, interval: float, stop_attempts_after_mins: float, free_window_mins: int, scheduler=None):
        super().__init__("JobSchedulingService", interval)
        from .scheduling import GreedyScheduler

        self.stop_attempts_after = timedelta(minutes=stop_attempts_after_mins)
        self.window = timedelta(minutes=free_window_mins)
        self.free_window_mins = free_window_mins
        self.scheduler = scheduler or GreedyScheduler(free_window_mins)
        self.stubborn: set[int] = set()
        self.launch_log: list[tuple[int, float]] = []  # (job id, unix time of execute)
        self._fast_until = 0.0  # monotonic deadline of the post-"device freed" re-checks
        self._queue_left = 0  # queued jobs the last tick could not start
        self._idle_claims = False  # the last tick saw a claimed device without a process

    # A device that lost its last process (MonitoringService) is usually free for the queue, but
    # the task's exit can reach th-run's session state a moment after the process left the
    # device, and then this tick still sees the device claimed.  So after such a wake-up the
    # service re-checks every FAST_RECHECK_S for up to FAST_WINDOW_S while queued jobs remain or
    # a claimed device shows no process (its task not yet seen as ended), instead of sleeping for
    # its full interval (30 s by default).
    FAST_RECHECK_S = 0.5
    FAST_WINDOW_S = 10.0

    def device_freed(self) -> None:
        self._fast_until = time.monotonic() + self.FAST_WINDOW_S
        self.wake()

    def next_wait(self, dt: float) -> float:
        w = super().next_wait(dt)
        if (self._queue_left or self._idle_claims) and time.monotonic() < self._fast_until:
            return min(w, self.FAST_RECHECK_S)
        return w

    # ---- helpers
    def occupancy(self) -> dict:
        """{host: {uuid: [processes]}} ordered by HIP index, from the latest snapshot."""
        infra = self.d.infrastructure
        out = {}
        for host in infra.hosts():
            procs = infra.node_gpu_processes(host)
            out[host] = {u: procs.get(u, []) for u in infra.gpu_uuids(host)}
        return out

    def claimed(self, occ: dict) -> set[tuple[str, str]]:
        """GPUs held by launching/running tasks (``gpu_allocations``; monitoring may not show
        the processes yet), plus pinned running tasks from before allocations existed."""
        from ..models.orm import Task, TaskStatus
        from .allocation import held_uuids
        from .scheduling import assigned_gpu_uuids

        out = held_uuids(self.d.infrastructure.snapshot().data)
        for t in Task.query.filter(Task._status == TaskStatus.running).all():
            for u in assigned_gpu_uuids(t, occ):
                if u:
                    out.add((t.hostname, u))
        return out

    def gpu_slots(self, occ: dict) -> dict:
        from ..models.orm import Reservation

        claimed = self.claimed(occ)
        now = dates.utcnow()
        out: dict = {}
        for host, gpus in occ.items():
            out[host] = {}
            for uuid, procs in gpus.items():
                if procs or (host, uuid) in claimed:
                    out[host][uuid] = 0
                    continue
                near = Reservation.upcoming_events_for_resource(uuid, self.window)
                if near:
                    start = near[0].start
                    out[host][uuid] = (start - now).total_seconds() / 60 if start > now else 0
                else:
                    out[host][uuid] = None
        return out

    def eligible(self, jobs) -> dict:
        from ..controllers.nodes import filtered_view

        base = self.d.infrastructure.snapshot().data
        out = {}
        for job in jobs:
            infra = filtered_view(base, job.user.allowed_gpu_uuids()) if job.user else {}
            out[job] = {h: list(((e or {}).get("GPU") or {}).keys()) for h, e in infra.items()}
        return out

    def _execute(self, job, placements: dict | None = None) -> bool:
        from ..controllers.job import business_execute

        content, status = business_execute(job.id, placements=placements, daemon=self.d)
        if status == 200:
            self.launch_log.append((job.id, time.time()))
            return True
        log.warning("scheduler could not execute job %s: %s", job.id, content.get("msg"))
        return False

    def gpu_info(self) -> dict:
        """{host: {uuid: {index, numa_node}}} for placing ``auto:N`` tasks."""
        data = self.d.infrastructure.snapshot().data
        return {h: {u: {"index": g.get("index"), "numa_node": g.get("numa_node")}
                    for u, g in (((e or {}).get("GPU")) or {}).items()} for h, e in data.items()}

    def refresh_allocations(self) -> None:
        """Re-sync every task that holds devices (one ``th-run ls`` per host and user), so the
        devices of finished tasks are released within one tick; then drop orphaned claims."""
        from ..controllers import task as task_ctl
        from ..models.orm import GpuAllocation
        from . import allocation

        cache = task_ctl.SessionCache()
        for tid in sorted({a.task_id for a in GpuAllocation.query.all()}):
            task_ctl.synchronize(tid, cache)
        allocation.reap()

    def interferes_with_reservations(self, job, occ, period=timedelta(0)) -> bool:
        from ..models.orm import Reservation
        from .scheduling import assigned_gpu_uuids

        for t in job.tasks:
            for u in assigned_gpu_uuids(t, occ):
                if u and any(r.user_id != job.user_id for r in Reservation.upcoming_events_for_resource(u, period)):
                    return True
        return False

    # ---- phases
    def execute_scheduled(self, occ) -> bool:
        from sqlalchemy import and_, or_

        from ..models.orm import Job, JobStatus
        from .allocation import device_request
        from .scheduling import assigned_gpu_uuids

        now = dates.utcnow()
        jobs = Job.query.filter(Job._start_at.isnot(None), or_(Job._stop_at.is_(None), Job._start_at < Job._stop_at),
                                Job._start_at < now, or_(Job._stop_at.is_(None), now < Job._stop_at)).all()
        claimed = self.claimed(occ)
        taken: set = set()
        ran = False
        for job in jobs:
            if job.status is JobStatus.running:
                continue
            keys = set()
            ok = True
            for t in job.tasks:
                req = device_request(t)
                if req is None or req.auto:
                    continue  # CPU-only, or placed (and checked) by business_execute's allocator
                uu = assigned_gpu_uuids(t, occ)
                if not uu or None in uu:
                    ok = False
                    break
                for u in uu:
                    k = (t.hostname, u)
                    if occ.get(t.hostname, {}).get(u) or k in claimed or k in taken:
                        ok = False
                    keys.add(k)
            if not ok or self.interferes_with_reservations(job, occ):
                continue
            if self._execute(job):
                job._start_at = None
                job.save()
                taken |= keys
                ran = True
        return ran

    def execute_queued(self, occ) -> None:
        from ..models.orm import Job

        queue = Job.get_job_queue()
        self._queue_left = len(queue)
        if not queue:
            return
        sched = self.scheduler
        try:
            jobs = sched.schedule_jobs(self.eligible(queue), self.gpu_slots(occ), self.gpu_info())
        except TypeError:  # a custom Scheduler with the reference's two-argument signature
            jobs = sched.schedule_jobs(self.eligible(queue), self.gpu_slots(occ))
        started = sum(1 for job in jobs if self._execute(job, (getattr(sched, "placements", None) or {}).get(job.id)))
        self._queue_left = len(queue) - started

    def stop_with_grace(self, job_id: int):
        from ..controllers.job import business_stop

        if job_id in self.stubborn:
            self.stubborn.discard(job_id)
            return business_stop(job_id, gracefully=False)
        content, status = business_stop(job_id, gracefully=True)
        if status != 200:
            self.stubborn.add(job_id)
        return content, status

    def stop_scheduled(self) -> None:
        from ..models.orm import Job, JobStatus

        now = dates.utcnow()
        jobs = Job.query.filter(Job._stop_at.isnot(None), Job._stop_at > now - self.stop_attempts_after,
                                Job._stop_at < now).all()
        for job in jobs:
            if job.status is JobStatus.running or job.id in self.stubborn:
                self.stop_with_grace(job.id)

    def sync_running_from_queue(self, occ) -> None:
        from ..models.orm import Job
        from .scheduling import assigned_gpu_uuids

        for job in Job.get_jobs_running_from_queue():
            task_ids = {str(t.id) for t in job.tasks}
            stop = False
            for t in job.tasks:
                for u in assigned_gpu_uuids(t, occ):
                    procs = occ.get(t.hostname, {}).get(u) or []
                    owner = job.user.username if job.user else None
                    if any(p.get("task_id") not in task_ids and p.get("owner") != owner for p in procs):
                        stop = True
            if stop or self.interferes_with_reservations(job, occ, self.window):
                log.info("stopping queued job %s (GPU contention or upcoming reservation)", job.id)
                self.stop_with_grace(job.id)

    def do_run(self) -> None:
        self.refresh_allocations()
        occ = self.occupancy()
        self._idle_claims = any(not occ.get(h, {}).get(u) for h, u in self.claimed(occ))
        if not self.execute_scheduled(occ):
            self.execute_queued(occ)
        self.stop_scheduled()
        self.sync_running_from_queue(occ)
