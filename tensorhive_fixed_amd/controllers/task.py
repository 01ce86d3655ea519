"""Tasks: create/update/destroy, spawn/terminate through th-run, log fetch, state sync
(reference ``controllers/task.py``).

Synchronisation compares ``task.pid`` with the live ``th-run`` sessions of the job owner on the
task's host.  Transitions: running -> terminated and unsynchronized -> not_running when the pid
is gone; any transport failure -> unsynchronized.  Sessions are listed ONCE per (host, user)
per request (:class:`SessionCache`) instead of one SSH round trip per task
(``GET /jobs`` used to sync every task of every job serially, ``controllers/job.py:64-67``).

GPU ids: ``HIP_VISIBLE_DEVICES=<list>`` (env segment or command prefix) is parsed into a list;
``task.gpu_id`` keeps the first index for schema compatibility.  ``CUDA_VISIBLE_DEVICES`` is
not interpreted (north star: no CUDA paths).
"""
from __future__ import annotations

import logging
import re
import time

from sqlalchemy.exc import NoResultFound

from ..core import allocation, task_nursery
from ..database import db_session
from ..core.scheduling import parse_device_list
from ..models.orm import CommandSegment, Job, SegmentType, Task, TaskStatus
from ._common import Abort, M, guarded, is_admin, me

log = logging.getLogger(__name__)


class SessionCache:
    """(host, user) -> live task sessions keyed by pid (current and spawn-time), fetched lazily once.  The monotonic time each list
    was fetched is kept: a launch that finished after it is not judged by that list."""

    def __init__(self):
        self._d: dict[tuple[str, str], dict[int, dict] | Exception] = {}
        self.fetched_at: dict[tuple[str, str], float] = {}

    def pids(self, host: str, user: str) -> dict[int, dict]:
        key = (host, user)
        if key not in self._d:
            self.fetched_at[key] = time.monotonic()
            try:
                self._d[key] = task_nursery.running_sessions(host, user)
            except Exception as e:  # noqa: BLE001
                self._d[key] = e
        v = self._d[key]
        if isinstance(v, Exception):
            raise v
        return v


def synchronize(task_id: int, cache: SessionCache | None = None) -> None:
    """Reconcile one task with the live sessions on its node.

    The transition is decided under the allocation lock on a fresh read of the task, and is
    skipped while the job is launching or when its launch finished after the session list was
    fetched -- otherwise a stale view could erase a just-spawned pid and release the devices of
    a running task (tests/test_allocation.py::test_concurrent_executes_and_ticks_never_double_allocate)."""
    cache = cache or SessionCache()
    try:
        task = Task.get(task_id)
    except NoResultFound:
        return
    try:
        job = task.job
        assert task.hostname, "hostname is empty"
        assert job is not None and job.user is not None, "user does not exist"
        live = cache.pids(task.hostname, job.user.username)
        fetched = cache.fetched_at.get((task.hostname, job.user.username), 0.0)
    except Exception as e:  # noqa: BLE001 -- unreachable node, bad config, ...
        log.debug("task %s unsynchronized: %s", task_id, e)
        task.status = TaskStatus.unsynchronized
        task.save()
        return
    with allocation.ALLOC_LOCK:
        try:
            db_session.refresh(task)
        except Exception:  # noqa: BLE001 -- deleted meanwhile
            db_session.rollback()
            return
        if task.job_id in allocation.launching or allocation.launched_at.get(task.job_id, -1.0) >= fetched:
            return
        # By session name first: it survives any number of restarts, whatever pid was stored.
        sess = live.get(task_nursery.session_name(task.id)) if task.pid is not None else None
        if sess is None and task.pid is not None:
            sess = live.get(task.pid)
        if sess is None:
            if task.status is TaskStatus.running:
                task.status = TaskStatus.terminated
            elif task.status is TaskStatus.unsynchronized:
                task.status = TaskStatus.not_running
            task.pid = None
            task.save()
            allocation.release_task(task.id)  # the task's devices are free again
        else:
            if isinstance(sess, dict):  # the restart policy may have replaced the process
                cur = int(sess.get("pid") or task.pid)
                if cur != task.pid:
                    task.pid = cur
                    task.save()
                if sess.get("restarts") not in (None, ""):
                    lec = sess.get("last_exit_code")
                    task.record_restarts(int(sess["restarts"]), int(lec) if lec not in (None, "") else None)
            if task.status is not TaskStatus.running:
                task.status = TaskStatus.running  # re-adopt a live session after a daemon restart
                task.save()


def parse_gpu_id_from_command(value: str | None) -> int | None:
    """First GPU index of a leading ``HIP_VISIBLE_DEVICES=`` prefix (multi-digit, lists)."""
    if value and value.lstrip().startswith(("HIP_VISIBLE_DEVICES=", "ROCR_VISIBLE_DEVICES=")):
        ids = parse_device_list(value.lstrip().split("=", 1)[1].split(" ", 1)[0])
        return ids[0] if ids else None
    return None


def _segment(name: str, kind: SegmentType) -> CommandSegment:
    seg = CommandSegment.query.filter(CommandSegment._segment_type == kind, CommandSegment.name == name).first()
    return seg or CommandSegment(name=name, segment_type=kind)


def _apply_segments(task: Task, segs: dict) -> None:
    for s in segs.get("envs", []) or []:
        task.add_cmd_segment(_segment(s["name"], SegmentType.env_variable), s.get("value", ""))
    for s in segs.get("params", []) or []:
        task.add_cmd_segment(_segment(s["name"], SegmentType.parameter), s.get("value", ""))
    for name, value in task.envs():
        if name in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES"):
            ids = parse_device_list(value)
            task.gpu_id = ids[0] if ids else task.gpu_id


def _owned_task(id: int) -> Task:
    task = Task.get(id)
    if not is_admin() and task.job.user_id != me():
        raise Abort(403, M("general.unprivileged"))
    return task


# ------------------------------------------------------------------------------ controllers
@guarded(not_found="task.not_found")
def create(task: dict, job_id: int):
    job = Job.get(job_id)
    if not is_admin() and job.user_id != me():
        raise Abort(403, M("general.unprivileged"))
    return business_create(task, job_id)


@guarded(not_found="task.not_found")
def get(id: int):
    _owned_task(id)
    return business_get(id)


@guarded(not_found="task.not_found")
def get_all(jobId: int | None = None, syncAll: bool | None = None):
    if jobId is not None:
        job = Job.get(jobId)
        if not is_admin() and job.user_id != me():
            raise Abort(403, M("general.unprivileged"))
    return business_get_all(jobId, syncAll)


@guarded(not_found="task.not_found")
def update(id: int, newValues: dict):
    _owned_task(id)
    return business_update(id, newValues)


@guarded(not_found="task.not_found")
def destroy(id: int):
    _owned_task(id)
    return business_destroy(id)


@guarded(not_found="task.not_found")
def get_log(id: int, tail: bool = False):
    _owned_task(id)
    return business_get_log(id, tail)


@guarded(not_found="task.not_found")
def get_training_metrics(id: int, lines: int = 400):
    _owned_task(id)
    return business_get_training_metrics(id, lines)


# ------------------------------------------------------------------- business functions
def business_get_all(job_id: int | None, sync_all: bool | None):
    if job_id is not None:
        tasks = Task.query.filter(Task.job_id == job_id).all()
    else:
        tasks = [t for j in Job.query.filter(Job.user_id == me()).all() for t in j.tasks]
    cache = SessionCache()
    out = []
    for t in tasks:
        if sync_all:
            synchronize(t.id, cache)
        out.append(t.as_dict())
    return {"msg": M("task.all.success"), "tasks": out}, 200


@guarded(assertion="task.create.failure.invalid")
def business_create(task: dict, job_id: int):
    try:
        t = Task(hostname=task["hostname"], command=task["command"])
    except KeyError:
        return {"msg": M("general.bad_request")}, 422
    t.gpu_id = parse_gpu_id_from_command(task["command"])
    job = Job.get(job_id)
    t.save()
    _apply_segments(t, task.get("cmdsegments") or {})
    if task.get("maxRestarts") is not None:
        t.set_max_restarts(task["maxRestarts"])
    t.save()
    job.add_task(t)
    return {"msg": M("task.create.success"), "task": t.as_dict()}, 201


@guarded(not_found="task.not_found")
def business_get(id: int):
    synchronize(id)
    return {"msg": M("task.get.success"), "task": Task.get(id).as_dict()}, 200


@guarded(not_found="task.not_found", assertion="task.update.failure.assertions")
def business_update(id: int, newValues: dict):
    t = Task.get(id)
    assert t.status is not TaskStatus.running, "Cannot update task which is already running"
    for key, value in newValues.items():
        if key == "hostname":
            t.hostname = value
        elif key == "command":
            t.gpu_id = parse_gpu_id_from_command(value)
            t.command = value
        elif key == "cmdsegments":
            for lk in list(t.segment_links):
                t.segment_links.remove(lk)
            t.save()
            _apply_segments(t, value or {})
        elif key == "maxRestarts":
            t.set_max_restarts(value)
    t.save()
    return {"msg": M("task.update.success"), "task": t.as_dict()}, 201


@guarded(not_found="task.not_found", assertion="task.delete.failure.assertions")
def business_destroy(id: int):
    synchronize(id)
    t = Task.get(id)
    assert t.status is not TaskStatus.running, "must be terminated first"
    segs = t.cmd_segments
    t.destroy()
    for s in segs:
        if not s.links:
            s.destroy()
    return {"msg": M("task.delete.success")}, 200


@guarded(not_found="task.not_found", assertion="task.spawn.failure.assertions")
def business_spawn(id: int, cache: SessionCache | None = None):
    synchronize(id, cache)
    t = Task.get(id)
    job = t.job
    assert t.status is not TaskStatus.running, "task is already running"
    assert t.full_command, "command is empty"
    assert t.hostname, "hostname is empty"
    assert job is not None and job.user is not None, "user does not exist"
    try:
        pid = task_nursery.spawn(t.full_command, t.hostname, job.user.username, name_appendix=str(t.id),
                                 max_restarts=t.max_restarts)
    except (task_nursery.SpawnError, ConnectionError, KeyError, AssertionError) as e:
        return {"msg": M("task.spawn.failure.backend", reason=e)}, 500
    t.pid = pid
    t.status = TaskStatus.running
    t.save()
    return {"msg": M("task.spawn.success"), "pid": pid}, 200


@guarded(not_found="task.not_found", assertion="task.terminate.failure.state", assertion_status=409)
def business_terminate(id: int, gracefully: bool | None = True, cache: SessionCache | None = None):
    synchronize(id, cache)
    t = Task.get(id)
    assert t.status is TaskStatus.running, "only running tasks can be terminated"
    assert t.pid, "task has no pid assigned"
    try:
        code = task_nursery.terminate(t.pid, t.hostname, t.job.user.username, gracefully=gracefully)
    except ConnectionError as e:
        return {"msg": M("task.terminate.failure.connection", reason=e)}, 500
    if code != 0:
        return {"msg": M("task.terminate.failure.exit_code"), "exit_code": code}, 202
    return {"msg": M("task.terminate.success"), "exit_code": code}, 200


_TRAIN_LINE = re.compile(r"\[th-train\] step=(\d+) loss=([-+0-9.eEnainf]+) tokens/s=([0-9.]+)(?: world=(\d+))?")


def parse_training_lines(lines) -> list[dict]:
    """``[th-train] step=S loss=L tokens/s=T world=W`` lines of the Llama payload
    (``workloads/llama3_ddp.py``) -> [{step, loss, tokensPerSec, world}] in log order."""
    out = []
    for line in lines:
        m = _TRAIN_LINE.search(line)
        if m:
            out.append({"step": int(m.group(1)), "loss": float(m.group(2)), "tokensPerSec": float(m.group(3)),
                        "world": int(m.group(4)) if m.group(4) else None})
    return out


@guarded(not_found="task.not_found", assertion="task.get_log.failure.assertions")
def business_get_training_metrics(id: int, lines: int = 400):
    """Training progress read from the task's log tail: the series of ``[th-train]`` lines and
    the latest tokens/s, which the dashboard charts next to the task (SURVEY §5 metrics row)."""
    t = Task.get(id)
    job = t.job
    assert t.hostname, "hostname is empty"
    assert job is not None and job.user is not None, "user does not exist"
    try:
        out, path = task_nursery.fetch_log(t.hostname, job.user.username, t.id, tail=True,
                                           tail_lines=max(1, min(int(lines), 5000)))
    except FileNotFoundError as e:
        return {"msg": M("task.get_log.failure.not_found", location=e)}, 404
    except ConnectionError as e:
        return {"msg": M("task.get_log.failure.assertions", reason=e)}, 500
    series = parse_training_lines(out)
    last = series[-1] if series else None
    return {"msg": M("task.get_log.success"), "path": path, "series": series, "last": last,
            "tokensPerSec": last["tokensPerSec"] if last else None}, 200


@guarded(not_found="task.not_found", assertion="task.get_log.failure.assertions")
def business_get_log(id: int, tail: bool = False):
    t = Task.get(id)
    job = t.job
    assert t.hostname, "hostname is empty"
    assert job is not None and job.user is not None, "user does not exist"
    try:
        lines, path = task_nursery.fetch_log(t.hostname, job.user.username, t.id, bool(tail))
    except FileNotFoundError as e:
        return {"msg": M("task.get_log.failure.not_found", location=e)}, 404
    except ConnectionError as e:
        return {"msg": M("task.get_log.failure.assertions", reason=e)}, 500
    return {"msg": M("task.get_log.success"), "path": path, "output_lines": lines}, 200
