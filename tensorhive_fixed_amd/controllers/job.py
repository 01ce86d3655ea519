"""Jobs: CRUD, execute/stop, enqueue/dequeue, task membership (reference ``controllers/job.py``).

``business_execute`` spawns every task of the job in PARALLEL (one thread per task; the
reference spawned serially, 2 SSH round trips per task) and wakes the scheduler on queue
changes so a queued job starts in well under a second when GPUs are free.
"""
from __future__ import annotations

import concurrent.futures as cf
import logging
import time

from ..models.orm import Job, JobStatus, Task
from ..utils.exceptions import ForbiddenException
from . import task as task_ctl
from ._common import Abort, M, check_fields, guarded, is_admin, me, snake

log = logging.getLogger(__name__)


def _owned(id: int, admin_ok: bool = True) -> Job:
    job = Job.get(id)
    if not ((admin_ok and is_admin()) or job.user_id == me()):
        raise Abort(403, M("general.unprivileged"))
    return job


@guarded(not_found="job.not_found")
def get_by_id(id: int):
    job = _owned(id)
    return {"msg": M("job.get.success"), "job": job.as_dict()}, 200


@guarded(not_found="job.not_found", forbidden="job.all.forbidden")
def get_all(userId: int | None = None):
    if userId:
        if not (is_admin() or me() == userId):
            raise ForbiddenException("not an owner")
        jobs = Job.query.filter(Job.user_id == userId).all()
    else:
        if not is_admin():
            raise ForbiddenException("unauthorized")
        jobs = Job.all()
    cache = task_ctl.SessionCache()
    for j in jobs:
        for t in j.tasks:
            task_ctl.synchronize(t.id, cache)
    return {"msg": M("job.all.success"), "jobs": [j.as_dict() for j in jobs]}, 200


@guarded(assertion="job.create.failure.invalid")
def create(job: dict):
    if job["userId"] != me():
        raise Abort(403, M("general.unprivileged"))
    try:
        j = Job(name=job["name"], description=job.get("description"), user_id=job["userId"],
                start_at=job.get("startAt"), stop_at=job.get("stopAt"))
    except ValueError:
        return {"msg": M("job.create.failure.invalid", reason="invalid date format")}, 422
    j.save()
    _wake("job")
    return {"msg": M("job.create.success"), "job": j.as_dict()}, 201


@guarded(not_found="job.not_found", forbidden="job.update.failure.forbidden",
         assertion="job.update.failure.assertions")
def update(id: int, newValues: dict):
    job = Job.get(id)
    if not (is_admin() or job.user_id == me()):
        raise ForbiddenException("not an owner")
    check_fields(newValues, {"name", "description", "startAt", "stopAt"})
    assert job.status is not JobStatus.running, "must be stopped first"
    for k, v in newValues.items():
        if v is not None:
            setattr(job, snake(k), v)
    job.save()
    _wake("job")
    return {"msg": M("job.update.success"), "job": job.as_dict()}, 200


@guarded(not_found="job.not_found", forbidden="job.update.failure.forbidden",
         assertion="job.delete.failure.assertions")
def delete(id: int):
    job = Job.get(id)
    if not (is_admin() or job.user_id == me()):
        raise ForbiddenException("not an owner")
    assert job.status is not JobStatus.running, "must be stopped first"
    job.destroy()
    return {"msg": M("job.delete.success")}, 200


def _job_and_task(job_id: int, task_id: int):
    from sqlalchemy.exc import NoResultFound

    try:
        job = Job.get(job_id)
    except NoResultFound:
        raise Abort(404, M("job.not_found"))
    try:
        task = Task.get(task_id)
    except NoResultFound:
        raise Abort(404, M("task.not_found"))
    if job.user_id != me():
        raise Abort(403, M("job.tasks.add.failure.assertions", reason="Not an owner"))
    return job, task


@guarded(invalid="job.tasks.add.failure.duplicate", assertion="job.tasks.add.failure.assertions",
         assertion_status=403)
def add_task(job_id: int, task_id: int):
    job, task = _job_and_task(job_id, task_id)
    job.add_task(task)
    return {"msg": M("job.tasks.add.success"), "job": job.as_dict()}, 200


@guarded(invalid="job.tasks.remove.failure.not_found", invalid_status=404,
         assertion="job.tasks.remove.failure.assertions", assertion_status=403)
def remove_task(job_id: int, task_id: int):
    job, task = _job_and_task(job_id, task_id)
    job.remove_task(task)
    return {"msg": M("job.tasks.remove.success"), "job": job.as_dict()}, 200


@guarded(not_found="job.not_found")
def execute(id: int):
    job = Job.get(id)
    if job.user_id != me():
        raise Abort(403, M("general.unprivileged"))
    return business_execute(id)


def _fan_out(fn, items):
    """Run blocking node operations (spawn/terminate over the transports) concurrently; the DB
    work around them stays on the calling thread."""
    if len(items) <= 1:
        return [fn(*it) for it in items]
    with cf.ThreadPoolExecutor(max_workers=min(16, len(items))) as ex:
        return list(ex.map(lambda it: fn(*it), items))


@guarded(not_found="job.not_found")
def business_execute(id: int, placements: dict | None = None, daemon=None):
    """Claim devices for every task, then spawn them all in parallel.

    Allocation (``core/allocation.py``) runs under the lock shared with the scheduler tick: the
    running check, the device choice for ``auto:N`` tasks and the ``gpu_allocations`` insert
    are one atomic step, so a double execute, or an execute racing a queue tick, gets 409
    instead of a second process on the same GPU.  ``placements`` (task id -> [uuid]) carries
    the scheduler's choices for ``auto`` tasks; they are re-validated under the lock."""
    from ..core import allocation, task_nursery
    from ..database import db_session
    from ..models.orm import GpuAllocation, TaskStatus

    d = daemon if daemon is not None else _daemon()
    job = Job.get(id)
    cache = task_ctl.SessionCache()
    for t in job.tasks:
        task_ctl.synchronize(t.id, cache)
    with allocation.ALLOC_LOCK:
        db_session.expire_all()
        job = Job.get(id)
        if (job.status is JobStatus.running or job.id in allocation.launching
                or GpuAllocation.query.filter(GpuAllocation.job_id == job.id).count()):
            return {"msg": M("job.execute.failure.state", reason="Job is already running")}, 409
        snapshot = d.infrastructure.snapshot().data if d is not None else {}
        window = d.scheduling_window() if d is not None else None
        try:
            plan = allocation.plan_job(job, snapshot, placements, **({"window": window} if window else {}))
            allocation.claim(job, plan)
        except allocation.AllocationError as e:
            return {"msg": M("job.execute.failure.state", reason=e.reason)}, e.status
        allocation.launching.add(job.id)
    try:
        failed, todo = [], []
        for t in job.tasks:
            if t.status is TaskStatus.running or not t.full_command or not t.hostname or job.user is None:
                failed.append(t.id)
                continue
            devices = [i for i, _u in plan.get(t.id, [])]
            cmd = allocation.render_command(t, devices)
            todo.append((t, (cmd, t.hostname, job.user.username, str(t.id), t.max_restarts)))

        def spawn(cmd, host, user, tid, max_restarts):
            try:
                return task_nursery.spawn(cmd, host, user, name_appendix=tid, max_restarts=max_restarts)
            except Exception as e:  # noqa: BLE001
                log.warning("spawn of task %s failed: %s", tid, e)
                return None

        pids = _fan_out(spawn, [args for _t, args in todo])
        for (t, _args), pid in zip(todo, pids):
            if pid is None:
                failed.append(t.id)
                continue
            t.pid = pid
            t.status = TaskStatus.running
            t.save()
        for tid in failed:
            allocation.release_task(tid)
        job.synchronize_status()
        job.save()
    finally:
        with allocation.ALLOC_LOCK:
            allocation.launching.discard(job.id)
            allocation.launched_at[job.id] = time.monotonic()
    if failed:
        return {"msg": M("job.execute.failure.tasks", reason="Could not spawn some tasks"),
                "not_spawned_list": failed}, 422
    return {"msg": M("job.execute.success"), "job": job.as_dict()}, 200


def _daemon():
    from ..api.app import daemon

    return daemon()


@guarded(not_found="job.not_found", assertion="job.enqueue.failure", assertion_status=409)
def enqueue(id: int):
    job = _owned(id)
    job.enqueue()
    _wake("enqueue")
    return {"msg": M("job.enqueue.success"), "job": job.as_dict()}, 200


@guarded(not_found="job.not_found", assertion="job.dequeue.failure", assertion_status=409)
def dequeue(id: int):
    job = _owned(id)
    job.dequeue()
    return {"msg": M("job.dequeue.success"), "job": job.as_dict()}, 200


@guarded(not_found="job.not_found")
def stop(id: int, gracefully: bool | None = True):
    job = Job.get(id)
    if not (me() == job.user_id or is_admin()):
        raise Abort(403, M("general.unprivileged"))
    if job.status is not JobStatus.running:
        return {"msg": M("job.stop.failure.state", reason="Only running jobs can be stopped")}, 409
    return business_stop(id, gracefully)


@guarded(not_found="job.not_found")
def business_stop(id: int, gracefully: bool | None = True):
    from ..core import task_nursery
    from ..models.orm import TaskStatus

    job = Job.get(id)
    cache = task_ctl.SessionCache()
    bad, todo = 0, []
    for t in job.tasks:
        task_ctl.synchronize(t.id, cache)
        if t.status is not TaskStatus.running or not t.pid:
            continue
        todo.append((t.pid, t.hostname, job.user.username))

    def term(pid, host, user):
        try:
            return task_nursery.terminate(pid, host, user, gracefully=gracefully)
        except Exception as e:  # noqa: BLE001
            log.warning("terminate of pid %s on %s failed: %s", pid, host, e)
            return -1

    bad = sum(1 for code in _fan_out(term, todo) if code != 0)
    if bad:
        return {"msg": M("job.stop.failure.tasks", reason="Not all tasks could be terminated")}, 422
    fresh = task_ctl.SessionCache()  # processes that already exited show up as terminated now
    for t in job.tasks:
        task_ctl.synchronize(t.id, fresh)
    if job.start_at:
        job.start_at = None  # a manually stopped job is not auto-started again
    job.synchronize_status()
    job.save()
    _wake("stop")
    return {"msg": M("job.stop.success"), "job": job.as_dict()}, 200


@guarded(not_found="job.not_found", forbidden="job.update.failure.forbidden",
         assertion="job.update.failure.assertions")
def attach_to_reservation(id: int, reservation_id: int, siblings: bool | None = True):
    """Run a job inside a reservation (the reservation card's "attach jobs", reference
    ``FullCalendarInfo.vue:510-548``), done server-side in one transaction: the job's window
    becomes the reservation's, and every task moves to the reserved node with
    ``HIP_VISIBLE_DEVICES`` set to the reserved GPUs' HIP indices in xGMI ring order
    (``--nproc_per_node=`` follows).  ``siblings`` (default on) also takes the owner's other
    reservations on the same node with the same window -- a multi-GPU reservation made in one
    go -- so a torchrun task gets all of them.  The reference rewrote the first word of the
    command to ``CUDA_VISIBLE_DEVICES=<one index>``, clobbering commands that had no prefix."""
    from ..api.app import daemon
    from ..core.launcher import devices_for_uuids, hip_visible_devices, order_for_rings
    from ..models.orm import Reservation, Resource
    from . import task as task_ctl

    job = Job.get(id)
    if not (is_admin() or job.user_id == me()):
        raise ForbiddenException("not an owner")
    assert job.status is not JobStatus.running, "must be stopped first"
    res = Reservation.get(reservation_id)
    assert res.user_id == job.user_id, "reservation belongs to another user"
    assert not res.is_cancelled, "reservation is cancelled"
    resource = Resource.get(res.resource_id)
    chosen = [res]
    if siblings is None or siblings:
        for r in Reservation.query.filter(Reservation.user_id == res.user_id, Reservation.id != res.id).all():
            if r.is_cancelled or r.start != res.start or r.end != res.end:
                continue
            other = Resource.query.filter(Resource.id == r.resource_id).first()
            if other is not None and other.hostname == resource.hostname:
                chosen.append(r)
    d = daemon()
    snap = d.infrastructure.snapshot().data if d is not None else {}
    topo = d.topology().get(resource.hostname) if d is not None else None
    try:
        idx = devices_for_uuids(snap, resource.hostname, [r.resource_id for r in chosen])
    except KeyError:
        raise AssertionError("reserved GPUs are not visible on the node right now")
    idx = order_for_rings(idx, topo)
    job.start_at, job.stop_at = res.start, res.end
    job.save()
    for t in job.tasks:
        assert t.status is not task_ctl.TaskStatus.running, "must be stopped first"
        form = {"envs": [{"name": n, "value": v} for n, v in t.envs()
                         if n not in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")],
                "params": [{"name": n, "value": str(len(idx)) if n == "--nproc_per_node=" else v}
                           for n, v in t.params()]}
        form["envs"].insert(0, {"name": "HIP_VISIBLE_DEVICES", "value": hip_visible_devices(idx)})
        words = t.command.split(" ")
        command = " ".join(words[1:]) if words[0].startswith(("HIP_VISIBLE_DEVICES=", "CUDA_VISIBLE_DEVICES=",
                                                               "ROCR_VISIBLE_DEVICES=")) else t.command
        task_ctl.business_update(t.id, {"hostname": resource.hostname, "command": command, "cmdsegments": form})
    _wake("job")
    return {"msg": M("job.update.success"), "job": Job.get(id).as_dict()}, 200


def _placements(form: dict) -> list[dict]:
    out = []
    for p in form["placements"]:
        assert isinstance(p, dict) and isinstance(p.get("hostname"), str), "placement needs a hostname"
        gpus = p.get("gpus", [p["gpu"]] if "gpu" in p else [])
        count = p.get("gpuCount")
        if isinstance(gpus, str) and gpus.startswith("auto"):  # "auto:4": the scheduler picks
            if ":" in gpus:
                n = gpus.split(":", 1)[1]
                assert n.isdigit(), "auto placement needs a count: auto:N"
                count = int(n)
            assert count is not None, "auto placement needs a count: auto:N or gpuCount"
            gpus = []
        if count is not None:
            assert isinstance(count, int) and count >= 1, "gpuCount must be a positive integer"
            assert not gpus, "give either gpus or gpuCount"
        else:
            assert all(isinstance(g, int) and g >= 0 for g in gpus), "gpus must be device indices"
        out.append({"hostname": p["hostname"], "gpus": gpus, "count": count, "role": p.get("role", "worker")})
    assert out, "no placements"
    return out


@guarded(not_found="job.not_found", forbidden="job.update.failure.forbidden",
         assertion="task.create.failure.invalid")
def generate_tasks(id: int, form: dict):
    """Create every task of a distributed launch in one call (the reference's task creator did
    this in the browser, ``TaskCreate.vue:201-215,617-670``, and never persisted TF_CONFIG).

    ``template``: ``torchrun`` (one task per host, all its GPUs, c10d rendezvous on the first
    host), ``torch`` (one task per GPU with explicit ``--rank``/``--world-size``), ``tf2``
    (TF_CONFIG per task, ports auto-increment per host from 2222; ``role`` chief/worker/ps/
    evaluator), ``tf1`` (ClusterSpec ``--ps_hosts/--worker_hosts``; ``role`` ps/worker).
    ``placements``: ``[{"hostname": h, "gpus": [i, ...] | "gpu": i | "auto:N", "gpuCount": N, "role": r}]``;
    a count (``torchrun`` only) leaves the choice of devices to the allocator at launch time."""
    from ..core import launcher
    from . import task as task_ctl

    job = Job.get(id)
    if not (is_admin() or job.user_id == me()):
        raise ForbiddenException("not an owner")
    assert job.status is not JobStatus.running, "must be stopped first"
    pl = _placements(form)
    kind = form["template"]
    # Only torchrun defers device choice to the allocator (one task owns all its devices); the
    # per-GPU templates need concrete indices -- a count there would pin every task to GPU 0 or
    # create no task at all.
    assert kind == "torchrun" or all(p["count"] is None for p in pl), \
        "gpuCount / auto:N placements are supported by the torchrun template only"
    command = form.get("command") or "python train.py"
    master = pl[0]["hostname"]
    if kind == "torchrun":
        port = form.get("masterPort") or 29500
        forms = [launcher.torchrun_task(p["hostname"], p["gpus"] or p["count"], master, port, nnodes=len(pl),
                                        module=form.get("module") or "tensorhive_fixed_amd.workloads.llama3_ddp")
                 for p in pl]
    elif kind == "torch":
        port = form.get("masterPort") or 29500
        forms = launcher.pytorch_tcp_tasks([(p["hostname"], g) for p in pl for g in p["gpus"]], master, port, command)
    elif kind == "tf2":
        forms = launcher.tf2_tasks([(p["hostname"], p["role"], p["gpus"][0] if p["gpus"] else 0) for p in pl],
                                   form.get("masterPort") or 2222, command)
    elif kind == "tf1":
        forms = launcher.tf1_tasks([p["hostname"] for p in pl if p["role"] == "ps"],
                                   [(p["hostname"], p["gpus"][0] if p["gpus"] else 0) for p in pl if p["role"] != "ps"],
                                   form.get("masterPort") or 2222, command)
    else:
        raise AssertionError(f"unknown template {kind!r}")
    created = []
    for f in forms:
        body, status = task_ctl.business_create(f, id)
        assert status == 201, body.get("msg")
        created.append(body["task"])
    _wake("job")
    return {"msg": M("task.create.success"), "tasks": created}, 201


def get_templates():
    """Launch templates for the task creator (PyTorch-ROCm torchrun, TF_CONFIG, ClusterSpec)."""
    from ..core.launcher import TEMPLATES

    return {"msg": M("general.success"), "templates": TEMPLATES}, 200


def _wake(reason: str) -> None:
    from ..api.app import daemon

    d = daemon()
    if d is not None:
        d.wake(reason)
