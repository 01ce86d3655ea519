"""Gang GPU allocation (core/allocation.py): device picking, atomic claims shared by manual
execute and the scheduler tick, release, and the API surface of ``auto:N`` requests.

Reference behaviour being replaced: a task named one GPU (``CUDA_VISIBLE_DEVICES=<n>``), the
scheduler deduplicated GPUs within one round only (``tensorhive/core/services/
JobSchedulingService.py:140-168``) and nothing serialised execute against a scheduler tick."""
import datetime
import threading
from datetime import timedelta

import pytest

from tensorhive_fixed_amd.core import allocation as A
from tensorhive_fixed_amd.core.allocation import Candidate, pick
from tensorhive_fixed_amd.models.orm import (CommandSegment, GpuAllocation, Job, JobStatus, Reservation, Resource,
                                             Restriction, Role, SegmentType, Task, User)

UTC = datetime.datetime.utcnow


# ------------------------------------------------------------------------------- picking
def _c(i, numa, tier=1):
    return Candidate(i, f"u{i}", numa, tier)


def test_pick_prefers_one_numa_node_best_fit():
    # node 0 has 1 free GPU, node 1 has 4: a pair goes to node 1, a single to node 0 (best fit)
    cands = [_c(3, 0), _c(4, 1), _c(5, 1), _c(6, 1), _c(7, 1)]
    assert [c.index for c in pick(cands, 2)] == [4, 5]
    assert [c.index for c in pick(cands, 1)] == [3]
    # more than any one node holds: the larger node is used whole, then the rest
    assert sorted(c.index for c in pick(cands, 5)) == [3, 4, 5, 6, 7]
    assert pick(cands, 6) is None


def test_pick_takes_own_reservation_first_then_fills_on_its_numa_node():
    cands = [_c(0, 0, tier=1), _c(1, 0, tier=1), _c(5, 1, tier=0), _c(6, 1, tier=1), _c(7, 1, tier=1)]
    got = pick(cands, 3)
    assert [c.index for c in got] == [5, 6, 7]  # reserved GPU 5, then its socket-mates
    assert got[0].tier == 0


def test_best_fit_leaves_whole_sockets_for_big_gangs():
    # node 0: 2 free, node 1: 4 free -> a pair takes node 0, so node 1 still fits a 4-GPU gang
    cands = [_c(2, 0), _c(3, 0), _c(4, 1), _c(5, 1), _c(6, 1), _c(7, 1)]
    assert [c.index for c in pick(cands, 2)] == [2, 3]


# --------------------------------------------------------------------------- fixtures
def _user(name, admin=False):
    roles = [Role(name="user")] + ([Role(name="admin")] if admin else [])
    u = User(username=name, password="password1", email=f"{name}@example.org", roles=roles)
    u.save()
    return u


def _seg(name, kind):
    return CommandSegment.query.filter(CommandSegment.name == name).first() or \
        CommandSegment(name=name, segment_type=kind)


def _job(user, devices, host="node-a", name="j", nproc=False):
    j = Job(name=name, description="", user_id=user.id)
    j.save()
    t = Task(command="torchrun" if nproc else "python train.py", hostname=host)
    t.save()
    t.add_cmd_segment(_seg("HIP_VISIBLE_DEVICES", SegmentType.env_variable), devices)
    if nproc:
        t.add_cmd_segment(_seg("--nproc_per_node=", SegmentType.parameter), "auto")
        t.add_cmd_segment(_seg("-m", SegmentType.parameter), "tensorhive_fixed_amd.workloads.llama3_ddp")
    j.add_task(t)
    return j


@pytest.fixture()
def world(daemon):
    """8-GPU node-a (NUMA 0: GPUs 0-3, NUMA 1: 4-7), a permissive global restriction."""
    g = Restriction(name="everyone", starts_at=UTC() - timedelta(days=1), is_global=True)
    g.save()
    users = {n: _user(n) for n in ("alice", "bob", "carol")}
    for u in users.values():
        g.apply_to_user(u)
    uuids = [daemon.stub.gpu_uuid("node-a", i) for i in range(8)]
    for u in uuids:
        Resource(id=u, name="MI355X", hostname="node-a").save()
    return daemon, users, uuids


def _execute(d, job_id, placements=None):
    from tensorhive_fixed_amd.controllers.job import business_execute

    return business_execute(job_id, placements=placements, daemon=d)


def _spawned_cmd(d, pid):
    return d.transports.get("node-a").sessions[pid]["command"]


# --------------------------------------------------------------------------- manual execute
def test_auto_request_renders_devices_and_nproc(world):
    d, users, _ = world
    j = _job(users["alice"], "auto:2", nproc=True)
    body, status = _execute(d, j.id)
    assert status == 200, body
    t = Job.get(j.id).tasks[0]
    cmd = _spawned_cmd(d, t.pid)
    assert "HIP_VISIBLE_DEVICES=0,1 torchrun --nproc_per_node=2" in cmd
    assert t.as_dict()["allocatedGpus"] == [0, 1]
    assert t.as_dict()["cmdsegments"]["envs"][0]["value"] == "auto:2"  # the request is kept
    # the stub telemetry shows the task's processes on exactly those GPUs
    procs = d.stub.sample("node-a")["GPU"]
    busy = sorted(g["index"] for g in procs.values() if g["processes"])
    assert busy == [0, 1]


def test_double_execute_is_rejected(world):
    d, users, _ = world
    j = _job(users["alice"], "auto:2")
    assert _execute(d, j.id)[1] == 200
    body, status = _execute(d, j.id)
    assert status == 409 and "already running" in body["msg"].lower()
    assert len(d.transports.get("node-a").sessions) == 1


def test_pinned_gpu_held_by_another_task_is_refused(world):
    d, users, _ = world
    a = _job(users["alice"], "3", name="a")
    b = _job(users["bob"], "2,3", name="b")
    assert _execute(d, a.id)[1] == 200
    body, status = _execute(d, b.id)
    assert status == 409 and "node-a:3" in body["msg"]
    assert Job.get(b.id).status is not JobStatus.running


def test_auto_skips_busy_foreign_reserved_and_forbidden_gpus(world):
    d, users, uuids = world
    alice, bob = users["alice"], users["bob"]
    d.stub.add_process("node-a", 0, 5555, "mallory")  # a foreign process on GPU 0
    Reservation(user_id=bob.id, title="bob", description="", resource_id=uuids[1], start=UTC() - timedelta(minutes=1),
                end=UTC() + timedelta(hours=1)).save()
    d.infrastructure.publish("node-a", d.stub.sample("node-a"))
    j = _job(alice, "auto:2")
    assert _execute(d, j.id)[1] == 200
    assert Job.get(j.id).tasks[0].as_dict()["allocatedGpus"] == [2, 3]


def test_auto_prefers_owner_reservation(world):
    d, users, uuids = world
    alice = users["alice"]
    for i in (6, 7):
        Reservation(user_id=alice.id, title="mine", description="", resource_id=uuids[i],
                    start=UTC() - timedelta(minutes=1), end=UTC() + timedelta(hours=1)).save()
    j = _job(alice, "auto:2")
    assert _execute(d, j.id)[1] == 200
    assert Job.get(j.id).tasks[0].as_dict()["allocatedGpus"] == [6, 7]


def test_restricted_user_gets_only_permitted_gpus(world):
    d, _users, uuids = world
    dave = _user("dave")  # not in the global restriction
    r = Restriction(name="dave-4-5", starts_at=UTC() - timedelta(days=1), is_global=False)
    r.save()
    r.apply_to_user(dave)
    r.apply_to_resource(Resource.get(uuids[4]))
    r.apply_to_resource(Resource.get(uuids[5]))
    ok, too_many = _job(dave, "auto:2", name="ok"), _job(dave, "auto:1", name="more")
    assert _execute(d, ok.id)[1] == 200
    assert Job.get(ok.id).tasks[0].as_dict()["allocatedGpus"] == [4, 5]
    body, status = _execute(d, too_many.id)
    assert status == 409 and "0 free" in body["msg"]


def test_claims_are_released_when_the_task_ends(world):
    from tensorhive_fixed_amd.controllers import task as task_ctl

    d, users, _ = world
    node = d.transports.get("node-a")
    jobs = [_job(users["alice"], "auto:4", name=f"j{i}") for i in range(3)]
    assert _execute(d, jobs[0].id)[1] == 200
    assert _execute(d, jobs[1].id)[1] == 200
    assert _execute(d, jobs[2].id)[1] == 409  # node full
    assert GpuAllocation.held() == {("node-a", i) for i in range(8)}
    node.exit_task(Job.get(jobs[0].id).tasks[0].pid)
    task_ctl.synchronize(Job.get(jobs[0].id).tasks[0].id)
    assert {i for _h, i in GpuAllocation.held()} == {4, 5, 6, 7}
    d.infrastructure.publish("node-a", d.stub.sample("node-a"))
    assert _execute(d, jobs[2].id)[1] == 200
    assert Job.get(jobs[2].id).tasks[0].as_dict()["allocatedGpus"] == [0, 1, 2, 3]


def test_failed_spawn_releases_claims(world):
    d, users, _ = world
    node = d.transports.get("node-a")
    node.down = True
    j = _job(users["alice"], "auto:2")
    body, status = _execute(d, j.id)
    assert status == 422 and body["not_spawned_list"]
    assert GpuAllocation.held() == set()
    node.down = False
    assert _execute(d, j.id)[1] == 200


def test_reap_drops_claims_of_dead_tasks(world):
    d, users, _ = world
    j = _job(users["alice"], "0")
    t = j.tasks[0]
    GpuAllocation(task_id=t.id, job_id=j.id, hostname="node-a", gpu_index=0,
                  created_at=UTC() - timedelta(minutes=10)).save()
    assert A.reap() == 1 and GpuAllocation.held() == set()


def test_api_execute_and_task_view(world, app, auth_headers):
    d, users, _ = world
    client = app.test_client()
    alice = users["alice"]
    h = auth_headers(alice)
    j = client.post("/api/jobs", json={"name": "gang", "description": "", "userId": alice.id}, headers=h).get_json()
    tid = client.post(f"/api/jobs/{j['job']['id']}/tasks", headers=h, json={
        "command": "torchrun", "hostname": "node-a",
        "cmdsegments": {"envs": [{"name": "HIP_VISIBLE_DEVICES", "value": "auto:4"}],
                        "params": [{"name": "--nproc_per_node=", "value": "auto"}]}}).get_json()["task"]["id"]
    r = client.get(f"/api/jobs/{j['job']['id']}/execute", headers=h)
    assert r.status_code == 200, r.get_json()
    r2 = client.get(f"/api/jobs/{j['job']['id']}/execute", headers=h)
    assert r2.status_code == 409
    task = client.get(f"/api/tasks/{tid}", headers=h).get_json()["task"]
    assert task["allocatedGpus"] == [0, 1, 2, 3] and task["status"] == "running"


def test_generate_torchrun_with_gpu_count(world, app, auth_headers):
    d, users, _ = world
    client = app.test_client()
    alice = users["alice"]
    h = auth_headers(alice)
    j = client.post("/api/jobs", json={"name": "gen", "description": "", "userId": alice.id}, headers=h).get_json()
    r = client.post(f"/api/jobs/{j['job']['id']}/tasks/generate", headers=h, json={
        "template": "torchrun", "placements": [{"hostname": "node-a", "gpus": "auto:4"}]})
    assert r.status_code == 201, r.get_json()
    t = r.get_json()["tasks"][0]
    assert t["cmdsegments"]["envs"][0]["value"] == "auto:4"
    assert any(p["name"] == "--nproc_per_node=" and p["value"] == "4" for p in t["cmdsegments"]["params"])


# --------------------------------------------------------------------------- scheduler
def test_scheduler_places_unpinned_gang_jobs(world):
    from tensorhive_fixed_amd.core.services import JobSchedulingService

    d, users, uuids = world
    jobs = [_job(users[n], "auto:2", name=n) for n in ("alice", "bob", "carol")]
    big = _job(users["alice"], "auto:4", name="big")
    for j in jobs + [big]:
        j.enqueue()
    sched = JobSchedulingService(3600.0, 5, 30)
    d.add_service(sched)
    sched.do_run()
    got = {j.name: Job.get(j.id).tasks[0].as_dict()["allocatedGpus"] for j in jobs}
    assert all(Job.get(j.id).status is JobStatus.running for j in jobs)
    assert Job.get(big.id).status is JobStatus.pending  # 2 GPUs left, 4 wanted
    flat = sorted(i for v in got.values() for i in v)
    assert len(flat) == len(set(flat)) == 6
    assert all(len({0 if i < 4 else 1 for i in v}) == 1 for v in got.values())  # each pair on one socket


def test_scheduler_keeps_clear_of_upcoming_foreign_reservation(world):
    from tensorhive_fixed_amd.core.services import JobSchedulingService

    d, users, uuids = world
    for i in range(6):  # carol's reservation on GPUs 0-5 starts in 10 minutes (inside the 30-min window)
        Reservation(user_id=users["carol"].id, title="c", description="", resource_id=uuids[i],
                    start=UTC() + timedelta(minutes=10), end=UTC() + timedelta(hours=2)).save()
    j = _job(users["bob"], "auto:2")
    k = _job(users["bob"], "auto:2", name="k")
    j.enqueue()
    k.enqueue()
    sched = JobSchedulingService(3600.0, 5, 30)
    d.add_service(sched)
    sched.do_run()
    assert Job.get(j.id).tasks[0].as_dict()["allocatedGpus"] == [6, 7]
    assert Job.get(k.id).status is JobStatus.pending


# --------------------------------------------------------------------------- concurrency
def test_concurrent_executes_and_ticks_never_double_allocate(tmp_path, world):
    """20 manual executes from 20 threads race 4 scheduler ticks over 12 two-GPU jobs on 8 GPUs:
    every GPU ends up with at most one task, on the node and in the table."""
    from tensorhive_fixed_amd import database as D
    from tensorhive_fixed_amd.core.services import JobSchedulingService

    d, users, uuids = world
    # a file database: each thread gets its own connection (the in-memory fixture shares one)
    D.db_session.remove()
    D.configure(f"sqlite:///{tmp_path / 'race.sqlite'}")
    D.create_all()
    g = Restriction(name="everyone", starts_at=UTC() - timedelta(days=1), is_global=True)
    g.save()
    users = {n: _user(n) for n in ("alice", "bob", "carol")}
    for u in users.values():
        g.apply_to_user(u)
    for u in uuids:
        Resource(id=u, name="MI355X", hostname="node-a").save()
    names = list(users)
    jobs = [_job(users[names[i % 3]], "auto:2", name=f"j{i}") for i in range(12)]
    ids = [j.id for j in jobs]
    for j in jobs[8:]:
        j.enqueue()
    D.db_session.remove()
    sched = JobSchedulingService(3600.0, 5, 30)
    d.add_service(sched)
    barrier = threading.Barrier(24)
    errors = []

    def execute(jid):
        try:
            barrier.wait()
            _execute(d, jid)
        except Exception as e:  # noqa: BLE001
            errors.append(e)
        finally:
            D.db_session.remove()

    def tick():
        try:
            barrier.wait()
            sched.do_run()
        except Exception as e:  # noqa: BLE001
            errors.append(e)
        finally:
            D.db_session.remove()

    threads = [threading.Thread(target=execute, args=(ids[i % 8],)) for i in range(20)]
    threads += [threading.Thread(target=tick) for _ in range(4)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(60)
    assert not errors, errors
    node = d.transports.get("node-a")
    per_gpu: dict[int, list[int]] = {}
    for s in node.sessions.values():
        for gi in s["gpus"]:
            per_gpu.setdefault(gi, []).append(s["pid"])
    assert all(len(v) == 1 for v in per_gpu.values()), per_gpu
    assert len(per_gpu) == 8  # the node is full
    rows = GpuAllocation.query.all()
    assert len(rows) == 8 and len({(r.hostname, r.gpu_index) for r in rows}) == 8
    running = [Job.get(i) for i in ids if Job.get(i).status is JobStatus.running]
    assert len(running) == 4 and len(node.sessions) == 4
    D.db_session.remove()
