"""BASELINE config 5 on a simulated 8-GPU MI355X node: three users with overlapping reservations,
queued two-GPU jobs, the gang scheduler's decisions, node GPU occupancy, and the violation path
(terminal wall) for a process nobody reserved."""
import datetime
from datetime import timedelta

from tensorhive_fixed_amd.core.services import JobSchedulingService, ProtectionService
from tensorhive_fixed_amd.core.violation_handlers import MessageSendingBehaviour, ProtectionHandler
from tensorhive_fixed_amd.models.orm import (CommandSegment, Job, JobStatus, Reservation, Resource, Restriction,
                                             Role, SegmentType, Task, User)

UTC = datetime.datetime.utcnow


def _user(name):
    u = User(username=name, password="password1", email=f"{name}@example.org", roles=[Role(name="user")])
    u.save()
    return u


def _job(user, gpus, name):
    j = Job(name=name, description="", user_id=user.id)
    j.save()
    t = Task(command="python train.py", hostname="node-a")
    t.save()
    seg = CommandSegment.query.filter(CommandSegment.name == "HIP_VISIBLE_DEVICES").first() or \
        CommandSegment(name="HIP_VISIBLE_DEVICES", segment_type=SegmentType.env_variable)
    t.add_cmd_segment(seg, gpus)
    j.add_task(t)
    j.enqueue()
    return j


def test_three_tenants(daemon):
    stub = daemon.stub
    alice, bob, carol = _user("alice"), _user("bob"), _user("carol")
    g = Restriction(name="everyone", starts_at=UTC() - timedelta(days=1), is_global=True)
    g.save()
    for u in (alice, bob, carol):
        g.apply_to_user(u)
    uuid = [stub.gpu_uuid("node-a", i) for i in range(8)]
    for i, u in enumerate(uuid):
        Resource(id=u, name="MI355X", hostname="node-a").save()

    def reserve(user, gpus, start, hours):
        for i in gpus:
            Reservation(user_id=user.id, title=f"{user.username}-{i}", description="", resource_id=uuid[i],
                        start=start, end=start + timedelta(hours=hours)).save()

    reserve(alice, [0, 1], UTC() - timedelta(minutes=5), 2)
    reserve(bob, [2, 3], UTC() - timedelta(minutes=5), 2)
    reserve(carol, [4], UTC() + timedelta(minutes=10), 2)  # upcoming, inside the 30-min window

    jobs = {
        "alice-own": _job(alice, "0,1", "alice-own"),      # her reservation -> runs
        "bob-on-alice": _job(bob, "0,1", "bob-on-alice"),  # alice holds them -> waits
        "carol-own": _job(carol, "4", "carol-own"),        # her upcoming reservation -> runs
        "carol-free": _job(carol, "6,7", "carol-free"),    # nobody's -> runs
        "bob-on-carol": _job(bob, "4,5", "bob-on-carol"),  # carol's reservation starts soon -> waits
    }
    for h in ("node-a", "node-b"):
        daemon.infrastructure.publish(h, stub.sample(h))
    sched = JobSchedulingService(3600.0, 5, 30)
    daemon.add_service(sched)
    sched.do_run()
    status = {k: Job.get(j.id).status for k, j in jobs.items()}
    assert status == {"alice-own": JobStatus.running, "bob-on-alice": JobStatus.pending,
                      "carol-own": JobStatus.running, "carol-free": JobStatus.running,
                      "bob-on-carol": JobStatus.pending}, status
    # achieved node occupancy: 5 of 8 GPUs busy with the tenants' own work
    busy = [i for i, u in enumerate(uuid) if stub.sample("node-a")["GPU"][u]["processes"]]
    assert busy == [0, 1, 4, 6, 7]

    # a foreign process on bob's reserved GPU 2: detected and walled on the intruder's terminals
    node = daemon.transports.get("node-a")
    node.ttys = [("mallory", "pts/3")]
    stub.add_process("node-a", 2, 66666, "mallory")
    daemon.infrastructure.publish("node-a", stub.sample("node-a"))
    prot = ProtectionService(1.0, [ProtectionHandler(MessageSendingBehaviour(daemon.transports))], level=1)
    prot.inject(daemon)
    prot.do_run()
    assert set(prot.last_violations) == {"mallory"}
    assert prot.last_violations["mallory"]["RESERVATIONS"][0]["OWNER_USERNAME"] == "bob"
    assert [t for t, _ in node.tty_messages] == ["pts/3"]

    # alice's job finishes -> bob's waiting job gets the GPUs only once alice's reservation is over
    for t in Job.get(jobs["alice-own"].id).tasks:
        node.exit_task(t.pid)
    daemon.infrastructure.publish("node-a", stub.sample("node-a"))
    sched.do_run()
    assert Job.get(jobs["bob-on-alice"].id).status is JobStatus.pending


def test_three_tenants_unpinned_gang_jobs(daemon):
    """The same node with jobs that ask for a COUNT of GPUs (``HIP_VISIBLE_DEVICES=auto:2``):
    the scheduler picks pairs that respect every reservation, never overlaps them, and the
    node fills up except where a reservation fences GPUs off."""
    from tensorhive_fixed_amd.models.orm import GpuAllocation

    stub = daemon.stub
    alice, bob, carol = _user("alice"), _user("bob"), _user("carol")
    g = Restriction(name="everyone", starts_at=UTC() - timedelta(days=1), is_global=True)
    g.save()
    for u in (alice, bob, carol):
        g.apply_to_user(u)
    uuid = [stub.gpu_uuid("node-a", i) for i in range(8)]
    for u in uuid:
        Resource(id=u, name="MI355X", hostname="node-a").save()
    for user, gpus, start in ((alice, [0, 1], UTC() - timedelta(minutes=5)), (bob, [2, 3], UTC() - timedelta(minutes=5)),
                              (carol, [4], UTC() + timedelta(minutes=10))):
        for i in gpus:
            Reservation(user_id=user.id, title=f"{user.username}-{i}", description="", resource_id=uuid[i],
                        start=start, end=start + timedelta(hours=2)).save()
    jobs = {n: _job(u, "auto:2", n) for n, u in (("a1", alice), ("b1", bob), ("c1", carol), ("b2", bob),
                                                 ("a2", alice))}
    sched = JobSchedulingService(3600.0, 5, 30)
    daemon.add_service(sched)
    sched.do_run()
    got = {k: Job.get(j.id).tasks[0].as_dict()["allocatedGpus"] for k, j in jobs.items()}
    status = {k: Job.get(j.id).status for k, j in jobs.items()}
    assert got["a1"] == [0, 1]   # alice's own reservation first
    assert got["b1"] == [2, 3]   # bob's own reservation first
    assert got["c1"] in ([4, 5], [4, 6], [4, 7])  # carol's upcoming GPU 4 is hers to use
    assert status["b2"] is JobStatus.running and status["a2"] is JobStatus.pending
    flat = [i for v in got.values() for i in v]
    assert len(flat) == len(set(flat)) == 8  # no GPU twice, node full
    assert 4 not in got["b2"]  # carol's upcoming reservation is fenced off for bob
    held = {i for _h, i in GpuAllocation.held()}
    assert held == set(range(8))
    # a1 finishes -> its pair goes back to alice's queue entry a2 on the next tick
    node = daemon.transports.get("node-a")
    node.exit_task(Job.get(jobs["a1"].id).tasks[0].pid)
    daemon.infrastructure.publish("node-a", stub.sample("node-a"))
    sched.do_run()
    assert Job.get(jobs["a2"].id).tasks[0].as_dict()["allocatedGpus"] == [0, 1]
