"""Daemon services against simulated MI355X nodes (reference ``core/services/*``; the reference
has no tests for these -- SURVEY §4 lists them as untested)."""
import datetime
import json
import time
from datetime import timedelta

import pytest

from tensorhive_fixed_amd.core.services import (JobSchedulingService, MonitoringService, ProtectionService,
                                                UsageLoggingService)
from tensorhive_fixed_amd.core.violation_handlers import (EmailSendingBehaviour, MessageSendingBehaviour,
                                                          ProtectionHandler, SudoProcessKillingBehaviour,
                                                          UserProcessKillingBehaviour)
from tensorhive_fixed_amd.models.orm import (CommandSegment, Job, JobStatus, Reservation, Resource, Restriction,
                                             SegmentType, Task, TaskStatus)

UTC = datetime.datetime.utcnow


def publish(daemon):
    for h in daemon.cfg.ssh.available_nodes:
        daemon.infrastructure.publish(h, daemon.stub.sample(h))


def gpu(daemon, host="node-a", i=0):
    uuid = daemon.stub.gpu_uuid(host, i)
    try:
        return Resource.get(uuid)
    except Exception:  # noqa: BLE001
        r = Resource(id=uuid, name="MI355X", hostname=host)
        r.save()
        return r


def reserve(user, res, start, dur):
    r = Reservation(user_id=user.id, title="t", description="d", resource_id=res.id, start=start, end=start + dur)
    r.save()
    return r


# ------------------------------------------------------------------------- monitoring
def test_monitoring_publishes_and_isolates_hosts(daemon):
    mon = MonitoringService(1.0, daemon.backends)
    mon.inject(daemon)
    daemon.stub.down.add("node-b")
    mon.do_run()
    snap = daemon.infrastructure.snapshot()
    assert len(snap.data["node-a"]["GPU"]) == 8
    assert snap.data["node-b"] == {"CPU": None, "GPU": None}
    v1 = snap.version
    mon.do_run()
    assert daemon.infrastructure.snapshot().version > v1


# ------------------------------------------------------------------------- protection
def test_protection_detects_intruder(daemon, new_user, new_admin):
    res = gpu(daemon)
    reserve(new_user, res, UTC() - timedelta(minutes=10), timedelta(hours=1))
    daemon.stub.add_process("node-a", 0, 1111, "justuser")
    daemon.stub.add_process("node-a", 0, 2222, "administrantee")
    publish(daemon)
    svc = ProtectionService(1.0, [], level=1)
    svc.inject(daemon)
    v = svc.find_violations()
    assert set(v) == {"justuser"}
    assert v["justuser"]["VIOLATION_PIDS"] == {"node-a": {1111}}
    assert v["justuser"]["RESERVATIONS"][0]["OWNER_USERNAME"] == "administrantee"
    assert v["justuser"]["HOSTNAMES"] == ["node-a"]


def test_protection_accepts_owners_tasks_and_levels(daemon, new_user, new_job_with_task):
    """A genuine process of the owner's task is fine even under a service account: it is in the
    task's th-run session and runs as the task's user (``core/attribution.py``)."""
    from tensorhive_fixed_amd.core.attribution import REGISTRY

    res = gpu(daemon)
    reserve(new_user, res, UTC() - timedelta(minutes=10), timedelta(hours=1))
    tid = new_job_with_task.tasks[0].id
    REGISTRY.record("node-a", {"name": f"tensorhive_task_{tid}", "sid": 7000, "monitor_pid": 6999,
                               "pid": 3333, "user": "svc-account"})
    daemon.stub.add_process("node-a", 0, 3333, "svc-account", task_id=str(tid), sid=7000)
    # a rank that called setsid itself: attested through its parent chain (th-run's monitor)
    daemon.stub.add_process("node-a", 0, 3334, "svc-account", task_id=str(tid), sid=3334, ancestors=[3333, 6999])
    daemon.stub.add_process("node-a", 5, 4444, "someone")  # unreserved GPU
    publish(daemon)
    lenient = ProtectionService(1.0, [], level=1)
    lenient.inject(daemon)
    assert lenient.find_violations() == {}
    strict = ProtectionService(1.0, [], level=2)
    strict.inject(daemon)
    v = strict.find_violations()
    assert set(v) == {"someone"} and v["someone"]["VIOLATION_PIDS"] == {"node-a": {4444}}


def test_forged_task_id_is_a_violation(daemon, new_user, new_job_with_task):
    """Round-4 bypass: ``TENSORHIVE_TASK_ID=<victim's task> python train.py`` on a reserved GPU.
    The claim is checked against the task's th-run session and uid, so an intruder -- or a
    process of the same service account outside the task's session -- is still a violation, and
    the published process carries ``claimed_task_id`` instead of ``task_id``."""
    from tensorhive_fixed_amd.core.attribution import REGISTRY

    res = gpu(daemon)
    reserve(new_user, res, UTC() - timedelta(minutes=10), timedelta(hours=1))
    tid = str(new_job_with_task.tasks[0].id)
    REGISTRY.record("node-a", {"name": f"tensorhive_task_{tid}", "sid": 7000, "monitor_pid": 6999,
                               "pid": 3333, "user": "svc-account"})
    daemon.stub.add_process("node-a", 0, 3333, "svc-account", task_id=tid, sid=7000)  # genuine
    daemon.stub.add_process("node-a", 0, 5001, "intruder", task_id=tid, sid=5001)  # other uid
    daemon.stub.add_process("node-a", 0, 5002, "intruder", task_id=tid, sid=7000)  # other uid, same sid number
    daemon.stub.add_process("node-a", 0, 5003, "svc-account", task_id=tid, sid=5003)  # same uid, outside
    daemon.stub.add_process("node-a", 0, 5004, "svc-account", task_id="999", sid=7000)  # unknown task
    publish(daemon)
    svc = ProtectionService(1.0, [], level=1)
    svc.inject(daemon)
    v = svc.find_violations()
    assert set(v) == {"intruder", "svc-account"}
    assert v["intruder"]["VIOLATION_PIDS"] == {"node-a": {5001, 5002}}
    assert v["svc-account"]["VIOLATION_PIDS"] == {"node-a": {5003, 5004}}
    procs = {p["pid"]: p for p in daemon.infrastructure.node_gpu_processes("node-a")[res.id]}
    assert procs[3333]["task_id"] == tid and "claimed_task_id" not in procs[3333]
    assert procs[5001]["task_id"] is None and procs[5001]["claimed_task_id"] == tid


def test_claim_of_unseen_task_triggers_one_session_lookup(daemon, new_user, new_job_with_task):
    """A daemon restarted under a running task has not seen its session yet: the first claim
    lists the owner's th-run sessions on that node once (rate-limited), then attests."""
    from tensorhive_fixed_amd.core.attribution import REGISTRY

    REGISTRY.clear()
    task = new_job_with_task.tasks[0]
    node = daemon.transports.get(task.hostname)
    user = new_job_with_task.user.username
    node.sessions[4242] = {"name": f"tensorhive_task_{task.id}", "pid": 4242, "pgid": 4242, "user": user,
                           "sid": 9100, "monitor_pid": 9099, "status": "running", "gpus": [], "env": {}}
    daemon.stub.add_process(task.hostname, 1, 4242, user, task_id=str(task.id), sid=9100)
    daemon.stub.add_process(task.hostname, 2, 4243, "intruder", task_id=str(task.id), sid=4243)
    n0 = sum(1 for c, _ in node.calls if " ls" in c)
    publish(daemon)  # queues the lookup on the attestor's worker (never on the publishing thread)
    assert daemon.attestor.drain()
    publish(daemon)
    assert daemon.attestor.drain()
    assert sum(1 for c, _ in node.calls if " ls" in c) - n0 == 1  # the intruder's claim does not re-list
    procs = daemon.infrastructure.node_gpu_processes(task.hostname)
    by_pid = {p["pid"]: p for ps in procs.values() for p in ps}
    assert by_pid[4242]["task_id"] == str(task.id)
    assert by_pid[4243]["task_id"] is None and by_pid[4243]["claimed_task_id"] == str(task.id)


def test_protection_handlers_warn_and_kill(daemon, new_user):
    res = gpu(daemon, "node-b", 3)
    reserve(new_user, res, UTC() - timedelta(minutes=10), timedelta(hours=1))
    node = daemon.transports.get("node-b")
    node.ttys = [("intruder", "pts/7"), ("intruder", "pts/9"), ("other", "pts/1")]
    daemon.stub.add_process("node-b", 3, 5555, "intruder")
    publish(daemon)
    handlers = [ProtectionHandler(MessageSendingBehaviour(daemon.transports)),
                ProtectionHandler(UserProcessKillingBehaviour(daemon.transports))]
    svc = ProtectionService(1.0, handlers, level=1)
    svc.inject(daemon)
    svc.do_run()
    assert sorted(t for t, _ in node.tty_messages) == ["pts/7", "pts/9"]
    assert "reserved by someone else" in node.tty_messages[0][1]
    assert node.killed == [(5555, "intruder", False)]
    publish(daemon)
    assert svc.find_violations() == {}  # killed process no longer reported


def test_sudo_kill_runs_once(daemon):
    node = daemon.transports.get("node-a")
    SudoProcessKillingBehaviour(daemon.transports).trigger_action(
        {"INTRUDER_USERNAME": "x", "VIOLATION_PIDS": {"node-a": {7, 8}}})
    assert node.killed == [(7, None, True), (8, None, True)]
    assert sum(1 for c, _ in node.calls if "kill" in c) == 1


def test_message_behaviour_skips_hosts_without_tty(daemon):
    """Reference bug: one host without a terminal aborted the remaining hosts."""
    a, b = daemon.transports.get("node-a"), daemon.transports.get("node-b")
    b.ttys = [("intruder", "pts/2")]
    MessageSendingBehaviour(daemon.transports).trigger_action(
        {"INTRUDER_USERNAME": "intruder", "GPUS": "x", "HOSTNAMES": ["node-a", "node-b"]})
    assert a.tty_messages == [] and [t for t, _ in b.tty_messages] == ["pts/2"]


class FakeSMTP:
    sent = []

    def __init__(self, host, port):
        self.host, self.port = host, port

    def ehlo(self):
        pass

    def starttls(self):
        pass

    def login(self, u, p):
        self.user = u

    def sendmail(self, frm, to, msg):
        FakeSMTP.sent.append((frm, to, msg))

    def quit(self):
        pass


def test_email_behaviour_timers(cfg, tables, new_user):
    import dataclasses

    FakeSMTP.sent = []
    mb = dataclasses.replace(cfg.mailbot, smtp_server="smtp.example.org", smtp_port=587, smtp_login="bot@example.org",
                             smtp_password="pw", notify_admin=True, notify_intruder=True,
                             admin_email="admin1@example.org, admin2@example.org", interval=10,
                             max_emails_per_protection_interval=50)
    beh = EmailSendingBehaviour(mb, smtp_factory=FakeSMTP)
    data = {"INTRUDER_USERNAME": "administrantee", "GPUS": "node-a - GPU0: MI355X", "OWNERS": "x (y)",
            "HOSTNAMES": ["node-a"], "RESERVATIONS": []}
    beh.trigger_action(dict(data))
    to = sorted(t for _, t, _ in FakeSMTP.sent)
    assert to == ["admin1@example.org", "admin2@example.org", "administrantee@example.org"]
    beh.trigger_action(dict(data))  # within the resend interval -> nothing new
    assert len(FakeSMTP.sent) == 3


def test_email_behaviour_incomplete_config_is_noop(cfg, tables):
    FakeSMTP.sent = []
    beh = EmailSendingBehaviour(cfg.mailbot, smtp_factory=FakeSMTP)
    beh.trigger_action({"INTRUDER_USERNAME": "nobody", "GPUS": "g"})
    assert FakeSMTP.sent == []


def test_mailer_and_message():
    from tensorhive_fixed_amd.core.mailer import Mailer, Message

    with pytest.raises(AssertionError):
        Mailer("foo", 123).send(Message("a", "b", "c", "d"))
    m = Message(author="foo", to=["foo", "bar", "fizz"], subject="s", body="b")
    assert m.recipients == "foo, bar, fizz"
    mailer = Mailer("smtp", 1, smtp_factory=FakeSMTP)
    mailer.connect("u", "p")
    with pytest.raises(AssertionError):
        mailer.send(Message(None, None, None, None))
    FakeSMTP.sent = []
    mailer.send(Message(author="foo", to="bar", subject="foo", body="bar"))
    assert len(FakeSMTP.sent) == 1


# ------------------------------------------------------------------------- usage logging
@pytest.mark.parametrize("action,expect", [(0, None), (1, ".{id}.json"), (2, "old_{id}.json")])
def test_usage_logging_lifecycle(daemon, new_user, tmp_path, action, expect):
    res = gpu(daemon)
    r = reserve(new_user, res, UTC() - timedelta(minutes=40), timedelta(hours=1))
    daemon.stub.util_override[("node-a", 0)] = 50.0
    publish(daemon)
    svc = UsageLoggingService(1.0, str(tmp_path / "usage"), action)
    svc.inject(daemon)
    svc.do_run()
    daemon.stub.util_override[("node-a", 0)] = 100.0
    publish(daemon)
    svc.do_run()
    doc = json.loads((tmp_path / "usage" / f"{r.id}.json").read_text())
    assert doc["metrics"]["utilization"]["values"] == [50.0, 100.0] and len(doc["timestamps"]) == 2
    assert doc["metrics"]["power"]["values"]  # MI355X extras are logged too
    r._end = UTC() - timedelta(seconds=1)  # the reservation ends
    r.save()
    svc.handle_expired_logs()
    assert Reservation.get(r.id).gpu_util_avg == 75 and Reservation.get(r.id).mem_util_avg == 45
    summary = json.loads((tmp_path / "usage" / f"{r.id}.summary.json").read_text())
    assert summary["utilization"] == 75
    assert not (tmp_path / "usage" / f"{r.id}.json").exists()
    if expect:
        assert (tmp_path / "usage" / expect.format(id=r.id)).exists()


def test_usage_logging_drops_logs_of_deleted_reservations(daemon, tmp_path):
    d = tmp_path / "usage"
    d.mkdir()
    (d / "999.json").write_text("{}")
    svc = UsageLoggingService(1.0, str(d), 0)
    svc.inject(daemon)
    svc.handle_expired_logs()
    assert not (d / "999.json").exists()


# ------------------------------------------------------------------------- job scheduling
def _task(job, host, gpus, command="python train.py"):
    t = Task(command=command, hostname=host)
    t.save()
    seg = CommandSegment.query.filter(CommandSegment.name == "HIP_VISIBLE_DEVICES").first() or \
        CommandSegment(name="HIP_VISIBLE_DEVICES", segment_type=SegmentType.env_variable)
    t.add_cmd_segment(seg, gpus)
    job.add_task(t)
    return t


def _queued(user, *tasks, name="q"):
    j = Job(name=name, description="", user_id=user.id)
    j.save()
    for host, gpus in tasks:
        _task(j, host, gpus)
    j.enqueue()
    return j


@pytest.fixture()
def sched(daemon, new_user, permissive_restriction):
    permissive_restriction.apply_to_user(new_user)
    for h in ("node-a", "node-b"):
        for i in range(8):
            gpu(daemon, h, i)
    publish(daemon)
    s = JobSchedulingService(3600.0, 5, 30)
    daemon.add_service(s)
    return s


def test_queued_job_runs_on_free_gpus(sched, daemon, new_user):
    j = _queued(new_user, ("node-a", "0,1"), ("node-b", "0"))
    sched.do_run()
    j = Job.get(j.id)
    assert j.status is JobStatus.running and all(t.status is TaskStatus.running for t in j.tasks)
    procs = daemon.stub.sample("node-a")["GPU"][daemon.stub.gpu_uuid("node-a", 1)]["processes"]
    assert procs and procs[0]["task_id"] == str(j.tasks[0].id)
    assert j in Job.get_jobs_running_from_queue()


def test_gang_scheduling_is_all_or_nothing(sched, daemon, new_user):
    daemon.stub.add_process("node-b", 0, 999, "someone")
    publish(daemon)
    j = _queued(new_user, ("node-a", "0"), ("node-b", "0"))
    sched.do_run()
    assert Job.get(j.id).status is JobStatus.pending
    assert daemon.transports.get("node-a").sessions == {}  # nothing half-started


def test_queue_respects_other_users_reservations(sched, daemon, new_user, new_admin):
    reserve(new_admin, gpu(daemon, "node-a", 2), UTC() + timedelta(minutes=10), timedelta(hours=1))
    blocked = _queued(new_user, ("node-a", "2"), name="blocked")
    sched.do_run()
    assert Job.get(blocked.id).status is JobStatus.pending
    reserve(new_user, gpu(daemon, "node-a", 3), UTC() + timedelta(minutes=10), timedelta(hours=1))
    own = _queued(new_user, ("node-a", "3"), name="own")
    sched.do_run()
    assert Job.get(own.id).status is JobStatus.running  # the owner's own reservation does not block


def test_two_queued_jobs_do_not_share_a_gpu(sched, new_user):
    a = _queued(new_user, ("node-a", "4"), name="a")
    b = _queued(new_user, ("node-a", "4,5"), name="b")
    sched.do_run()
    assert Job.get(a.id).status is JobStatus.running and Job.get(b.id).status is JobStatus.pending
    sched.do_run()  # the task is known to be running even before monitoring shows it
    assert Job.get(b.id).status is JobStatus.pending


def test_scheduled_start_and_stop(sched, daemon, new_user):
    j = Job(name="timed", description="", user_id=new_user.id, start_at=UTC() + timedelta(hours=1))
    j.save()
    _task(j, "node-a", "6")
    sched.do_run()
    assert Job.get(j.id).status is JobStatus.not_running
    j._start_at = UTC() - timedelta(seconds=1)
    j._stop_at = UTC() + timedelta(hours=1)
    j.save()
    sched.do_run()
    j = Job.get(j.id)
    assert j.status is JobStatus.running and j.start_at is None
    j._stop_at = UTC() - timedelta(seconds=1)
    j.save()
    sched.do_run()
    from tensorhive_fixed_amd.controllers import task as task_ctl

    task_ctl.synchronize(j.tasks[0].id)
    assert Job.get(j.id).status is JobStatus.terminated


def test_queued_job_stopped_on_contention(sched, daemon, new_user):
    j = _queued(new_user, ("node-b", "7"))
    sched.do_run()
    assert Job.get(j.id).status is JobStatus.running
    daemon.stub.add_process("node-b", 7, 31337, "intruder")
    publish(daemon)
    sched.do_run()
    from tensorhive_fixed_amd.controllers import task as task_ctl

    task_ctl.synchronize(Job.get(j.id).tasks[0].id)
    assert Job.get(j.id).status is JobStatus.terminated


def test_event_driven_wake(sched, daemon, new_user):
    """The scheduler thread sleeps for an hour but an enqueue wakes it immediately."""
    sched.start()
    time.sleep(0.2)
    j = _queued(new_user, ("node-a", "7"))
    t0 = time.time()
    daemon.wake("enqueue")
    while time.time() - t0 < 5 and not any(jid == j.id for jid, _ in sched.launch_log):
        time.sleep(0.01)
    assert any(jid == j.id for jid, _ in sched.launch_log)
    assert time.time() - t0 < 2.0


def test_greedy_scheduler_unit():
    from tensorhive_fixed_amd.core.scheduling import GreedyScheduler

    class T:
        def __init__(self, host, env):
            self.hostname = host
            self._env = env

        def envs(self):
            return [("HIP_VISIBLE_DEVICES", self._env)]

        gpu_id = None
        command = "x"

    class J:
        def __init__(self, *tasks):
            self.tasks = list(tasks)
            self.user_id = 1

    slots = {"h": {"u0": None, "u1": 5, "u2": 60}}
    s = GreedyScheduler(30, own_reservations=lambda u, j, w: False)
    ok, busy, long_enough = J(T("h", "0")), J(T("h", "1")), J(T("h", "2"))
    dup = J(T("h", "0"))
    assert s.schedule_jobs({ok: None, busy: None, long_enough: None, dup: None}, slots) == [ok, long_enough]


def test_monitoring_wakes_the_scheduler_when_a_gpu_is_freed(daemon):
    """A device that loses its last process wakes the job scheduler (queued jobs start at the next
    telemetry sample, not at the scheduler's periodic tick); a host that stops answering does not."""
    woken = []
    daemon.wake = lambda reason="": woken.append(reason)
    mon = MonitoringService(1.0, daemon.backends)
    mon.inject(daemon)
    daemon.stub.add_process("node-a", 3, 4242, "alice")
    mon.do_run()
    assert woken == []
    mon.do_run()
    assert woken == []  # still busy
    daemon.stub.clear_processes("node-a")
    mon.do_run()
    assert woken == ["gpu_freed"]
    daemon.stub.add_process("node-a", 3, 4243, "alice")
    mon.do_run()
    daemon.stub.down.add("node-a")
    mon.do_run()
    assert woken == ["gpu_freed"]


def test_device_freed_wake_rechecks_while_jobs_wait(sched):
    """After a "device freed" wake-up the scheduler re-checks every FAST_RECHECK_S (the exit may
    reach th-run's state after the process left the device) while queued jobs remain, within the
    window only; otherwise it sleeps its interval."""
    sched.interval = 3600.0
    assert sched.next_wait(0.0) == 3600.0
    sched._queue_left = 2
    assert sched.next_wait(0.0) == 3600.0  # no device was freed
    sched.device_freed()
    assert sched.next_wait(0.0) == sched.FAST_RECHECK_S
    sched._queue_left = 0
    assert sched.next_wait(0.0) == 3600.0  # nothing waits
    sched._idle_claims = True
    assert sched.next_wait(0.0) == sched.FAST_RECHECK_S  # a finished task not yet seen as ended
    sched._idle_claims = False
    sched._queue_left = 1
    sched._fast_until = 0.0
    assert sched.next_wait(0.0) == 3600.0  # window over
