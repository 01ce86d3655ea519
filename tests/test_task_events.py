"""Task exit as an event (``core/events.py``; round-4 verdict item 5).

th-run sends one datagram when a task has exited; the daemon samples that host and runs the
scheduler at once, so a queued job takes the freed devices without waiting for the periodic tick
(30 s in the reference, ``tensorhive/core/services/JobSchedulingService.py:286-297``) or for
re-polling th-run."""
import json
import os
import shutil
import socket
import subprocess
import sys
import time

import pytest

from tensorhive_fixed_amd.core.events import EventListener, open_event_socket, parse_event
from tensorhive_fixed_amd.models.orm import Job, JobStatus
from tensorhive_fixed_amd.native.build import build_all, path_of
from tests.test_allocation import _job, world  # noqa: F401  (fixture re-export)

native = pytest.mark.skipif(shutil.which("g++") is None, reason="needs a C++ compiler for th-run")


@native
def test_th_run_notifies_after_its_state_says_exited(tmp_path):
    build_all(strict=False)
    got = []

    def on(ev):
        # the state file already says exited when the event arrives
        st = json.loads(subprocess.run([str(path_of("th-run")), "status", "--name", ev["name"], "--state-dir",
                                        str(tmp_path)], capture_output=True, text=True).stdout)
        got.append((time.time(), ev, st))

    lst = EventListener(on)
    try:
        assert oct(os.stat(lst.path).st_mode & 0o777) == "0o666"
        r = subprocess.run([str(path_of("th-run")), "spawn", "--name", "tensorhive_task_5", "--log",
                            str(tmp_path / "t.log"), "--state-dir", str(tmp_path), "--notify", lst.path, "--",
                            "bash", "-c", "sleep 0.3; exit 3"], capture_output=True, text=True, timeout=30)
        assert r.returncode == 0
        t0 = time.time()
        while not got and time.time() - t0 < 10:
            time.sleep(0.01)
        assert got, "no task-exit event"
        at, ev, st = got[0]
        assert ev["event"] == "task_exit" and ev["name"] == "tensorhive_task_5" and ev["exit_code"] == 3
        assert st["status"] == "exited" and st["exit_code"] == 3 and st["ended_ms"] == ev["ended_ms"]
        assert at * 1000 - ev["ended_ms"] < 1000  # delivered at once
    finally:
        lst.close()
    assert not os.path.exists(lst.path)


def test_garbage_datagrams_are_ignored(tmp_path):
    seen = []
    lst = EventListener(seen.append)
    try:
        c = socket.socket(socket.AF_UNIX, socket.SOCK_DGRAM)
        for msg in (b"x", b"[1]", b'{"event": "other"}', b'{"event": "task_exit", "name": "tensorhive_task_1"}'):
            c.sendto(msg, lst.path)
        t0 = time.time()
        while not seen and time.time() - t0 < 5:
            time.sleep(0.01)
        assert [e["name"] for e in seen] == ["tensorhive_task_1"] and lst.received == 1
    finally:
        lst.close()
    assert parse_event(b"{") is None


def test_node_socket_refuses_a_foreign_path(tmp_path):
    squat = tmp_path / "events.sock"
    squat.write_text("not a socket")
    with pytest.raises(OSError):
        open_event_socket(str(squat))


def test_queued_job_starts_on_the_exit_event_without_a_tick(world):
    """A one-device queue on a busy GPU: the job's exit is the only trigger -- the scheduler's
    period is an hour and no monitoring service is running."""
    from tensorhive_fixed_amd.core.services import JobSchedulingService, MonitoringService

    d, users, uuids = world
    node = d.transports.get("node-a")
    mon = MonitoringService(3600.0, d.backends)
    d.add_service(mon)
    sched = JobSchedulingService(3600.0, 5, 30)
    d.add_service(sched)
    first = _job(users["alice"], "auto:8", name="first")
    first.enqueue()
    sched.do_run()
    assert Job.get(first.id).status is JobStatus.running
    second = _job(users["bob"], "auto:8", name="second")
    second.enqueue()
    sched.start()
    try:
        time.sleep(0.3)
        assert Job.get(second.id).status is JobStatus.pending  # all 8 GPUs are taken
        pid = Job.get(first.id).tasks[0].pid
        t0 = time.time()
        node.exit_task(pid)  # th-run would send the datagram now
        while time.time() - t0 < 5:
            from tensorhive_fixed_amd.database import db_session

            db_session.expire_all()
            if Job.get(second.id).status is JobStatus.running:
                break
            time.sleep(0.01)
        assert Job.get(second.id).status is JobStatus.running
        assert time.time() - t0 < 2.0
        assert d.task_events and d.task_events[-1][2]["name"].startswith("tensorhive_task_")
    finally:
        sched.stop()
        sched.join(5)


def test_spawn_passes_the_event_socket(world, monkeypatch):
    from tensorhive_fixed_amd.core import task_nursery

    d, users, _ = world
    cmd = task_nursery.build_spawn_command("python t.py", 9, "th-run", notify="/run/x.sock")
    assert " --notify /run/x.sock " in cmd
    assert "--notify" not in task_nursery.build_spawn_command("python t.py", 9, "th-run")
    # simulated nodes report exits in-process; local nodes get the daemon's listener socket
    assert d.event_socket_for("node-a") is None


def test_agent_forwards_exit_events(tmp_path):
    """Remote nodes: the node agent listens on the node's socket, samples at once and forwards the
    event on its stream, after a fresh entry."""
    sock = str(tmp_path / "ev.sock")
    p = subprocess.Popen([sys.executable, "-m", "tensorhive_fixed_amd.agent", "--stream", "2000", "--backend", "stub",
                          "--stub-gpus", "1", "--host", "n9", "--events", sock], stdout=subprocess.PIPE, text=True,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    try:
        bound = json.loads(p.stdout.readline())
        assert bound["events_socket"] == sock  # reported before the first entry
        first = json.loads(p.stdout.readline())
        assert "entry" in first
        t0 = time.time()
        while not os.path.exists(sock) and time.time() - t0 < 10:
            time.sleep(0.02)
        c = socket.socket(socket.AF_UNIX, socket.SOCK_DGRAM)
        t_send = time.time()
        c.sendto(b'{"event": "task_exit", "name": "tensorhive_task_3", "exit_code": 0}', sock)
        a = json.loads(p.stdout.readline())
        b = json.loads(p.stdout.readline())
        assert "entry" in a and b["event"]["name"] == "tensorhive_task_3"
        assert time.time() - t_send < 1.0  # not after the 2 s period
    finally:
        p.terminate()
        p.wait(10)
    assert not os.path.exists(sock)


def test_an_event_flood_is_not_a_sampling_flood(world, monkeypatch):
    """The node socket takes datagrams from any local user: 200 events in a burst re-sample the host
    (and wake the scheduler) a bounded number of times -- at most once per Daemon.EVENT_SAMPLE_MIN_S,
    plus one trailing sample at the end of the burst, so the last event is never left unseen."""
    from tensorhive_fixed_amd.core.services import MonitoringService

    d, _, _ = world
    mon = MonitoringService(3600.0, d.backends)
    d.add_service(mon)
    samples, wakes = [], []
    monkeypatch.setattr(mon, "sample_host", lambda host: samples.append(host))
    monkeypatch.setattr(d, "wake", lambda reason="": wakes.append(reason))
    t0 = time.time()
    for i in range(200):
        d.on_task_event("node-a", {"event": "task_exit", "name": f"x{i}"})
    elapsed = time.time() - t0
    time.sleep(3 * d.EVENT_SAMPLE_MIN_S)  # the trailing sample of the burst
    assert len(d.task_events) == 200
    assert 2 <= len(samples) <= 3 + int(elapsed / d.EVENT_SAMPLE_MIN_S)
    assert len(samples) == len(wakes) and len(samples) < 50
    assert time.time() - t0 < 2.0


def test_agent_coalesces_an_event_flood(tmp_path):
    """A burst of 300 datagrams at the node agent turns into a bounded number of samples (one per
    agent.EVENT_MIN_GAP_S at most) and at most agent.MAX_EVENTS_PER_SAMPLE events per sample."""
    import threading

    from tensorhive_fixed_amd import agent

    sock = str(tmp_path / "ev.sock")
    p = subprocess.Popen([sys.executable, "-m", "tensorhive_fixed_amd.agent", "--stream", "5000", "--backend", "stub",
                          "--stub-gpus", "1", "--host", "n9", "--events", sock], stdout=subprocess.PIPE, text=True,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    try:
        assert json.loads(p.stdout.readline())["events_socket"] == sock
        assert "entry" in json.loads(p.stdout.readline())
        t0 = time.time()
        while not os.path.exists(sock) and time.time() - t0 < 10:
            time.sleep(0.02)
        c = socket.socket(socket.AF_UNIX, socket.SOCK_DGRAM)
        t_send = time.time()
        for i in range(300):
            c.sendto(json.dumps({"event": "task_exit", "name": f"t{i}"}).encode(), sock)
        burst = time.time() - t_send
        lines: list[dict] = []
        reader = threading.Thread(target=lambda: [lines.append(json.loads(ln)) for ln in p.stdout], daemon=True)
        reader.start()
        time.sleep(1.0)
        docs = list(lines)
        entries = sum("entry" in d for d in docs)
        events = sum("event" in d for d in docs)
        assert events >= 1
        assert entries <= 3 + int((burst + 1.0) / agent.EVENT_MIN_GAP_S)
        assert events <= entries * agent.MAX_EVENTS_PER_SAMPLE
    finally:
        p.terminate()
        p.wait(10)


def test_agent_auto_socket_is_private_and_reported(tmp_path):
    """``--events auto`` binds in a fresh 0711 directory (no other user can pre-create or swap the
    socket) and reports the path; the directory is gone when the agent exits."""
    env = {**os.environ, "XDG_RUNTIME_DIR": str(tmp_path)}
    p = subprocess.Popen([sys.executable, "-m", "tensorhive_fixed_amd.agent", "--stream", "2000", "--backend", "stub",
                          "--stub-gpus", "1", "--host", "n9", "--events", "auto"], stdout=subprocess.PIPE, text=True,
                         env=env, cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    try:
        sock = json.loads(p.stdout.readline())["events_socket"]
        d = os.path.dirname(sock)
        assert os.path.dirname(d) == str(tmp_path) and os.path.basename(d).startswith("tensorhive-events-")
        assert (os.stat(d).st_mode & 0o777) == 0o711
        assert "entry" in json.loads(p.stdout.readline())
        c = socket.socket(socket.AF_UNIX, socket.SOCK_DGRAM)
        c.sendto(b'{"event": "task_exit", "name": "tensorhive_task_4", "exit_code": 0}', sock)
        json.loads(p.stdout.readline())
        assert json.loads(p.stdout.readline())["event"]["name"] == "tensorhive_task_4"
    finally:
        p.terminate()
        p.wait(10)
    assert not os.path.exists(d)


def test_squatted_socket_path_is_never_handed_to_tasks(tmp_path):
    """An explicit path another process already holds: the agent warns and binds nothing, so it reports no
    socket and the daemon passes no --notify path for that node (exits are found by polling)."""
    from tensorhive_fixed_amd.core.telemetry import RemoteBackend

    squat = str(tmp_path / "ev.sock")
    with open(squat, "w") as f:
        f.write("not a socket")
    argv = [sys.executable, "-m", "tensorhive_fixed_amd.agent", "--stream", "300", "--backend", "stub", "--stub-gpus",
            "1", "--host", "n9", "--events", squat]

    class T:
        def get(self, host):
            return self

        def stream_argv(self, cmd):
            return argv

    b = RemoteBackend(T(), stream_ms=300, mode="agent")
    try:
        t0 = time.time()
        while b.sample("n9") is None and time.time() - t0 < 20:
            time.sleep(0.1)
        assert b.sample("n9") is not None
        assert b.event_socket("n9") is None
    finally:
        b.close()
    # and a well-behaved agent's reported path is what the backend hands out
    argv[-1] = str(tmp_path / "ok.sock")
    b = RemoteBackend(T(), stream_ms=300, mode="agent")
    try:
        t0 = time.time()
        while b.event_socket("n9") is None and time.time() - t0 < 20:
            b.sample("n9")
            time.sleep(0.1)
        assert b.event_socket("n9") == str(tmp_path / "ok.sock")
    finally:
        b.close()
