"""Task restart policy (SURVEY §5 failure-recovery row; round-1 verdict missing item 6).

``th-run spawn --max-restarts N`` starts a run that exited non-zero again (new pid, same log and
session), at most N times, and never after a stop requested through th-run.  The daemon keeps
the task ``running`` across a restart, follows the new pid and keeps the GPU claim; when the
restarts are used up the task ends and its devices are released."""
import getpass
import shutil
import subprocess
import time

import pytest

from tensorhive_fixed_amd.models.orm import GpuAllocation, Job, TaskStatus
from tensorhive_fixed_amd.native.build import build_all, path_of
from tests.test_allocation import _execute, _job, world  # noqa: F401  (fixture re-export)

native = pytest.mark.skipif(shutil.which("g++") is None, reason="needs a C++ compiler for th-run")


def _th_run(*args, state):
    return subprocess.run([str(path_of("th-run")), args[0], "--state-dir", str(state), *args[1:]],
                          capture_output=True, text=True, timeout=30)


def _status(name, state):
    import json

    return json.loads(_th_run("status", "--name", name, state=state).stdout)


@native
def test_th_run_restarts_a_failing_run_up_to_the_limit(tmp_path):
    build_all(strict=False)
    log = tmp_path / "t.log"
    r = _th_run("spawn", "--name", "t1", "--log", str(log), "--max-restarts", "2", "--restart-delay", "0.1",
                "--", "bash", "-c", "echo run $TH_RUN_RESTART; exit 3", state=tmp_path)
    first = int(r.stdout.strip())
    assert _th_run("wait", "--name", "t1", "--timeout", "15", state=tmp_path).returncode == 3
    st = _status("t1", tmp_path)
    assert st["restarts"] == 2 and st["exit_code"] == 3 and st["first_pid"] == first and st["pid"] != first
    lines = log.read_text().splitlines()
    assert [l for l in lines if l.startswith("run")] == ["run 0", "run 1", "run 2"]
    assert sum("restart" in l for l in lines) == 2


@native
def test_th_run_success_is_not_restarted(tmp_path):
    build_all(strict=False)
    _th_run("spawn", "--name", "ok", "--log", str(tmp_path / "ok.log"), "--max-restarts", "3",
            "--", "true", state=tmp_path)
    assert _th_run("wait", "--name", "ok", "--timeout", "15", state=tmp_path).returncode == 0
    assert _status("ok", tmp_path)["restarts"] == 0


@native
def test_requested_stop_is_never_restarted_and_pid_signals_follow_restarts(tmp_path):
    build_all(strict=False)
    r = _th_run("spawn", "--name", "t3", "--log", str(tmp_path / "t3.log"), "--max-restarts", "5",
                "--restart-delay", "0.1", "--", "bash", "-c", "sleep 30", state=tmp_path)
    first = int(r.stdout.strip())
    time.sleep(0.3)
    subprocess.run(["kill", "-9", "--", f"-{first}"], check=True)  # a crash (e.g. the OOM killer)
    t0 = time.time()
    while time.time() - t0 < 10 and _status("t3", tmp_path).get("restarts") != 1:
        time.sleep(0.05)
    st = _status("t3", tmp_path)
    assert st["restarts"] == 1 and st["alive"] and st["pid"] != first
    # the daemon only knows the spawn-time pid: a stop through it reaches the current run
    assert _th_run("terminate", "--pid", str(first), state=tmp_path).returncode == 0
    assert _th_run("wait", "--name", "t3", "--timeout", "15", state=tmp_path).returncode == 143
    assert _status("t3", tmp_path)["restarts"] == 1


def test_daemon_follows_a_restarted_task_and_releases_after_the_last_failure(world):  # noqa: F811
    from tensorhive_fixed_amd.controllers import task as task_ctl

    d, users, _ = world
    node = d.transports.get("node-a")
    j = _job(users["alice"], "auto:2")
    t = j.tasks[0]
    t.set_max_restarts(1)
    assert _execute(d, j.id)[1] == 200
    t = Job.get(j.id).tasks[0]
    first = t.pid
    assert "--max-restarts 1" in next(c for c, _u in node.calls if "spawn --name" in c)
    new = node.crash_task(first, code=1)
    assert new is not None and new != first
    task_ctl.synchronize(t.id)
    t = Job.get(j.id).tasks[0]
    assert t.status is TaskStatus.running and t.pid == new
    assert t.as_dict()["restarts"] == 1 and t.as_dict()["maxRestarts"] == 1
    assert {i for _h, i in GpuAllocation.held()} == {0, 1}  # the claim survives the restart
    assert node.crash_task(new, code=1) is None  # restarts used up
    task_ctl.synchronize(t.id)
    t = Job.get(j.id).tasks[0]
    assert t.status is TaskStatus.terminated and GpuAllocation.held() == set()


def test_max_restarts_through_the_api(world, client, auth_headers):  # noqa: F811
    d, users, _ = world
    hdr = auth_headers(users["alice"])
    app = client
    r = app.post("/api/jobs", json={"name": "r", "description": "", "userId": users["alice"].id}, headers=hdr)
    jid = r.get_json()["job"]["id"]
    r = app.post(f"/api/jobs/{jid}/tasks", json={"command": "python t.py", "hostname": "node-a", "maxRestarts": 3},
                 headers=hdr)
    assert r.status_code == 201, r.get_json()
    tid = r.get_json()["task"]["id"]
    assert r.get_json()["task"]["maxRestarts"] == 3
    r = app.put(f"/api/tasks/{tid}", json={"maxRestarts": 0}, headers=hdr)
    assert r.status_code == 201 and r.get_json()["task"]["maxRestarts"] == 0
    r = app.put(f"/api/tasks/{tid}", json={"maxRestarts": -1}, headers=hdr)
    assert r.status_code in (400, 422)


def test_training_metrics_are_parsed_from_the_task_log(world, client, auth_headers):  # noqa: F811
    from tensorhive_fixed_amd.controllers.task import parse_training_lines

    assert parse_training_lines(["noise", "[th-train] step=10 loss=7.1234 tokens/s=24777.5 world=1"]) == [
        {"step": 10, "loss": 7.1234, "tokensPerSec": 24777.5, "world": 1}]
    d, users, _ = world
    node = d.transports.get("node-a")
    j = _job(users["alice"], "0")
    assert _execute(d, j.id)[1] == 200
    t = Job.get(j.id).tasks[0]
    logf = node.sessions[t.pid]["log"]
    node.logs[logf] += [f"[th-train] step={s} loss={9 - s / 10:.4f} tokens/s={24000 + s:.1f} world=8"
                        for s in (10, 20)]
    r = client.get(f"/api/tasks/{t.id}/training", headers=auth_headers(users["alice"]))
    body = r.get_json()
    assert r.status_code == 200, body
    assert [p["step"] for p in body["series"]] == [10, 20] and body["tokensPerSec"] == 24020.0
    assert client.get(f"/api/tasks/{t.id}/training", headers=auth_headers(users["bob"])).status_code == 403


@native
def test_th_run_pid_history_and_stop_between_runs(tmp_path):
    """Every incarnation's pid finds the session; a stop landing between a failed run and its
    restart succeeds (exit 0) and no further run starts (th_run.cpp:443)."""
    build_all(strict=False)
    r = _th_run("spawn", "--name", "t4", "--log", str(tmp_path / "t4.log"), "--max-restarts", "5",
                "--restart-delay", "0.1", "--", "bash", "-c", "sleep 30", state=tmp_path)
    pids = [int(r.stdout.strip())]
    for k in (1, 2):  # two crashes -> three incarnations
        time.sleep(0.3)
        subprocess.run(["kill", "-9", "--", f"-{pids[-1]}"], check=True)
        t0 = time.time()
        while time.time() - t0 < 10 and _status("t4", tmp_path).get("restarts") != k:
            time.sleep(0.05)
        pids.append(_status("t4", tmp_path)["pid"])
    st = _status("t4", tmp_path)
    assert st["restarts"] == 2 and [int(p) for p in st["pids"].split(",")] == pids
    # the MIDDLE pid (neither first nor current) still reaches the live run
    assert _th_run("terminate", "--pid", str(pids[1]), state=tmp_path).returncode == 0
    assert _th_run("wait", "--name", "t4", "--timeout", "15", state=tmp_path).returncode == 143

    r = _th_run("spawn", "--name", "t5", "--log", str(tmp_path / "t5.log"), "--max-restarts", "5",
                "--restart-delay", "2", "--", "bash", "-c", "exit 7", state=tmp_path)
    first = int(r.stdout.strip())
    t0 = time.time()
    while time.time() - t0 < 10 and _status("t5", tmp_path).get("status") != "restarting":
        time.sleep(0.02)
    assert _th_run("interrupt", "--pid", str(first), state=tmp_path).returncode == 0
    assert _th_run("wait", "--name", "t5", "--timeout", "15", state=tmp_path).returncode == 7
    assert _status("t5", tmp_path)["restarts"] == 1  # the pending restart was abandoned, no new run


def test_daemon_tracks_a_task_across_several_restarts(world, client, auth_headers):  # noqa: F811
    """after >= 2 restarts the stored pid must still resolve, the claim must be
    kept, and a stop must reach the live run -- with and without a sync between the crashes."""
    from tensorhive_fixed_amd.controllers import task as task_ctl

    d, users, _ = world
    node = d.transports.get("node-a")
    j = _job(users["alice"], "auto:2")
    t = j.tasks[0]
    t.set_max_restarts(4)
    assert _execute(d, j.id)[1] == 200
    t = Job.get(j.id).tasks[0]
    p1 = t.pid
    p2 = node.crash_task(p1, code=1)
    task_ctl.synchronize(t.id)  # the daemon sees the middle incarnation
    assert Job.get(j.id).tasks[0].pid == p2
    p3 = node.crash_task(p2, code=1)
    p4 = node.crash_task(p3, code=1)  # two crashes with no sync between them
    task_ctl.synchronize(t.id)
    t = Job.get(j.id).tasks[0]
    assert t.status is TaskStatus.running and t.pid == p4
    assert {i for _h, i in GpuAllocation.held()} == {0, 1}
    r = client.get(f"/api/jobs/{j.id}/stop", query_string={"gracefully": "true"},
                   headers=auth_headers(users["alice"]))
    assert r.status_code == 200, r.get_json()
    assert p4 not in node.sessions  # the stop reached the current run
    task_ctl.synchronize(t.id)
    t = Job.get(j.id).tasks[0]
    assert t.status is TaskStatus.terminated and GpuAllocation.held() == set()
