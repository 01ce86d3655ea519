"""Task attribution against REAL th-run sessions (``core/attribution.py``; round-4 verdict item 1).

th-run records the session id, uid and user of every task; a process claiming the task through
``TENSORHIVE_TASK_ID`` is accepted only inside that session (or below its monitor) and as that
uid.  These tests read the same /proc facts libthsmi reports (``native/thsmi.cpp::resolve_pid``)."""
import json
import os
import shutil
import subprocess
import sys
import time

import pytest

from tensorhive_fixed_amd.core import attribution
from tensorhive_fixed_amd.native.build import build_all, path_of

native = pytest.mark.skipif(shutil.which("g++") is None, reason="needs a C++ compiler for th-run")


def proc_facts(pid: int) -> dict:
    """What libthsmi reports for a pid: uid, sid, pgid and the parent chain."""
    stat = open(f"/proc/{pid}/stat").read()
    f = stat[stat.rindex(")") + 2:].split()
    ppid, pgid, sid = int(f[1]), int(f[2]), int(f[3])
    anc, cur = [], ppid
    while cur > 1 and len(anc) < 64:
        anc.append(cur)
        s = open(f"/proc/{cur}/stat").read()
        cur = int(s[s.rindex(")") + 2:].split()[1])
    return {"pid": pid, "uid": os.stat(f"/proc/{pid}").st_uid, "sid": sid, "pgid": pgid, "ancestors": anc,
            "task_id": "41"}


def _th_run(*args, state):
    return subprocess.run([str(path_of("th-run")), args[0], "--state-dir", str(state), *args[1:]],
                          capture_output=True, text=True, timeout=30)


def _wait_child(pid: int, timeout: float = 10.0) -> int:
    """pid of the first child of ``pid`` (the task's own forked rank)."""
    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            kids = open(f"/proc/{pid}/task/{pid}/children").read().split()
        except OSError:
            kids = []
        if kids:
            return int(kids[0])
        time.sleep(0.05)
    raise AssertionError("no child")


@native
def test_th_run_session_attests_its_processes_and_not_a_forger(tmp_path):
    build_all(strict=False)
    state = tmp_path / "state"
    # the task forks a rank that calls setsid (leaves the session) -> attested by parent chain
    script = ("import os,subprocess,sys,time; "
              "subprocess.Popen([sys.executable,'-c','import time; time.sleep(60)'], start_new_session=True); "
              "time.sleep(60)")
    r = _th_run("spawn", "--name", "tensorhive_task_41", "--log", str(tmp_path / "t.log"),
                "--env", "TENSORHIVE_TASK_ID=41", "--", sys.executable, "-c", script, state=state)
    assert r.returncode == 0, r.stderr
    pid = int(r.stdout.strip().splitlines()[-1])
    forger = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(60)"],
                              env={**os.environ, "TENSORHIVE_TASK_ID": "41"}, start_new_session=True)
    try:
        sess = json.loads(_th_run("status", "--name", "tensorhive_task_41", state=state).stdout)
        assert sess["sid"] == os.getsid(pid) and sess["uid"] == os.getuid() and sess["user"]
        assert sess["sid"] != pid  # the task leads its own process GROUP, inside th-run's session
        reg = attribution.SessionRegistry()
        reg.record("n", sess)
        rank = _wait_child(pid)
        assert os.getsid(rank) == rank  # left the session ...
        assert attribution.check(proc_facts(pid), reg.get("n", "41")) is None
        assert attribution.check(proc_facts(rank), reg.get("n", "41")) is None  # ... still below the monitor
        why = attribution.check(proc_facts(forger.pid), reg.get("n", "41"))
        assert why == "not in the task's th-run session"
        other_uid = dict(proc_facts(pid), uid=os.getuid() + 1)
        assert "uid" in attribution.check(other_uid, reg.get("n", "41"))
        # what the daemon sees end to end: a GPU entry with all three claiming task 41
        entry = {"GPU": {"u": {"index": 0, "bdf": "b", "metrics": {},
                               "processes": [proc_facts(pid), proc_facts(rank), proc_facts(forger.pid)]}}}
        attribution.Attestor(reg).attest_entry("n", entry)
        got = {p["pid"]: p["task_id"] for p in entry["GPU"]["u"]["processes"]}
        assert got == {pid: "41", rank: "41", forger.pid: None}
    finally:
        forger.kill()
        forger.wait()
        _th_run("kill", "--name", "tensorhive_task_41", state=state)


@native
def test_spawn_records_the_session_in_the_same_round_trip(tmp_path, monkeypatch):
    """``task_nursery.spawn`` on a local node prints th-run's status after the pid: the registry
    knows the new session before the first telemetry sample."""
    from tensorhive_fixed_amd.core import task_nursery
    from tensorhive_fixed_amd.core.transport import LocalTransport, TransportManager

    build_all(strict=False)
    monkeypatch.setenv("TH_RUN_STATE_DIR", str(tmp_path / "state"))
    th = str(path_of("th-run"))
    monkeypatch.setattr(task_nursery, "_th_run", lambda host: th)
    monkeypatch.setattr(task_nursery, "log_path", lambda tid: str(tmp_path / f"task_{tid}.log"))
    tm = TransportManager({"localnode": LocalTransport("localnode")})
    task_nursery.use_transports(tm)
    try:
        attribution.REGISTRY.forget("localnode", "77")
        pid = task_nursery.spawn("sleep 30", "localnode", None, name_appendix="77")
        rec = attribution.REGISTRY.get("localnode", "77")
        assert rec is not None and rec["sid"] == os.getsid(pid) and rec["uid"] == os.getuid()
        task_nursery.terminate(pid, "localnode", None, gracefully=False)
        t0 = time.time()
        while task_nursery.running("localnode", None) and time.time() - t0 < 10:
            time.sleep(0.05)
    finally:
        task_nursery.use_transports(None)


def test_many_forged_task_ids_do_not_become_many_lookups():
    """Claims are free to forge: 500 processes each claiming a different unknown task id trigger at
    most Attestor.MAX_LOOKUPS_PER_S session lookups per second, and the bookkeeping stays bounded."""
    from tensorhive_fixed_amd.core.attribution import Attestor, SessionRegistry

    calls = []
    att = Attestor(SessionRegistry(), lookup=lambda host, tid: calls.append(tid), refetch_s=5.0)
    entry = {"GPU": {"g0": {"processes": [{"pid": 10000 + i, "uid": 1001, "owner": "mallory", "sid": 10000 + i,
                                            "task_id": str(i)} for i in range(500)]}}}
    att.attest_entry("node-x", entry)
    assert len(calls) <= Attestor.MAX_LOOKUPS_PER_S
    assert all(p["task_id"] is None for p in entry["GPU"]["g0"]["processes"])
    for i in range(6000):  # warning bookkeeping for many distinct pids stays bounded
        att.verify("node-x", {"pid": 20000 + i, "uid": 1001, "sid": 1, "task_id": "x"})
    assert len(att._warned) <= Attestor._MAX_TRACKED
