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


def test_attestor_bookkeeping_is_thread_safe_under_many_forged_claims():
    """publish() runs attest_entry from the monitoring pool, the event listener and the agents'
    stream readers at once.  Many threads x more forged claims than _MAX_TRACKED must neither raise nor
    exceed the lookup rate limit, and every forged claim stays rejected."""
    import threading

    from tensorhive_fixed_amd.core.attribution import Attestor, SessionRegistry

    calls = []
    lock = threading.Lock()

    def lookup(host, tid):
        with lock:
            calls.append(time.monotonic())

    att = Attestor(SessionRegistry(), lookup=lookup, refetch_s=0.0)
    n = Attestor._MAX_TRACKED + 500
    errors = []

    def worker(w):
        try:
            for chunk in range(0, n, 250):
                entry = {"GPU": {"g": {"processes": [
                    {"pid": 100000 * w + i, "uid": 1001, "owner": "mallory", "sid": 5, "task_id": f"{w}-{i}"}
                    for i in range(chunk, min(n, chunk + 250))]}}}
                att.attest_entry(f"node-{w % 3}", entry)
                assert all(p["task_id"] is None for p in entry["GPU"]["g"]["processes"])
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    t0 = time.monotonic()
    ts = [threading.Thread(target=worker, args=(w,)) for w in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors[:3]
    dt = time.monotonic() - t0
    assert len(calls) <= Attestor.MAX_LOOKUPS_PER_S * (dt + 1.0) + 1e-9, (len(calls), dt)
    assert len(att._warned) <= Attestor._MAX_TRACKED and len(att._fetched) <= Attestor._MAX_TRACKED
    assert att.rejected >= 8 * n


def test_background_lookup_never_runs_on_the_publishing_thread():
    """an unseen claim is looked up on the attestor's worker, not on the thread that publishes
    the sample; that sample carries the claim unattested (pending), the next one attests it."""
    import threading

    from tensorhive_fixed_amd.core.attribution import Attestor, SessionRegistry

    reg = SessionRegistry()
    release = threading.Event()
    seen_threads = []

    def slow_lookup(host, tid):  # an unreachable node's SSH timeout
        seen_threads.append(threading.current_thread().name)
        release.wait(5)
        reg.record(host, {"name": f"tensorhive_task_{tid}", "sid": 4242, "uid": 1000, "user": "alice",
                          "monitor_pid": 4241, "pid": 4243})

    att = Attestor(reg, lookup=slow_lookup, background=True)
    proc = {"pid": 4243, "uid": 1000, "owner": "alice", "sid": 4242, "task_id": "9"}
    entry = {"GPU": {"g": {"processes": [dict(proc)]}}}
    t0 = time.monotonic()
    att.attest_entry("n1", entry)
    assert time.monotonic() - t0 < 0.5  # did not wait for the lookup
    p = entry["GPU"]["g"]["processes"][0]
    assert p["task_id"] is None and p["claimed_task_id"] == "9" and p["attestation_pending"] is True
    # still pending: the same claim does not queue a second lookup
    att.attest_entry("n1", {"GPU": {"g": {"processes": [dict(proc)]}}})
    release.set()
    deadline = time.monotonic() + 5
    while att.pending("n1", "9") and time.monotonic() < deadline:
        time.sleep(0.01)
    entry2 = {"GPU": {"g": {"processes": [dict(proc)]}}}
    att.attest_entry("n1", entry2)
    p2 = entry2["GPU"]["g"]["processes"][0]
    assert p2["task_id"] == "9" and "attestation_pending" not in p2
    assert seen_threads == ["th-attest-lookup"]
    att.close()


def test_pending_claims_do_not_exempt_a_process_from_protection():
    """A claim whose lookup has not run yet is judged like a rejected one (by the UNIX owner)."""
    from tensorhive_fixed_amd.core.attribution import Attestor, SessionRegistry

    att = Attestor(SessionRegistry(), lookup=lambda h, t: time.sleep(0.2), background=True)
    entry = {"GPU": {"g": {"processes": [{"pid": 1, "uid": 1001, "owner": "mallory", "sid": 1, "task_id": "5"}]}}}
    att.attest_entry("n", entry)
    p = entry["GPU"]["g"]["processes"][0]
    assert p["task_id"] is None  # ProtectionService and the queue's eviction check read task_id only
    att.close()


def test_fallback_session_without_sid_or_uid_warns_once(caplog):
    from tensorhive_fixed_amd.core.attribution import Attestor, SessionRegistry

    reg = SessionRegistry()
    reg.record("n", {"name": "tensorhive_task_3", "pid": 10})  # setsid fallback: no sid / uid recorded
    att = Attestor(reg)
    with caplog.at_level("WARNING"):
        for _ in range(3):
            att.attest_entry("n", {"GPU": {"g": {"processes": [{"pid": 11, "uid": 1000, "sid": 10, "task_id": "3"}]}}})
    msgs = [r.getMessage() for r in caplog.records if "not started by th-run" in r.getMessage()]
    assert len(msgs) == 1
