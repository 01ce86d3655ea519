"""Trust boundaries (round-3 verdict item 1).

* JWT signing key: a fresh install gets a random 256-bit key; the reference's public default
  ``jwt-some-secret`` (``tensorhive/config.py:289``, ``main_config.ini:75``) and an empty key are
  refused by the daemon and by the token layer; tokens without ``exp`` are rejected.
* In-task HBM counter files in the world-writable ``/dev/shm``: taken only from a file whose owner
  owns the pid it names, whose pid is a th-run task process (``TENSORHIVE_TASK_ID``) listed by
  libthsmi on that very GPU; a GPU with an uncounted process is labelled ``partial``.
"""
import json
import os
import re
import stat
import time
from datetime import timedelta

import click
import pytest

from tensorhive_fixed_amd import config as C
from tensorhive_fixed_amd.utils import jwt


# ----------------------------------------------------------------------------- signing key
def test_fresh_install_writes_a_random_private_key(tmp_path):
    C.init_config_files(tmp_path)
    p = tmp_path / "main_config.ini"
    key = C.load_config(tmp_path).auth.secret_key
    assert re.fullmatch(r"[0-9a-f]{64}", key)
    assert stat.S_IMODE(os.stat(p).st_mode) == 0o600
    other = tmp_path / "b"
    C.init_config_files(other)
    assert C.load_config(other).auth.secret_key != key  # per install
    C.init_config_files(tmp_path)  # never overwritten
    assert C.load_config(tmp_path).auth.secret_key == key


def test_upgraded_install_with_the_public_key_is_rotated(tmp_path):
    p = tmp_path / "main_config.ini"
    p.write_text("[api]\nurl_port = 1234\n\n[auth]\nsecret_key = jwt-some-secret\njwt_blacklist_enabled = yes\n")
    assert C.secret_is_insecure(C.load_config(tmp_path).auth.secret_key)
    assert C.ensure_secret_key(p) is True
    cfg = C.load_config(tmp_path)
    assert not C.secret_is_insecure(cfg.auth.secret_key) and cfg.api.url_port == "1234"
    assert cfg.auth.blacklist_enabled is True
    assert C.ensure_secret_key(p) is False  # a real key is kept
    # the typo spelling of the reference, and a file with no [auth] section at all
    q = tmp_path / "q" / "main_config.ini"
    q.parent.mkdir()
    q.write_text("[auth]\nsecrect_key = jwt-some-secret\n")
    assert C.ensure_secret_key(q) and not C.secret_is_insecure(C.load_config(q.parent).auth.secret_key)
    r = tmp_path / "r" / "main_config.ini"
    r.parent.mkdir()
    r.write_text("[api]\nurl_port = 1\n")
    assert C.ensure_secret_key(r) and not C.secret_is_insecure(C.load_config(r.parent).auth.secret_key)


@pytest.mark.parametrize("key", ["jwt-some-secret", "", "x", "a" * 31])
def test_daemon_refuses_to_start_with_a_public_or_empty_key(cfg, monkeypatch, key):
    from tensorhive_fixed_amd.cli import refuse_insecure_secret

    monkeypatch.delenv(C.ALLOW_INSECURE_ENV, raising=False)
    cfg.auth.secret_key = key
    with pytest.raises(click.ClickException, match="secret_key"):
        refuse_insecure_secret(cfg)
    monkeypatch.setenv(C.ALLOW_INSECURE_ENV, "1")
    refuse_insecure_secret(cfg)  # tests may opt in


def test_a_long_operator_key_is_kept_and_accepted(tmp_path, cfg, monkeypatch):
    """The minimum is a length, not a pattern: the operator's own 32+ character key is neither
    replaced on startup nor refused; a short one is kept in the file but refused."""
    from tensorhive_fixed_amd.cli import refuse_insecure_secret

    monkeypatch.delenv(C.ALLOW_INSECURE_ENV, raising=False)
    p = tmp_path / "m.ini"
    for key, ok in (("k" * 32, True), ("short-but-mine", False)):
        p.write_text(f"[auth]\nsecret_key = {key}\n")
        assert C.ensure_secret_key(p) is False and key in p.read_text()
        cfg.auth.secret_key = key
        if ok:
            refuse_insecure_secret(cfg)
        else:
            with pytest.raises(click.ClickException, match="32 characters"):
                refuse_insecure_secret(cfg)


def _get_jobs(client, token):
    return client.get("/api/jobs", headers={"Authorization": f"Bearer {token}"})


def test_token_signed_with_the_old_default_is_401(client, new_admin, auth_headers):
    forged = jwt.create_token(new_admin.id, "access", "jwt-some-secret", timedelta(minutes=5), fresh=True,
                              user_claims={"roles": ["user", "admin"]})
    assert _get_jobs(client, forged).status_code == 401
    good = auth_headers(new_admin)["Authorization"].split()[1]
    assert _get_jobs(client, good).status_code == 200


def test_token_without_exp_is_401(client, new_admin, cfg):
    now = int(time.time())
    claims = {"iat": now, "nbf": now, "jti": "x" * 8, "identity": new_admin.id, "type": "access", "fresh": True,
              "user_claims": {"roles": ["user", "admin"]}}
    tok = jwt.encode(claims, cfg.auth.secret_key)
    assert _get_jobs(client, tok).status_code == 401
    with pytest.raises(jwt.MissingClaim):
        jwt.decode(tok, cfg.auth.secret_key)
    claims["exp"] = "never"
    with pytest.raises(jwt.MissingClaim):
        jwt.decode(jwt.encode(claims, cfg.auth.secret_key), cfg.auth.secret_key)


def test_no_token_is_signed_or_accepted_under_a_public_key(client, new_admin, cfg, monkeypatch):
    from tensorhive_fixed_amd.api import auth

    monkeypatch.delenv(C.ALLOW_INSECURE_ENV, raising=False)
    cfg.auth.secret_key = "jwt-some-secret"
    forged = jwt.create_token(new_admin.id, "access", "jwt-some-secret", timedelta(minutes=5), fresh=True,
                              user_claims={"roles": ["user", "admin"]})
    assert _get_jobs(client, forged).status_code == 401
    with pytest.raises(auth.InsecureSecret):
        auth.create_access_token(new_admin.id, ["admin"])
    r = client.post("/api/user/login", json={"username": new_admin.username, "password": "TEST PASSWORD"})
    assert r.status_code >= 500 or r.status_code == 401
    monkeypatch.setenv(C.ALLOW_INSECURE_ENV, "1")
    assert _get_jobs(client, forged).status_code == 200


# ----------------------------------------------------------------------------- HBM counter files
from tensorhive_fixed_amd.core import hbm  # noqa: E402

BDF0, BDF1 = "0000:05:00.0", "0000:15:00.0"


def _file(tmp_path, pid, bdf, rd, wr, name=None):
    f = tmp_path / (name or f"th-hbm-{pid}.json")
    f.write_text(json.dumps({"pid": pid, "ts_ns": int(time.time() * 1e9), "window_ms": 1000.0,
                             "gpus": [{"bdf": bdf, "rd_bytes": rd, "wr_bytes": wr}]}))
    return f


def _gpu(index, bdf, procs, est=None):
    return {"index": index, "bdf": bdf, "processes": procs,
            "metrics": {"hbm_bw": {"value": est, "unit": "GB/s"}} if est is not None else {}}


def _rates(tmp_path):
    return hbm.read_rates(str(tmp_path / "th-hbm-*.json"))


def test_counted_task_on_its_gpu_is_labelled_counters(tmp_path):
    me = os.getpid()
    _file(tmp_path, me, BDF0, 2e12, 1e12)
    m = hbm.metrics_for([_gpu(0, BDF0, [{"pid": me, "task_id": "7"}], est=900.0)], _rates(tmp_path))
    assert m[0]["hbm_bw_source"]["value"] == "counters" and m[0]["hbm_bw"]["value"] == 3000.0


def test_file_owned_by_another_uid_is_ignored(tmp_path, monkeypatch):
    me = os.getpid()
    _file(tmp_path, me, BDF0, 2e12, 1e12)
    real = hbm._proc_uid
    monkeypatch.setattr(hbm, "_proc_uid", lambda pid: (real(pid) or 0) + 1)  # the pid belongs to someone else
    r = _rates(tmp_path)
    assert r == {}
    assert hbm.metrics_for([_gpu(0, BDF0, [{"pid": me, "task_id": "7"}], est=900.0)], r) == {}


def test_pid_that_is_not_a_task_process_changes_nothing(tmp_path):
    me = os.getpid()
    _file(tmp_path, me, BDF0, 9e12, 9e12)
    gpus = [_gpu(0, BDF0, [{"pid": me, "task_id": None}], est=100.0)]
    assert hbm.metrics_for(gpus, _rates(tmp_path)) == {}


def test_pid_not_on_that_gpu_changes_nothing(tmp_path):
    me = os.getpid()
    _file(tmp_path, me, BDF1, 9e12, 9e12)  # claims traffic on GPU 1, but runs on GPU 0
    gpus = [_gpu(0, BDF0, [{"pid": me, "task_id": "3"}], est=100.0), _gpu(1, BDF1, [], est=0.0)]
    assert hbm.metrics_for(gpus, _rates(tmp_path)) == {}
    _file(tmp_path, 1, BDF1, 9e12, 9e12, name="th-hbm-init.json")  # pid 1: alive, not ours
    assert hbm.metrics_for(gpus, _rates(tmp_path)) == {}


def test_uncounted_tenant_makes_the_gpu_partial(tmp_path):
    me = os.getpid()
    _file(tmp_path, me, BDF0, 1.0e12, 0.0)  # the counted task: 1000 GB/s
    foreign = {"pid": 424242, "task_id": None}  # a tenant th-run did not start
    gpus = [_gpu(0, BDF0, [{"pid": me, "task_id": "7"}, foreign], est=2600.0)]
    m = hbm.metrics_for(gpus, _rates(tmp_path))[0]
    assert m["hbm_bw_source"]["value"] == "partial"
    assert m["hbm_bw"]["value"] == 2600.0 and m["hbm_counted"]["value"] == 1000.0
    assert m["hbm_uncounted_pids"]["value"] == 1
    gpus[0]["metrics"]["hbm_bw"]["value"] = 400.0  # the estimate never hides counted bytes
    assert hbm.metrics_for(gpus, _rates(tmp_path))[0]["hbm_bw"]["value"] == 1000.0


def test_counts_of_a_forged_task_id_are_not_accepted(tmp_path):
    """The counter files are authenticated per pid, but whether the pid is a task process is a
    CLAIM: after attestation (``core/attribution.py``) a process carrying a task id it does not
    own neither gets its counts accepted nor hides its traffic behind a ``counters`` label."""
    from tensorhive_fixed_amd.core.attribution import Attestor, SessionRegistry
    from tensorhive_fixed_amd.core.telemetry import apply_task_hbm

    me = os.getpid()
    _file(tmp_path, me, BDF0, 1.0e12, 0.0)
    reg = SessionRegistry()
    reg.record("n", {"name": "tensorhive_task_7", "sid": 1, "monitor_pid": 2, "uid": os.getuid()})

    def entry(sid):
        return {"GPU": {"u0": _gpu(0, BDF0, [{"pid": me, "task_id": "7", "uid": os.getuid(), "sid": sid}],
                                   est=2600.0)}}

    e = apply_task_hbm(entry(sid=12345), str(tmp_path / "th-hbm-*.json"))  # node view: the claim
    assert e["GPU"]["u0"]["metrics"]["hbm_bw_source"]["value"] == "counters"
    Attestor(reg).attest_entry("n", e)  # daemon view: not in task 7's session
    m = e["GPU"]["u0"]["metrics"]
    assert m["hbm_bw_source"]["value"] == "umc_activity" and m["hbm_bw"]["value"] == 2600.0
    assert "hbm_read" not in m and "_hbm" not in e["GPU"]["u0"]
    e = apply_task_hbm(entry(sid=1), str(tmp_path / "th-hbm-*.json"))  # genuinely in the session
    Attestor(reg).attest_entry("n", e)
    m = e["GPU"]["u0"]["metrics"]
    assert m["hbm_bw_source"]["value"] == "counters" and m["hbm_bw"]["value"] == 1000.0


def test_planted_fifo_symlink_and_huge_files_neither_block_nor_count(tmp_path):
    """``/dev/shm`` is world-writable: a FIFO would block a plain open, a symlink to /dev/zero or a
    huge file would make the read unbounded.  None of them is read; the real file still counts."""
    import threading

    me = os.getpid()
    _file(tmp_path, me, BDF0, 1e12, 0.0)
    os.mkfifo(tmp_path / "th-hbm-fifo.json")
    os.symlink("/dev/zero", tmp_path / "th-hbm-zero.json")
    os.symlink(tmp_path / f"th-hbm-{me}.json", tmp_path / "th-hbm-link.json")
    (tmp_path / "th-hbm-big.json").write_bytes(b" " * (hbm.MAX_FILE_BYTES + 1))
    out = {}
    t = threading.Thread(target=lambda: out.update(r=_rates(tmp_path)), daemon=True)
    t.start()
    t.join(10)
    assert not t.is_alive(), "read_rates blocked on a planted file"
    assert out["r"][BDF0]["pids"] == [me]  # the symlink to the genuine file is not read twice


def test_profiler_tasks_do_not_get_the_counter_tool(cfg, monkeypatch):
    from tensorhive_fixed_amd.cli import rocprof_prefix
    from tensorhive_fixed_amd.core import task_nursery

    monkeypatch.setattr(hbm, "tool_path", lambda: "/opt/th/libthhbm.so")
    cfg.ssh.available_nodes["localnode"] = {"transport": "local"}
    assert task_nursery.spawn_env("localnode", "python train.py")
    prof = rocprof_prefix(5, "SQ_WAVES") + " python train.py"
    assert task_nursery.spawn_env("localnode", prof) == {}
    assert task_nursery.spawn_env("localnode", "/opt/rocm/bin/rocprofv3 --stats -- ./a") == {}
    assert task_nursery.spawn_env("localnode", "TENSORHIVE_HBM_COUNTERS=0 python t.py") == {}


def test_remote_tasks_get_the_node_local_tool_when_configured(cfg):
    from tensorhive_fixed_amd.core import task_nursery

    cfg.ssh.available_nodes["gpu7"] = {"transport": "ssh", "user": "u", "port": 22}
    assert task_nursery.spawn_env("gpu7", "python t.py") == {}
    cfg.launcher.hbm_tool = "/opt/tensorhive/lib/libthhbm.so"
    assert task_nursery.spawn_env("gpu7", "python t.py") == {"ROCP_TOOL_LIBRARIES": "/opt/tensorhive/lib/libthhbm.so"}
    assert task_nursery.spawn_env("gpu7", "rocprofv3 --pmc SQ_WAVES -- python t.py") == {}
    assert task_nursery.spawn_env("node-a", "python t.py") == {}  # simulated nodes: nothing to count
