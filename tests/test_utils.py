"""Pure units: dates, JWT, password hashes, memoize, SSH helpers, config parsing, launcher
templates/placement, reservation verifier corner cases (reference ``tests/unit/test_*``)."""
import datetime
import json
import os
import stat
import time
from datetime import timedelta
from types import SimpleNamespace
from unittest.mock import patch

import pytest

from tensorhive_fixed_amd.utils import dates, jwt, passwords
from tensorhive_fixed_amd.utils.decorators import memoize


# ----------------------------------------------------------------------------- dates
def test_dates_roundtrip():
    d = dates.parse("2101-01-02T10:00:00.000Z")
    assert d == datetime.datetime(2101, 1, 2, 10) and d.tzinfo is None
    assert dates.stringify(d).endswith("+00:00")
    assert dates.try_parse(None) is None
    with pytest.raises(ValueError):
        dates.parse("2101_01_02T10:00:00.000Z")
    assert dates.try_parse(d) is d


# ----------------------------------------------------------------------------- jwt
def test_jwt_roundtrip_and_claims():
    tok = jwt.create_token(7, "access", "secret", timedelta(minutes=1), fresh=True, user_claims={"roles": ["user"]})
    c = jwt.decode(tok, "secret")
    assert c["identity"] == 7 and c["type"] == "access" and c["fresh"] is True
    assert c["user_claims"] == {"roles": ["user"]} and c["jti"] and c["exp"] > c["iat"]
    with pytest.raises(jwt.JWTError):
        jwt.decode(tok, "other-secret")
    with pytest.raises(jwt.ExpiredSignature):
        jwt.decode(tok, "secret", now=time.time() + 3600)
    head, body, sig = tok.split(".")
    with pytest.raises(jwt.JWTError):
        jwt.decode(".".join([head, body[:-2] + "AA", sig]), "secret")


# ----------------------------------------------------------------------------- passwords
def test_password_hash_format_and_verify():
    h = passwords.hash_password("correct horse", rounds=1000, salt=b"0123456789abcdef")
    assert h.startswith("$pbkdf2-sha256$1000$")
    assert passwords.verify_password("correct horse", h)
    assert not passwords.verify_password("wrong", h)
    assert not passwords.verify_password("x", "garbage")


def test_password_compatible_with_passlib_vector():
    """A hash produced by passlib's pbkdf2_sha256 (the reference's scheme) verifies here
    (vector computed with hashlib: pbkdf2_hmac('sha256', b'password', b'salt', 1000))."""
    import hashlib

    dk = hashlib.pbkdf2_hmac("sha256", b"password", b"salt", 1000)
    h = f"$pbkdf2-sha256$1000${passwords.ab64_encode(b'salt')}${passwords.ab64_encode(dk)}"
    assert passwords.verify_password("password", h)


# ----------------------------------------------------------------------------- memoize
def test_memoize_call_counts():
    calls = []

    @memoize
    def add(x, y):
        calls.append(1)
        return x + y

    assert [add(1, 2) for _ in range(10)] == [3] * 10 and len(calls) == 1

    @memoize
    def foo(a, b, c):
        calls.append(2)
        return bool(a and b and c)

    foo({"a": 1}, {"b": 2}, True)
    foo({"a": 1}, {"b": 2}, "True")  # same value, different type -> different key
    assert calls.count(2) == 2


# ----------------------------------------------------------------------------- ssh helpers
def test_dedicated_config(cfg):
    from tensorhive_fixed_amd.core import ssh

    conf, proxy = ssh.build_dedicated_config_for("node-a", "someone")
    assert conf["node-a"]["user"] == "someone" and conf["node-a"]["pkey"] == cfg.ssh.key_file
    assert proxy is None
    for host, user in ((None, None), ("node-a", None), (None, "bar")):
        with pytest.raises(AssertionError):
            ssh.build_dedicated_config_for(host, user)


@pytest.mark.skipif(not os.path.exists("/usr/bin/ssh-keygen"), reason="ssh-keygen missing")
def test_generate_key(tmp_path):
    from tensorhive_fixed_amd.core import ssh

    p = ssh.generate_key(tmp_path / "key")
    assert stat.S_IMODE(os.stat(p).st_mode) == 0o600
    pub = ssh.public_key(p)
    assert pub.startswith("ssh-")
    with pytest.raises(FileExistsError):
        ssh.generate_key(tmp_path / "key")
    ssh.generate_key(tmp_path / "key", replace=True)
    assert ssh.public_key(p) != pub
    assert ssh.authorized_keys_entry(p, "host").startswith("ssh-")


def test_parse_who():
    from tensorhive_fixed_amd.core.ssh import parse_who

    out = parse_who("alice pts/0 2026-01-01 10:00 (10.0.0.1)\nbob   tty1  2026-01-01 09:00\n\n")
    assert out == [{"USER": "alice", "TTY": "pts/0"}, {"USER": "bob", "TTY": "tty1"}]


# ----------------------------------------------------------------------------- config
def test_config_env_override_and_aliases(tmp_path, monkeypatch):
    from tensorhive_fixed_amd import config as C

    C.init_config_files(tmp_path)
    main = (tmp_path / "main_config.ini").read_text()
    main += "\n[task_scheduling_service]\nupdate_interval = 7\n"
    (tmp_path / "main_config.ini").write_text(main.replace("[job_scheduling_service]", "[unused_section]"))
    (tmp_path / "hosts_config.ini").write_text("[gpu1]\nuser = alice\nport = 2222\n[proxy_tunneling]\n"
                                               "enabled = on\nproxy_host = gw\nproxy_user = bob\n")
    monkeypatch.setenv("TENSORHIVE_MONITORING_SERVICE_UPDATE_INTERVAL", "0.25")
    c = C.load_config(tmp_path)
    assert c.monitoring.update_interval == 0.25
    assert c.job_scheduling.update_interval == 7.0  # the reference's misnamed section is honoured
    assert c.ssh.available_nodes == {"gpu1": {"user": "alice", "port": 2222, "transport": "ssh"}}
    assert c.ssh.proxy == {"proxy_host": "gw", "proxy_user": "bob", "proxy_port": 22}


def test_config_templates_have_reference_keys(tmp_path):
    import configparser

    from tensorhive_fixed_amd import config as C

    C.init_config_files(tmp_path)
    cp = configparser.ConfigParser()
    cp.read(tmp_path / "main_config.ini")
    for section in ("web_app.server", "api", "ssh", "monitoring_service", "protection_service",
                    "usage_logging_service", "job_scheduling_service", "auth", "database"):
        assert cp.has_section(section), section
    assert cp.has_section("amd_monitor") and cp.has_section("launcher")


# ----------------------------------------------------------------------------- launcher
def _snap():
    from tensorhive_fixed_amd.core.telemetry import StubBackend

    s = StubBackend(8)
    return s, {"h": s.sample("h")}, s.topology("h")


def test_attach_to_reservation_uses_hip_indices_and_numa_order():
    from tensorhive_fixed_amd.core.launcher import attach_to_reservation, torchrun_task

    stub, snap, topo = _snap()
    uuids = [stub.gpu_uuid("h", i) for i in (6, 1, 5)]
    form = torchrun_task("h", [0], "h")
    form["cmdsegments"]["envs"].append({"name": "CUDA_VISIBLE_DEVICES", "value": "0"})
    out = attach_to_reservation(form, snap, uuids, topo)
    envs = {e["name"]: e["value"] for e in out["cmdsegments"]["envs"]}
    assert envs["HIP_VISIBLE_DEVICES"] == "1,5,6" and "CUDA_VISIBLE_DEVICES" not in envs
    assert {p["name"]: p["value"] for p in out["cmdsegments"]["params"]}["--nproc_per_node="] == "3"
    assert envs["NCCL_MIN_NCHANNELS"] if "NCCL_MIN_NCHANNELS" in envs else True


def test_tf2_tasks_ports_and_config():
    from tensorhive_fixed_amd.core.launcher import tf2_tasks

    tasks = tf2_tasks([("a", "chief", 0), ("a", "worker", 1), ("b", "worker", 0)])
    cfgs = [json.loads(dict((e["name"], e["value"]) for e in t["cmdsegments"]["envs"])["TF_CONFIG"]) for t in tasks]
    assert cfgs[0]["cluster"] == {"chief": ["a:2222"], "worker": ["a:2223", "b:2222"]}
    assert [c["task"] for c in cfgs] == [{"type": "chief", "index": 0}, {"type": "worker", "index": 0},
                                        {"type": "worker", "index": 1}]


def test_pytorch_tcp_and_tf1_tasks():
    from tensorhive_fixed_amd.core.launcher import pytorch_tcp_tasks, tf1_tasks

    ts = pytorch_tcp_tasks([("a", 0), ("b", 3)], "a")
    p = {x["name"]: x["value"] for x in ts[1]["cmdsegments"]["params"]}
    assert p["--rank="] == "1" and p["--world-size="] == "2" and p["--init-method="] == "tcp://a:29500"
    ts = tf1_tasks(["a"], [("b", 0), ("c", 1)])
    assert [dict((x["name"], x["value"]) for x in t["cmdsegments"]["params"])["--job_name="] for t in ts] == \
        ["ps", "worker", "worker"]


def test_templates_never_mention_cuda():
    from tensorhive_fixed_amd.core.launcher import TEMPLATES

    assert "CUDA" not in json.dumps(TEMPLATES)


# ----------------------------------------------------------------------------- verifier
def _R(start, end=None, schedules=(), resources=(), is_global=False):
    return SimpleNamespace(starts_at=start, ends_at=end, schedules=list(schedules), resources=list(resources),
                           is_global=is_global)


def _S(days, a, b):
    return SimpleNamespace(schedule_days=days, hour_start=a, hour_end=b)


def _allowed(restrictions, start, end, res="R"):
    from tensorhive_fixed_amd.core import verifier

    user = SimpleNamespace(get_restrictions=lambda include_group=False: restrictions)
    reservation = SimpleNamespace(resource_id=res, start=start, end=end)
    with patch("tensorhive_fixed_amd.models.orm.Resource.get", return_value=res):
        return verifier.is_reservation_allowed(user, reservation)


D0 = datetime.datetime(2101, 1, 3)  # a Monday


def test_verifier_basic_windows():
    r = _R(D0, D0 + timedelta(days=2), resources=["R"])
    assert _allowed([r], D0 + timedelta(hours=1), D0 + timedelta(hours=5))
    assert not _allowed([r], D0 + timedelta(days=1), D0 + timedelta(days=3))
    assert not _allowed([_R(D0, None, resources=["other"])], D0 + timedelta(hours=1), D0 + timedelta(hours=2))
    assert _allowed([_R(D0, None, is_global=True)], D0 + timedelta(hours=1), D0 + timedelta(days=9))


def test_verifier_schedule_wraps_midnight():
    """A 22:00-06:00 window (hour_start > hour_end) covers a night reservation."""
    night = _S("1234567", datetime.time(22), datetime.time(6))
    r = _R(D0, None, schedules=[night], resources=["R"])
    assert _allowed([r], D0 + timedelta(hours=23), D0 + timedelta(days=1, hours=5))
    assert not _allowed([r], D0 + timedelta(hours=20), D0 + timedelta(hours=23))


def test_verifier_sunday_to_monday_and_end_of_day():
    """Fixed wrap Sunday(7) -> Monday(1) and the 23:59 'until end of day' convention."""
    sunday = D0 - timedelta(days=1)
    sch = [_S("7", datetime.time(8), datetime.time(23, 59)), _S("1", datetime.time(0), datetime.time(9))]
    r = _R(sunday - timedelta(days=7), None, schedules=sch, resources=["R"])
    assert _allowed([r], sunday + timedelta(hours=20), D0 + timedelta(hours=8))
    assert not _allowed([r], sunday + timedelta(hours=20), D0 + timedelta(hours=10))


def test_verifier_schedule_clamped_to_restriction_end():
    always = _S("1234567", datetime.time(0), datetime.time(23, 59))
    r = _R(D0, D0 + timedelta(hours=12), schedules=[always], resources=["R"])
    assert _allowed([r], D0 + timedelta(hours=1), D0 + timedelta(hours=11))
    assert not _allowed([r], D0 + timedelta(hours=1), D0 + timedelta(hours=13))


def test_config_accepts_both_secret_key_spellings(tmp_path):
    """the reference reads ``[auth] secrect_key`` (typo, config.py:289); both spellings work."""
    from tensorhive_fixed_amd import config as C

    C.init_config_files(tmp_path)
    main = (tmp_path / "main_config.ini").read_text()
    import re

    main = re.sub(r"(?m)^secre[c]?t_key\s*=.*$", "", main)
    (tmp_path / "main_config.ini").write_text(main + "\n[auth]\nsecrect_key = typo-spelling\n"
                                              if "[auth]" not in main else
                                              main.replace("[auth]", "[auth]\nsecrect_key = typo-spelling"))
    assert C.load_config(tmp_path).auth.secret_key == "typo-spelling"
    main2 = (tmp_path / "main_config.ini").read_text().replace("secrect_key", "secret_key")
    (tmp_path / "main_config.ini").write_text(main2)
    assert C.load_config(tmp_path).auth.secret_key == "typo-spelling"


def test_global_restrictions_exclude_expired(tables):
    """the reference discards its ``include_expired`` filter (Restriction.py:190-193)."""
    import datetime

    from tensorhive_fixed_amd.models.orm import Restriction

    now = datetime.datetime.utcnow()
    live = Restriction(name="live", starts_at=now - datetime.timedelta(days=2), is_global=True)
    live.save()
    old = Restriction(name="old", starts_at=now - datetime.timedelta(days=9), ends_at=now + datetime.timedelta(days=1),
                      is_global=True)
    old.save()
    from tensorhive_fixed_amd.database import db_session

    old._ends_at = now - datetime.timedelta(days=1)  # expire it behind the model's edit guard
    db_session.commit()
    assert [r.name for r in Restriction.get_global_restrictions()] == ["live"]
    assert sorted(r.name for r in Restriction.get_global_restrictions(include_expired=True)) == ["live", "old"]
