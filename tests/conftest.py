"""pytest configuration: the `gpu` marker, GPU-availability gating, shared fixtures."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

os.environ.setdefault("PYTEST", "1")  # in-memory SQLite, as the reference's pytest.ini does


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) and the built HIP kernels")
    config.addinivalue_line("markers", "slow: long-running test")


def _gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


# ----------------------------------------------------------------------------- daemon fixtures
import datetime  # noqa: E402
import json  # noqa: E402

HOSTS_INI = """
[node-a]
user = tester
transport = simulated

[node-b]
user = tester
transport = simulated
"""


@pytest.fixture()
def cfg(tmp_path, monkeypatch):
    """A private config dir (2 simulated MI355X nodes speaking the th-run protocol in-process),
    in-memory DB, installed as the global config."""
    from tensorhive_fixed_amd import config as C

    monkeypatch.setenv("TENSORHIVE_CONFIG_DIR", str(tmp_path))
    monkeypatch.setenv("PYTEST", "1")
    monkeypatch.setenv("TH_RUN_STATE_DIR", str(tmp_path / "th-run"))
    C.init_config_files(tmp_path)
    (tmp_path / "hosts_config.ini").write_text(HOSTS_INI)
    main = (tmp_path / "main_config.ini").read_text()
    main = main.replace("~/.config/TensorHive/hosts_config.ini", str(tmp_path / "hosts_config.ini"))
    main = main.replace("~/TensorHiveLogs", str(tmp_path / "TensorHiveLogs"))
    main = main.replace("~/.config/TensorHive/logs/", str(tmp_path / "usage_logs"))
    main = main.replace("key_file = ~/.config/TensorHive/ssh_key", f"key_file = {tmp_path / 'ssh_key'}")
    main = main.replace("test_on_startup = on", "test_on_startup = off")
    main = main.replace("backend = auto", "backend = stub")
    (tmp_path / "main_config.ini").write_text(main)
    c = C.load_config(tmp_path)
    C.set_config(c)
    yield c
    C.set_config(None)


@pytest.fixture()
def tables(cfg):
    from tensorhive_fixed_amd import database as D

    D.configure("sqlite://")
    D.create_all()
    D.db_session.remove()
    yield
    D.db_session.remove()
    D.drop_all()


@pytest.fixture()
def daemon(cfg, tables):
    from tensorhive_fixed_amd.core.daemon import Daemon
    from tensorhive_fixed_amd.core.telemetry import StubBackend

    from tensorhive_fixed_amd.core.attribution import REGISTRY

    REGISTRY.clear()  # th-run sessions seen by an earlier test's daemon
    stub = StubBackend(gpus_per_host=8)
    d = Daemon(cfg, backends={h: stub for h in cfg.ssh.available_nodes}, init_key=False, test_ssh=False)
    d.stub = stub
    for h in cfg.ssh.available_nodes:
        d.infrastructure.publish(h, stub.sample(h))
    yield d
    d.shutdown()


@pytest.fixture()
def app(daemon):
    from tensorhive_fixed_amd.api.app import create_app

    a = create_app(daemon)
    a.config["TH_REMOVE_SESSION"] = False
    a.config["TH_VALIDATE_RESPONSES"] = True  # every answer is checked against the OpenAPI document
    return a


@pytest.fixture()
def client(app):
    return app.test_client()


def _mk_user(name, admin=False, email=None):
    from tensorhive_fixed_amd.models.orm import Role, User

    roles = [Role(name="user")] + ([Role(name="admin")] if admin else [])
    u = User(username=name, password="TEST PASSWORD", email=email or f"{name}@example.org", roles=roles)
    u.save()
    return u


@pytest.fixture()
def new_user(tables):
    return _mk_user("administrantee")


@pytest.fixture()
def new_admin(tables):
    return _mk_user("justuser", admin=True)


@pytest.fixture()
def auth_headers():
    from tensorhive_fixed_amd.api import auth

    def make(user):
        tok = auth.create_access_token(user.id, user.role_names, fresh=True)
        return {"Authorization": f"Bearer {tok}", "Content-Type": "application/json"}
    return make


@pytest.fixture()
def resource1(tables):
    from tensorhive_fixed_amd.models.orm import Resource

    r = Resource(id="GPU-" + "0" * 36, name="MI355X", hostname="node-a")
    r.save()
    return r


@pytest.fixture()
def permissive_restriction(tables):
    from tensorhive_fixed_amd.models.orm import Restriction

    r = Restriction(name="everything", starts_at=datetime.datetime.utcnow() - datetime.timedelta(days=10),
                    is_global=True)
    r.save()
    return r




# ----------------------------------------------------------------------------- model fixtures
# Same scenarios as the reference's tests/fixtures/models.py (users, GPUs, restrictions, schedules,
# reservations, jobs, tasks); values chosen independently.
def _in(**kw):
    return datetime.datetime.utcnow() + datetime.timedelta(**kw)


@pytest.fixture()
def new_user_2(tables):
    return _mk_user("AnotherUser")


@pytest.fixture()
def resource2(tables):
    from tensorhive_fixed_amd.models.orm import Resource

    r = Resource(id="GPU-" + "1" * 36, name="Custom name", hostname="node-b")
    r.save()
    return r


@pytest.fixture()
def restriction(tables):
    from tensorhive_fixed_amd.models.orm import Restriction

    start = _in(minutes=5)
    r = Restriction(name="TestRestriction", starts_at=start, ends_at=start + datetime.timedelta(hours=8))
    r.save()
    return r


@pytest.fixture()
def new_group(tables):
    from tensorhive_fixed_amd.models.orm import Group

    return Group(name="TestGroup1")


@pytest.fixture()
def new_group_with_member(tables, new_user):
    from tensorhive_fixed_amd.models.orm import Group

    g = Group(name="TestGroup1")
    g.save()
    g.add_user(new_user)
    return g


def _schedule(days, a, b):
    from tensorhive_fixed_amd.models.orm import RestrictionSchedule

    s = RestrictionSchedule(schedule_days=days, hour_start=a, hour_end=b)
    s.save()
    return s


@pytest.fixture()
def active_schedule(tables):
    return _schedule("1234567", datetime.time(0, 0), datetime.time(23, 59, 59))


@pytest.fixture()
def inactive_schedule(tables):
    today = str(datetime.datetime.utcnow().weekday() + 1)
    return _schedule("1234567".replace(today, ""), datetime.time(8, 0), datetime.time(10, 0))


def _reservation(user, res, start, dur):
    from tensorhive_fixed_amd.models.orm import Reservation

    return Reservation(user_id=user.id, title="TEST TITLE", description="TEST_DESCRIPTION", resource_id=res.id,
                       start=start, end=start + dur)


@pytest.fixture()
def new_reservation(new_user, resource1):
    return _reservation(new_user, resource1, datetime.datetime.utcnow(), datetime.timedelta(minutes=60))


@pytest.fixture()
def new_reservation_2(new_user, new_admin, resource1):
    return _reservation(new_admin, resource1, datetime.datetime.utcnow(), datetime.timedelta(minutes=60))


@pytest.fixture()
def past_reservation(new_user, resource1):
    return _reservation(new_user, resource1, _in(hours=-5), datetime.timedelta(minutes=60))


@pytest.fixture()
def active_reservation(new_user, resource1):
    return _reservation(new_user, resource1, _in(hours=-5), datetime.timedelta(hours=10))


@pytest.fixture()
def future_reservation(new_user, resource1):
    return _reservation(new_user, resource1, _in(hours=5), datetime.timedelta(hours=10))


@pytest.fixture()
def new_task(tables):
    from tensorhive_fixed_amd.models.orm import CommandSegment, SegmentType, Task, TaskStatus

    t = Task(command="python train.py", hostname="node-a", _status=TaskStatus.not_running)
    t.add_cmd_segment(CommandSegment(name="--batch_size", segment_type=SegmentType.parameter), "32")
    t.save()
    return t


@pytest.fixture()
def new_task_2(tables):
    from tensorhive_fixed_amd.models.orm import CommandSegment, SegmentType, Task, TaskStatus

    t = Task(command="python eval.py", hostname="node-b", _status=TaskStatus.not_running)
    t.add_cmd_segment(CommandSegment(name="HIP_VISIBLE_DEVICES", segment_type=SegmentType.env_variable), "0")
    t.save()
    return t


def _job(user, name="job_name", status=None):
    from tensorhive_fixed_amd.models.orm import Job, JobStatus

    j = Job(name=name, description="testDescription", user_id=user.id, status=status or JobStatus.not_running)
    j.save()
    return j


@pytest.fixture()
def new_job(new_user):
    return _job(new_user)


@pytest.fixture()
def new_running_job(new_user):
    from tensorhive_fixed_amd.models.orm import JobStatus

    return _job(new_user, "running_job", JobStatus.running)


@pytest.fixture()
def new_job_with_task(new_user, new_task):
    j = _job(new_user)
    j.add_task(new_task)
    return j


@pytest.fixture()
def new_admin_job(new_user, new_admin, new_task):
    j = _job(new_admin, "admin_job")
    j.add_task(new_task)
    return j
