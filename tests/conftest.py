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
transport = local

[node-b]
user = tester
transport = local
"""


@pytest.fixture()
def cfg(tmp_path, monkeypatch):
    """A private config dir (2 local 'nodes'), in-memory DB, installed as the global config."""
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

    return create_app(daemon)


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

    r = Restriction(name="everything", starts_at=datetime.datetime.utcnow() - datetime.timedelta(days=1),
                    is_global=True)
    r.save()
    return r


