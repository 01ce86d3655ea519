"""Schema migration runner (reference ``tensorhive/migrations/versions/*``, 18 alembic revisions):
an existing TensorHive SQLite DB at ANY known revision upgrades in place to the schema the ORM
declares, keeping its data."""
import datetime

import pytest
from sqlalchemy import create_engine, inspect, text

from tensorhive_fixed_amd import migrations as M


def _db_at(tmp_path, rev):
    eng = create_engine(f"sqlite:///{tmp_path / 'th.sqlite'}")
    target = M._applied_closure([rev])
    with eng.connect() as c:
        for rid in M.ORDER:
            if rid in target:
                with c.begin():
                    M.BY_ID[rid].upgrade(c)
        with c.begin():
            M._set_revision(c, rev)
    return eng


def _schema(eng):
    insp = inspect(eng)
    return {t: sorted(col["name"] for col in insp.get_columns(t)) for t in insp.get_table_names()
            if t != "alembic_version"}


@pytest.fixture()
def orm_schema(tmp_path):
    from tensorhive_fixed_amd.database import Base, import_models

    import_models()
    eng = create_engine(f"sqlite:///{tmp_path / 'fresh.sqlite'}")
    Base.metadata.create_all(eng)
    return _schema(eng)


def test_history_is_complete():
    assert len(M.REVISIONS) == 18 and M.ORDER[-1] == M.HEAD
    assert M.pending([M.HEAD]) == []
    assert M.pending(["bffd7d81d326"])[0] == "05eca1c82f14"  # the other branch of the merge


@pytest.mark.parametrize("rev", M.ORDER)
def test_upgrade_from_every_revision_matches_orm(tmp_path, orm_schema, rev):
    eng = _db_at(tmp_path, rev)
    assert M.upgrade(eng) == M.HEAD
    with eng.connect() as c:
        assert M.current_revisions(c) == [M.HEAD]
    # the revision chain builds exactly the reference schema; daemon-owned tables come on top,
    # created next to it without a revision id (database.create_daemon_tables)
    from tensorhive_fixed_amd.database import DAEMON_TABLES, create_daemon_tables

    assert _schema(eng) == {t: c for t, c in orm_schema.items() if t not in DAEMON_TABLES}
    create_daemon_tables(eng)
    create_daemon_tables(eng)  # idempotent
    assert _schema(eng) == orm_schema


def test_data_survives_full_upgrade(tmp_path):
    eng = _db_at(tmp_path, "ce624ab2c458")
    with eng.begin() as c:
        c.execute(text("INSERT INTO users (id, username, created_at, _hashed_password) VALUES "
                       "(1, 'olduser', '2020-01-01 00:00:00', 'x')"))
        c.execute(text("INSERT INTO roles (id, name, user_id) VALUES (1, 'user', 1)"))
        c.execute(text("INSERT INTO reservations (id, user_id, title, description, protected_resource_id, _starts_at, "
                       "_ends_at, created_at) VALUES (1, 1, 't', 'd', :r, '2101-01-01 10:00:00', "
                       "'2101-01-01 12:00:00', '2020-01-01 00:00:00')"), {"r": "GPU-" + "1" * 36})
    M.upgrade(eng)
    from tensorhive_fixed_amd import database as D
    from tensorhive_fixed_amd.models.orm import Job, JobStatus, Reservation, User

    D.configure(f"sqlite:///{tmp_path / 'th.sqlite'}")
    try:
        u = User.get(1)
        assert u.username == "olduser" and u.email == "<email_missing>" and u.role_names == ["user"]
        r = Reservation.get(1)
        assert r.resource_id == "GPU-" + "1" * 36 and r.start == datetime.datetime(2101, 1, 1, 10)
        assert r.is_cancelled is False
        j = Job(name="after-migration", description="", user_id=1)
        j.save()
        j.enqueue()  # 'pending' must pass the relaxed CHECK constraint
        assert Job.get(j.id).status is JobStatus.pending
    finally:
        D.db_session.remove()
        D.configure("sqlite://")


def test_unknown_revision_is_refused(tmp_path):
    eng = create_engine(f"sqlite:///{tmp_path / 'x.sqlite'}")
    M.stamp(eng, "deadbeef0000")
    with pytest.raises(RuntimeError):
        M.upgrade(eng)


def test_ensure_db_creates_and_stamps(cfg, tmp_path):
    from tensorhive_fixed_amd import database as D

    D.configure(f"sqlite:///{tmp_path / 'new.sqlite'}")
    try:
        D.ensure_db_with_current_schema()
        with D.engine().connect() as c:
            assert M.current_revisions(c) == [M.HEAD]
        D.ensure_db_with_current_schema()  # idempotent
    finally:
        D.db_session.remove()
        D.configure("sqlite://")
