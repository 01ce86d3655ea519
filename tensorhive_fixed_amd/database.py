"""SQLite persistence: engine, thread-local session, schema lifecycle.

Reference: ``tensorhive/database.py`` -- scoped (thread-local) session, ``PYTEST=1`` -> in-memory
SQLite, FK pragma on every connection, ``create_all`` + stamp for a new DB else ``upgrade head``.
Here the migration runner is built in (alembic is not a dependency) and reads/writes the same
``alembic_version`` table with the same revision ids, so an existing TensorHive DB upgrades in
place (see :mod:`tensorhive_fixed_amd.migrations`).
"""
from __future__ import annotations

import logging
import threading
from pathlib import Path

from sqlalchemy import create_engine, event, inspect
from sqlalchemy.orm import declarative_base, scoped_session, sessionmaker
from sqlalchemy.pool import StaticPool

log = logging.getLogger(__name__)

db_session = scoped_session(sessionmaker(autoflush=False, expire_on_commit=False))
Base = declarative_base()
Base.query = db_session.query_property()

_engine = None
_engine_lock = threading.Lock()


def _fk_pragma(dbapi_conn, _record):
    cur = dbapi_conn.cursor()
    cur.execute("PRAGMA foreign_keys=ON")
    cur.close()


def _wal_pragma(dbapi_conn, _record):
    """File databases run in WAL mode.  The daemon writes from API threads and service threads
    at once; in the default rollback-journal mode a COMMIT must wait for every other
    connection's SHARED lock, and a reader that then wants to write waits for the committer's
    RESERVED lock -- a deadlock that only the 30 s busy timeout breaks (seen with concurrent
    executes and scheduler ticks, tests/test_allocation.py).  In WAL mode readers never block a
    commit.  WAL is a property of the database file; SQLite >= 3.7 (any TensorHive) opens it."""
    cur = dbapi_conn.cursor()
    cur.execute("PRAGMA journal_mode=WAL")
    cur.execute("PRAGMA synchronous=NORMAL")
    cur.close()


def configure(uri: str | None = None):
    """(Re)create the engine for ``uri`` (default: the configured DB) and bind the session."""
    global _engine
    from .config import get_config

    uri = uri or get_config().db_uri
    with _engine_lock:
        if _engine is not None:
            db_session.remove()
            _engine.dispose()
        if uri in ("sqlite://", "sqlite:///:memory:"):
            eng = create_engine(uri, connect_args={"check_same_thread": False}, poolclass=StaticPool)
        else:
            if uri.startswith("sqlite:///"):
                Path(uri[len("sqlite:///"):]).expanduser().parent.mkdir(parents=True, exist_ok=True)
            # one scoped session (= one pooled connection) per thread: API request threads, the
            # services and launch fan-outs run at once, so the pool is sized well above
            # SQLAlchemy's 5+10 default (SQLite connections are cheap file handles)
            eng = create_engine(uri, connect_args={"check_same_thread": False, "timeout": 30},
                                pool_size=32, max_overflow=64, pool_timeout=60)
            event.listen(eng, "connect", _wal_pragma)
        event.listen(eng, "connect", _fk_pragma)
        db_session.configure(bind=eng)
        _engine = eng
        return eng


def engine():
    if _engine is None:
        configure()
    return _engine


def import_models() -> None:
    """Import every ORM module so that ``Base.metadata`` knows all tables."""
    from .models import orm  # noqa: F401


def create_all() -> None:
    import_models()
    Base.metadata.create_all(engine())


def drop_all() -> None:
    import_models()
    Base.metadata.drop_all(engine())


def check_if_db_exists(path: str | None = None) -> bool:
    from .config import get_config

    p = Path(path or get_config().db_path).expanduser()
    return p.exists()


def ensure_db_with_current_schema() -> str:
    """Create + stamp a new DB, or run pending migrations; returns the final revision."""
    from . import migrations

    import_models()
    eng = engine()
    insp = inspect(eng)
    tables = set(insp.get_table_names())
    if not tables - {"alembic_version"}:
        Base.metadata.create_all(eng)
        migrations.stamp(eng, migrations.HEAD)
        log.info("created a new database at revision %s", migrations.HEAD)
        return migrations.HEAD
    rev = migrations.upgrade(eng)
    create_daemon_tables(eng)
    return rev


DAEMON_TABLES = ("gpu_allocations", "task_restart_policies")


def create_daemon_tables(eng=None) -> None:
    """Tables the daemon owns outside the alembic revision chain (``gpu_allocations``,
    ``task_restart_policies``): created
    idempotently so an upgraded TensorHive database gains them without a new revision id (the
    reference can still open it; it ignores tables it does not map)."""
    import_models()
    tables = [Base.metadata.tables[t] for t in DAEMON_TABLES if t in Base.metadata.tables]
    Base.metadata.create_all(eng or engine(), tables=tables)
