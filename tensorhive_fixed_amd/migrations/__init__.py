"""Built-in schema migration runner, revision-compatible with TensorHive's alembic history.

alembic is not a dependency; instead this module knows the reference's 18 revision ids
(``tensorhive/migrations/versions/*``) and, for each, how to move an SQLite database one step
forward with plain SQL.  It reads and writes the same ``alembic_version`` table, so:

* a new DB is created from the ORM metadata and stamped with :data:`HEAD`;
* an existing TensorHive DB at any known revision is upgraded in place, step by step;
* the final step also relaxes the ``jobs._status`` CHECK constraint that the reference's
  ``a44e0949e0a0`` created without ``pending``, by rebuilding the table.

History (``down -> up``)::

    ce624ab2c458 -> {bffd7d81d326, 05eca1c82f14} -> 5279ea22b197 (merge) -> 131eb148fd57
    -> ecd059f567b5 -> 81c2455baab1 -> e935d47c4cde -> 9d12594fe87b -> 06ce06e9bb85
    -> 58a12e45663e -> 72fb5b78625f -> 7110c972b137 -> e792ab930685 -> a44e0949e0a0
    -> 4d010fddad6f -> a16bb624004f -> 0a7b011e7b39 (head)
"""
from __future__ import annotations

import logging
from dataclasses import dataclass
from typing import Callable

from sqlalchemy import text
from sqlalchemy.engine import Connection, Engine

log = logging.getLogger(__name__)

HEAD = "0a7b011e7b39"


# ------------------------------------------------------------------------- sqlite helpers
def _cols(c: Connection, table: str) -> list[str]:
    return [r[1] for r in c.execute(text(f'PRAGMA table_info("{table}")'))]


def _has_table(c: Connection, table: str) -> bool:
    return c.execute(text("SELECT 1 FROM sqlite_master WHERE type='table' AND name=:n"), {"n": table}).first() is not None


def _add_column(c: Connection, table: str, ddl: str) -> None:
    name = ddl.split()[0].strip('"')
    if name not in _cols(c, table):
        c.execute(text(f'ALTER TABLE "{table}" ADD COLUMN {ddl}'))


def _rename_column(c: Connection, table: str, old: str, new: str) -> None:
    cols = _cols(c, table)
    if old in cols and new not in cols:
        c.execute(text(f'ALTER TABLE "{table}" RENAME COLUMN "{old}" TO "{new}"'))


def _rebuild(c: Connection, table: str, create_sql: str, mapping: dict[str, str] | None = None) -> None:
    """SQLite 12-step table rebuild: new table from ``create_sql``, copy the columns common to
    both (or ``mapping`` new<-old expressions), swap."""
    tmp = f"_th_new_{table}"
    c.execute(text(create_sql.replace(f'"{table}"', f'"{tmp}"', 1)))
    new_cols = _cols(c, tmp)
    old_cols = set(_cols(c, table))
    mapping = dict(mapping or {})
    pairs = [(n, mapping.get(n, f'"{n}"')) for n in new_cols if n in mapping or n in old_cols]
    if pairs:
        c.execute(text(f'INSERT INTO "{tmp}" ({", ".join(chr(34) + n + chr(34) for n, _ in pairs)}) '
                       f'SELECT {", ".join(e for _, e in pairs)} FROM "{table}"'))
    c.execute(text(f'DROP TABLE "{table}"'))
    c.execute(text(f'ALTER TABLE "{tmp}" RENAME TO "{table}"'))


# ------------------------------------------------------------------------------ revisions
def _r_ce624ab2c458(c):
    c.execute(text('CREATE TABLE IF NOT EXISTS revoked_tokens (id INTEGER NOT NULL PRIMARY KEY, '
                   'jti VARCHAR(120) NOT NULL UNIQUE)'))
    c.execute(text('CREATE TABLE IF NOT EXISTS users (id INTEGER NOT NULL PRIMARY KEY, username VARCHAR(40) NOT NULL '
                   'UNIQUE, created_at DATETIME, _hashed_password VARCHAR(120) NOT NULL)'))
    c.execute(text('CREATE TABLE IF NOT EXISTS reservations (id INTEGER NOT NULL PRIMARY KEY, user_id INTEGER NOT NULL '
                   'REFERENCES users(id), title VARCHAR(60) NOT NULL, description VARCHAR(200), '
                   'protected_resource_id VARCHAR(60) NOT NULL, _starts_at DATETIME NOT NULL, '
                   '_ends_at DATETIME NOT NULL, created_at DATETIME)'))
    c.execute(text('CREATE TABLE IF NOT EXISTS roles (id INTEGER NOT NULL PRIMARY KEY, name VARCHAR(40) NOT NULL, '
                   'user_id INTEGER REFERENCES users(id))'))


def _r_bffd7d81d326(c):
    _add_column(c, "reservations", "gpu_util_avg INTEGER")
    _add_column(c, "reservations", "mem_util_avg INTEGER")


def _r_05eca1c82f14(c):
    _add_column(c, "users", "email VARCHAR(64) NOT NULL DEFAULT '<email_missing>'")


def _r_5279ea22b197(c):  # merge point
    pass


def _r_131eb148fd57(c):
    c.execute(text('CREATE TABLE IF NOT EXISTS tasks (id INTEGER NOT NULL PRIMARY KEY, user_id INTEGER REFERENCES '
                   'users(id) ON DELETE CASCADE, host VARCHAR(40) NOT NULL, pid INTEGER, status VARCHAR(14) NOT NULL, '
                   'command VARCHAR(400) NOT NULL, spawn_at DATETIME, terminate_at DATETIME)'))
    # reservations.user_id gains ON DELETE CASCADE
    cols = _cols(c, "reservations")
    _rebuild(c, "reservations",
             'CREATE TABLE "reservations" (id INTEGER NOT NULL PRIMARY KEY, user_id INTEGER NOT NULL REFERENCES '
             'users(id) ON DELETE CASCADE, title VARCHAR(60) NOT NULL, description VARCHAR(200), '
             + ", ".join(f"{n} {t}" for n, t in [("protected_resource_id", "VARCHAR(60) NOT NULL"),
                                                 ("_starts_at", "DATETIME NOT NULL"), ("_ends_at", "DATETIME NOT NULL"),
                                                 ("created_at", "DATETIME"), ("gpu_util_avg", "INTEGER"),
                                                 ("mem_util_avg", "INTEGER")] if n in cols) + ")")


def _r_ecd059f567b5(c):
    c.execute(text('CREATE TABLE IF NOT EXISTS groups (id INTEGER NOT NULL PRIMARY KEY AUTOINCREMENT, '
                   'name VARCHAR(40), created_at DATETIME)'))
    c.execute(text('CREATE TABLE IF NOT EXISTS user2group (user_id INTEGER NOT NULL REFERENCES users(id) ON DELETE '
                   'CASCADE, group_id INTEGER NOT NULL REFERENCES groups(id) ON DELETE CASCADE, created_at DATETIME, '
                   'PRIMARY KEY (user_id, group_id))'))


def _r_81c2455baab1(c):
    c.execute(text('CREATE TABLE IF NOT EXISTS resources (id VARCHAR(64) NOT NULL PRIMARY KEY, name VARCHAR(40))'))


def _r_e935d47c4cde(c):
    c.execute(text('CREATE TABLE IF NOT EXISTS restrictions (id INTEGER NOT NULL PRIMARY KEY AUTOINCREMENT, '
                   'name VARCHAR(50), created_at DATETIME, starts_at DATETIME NOT NULL, ends_at DATETIME, '
                   'is_global BOOLEAN NOT NULL)'))
    c.execute(text('CREATE TABLE IF NOT EXISTS restriction2assignee (id INTEGER NOT NULL PRIMARY KEY AUTOINCREMENT, '
                   'restriction_id INTEGER NOT NULL REFERENCES restrictions(id) ON DELETE CASCADE, group_id INTEGER '
                   'REFERENCES groups(id) ON DELETE CASCADE, user_id INTEGER REFERENCES users(id) ON DELETE CASCADE)'))
    c.execute(text('CREATE TABLE IF NOT EXISTS restriction2resource (restriction_id INTEGER NOT NULL REFERENCES '
                   'restrictions(id) ON DELETE CASCADE, resource_id VARCHAR(64) NOT NULL REFERENCES resources(id) '
                   'ON DELETE CASCADE, PRIMARY KEY (restriction_id, resource_id))'))


def _r_9d12594fe87b(c):
    c.execute(text('CREATE TABLE IF NOT EXISTS restriction_schedules (id INTEGER NOT NULL PRIMARY KEY AUTOINCREMENT, '
                   'schedule_days VARCHAR(7) NOT NULL, hour_start TIME NOT NULL, hour_end TIME NOT NULL)'))
    c.execute(text('CREATE TABLE IF NOT EXISTS restriction2schedule (restriction_id INTEGER NOT NULL REFERENCES '
                   'restrictions(id) ON DELETE CASCADE, schedule_id INTEGER NOT NULL REFERENCES '
                   'restriction_schedules(id) ON DELETE CASCADE, PRIMARY KEY (restriction_id, schedule_id))'))


def _r_06ce06e9bb85(c):
    _add_column(c, "reservations", "is_cancelled BOOLEAN")


def _r_58a12e45663e(c):
    _add_column(c, "resources", "hostname VARCHAR(64)")


def _r_72fb5b78625f(c):
    _add_column(c, "groups", "is_default BOOLEAN")


def _r_7110c972b137(c):
    # the unique(is_default) constraint of 72fb5b78625f is dropped: rebuild groups without it
    _rebuild(c, "groups", 'CREATE TABLE "groups" (id INTEGER NOT NULL PRIMARY KEY AUTOINCREMENT, name VARCHAR(40), '
                          'created_at DATETIME, is_default BOOLEAN)')


def _r_e792ab930685(c):
    _rename_column(c, "reservations", "protected_resource_id", "resource_id")
    _rename_column(c, "reservations", "_starts_at", "_start")
    _rename_column(c, "reservations", "_ends_at", "_end")
    if _has_table(c, "tasks"):
        _rename_column(c, "tasks", "host", "hostname")


def _r_a44e0949e0a0(c):
    # the reference's enum had no 'pending'; we create it without a CHECK constraint
    c.execute(text('CREATE TABLE IF NOT EXISTS jobs (id INTEGER NOT NULL PRIMARY KEY AUTOINCREMENT, name VARCHAR(40) '
                   'NOT NULL, description TEXT, user_id INTEGER REFERENCES users(id) ON DELETE CASCADE, status '
                   'VARCHAR(14) NOT NULL, _start_at DATETIME, _stop_at DATETIME)'))


def _r_4d010fddad6f(c):
    c.execute(text('CREATE TABLE IF NOT EXISTS command_segments (id INTEGER NOT NULL PRIMARY KEY AUTOINCREMENT, '
                   'name VARCHAR(40) NOT NULL UNIQUE, segment_type VARCHAR(14) NOT NULL)'))
    c.execute(text('CREATE TABLE IF NOT EXISTS cmd_segment2task (task_id INTEGER NOT NULL REFERENCES tasks(id) ON '
                   'DELETE CASCADE, cmd_segment_id INTEGER NOT NULL REFERENCES command_segments(id) ON DELETE '
                   'CASCADE, _value VARCHAR(100), _index INTEGER, PRIMARY KEY (task_id, cmd_segment_id))'))


def _r_a16bb624004f(c):
    """Every pre-jobs task becomes a one-task job; tasks lose user_id/spawn_at/terminate_at."""
    cols = _cols(c, "tasks")
    if "job_id" in cols:
        return
    rows = c.execute(text("SELECT id, user_id, status, spawn_at, terminate_at FROM tasks")).fetchall() \
        if "user_id" in cols else []
    links = {}
    for tid, uid, st, sa, ta in rows:
        r = c.execute(text("INSERT INTO jobs (name, description, user_id, status, _start_at, _stop_at) VALUES "
                           "(:n, :d, :u, :s, :a, :b)"),
                      {"n": f"Job from Task {tid}", "d": f"Job auto-created from task with id: {tid}", "u": uid,
                       "s": st, "a": sa, "b": ta})
        links[tid] = r.lastrowid
    _rebuild(c, "tasks", 'CREATE TABLE "tasks" (id INTEGER NOT NULL PRIMARY KEY AUTOINCREMENT, job_id INTEGER '
                         'REFERENCES jobs(id) ON DELETE CASCADE, hostname VARCHAR(40) NOT NULL, pid INTEGER, '
                         'status VARCHAR(14) NOT NULL, command VARCHAR(400) NOT NULL)')
    for tid, jid in links.items():
        c.execute(text("UPDATE tasks SET job_id = :j WHERE id = :t"), {"j": jid, "t": tid})


def _r_0a7b011e7b39(c):
    _add_column(c, "jobs", "is_queued BOOLEAN")
    _rename_column(c, "jobs", "status", "_status")
    _rename_column(c, "tasks", "status", "_status")
    _add_column(c, "tasks", "gpu_id INTEGER")
    # relax any CHECK constraint on jobs._status so that 'pending' can be stored
    sql = c.execute(text("SELECT sql FROM sqlite_master WHERE type='table' AND name='jobs'")).scalar() or ""
    if "CHECK" in sql.upper():
        _rebuild(c, "jobs", 'CREATE TABLE "jobs" (id INTEGER NOT NULL PRIMARY KEY AUTOINCREMENT, name VARCHAR(40) NOT '
                            'NULL, description TEXT, user_id INTEGER REFERENCES users(id) ON DELETE CASCADE, _status '
                            'VARCHAR(14) NOT NULL, _start_at DATETIME, _stop_at DATETIME, is_queued BOOLEAN)')


@dataclass(frozen=True)
class Revision:
    id: str
    down: tuple[str, ...]
    title: str
    upgrade: Callable[[Connection], None]


REVISIONS: list[Revision] = [
    Revision("ce624ab2c458", (), "create tables", _r_ce624ab2c458),
    Revision("bffd7d81d326", ("ce624ab2c458",), "add summary fields to reservation", _r_bffd7d81d326),
    Revision("05eca1c82f14", ("ce624ab2c458",), "add email column to user", _r_05eca1c82f14),
    Revision("5279ea22b197", ("bffd7d81d326", "05eca1c82f14"), "merge emails and summaries", _r_5279ea22b197),
    Revision("131eb148fd57", ("5279ea22b197",), "add task table", _r_131eb148fd57),
    Revision("ecd059f567b5", ("131eb148fd57",), "create groups and user2group tables", _r_ecd059f567b5),
    Revision("81c2455baab1", ("ecd059f567b5",), "create resources table", _r_81c2455baab1),
    Revision("e935d47c4cde", ("81c2455baab1",), "create restrictions and secondary tables", _r_e935d47c4cde),
    Revision("9d12594fe87b", ("e935d47c4cde",), "create restriction schedules", _r_9d12594fe87b),
    Revision("06ce06e9bb85", ("9d12594fe87b",), "add is_cancelled to reservations", _r_06ce06e9bb85),
    Revision("58a12e45663e", ("06ce06e9bb85",), "add hostname to resources", _r_58a12e45663e),
    Revision("72fb5b78625f", ("58a12e45663e",), "add is_default to groups", _r_72fb5b78625f),
    Revision("7110c972b137", ("72fb5b78625f",), "remove unique constraint from is_default", _r_7110c972b137),
    Revision("e792ab930685", ("7110c972b137",), "rename columns to match api", _r_e792ab930685),
    Revision("a44e0949e0a0", ("e792ab930685",), "create jobs table", _r_a44e0949e0a0),
    Revision("4d010fddad6f", ("a44e0949e0a0",), "create command segments", _r_4d010fddad6f),
    Revision("a16bb624004f", ("4d010fddad6f",), "modify tasks table to match jobs table", _r_a16bb624004f),
    Revision("0a7b011e7b39", ("a16bb624004f",), "add and rename columns in jobs and tasks", _r_0a7b011e7b39),
]
BY_ID = {r.id: r for r in REVISIONS}
ORDER = [r.id for r in REVISIONS]  # a valid topological order of the history


def current_revisions(c: Connection) -> list[str]:
    if not _has_table(c, "alembic_version"):
        return []
    return [r[0] for r in c.execute(text("SELECT version_num FROM alembic_version"))]


def _set_revision(c: Connection, rev: str) -> None:
    c.execute(text("CREATE TABLE IF NOT EXISTS alembic_version (version_num VARCHAR(32) NOT NULL, "
                   "CONSTRAINT alembic_version_pkc PRIMARY KEY (version_num))"))
    c.execute(text("DELETE FROM alembic_version"))
    c.execute(text("INSERT INTO alembic_version (version_num) VALUES (:v)"), {"v": rev})


def stamp(engine: Engine, rev: str = HEAD) -> None:
    with engine.begin() as c:
        _set_revision(c, rev)


def _applied_closure(heads: list[str]) -> set[str]:
    done, stack = set(), list(heads)
    while stack:
        r = stack.pop()
        if r in done or r not in BY_ID:
            continue
        done.add(r)
        stack.extend(BY_ID[r].down)
    return done


def pending(heads: list[str]) -> list[str]:
    done = _applied_closure(heads)
    return [r for r in ORDER if r not in done]


def upgrade(engine: Engine) -> str:
    """Apply every pending revision in order; returns the new head revision."""
    with engine.connect() as c:
        heads = current_revisions(c)
    unknown = [h for h in heads if h not in BY_ID]
    if unknown:
        raise RuntimeError(f"database is at unknown revision(s) {unknown}")
    todo = pending(heads) if heads else []
    if not heads:
        # tables exist but no version table: assume a pre-alembic schema at the first revision
        todo = pending(["ce624ab2c458"])
    with engine.connect() as c:
        c.execute(text("PRAGMA foreign_keys=OFF"))
        c.commit()
        try:
            for rid in todo:
                with c.begin():
                    log.info("migrating database: %s (%s)", rid, BY_ID[rid].title)
                    BY_ID[rid].upgrade(c)
                    _set_revision(c, rid)
        finally:
            c.execute(text("PRAGMA foreign_keys=ON"))
            c.commit()
    return HEAD if (todo or HEAD in heads) else (heads[0] if heads else HEAD)
