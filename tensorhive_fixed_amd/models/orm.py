"""ORM entities -- the SQLite schema contract of TensorHive 1.1.

Tables, column names and enum storage (enum *names* as strings) match the reference models
(``tensorhive/models/*.py``) so an existing ``database.sqlite`` is read and written unchanged.
Behavioural notes, each covered by a test:

* ``Reservation``: 30 min .. 8 days, title 1..59 chars, description < 200, resource id of exactly
  40 chars, no overlap with a non-cancelled reservation on the same resource
  (``models/Reservation.py:39-55,120-130``).
* ``Job.start_at`` in the past is clamped to now (fork behaviour, ``models/Job.py:123-132``).
* ``Task.full_command`` renders ``ENV=v ... command param value ...``; a parameter whose name
  ends with ``=`` is joined without a space (fixes ``--rank= 0``, ``models/Task.py:95``).
* ``Restriction.get_global_restrictions(include_expired=False)`` really filters expired ones
  (the reference discards its filter, ``models/Restriction.py:190-193``).
* ``JobStatus.pending`` is stored without a CHECK constraint (the reference's migration
  ``a44e0949e0a0`` lacks it; see :mod:`..migrations`).
"""
from __future__ import annotations

import datetime
import enum
import json
import logging
import re
import shlex
import threading
from datetime import timedelta

from sqlalchemy import (Boolean, Column, DateTime, Enum, ForeignKey, Integer, String, Text, Time, UniqueConstraint,
                        and_, or_)
from sqlalchemy.exc import MultipleResultsFound, NoResultFound
from sqlalchemy import event
from sqlalchemy.orm import Session, relationship, validates

from ..database import Base, db_session
from ..utils import dates
from ..utils.exceptions import InvalidRequestException
from ..utils.passwords import hash_password, verify_password
from ..utils.weekday import Weekday
from .crud import CRUDModel

log = logging.getLogger(__name__)

_RESERVED_USERNAMES = {"root", "admin", "administrator", "api", "system", "null", "none", "daemon",
                       "login", "logout", "signup", "register", "static", "www", "tensorhive",
                       # insult words (the reference rejects them via the safe-usernames package)
                       "jerk", "idiot", "moron", "stupid", "loser", "dumbass", "asshole", "bastard", "retard"}
_USERNAME_RE = re.compile(r"^[A-Za-z0-9][A-Za-z0-9_.\-]*$")


def _utcnow():
    return dates.utcnow()


def _is_one_shell_word(v: str) -> bool:
    """Would ``bash`` read ``v`` as exactly one word with no unquoted control operator, no
    comment (a word starting with ``#``) and no brace expansion (``{a,b}``, ``{1..3}``)?
    (A small scanner, mirrored line for line by ``app/static/js/launch.js``.)"""
    # braces: one entry per open '{' -- whether that level saw an unquoted ',' or '..' (nested
    # levels are tracked separately: `{a,{c}}` expands through its OUTER level)
    words, in_word, quote, braces, i = 0, False, "", [], 0
    while i < len(v):
        c = v[i]
        if quote == "'":
            if c == "'":
                quote = ""
        elif quote == '"':
            if c == "\\":
                i += 1
            elif c == '"':
                quote = ""
        elif c in " \t\n":
            in_word, braces = False, []
        elif c in ";&|<>()":
            return False
        else:
            if not in_word:
                if c == "#":
                    return False
                words, in_word = words + 1, True
            if c == "\\":
                i += 1
            elif c in "'\"":
                quote = c
            elif c == "{":
                braces.append(False)
            elif braces and (c == "," or (c == "." and v[i + 1:i + 2] == ".")):
                braces[-1] = True
            elif c == "}" and braces:
                if braces.pop():
                    return False
        i += 1
    return words == 1 and quote == "" and i == len(v)


def _is_json_document(v: str) -> bool:
    if not v.lstrip().startswith(("{", "[")):
        return False
    try:
        json.loads(v)
        return True
    except ValueError:
        return False


def _shell_value(v) -> str:
    """A command-segment value as one shell word (see Task.render).

    A value that the shell already reads as exactly ONE word is left untouched, so values the
    user quoted themselves (``"a b"``), globs (``/data/*.tfrecord``) and ``$VARS`` keep the
    reference's semantics (``models/Task.py:77-98`` pasted values verbatim).  Single-quoted are
    only: a value that would split into several words, has an unbalanced quote or an unquoted
    control operator (``;`` ``&`` ``|`` ``<`` ``>`` parentheses), and a JSON document (a
    generated TF_CONFIG), whose quotes are data rather than shell syntax."""
    v = "" if v is None else str(v)
    if not v or (_is_one_shell_word(v) and not _is_json_document(v)):
        return v
    return "'" + v.replace("'", "'\\''") + "'"


# ------------------------------------------------------------------------------------ users
def _refresh_view(obj, attr: str) -> None:
    """The reverse side of a many-to-many is ``viewonly``: reload it after the owning side changed."""
    from sqlalchemy import inspect as sa_inspect

    if sa_inspect(obj).persistent:
        db_session.expire(obj, [attr])


class User2Group(Base):
    __tablename__ = "user2group"
    user_id = Column(Integer, ForeignKey("users.id", ondelete="CASCADE"), primary_key=True)
    group_id = Column(Integer, ForeignKey("groups.id", ondelete="CASCADE"), primary_key=True)
    created_at = Column(DateTime, default=_utcnow)


class Restriction2Assignee(Base):
    __tablename__ = "restriction2assignee"
    __table_args__ = {"sqlite_autoincrement": True}
    id = Column(Integer, primary_key=True, autoincrement=True)
    restriction_id = Column(Integer, ForeignKey("restrictions.id", ondelete="CASCADE"), nullable=False)
    group_id = Column(Integer, ForeignKey("groups.id", ondelete="CASCADE"))
    user_id = Column(Integer, ForeignKey("users.id", ondelete="CASCADE"))


class Restriction2Resource(Base):
    __tablename__ = "restriction2resource"
    restriction_id = Column(Integer, ForeignKey("restrictions.id", ondelete="CASCADE"), primary_key=True)
    resource_id = Column(String(64), ForeignKey("resources.id", ondelete="CASCADE"), primary_key=True)


class Restriction2Schedule(Base):
    __tablename__ = "restriction2schedule"
    restriction_id = Column(Integer, ForeignKey("restrictions.id", ondelete="CASCADE"), primary_key=True)
    schedule_id = Column(Integer, ForeignKey("restriction_schedules.id", ondelete="CASCADE"), primary_key=True)


class RestrictionAssignee:
    """Entities that restrictions can be assigned to (users, groups, resources)."""

    def get_restrictions(self, include_expired: bool = False):
        rs = list(self._restrictions)
        return rs if include_expired else [r for r in rs if not r.is_expired]

    def get_active_restrictions(self):
        return [r for r in self._restrictions if r.is_active]


class Role(CRUDModel, Base):
    __tablename__ = "roles"
    __public__ = ["id", "name"]
    id = Column(Integer, primary_key=True, autoincrement=True)
    name = Column(String(40), nullable=False)
    user_id = Column(Integer, ForeignKey("users.id"))

    @classmethod
    def find_by_name(cls, name):
        return cls.query.filter_by(name=name).first()

    @classmethod
    def find_by_user_id(cls, user_id):
        return cls.query.filter_by(user_id=user_id).all()

    def as_dict(self, include_private=False):
        d = super().as_dict(include_private)
        d["user_id"] = self.user_id
        return d


class RevokedToken(CRUDModel, Base):
    __tablename__ = "revoked_tokens"
    id = Column(Integer, primary_key=True, autoincrement=True)
    jti = Column(String(120), unique=True, nullable=False)

    # jtis already found absent from the table (per database): every authenticated request checks
    # its token, and revocations only ever ADD rows, so a "not revoked" answer stays true until the
    # next revocation -- which clears the set (after_flush listener below)
    _absent: dict = {}
    _absent_lock = threading.Lock()

    @classmethod
    def is_jti_blacklisted(cls, jti: str) -> bool:
        from .. import database

        key = id(database.engine())
        with cls._absent_lock:
            if jti in cls._absent.get(key, ()):
                return False
        revoked = db_session.query(cls.id).filter_by(jti=jti).first() is not None
        if not revoked:
            with cls._absent_lock:
                known = cls._absent.setdefault(key, set())
                if len(known) > 100_000:
                    known.clear()
                known.add(jti)
        return revoked


@event.listens_for(Session, "after_flush")
def _revocation_invalidates(session, _ctx):
    if any(isinstance(o, RevokedToken) for o in session.new):
        with RevokedToken._absent_lock:
            RevokedToken._absent.clear()


class User(CRUDModel, RestrictionAssignee, Base):
    __tablename__ = "users"
    __public__ = ["id", "username", "created_at"]
    __private__ = ["email"]
    min_password_length = 8

    id = Column(Integer, primary_key=True, autoincrement=True)
    username = Column(String(40), unique=True, nullable=False)
    email = Column(String(64), nullable=False, server_default="<email_missing>", default="<email_missing>")
    created_at = Column(DateTime, default=_utcnow)
    _hashed_password = Column(String(120), nullable=False)

    _roles = relationship("Role", cascade="all, delete-orphan", backref="user")
    _groups = relationship("Group", secondary="user2group", back_populates="_users", viewonly=True)
    _restrictions = relationship("Restriction", secondary="restriction2assignee", back_populates="_users",
                                 viewonly=True)
    reservations = relationship("Reservation", back_populates="user", cascade="all, delete-orphan",
                                passive_deletes=True)
    _jobs = relationship("Job", back_populates="user", cascade="all, delete-orphan", passive_deletes=True)

    def __init__(self, username=None, password=None, email=None, roles=None, **kw):
        super().__init__(**kw)
        if username is not None:
            self.username = username
        if email is not None:
            self.email = email
        if password is not None:
            self.password = password
        if roles is not None:
            self.roles = roles

    def __repr__(self):
        return f"<User id={self.id}, username={self.username} email={self.email}>"

    @property
    def roles(self):
        return self._roles

    @roles.setter
    def roles(self, value):
        self._roles = list(value)

    @property
    def role_names(self):
        return [r.name for r in self._roles]

    def has_role(self, name: str) -> bool:
        return name in self.role_names

    @property
    def groups(self):
        return self._groups

    @property
    def jobs(self):
        return self._jobs

    @property
    def password(self):
        return self._hashed_password

    @password.setter
    def password(self, raw: str):
        assert isinstance(raw, str) and len(raw) >= self.min_password_length, \
            f"Incorrect password, reason: password must be at least {self.min_password_length} characters long"
        self._hashed_password = hash_password(raw)

    @staticmethod
    def verify_hash(password: str, hashed: str) -> bool:
        return verify_password(password, hashed)

    @validates("username")
    def validate_username(self, _key, username):
        assert username and _USERNAME_RE.match(username) and username.lower() not in _RESERVED_USERNAMES, \
            "Username unsafe"
        assert 2 < len(username) < 16, "Username must be between 3 and 15 characters long"
        return username

    @validates("email")
    def validate_email(self, _key, email):
        assert re.search("[@.]", email or ""), "Email not correct"
        assert 3 < len(email) < 64, "Email must be between 3 and 64 characters long"
        return email

    @classmethod
    def find_by_username(cls, username):
        try:
            return db_session.query(cls).filter_by(username=username).one()
        except NoResultFound as e:
            raise NoResultFound(f"There is no user with username={username}!") from e

    def as_dict(self, include_private=False, include_groups=True):
        d = super().as_dict(include_private)
        d["roles"] = self.role_names
        if include_groups:
            d["groups"] = [g.as_dict(include_users=False) for g in self.groups]
        return d

    def get_restrictions(self, include_expired=False, include_group=False):
        rs = super().get_restrictions(include_expired=include_expired)
        if include_group:
            for g in self.groups:
                rs = rs + g.get_restrictions(include_expired=include_expired)
        return list(dict.fromkeys(rs))

    def get_active_restrictions(self, include_group=False):
        rs = super().get_active_restrictions()
        if include_group:
            for g in self.groups:
                rs = rs + g.get_active_restrictions()
        return list(dict.fromkeys(rs))

    def get_reservations(self, include_cancelled=False):
        return list(self.reservations) if include_cancelled else [r for r in self.reservations if not r.is_cancelled]

    def allowed_gpu_uuids(self) -> set[str] | None:
        """GPUs the user's restrictions (own and group, unexpired) cover; ``None`` = all of them
        (a global restriction)."""
        allowed: set[str] = set()
        for r in self.get_restrictions(include_expired=False, include_group=True):
            if r.is_global:
                return None
            allowed.update(res.id for res in r.resources)
        return allowed

    def filter_infrastructure_by_user_restrictions(self, infrastructure: dict) -> dict:
        """Drop GPUs the user may not use, then hosts left without GPUs, in place
        (reference ``models/User.py:166-186``)."""
        allowed = self.allowed_gpu_uuids()
        if allowed is None:
            return infrastructure
        for host in list(infrastructure):
            gpus = (infrastructure[host] or {}).get("GPU")
            if gpus is not None:
                for uuid in [u for u in gpus if u not in allowed]:
                    del gpus[uuid]
            if not gpus:
                del infrastructure[host]
        return infrastructure


class Group(CRUDModel, RestrictionAssignee, Base):
    __tablename__ = "groups"
    __table_args__ = {"sqlite_autoincrement": True}
    __public__ = ["id", "name", "is_default", "created_at"]
    id = Column(Integer, primary_key=True, autoincrement=True)
    name = Column(String(40), nullable=True)
    created_at = Column(DateTime, default=_utcnow)
    _is_default = Column("is_default", Boolean)
    _users = relationship("User", secondary="user2group", back_populates="_groups")
    _restrictions = relationship("Restriction", secondary="restriction2assignee", back_populates="_groups",
                                 viewonly=True)

    def __init__(self, name=None, is_default=None, **kw):
        super().__init__(**kw)
        self.name = name
        if is_default is not None:
            self.is_default = is_default

    def __repr__(self):
        return f"<Group id={self.id}, name={self.name}>"

    @property
    def is_default(self):
        return bool(self._is_default)

    @is_default.setter
    def is_default(self, value):
        self._is_default = bool(value)

    @property
    def users(self):
        return self._users

    def add_user(self, user):
        if user in self._users:
            raise InvalidRequestException(f"User {user} is already a member of group {self}!")
        self._users.append(user)
        self.save()
        _refresh_view(user, "_groups")

    def remove_user(self, user):
        if user not in self._users:
            raise InvalidRequestException(f"User {user} is not a member of group {self}!")
        self._users.remove(user)
        self.save()
        _refresh_view(user, "_groups")

    def as_dict(self, include_private=False, include_users=True):
        d = super().as_dict(include_private)
        if include_users:
            d["users"] = [u.as_dict(include_groups=False) for u in self._users]
        return d

    @classmethod
    def get_default_groups(cls):
        return cls.query.filter(cls._is_default.is_(True)).all()


class Resource(CRUDModel, RestrictionAssignee, Base):
    __tablename__ = "resources"
    __public__ = ["id", "name", "hostname"]
    id = Column(String(64), primary_key=True)
    name = Column(String(40), nullable=True)
    hostname = Column(String(64), nullable=True)
    _restrictions = relationship("Restriction", secondary="restriction2resource", back_populates="_resources",
                                 viewonly=True)

    def __repr__(self):
        return f"<Resource id={self.id}, name={self.name}>"

    def get_restrictions(self, include_expired=False, include_global=True):
        rs = super().get_restrictions(include_expired)
        if include_global:
            rs = rs + Restriction.get_global_restrictions(include_expired=include_expired)
        return list(dict.fromkeys(rs))

    def get_active_restrictions(self, include_global=True):
        rs = super().get_active_restrictions()
        if include_global:
            rs = rs + [r for r in Restriction.get_global_restrictions() if r.is_active]
        return list(dict.fromkeys(rs))

    @classmethod
    def get_by_name(cls, name):
        return db_session.query(cls).filter(cls.name == name).all()

    @classmethod
    def get_by_hostname(cls, hostname):
        return db_session.query(cls).filter(cls.hostname == hostname).all()


class RestrictionSchedule(CRUDModel, Base):
    __tablename__ = "restriction_schedules"
    __table_args__ = {"sqlite_autoincrement": True}
    __public__ = ["id"]
    id = Column(Integer, primary_key=True, autoincrement=True)
    _schedule_days = Column("schedule_days", String(7), nullable=False)
    hour_start = Column(Time(), nullable=False)
    hour_end = Column(Time(), nullable=False)
    _restrictions = relationship("Restriction", secondary="restriction2schedule", back_populates="_schedules",
                                 viewonly=True)

    def __init__(self, schedule_days, hour_start: datetime.time, hour_end: datetime.time, **kw):
        super().__init__(**kw)
        self.schedule_days = schedule_days
        self.hour_start = hour_start
        self.hour_end = hour_end

    def __repr__(self):
        return f"<RestrictionSchedule id={self.id} days={self.schedule_days} {self.hour_start}-{self.hour_end}>"

    def check_assertions(self):
        assert self.is_valid_schedule_expression(self.schedule_days), \
            "schedule_days must hold distinct digits 1-7 (1 = Monday ... 7 = Sunday)"

    @property
    def schedule_days(self):
        return self._schedule_days

    @schedule_days.setter
    def schedule_days(self, days):
        if isinstance(days, str):
            self._schedule_days = "".join(sorted(days))
        else:
            self._schedule_days = self.stringify_schedule_list(days)

    @property
    def restrictions(self):
        return self._restrictions

    @property
    def is_active(self) -> bool:
        now = dates.utcnow()
        today = str(now.weekday() + 1)
        return today in self.schedule_days and self.hour_start <= now.time() < self.hour_end

    @staticmethod
    def is_valid_schedule_expression(expr: str) -> bool:
        return bool(expr) and re.fullmatch("[1-7]{1,7}", expr) is not None and len(set(expr)) == len(expr)

    @staticmethod
    def parse_schedule_string(schedule: str):
        return [Weekday(int(d)) for d in sorted(schedule)]

    @staticmethod
    def stringify_schedule_list(schedule) -> str:
        return "".join(sorted(str(d.value) for d in schedule))

    def as_dict(self, include_private=False):
        d = super().as_dict(include_private)
        d["scheduleDays"] = [w.to_str() for w in self.parse_schedule_string(self.schedule_days)]
        d["hourStart"] = self.hour_start.strftime("%H:%M")
        d["hourEnd"] = self.hour_end.strftime("%H:%M")
        return d


class Restriction(CRUDModel, Base):
    __tablename__ = "restrictions"
    __table_args__ = {"sqlite_autoincrement": True}
    __public__ = ["id", "name", "created_at", "starts_at", "ends_at", "is_global"]
    id = Column(Integer, primary_key=True, autoincrement=True)
    name = Column(String(50))
    _created_at = Column("created_at", DateTime, default=_utcnow)
    _starts_at = Column("starts_at", DateTime, nullable=False)
    _ends_at = Column("ends_at", DateTime)
    is_global = Column(Boolean, nullable=False)
    _users = relationship("User", secondary="restriction2assignee", back_populates="_restrictions",
                          overlaps="_groups")
    _groups = relationship("Group", secondary="restriction2assignee", back_populates="_restrictions",
                           overlaps="_users")
    _resources = relationship("Resource", secondary="restriction2resource", back_populates="_restrictions")
    _schedules = relationship("RestrictionSchedule", secondary="restriction2schedule", back_populates="_restrictions")

    def __init__(self, name=None, starts_at=None, ends_at=None, is_global=False, **kw):
        super().__init__(**kw)
        self.name = name
        self.starts_at = starts_at
        self.ends_at = ends_at
        self.is_global = is_global

    def __repr__(self):
        return f"<Restriction id={self.id} name={self.name} {self.starts_at}..{self.ends_at} global={self.is_global}>"

    def check_assertions(self):
        if self.ends_at is not None:
            assert self.ends_at >= self.starts_at, "End date must happen after the start date!"
            assert self.ends_at > dates.utcnow(), \
                "You are trying to edit restriction that has already expired - please do not do that!"

    @property
    def starts_at(self):
        return self._starts_at

    @starts_at.setter
    def starts_at(self, value):
        self._starts_at = dates.try_parse(value)

    @property
    def ends_at(self):
        return self._ends_at

    @ends_at.setter
    def ends_at(self, value):
        self._ends_at = dates.try_parse(value)

    @property
    def created_at(self):
        return self._created_at

    @property
    def users(self):
        return self._users

    @property
    def groups(self):
        return self._groups

    @property
    def resources(self):
        return self._resources

    @property
    def schedules(self):
        return self._schedules

    def _add(self, coll, item, what):
        if item in coll:
            raise InvalidRequestException(f"Restriction {self} is already being applied to {what} {item}")
        coll.append(item)
        self.save()
        _refresh_view(item, "_restrictions")

    def _remove(self, coll, item, what):
        if item not in coll:
            raise InvalidRequestException(f"{what} {item} is not affected by restriction {self}")
        coll.remove(item)
        self.save()
        _refresh_view(item, "_restrictions")

    def apply_to_user(self, user):
        self._add(self._users, user, "user")

    def remove_from_user(self, user):
        self._remove(self._users, user, "User")

    def apply_to_group(self, group):
        self._add(self._groups, group, "group")

    def remove_from_group(self, group):
        self._remove(self._groups, group, "Group")

    def apply_to_resource(self, resource):
        self._add(self._resources, resource, "resource")

    def remove_from_resource(self, resource):
        self._remove(self._resources, resource, "Resource")

    def apply_to_resources(self, resources):
        for r in resources:
            if r not in self._resources:
                self._resources.append(r)
        self.save()

    def remove_from_resources(self, resources):
        for r in resources:
            if r in self._resources:
                self._resources.remove(r)
        self.save()

    def add_schedule(self, schedule):
        if schedule in self._schedules:
            raise InvalidRequestException(f"Schedule {schedule} is already applied to restriction {self}")
        self._schedules.append(schedule)
        self.save()

    def remove_schedule(self, schedule):
        if schedule not in self._schedules:
            raise InvalidRequestException(f"Schedule {schedule} is not assigned to restriction {self}")
        self._schedules.remove(schedule)
        self.save()

    def get_all_affected_users(self):
        users = list(self._users)
        for g in self._groups:
            users.extend(g.users)
        return list(dict.fromkeys(users))

    @classmethod
    def get_global_restrictions(cls, include_expired: bool = False):
        q = db_session.query(cls).filter(cls.is_global.is_(True))
        if not include_expired:
            now = dates.utcnow()
            q = q.filter(or_(cls._ends_at.is_(None), cls._ends_at > now))
        return q.all()

    @property
    def is_expired(self) -> bool:
        return self.ends_at is not None and self.ends_at <= dates.utcnow()

    @property
    def is_active(self) -> bool:
        active = self.starts_at <= dates.utcnow() and not self.is_expired
        if not self._schedules:
            return active
        return active and any(s.is_active for s in self._schedules)

    def as_dict(self, include_groups=False, include_users=False, include_resources=False, include_private=False):
        d = super().as_dict(include_private)
        d["schedules"] = [s.as_dict() for s in self._schedules]
        if include_groups:
            d["groups"] = [g.as_dict(include_users=False) for g in self._groups]
        if include_users:
            d["users"] = [u.as_dict(include_groups=False) for u in self._users]
        if include_resources:
            d["resources"] = [r.as_dict() for r in self._resources]
        return d


# ----------------------------------------------------------------------------- reservations
class Reservation(CRUDModel, Base):
    __tablename__ = "reservations"
    __table_args__ = {"sqlite_autoincrement": True}
    __public__ = ["id", "title", "description", "resource_id", "user_id", "gpu_util_avg", "mem_util_avg",
                  "start", "end", "created_at", "is_cancelled"]
    MIN_DURATION = timedelta(minutes=30)
    MAX_DURATION = timedelta(days=8)

    id = Column(Integer, primary_key=True, autoincrement=True)
    user_id = Column(Integer, ForeignKey("users.id", ondelete="CASCADE"), nullable=False)
    user = relationship("User", back_populates="reservations", lazy="joined")
    title = Column(String(60), nullable=False)
    description = Column(String(200), nullable=True)
    resource_id = Column(String(60), nullable=False)
    _is_cancelled = Column("is_cancelled", Boolean, nullable=True)
    gpu_util_avg = Column(Integer, nullable=True)
    mem_util_avg = Column(Integer, nullable=True)
    _start = Column(DateTime, nullable=False)
    _end = Column(DateTime, nullable=False)
    created_at = Column(DateTime, default=_utcnow)

    def __init__(self, start=None, end=None, is_cancelled=None, **kw):
        super().__init__(**kw)
        self.start = start
        self.end = end
        if is_cancelled is not None:
            self.is_cancelled = is_cancelled

    def __repr__(self):
        return f"<Reservation id={self.id} user={self.user_id} res={self.resource_id} {self.start}..{self.end}>"

    def check_assertions(self):
        assert self.user_id, "Reservation owner must be given!"
        assert self.resource_id, "Reservation must be related with a resource!"
        assert self.start, "Reservation start time is invalid!"
        assert self.end, "Reservation end time is invalid!"
        assert self.duration >= self.MIN_DURATION, "Reservation duration is too short!"
        assert self.duration <= self.MAX_DURATION, "Reservation duration is too long!"
        assert self.title is not None and 0 < len(self.title) < 60, "Reservation title length has incorrect length!"
        assert len(self.description or "") < 200, "Reservation description has incorrect length!"
        assert len(self.resource_id) == 40, "Protected resource UUID has incorrect length!"
        assert not self.would_interfere(), "Reservation would interfere with some other reservation!"

    @property
    def duration(self):
        return self.end - self.start

    @property
    def start(self):
        return self._start

    @start.setter
    def start(self, value):
        self._start = dates.try_parse(value)

    @property
    def end(self):
        return self._end

    @end.setter
    def end(self, value):
        self._end = dates.try_parse(value)

    @property
    def is_cancelled(self) -> bool:
        return bool(self._is_cancelled)

    @is_cancelled.setter
    def is_cancelled(self, value):
        self._is_cancelled = value

    @classmethod
    def current_events(cls, resource_id: str | None = None):
        now = dates.utcnow()
        q = cls.query.filter(and_(cls._start <= now, now <= cls._end))
        if resource_id is not None:
            q = q.filter(cls.resource_id == resource_id)
        return [e for e in q.all() if not e.is_cancelled]

    @classmethod
    def upcoming_events_for_resource(cls, resource_id: str, period_after: timedelta):
        now = dates.utcnow()
        q = cls.query.filter(and_(
            cls.resource_id == resource_id,
            or_(and_(cls._start < now, cls._end > now),
                and_(cls._start >= now, cls._start <= now + period_after)))).order_by(cls._start)
        return [e for e in q.all() if not e.is_cancelled]

    def would_interfere(self) -> bool:
        q = Reservation.query.filter(and_(self.start < Reservation._end, self.end > Reservation._start)) \
            .filter(Reservation.resource_id == self.resource_id)
        if self.id is not None:
            q = q.filter(Reservation.id != self.id)
        with db_session.no_autoflush:
            return any(not r.is_cancelled for r in q.all())

    @classmethod
    def filter_by_uuids_and_time_range(cls, uuids, start: datetime.datetime, end: datetime.datetime):
        assert isinstance(start, datetime.datetime) and isinstance(end, datetime.datetime), \
            "Argument must be of type datetime.datetime!"
        return cls.query.filter(and_(cls.resource_id.in_(list(uuids)), cls._start <= end, start <= cls._end)).all()

    def as_dict(self, include_private=False):
        d = super().as_dict(include_private)
        d["userName"] = self.user.username if self.user is not None else None
        return d


# ------------------------------------------------------------------------------- jobs/tasks
class JobStatus(enum.Enum):
    not_running = 1
    running = 2
    terminated = 3
    unsynchronized = 4
    pending = 5


class TaskStatus(enum.Enum):
    not_running = 1
    running = 2
    terminated = 3
    unsynchronized = 4


class SegmentType(enum.Enum):
    env_variable = 1
    parameter = 2


class CommandSegment(CRUDModel, Base):
    __tablename__ = "command_segments"
    __table_args__ = {"sqlite_autoincrement": True}
    __public__ = ["id", "name"]
    id = Column(Integer, primary_key=True, autoincrement=True)
    name = Column(String(50), unique=True, nullable=False)
    _segment_type = Column("segment_type", Enum(SegmentType), default=SegmentType.env_variable, nullable=False)
    links = relationship("CommandSegment2Task", back_populates="segment", cascade="all, delete-orphan",
                         passive_deletes=True)

    def __init__(self, name=None, segment_type=None, _segment_type=None, **kw):
        super().__init__(**kw)
        self.name = name
        st = segment_type or _segment_type
        if st is not None:
            self._segment_type = st

    def __repr__(self):
        return f"<Segment id={self.id}, name={self.name}, type={self.segment_type}>"

    @property
    def segment_type(self):
        return self._segment_type

    @property
    def tasks(self):
        return [lk.task for lk in self.links]

    @classmethod
    def find_by_name(cls, name):
        try:
            return db_session.query(cls).filter_by(name=name).one()
        except NoResultFound as e:
            raise NoResultFound(f"There is no command segment with name={name}!") from e
        except MultipleResultsFound as e:  # pragma: no cover - unique constraint
            raise MultipleResultsFound("duplicate command segment names") from e


class CommandSegment2Task(Base):
    __tablename__ = "cmd_segment2task"
    task_id = Column(Integer, ForeignKey("tasks.id", ondelete="CASCADE"), primary_key=True)
    cmd_segment_id = Column(Integer, ForeignKey("command_segments.id", ondelete="CASCADE"), primary_key=True)
    _value = Column(String(100))
    _index = Column(Integer)  # > 0: parameter position, < 0: env variable position
    task = relationship("Task", back_populates="segment_links")
    segment = relationship("CommandSegment", back_populates="links")

    @property
    def index(self):
        return self._index

    @property
    def value(self):
        return self._value


class Task(CRUDModel, Base):
    __tablename__ = "tasks"
    __table_args__ = {"sqlite_autoincrement": True}
    __public__ = ["id", "job_id", "hostname", "pid", "command"]
    id = Column(Integer, primary_key=True, autoincrement=True)
    job_id = Column(Integer, ForeignKey("jobs.id", ondelete="CASCADE"))
    job = relationship("Job", back_populates="_tasks")
    hostname = Column(String(40), nullable=False)
    pid = Column(Integer)
    _status = Column(Enum(TaskStatus), default=TaskStatus.not_running, nullable=False)
    command = Column(String(400), nullable=False)
    gpu_id = Column(Integer, nullable=True)
    segment_links = relationship("CommandSegment2Task", back_populates="task", cascade="all, delete-orphan",
                                 passive_deletes=True, order_by="CommandSegment2Task._index")

    def __init__(self, status=None, **kw):
        super().__init__(**kw)
        self._status = status or TaskStatus.not_running

    def __repr__(self):
        return f"<Task id={self.id} job={self.job_id} host={self.hostname} pid={self.pid} status={self._status.name}>"

    @property
    def status(self):
        return self._status

    @status.setter
    def status(self, value):
        self._status = value
        if self.job is not None:
            self.job.synchronize_status()

    @property
    def cmd_segments(self):
        return [lk.segment for lk in self.segment_links]

    @property
    def number_of_params(self):
        return sum(1 for lk in self.segment_links if lk.segment.segment_type == SegmentType.parameter)

    @property
    def number_of_env_vars(self):
        return sum(1 for lk in self.segment_links if lk.segment.segment_type == SegmentType.env_variable)

    def envs(self):
        """[(name, value)] in insertion order (index -1, -2, ...)."""
        return [(lk.segment.name, lk.value or "") for lk in
                sorted((lk for lk in self.segment_links if lk.index is not None and lk.index < 0),
                       key=lambda lk: -lk.index)]

    def params(self):
        return [(lk.segment.name, lk.value or "") for lk in
                sorted((lk for lk in self.segment_links if lk.index is not None and lk.index > 0),
                       key=lambda lk: lk.index)]

    @property
    def full_command(self) -> str:
        return self.render(self.envs(), self.params())

    def render(self, envs, params) -> str:
        """``ENV=v ... command param value ...`` from explicit segment lists (the launch path
        substitutes allocated devices before rendering, see ``core/allocation.py``).

        The line runs under ``bash -lc``: a value the shell would split -- unquoted spaces or
        control operators, an unbalanced quote -- and a TF_CONFIG JSON document are
        single-quoted; every other value stays as typed, so ``$HOME``, globs and the user's own
        quoting keep their shell meaning (see ``_shell_value``)."""
        parts = [f"{n}={_shell_value(v)}" for n, v in envs]
        parts.append(self.command)
        for n, v in params:
            v = _shell_value(v)
            if v == "":
                parts.append(n)
            elif n.endswith("=") or n.endswith(" "):
                parts.append(n + v)
            else:
                parts.append(f"{n} {v}")
        return " ".join(p for p in parts if p != "")

    def get_cmd_segment_link(self, segment):
        for lk in self.segment_links:
            if lk.segment is segment or (segment.id is not None and lk.cmd_segment_id == segment.id):
                return lk
        raise Exception(f"Segment {segment} is not assigned to task {self}!")

    def add_cmd_segment(self, segment, value: str):
        if segment in self.cmd_segments:
            raise Exception(f"Segment {segment} is already assigned to task {self}!")
        if segment.segment_type == SegmentType.env_variable:
            idx = -(self.number_of_env_vars + 1)
        else:
            idx = self.number_of_params + 1
        lk = CommandSegment2Task(_value=value, _index=idx)
        lk.segment = segment
        self.segment_links.append(lk)
        self.save()

    def remove_cmd_segment(self, segment):
        lk = self.get_cmd_segment_link(segment)
        removed = lk.index
        self.segment_links.remove(lk)
        for other in self.segment_links:
            if segment.segment_type == SegmentType.env_variable:
                if other.index < 0 and other.index < removed:
                    other._index = other.index + 1
            elif other.index > 0 and other.index > removed:
                other._index = other.index - 1
        self.save()

    def as_dict(self, include_private=None):
        d = super().as_dict(bool(include_private))
        d["status"] = self._status.name
        envs, params = [], []
        for lk in self.segment_links:
            seg = {"name": lk.segment.name, "value": lk.value, "index": lk.index}
            (envs if lk.segment.segment_type == SegmentType.env_variable else params).append(seg)
        d["cmdsegments"] = {"envs": envs, "params": params}
        d["fullCommand"] = self.full_command
        d["gpuId"] = self.gpu_id  # additive: first device of HIP_VISIBLE_DEVICES
        # additive: the HIP indices this task holds while launching/running (auto:N requests
        # resolve here; see core/allocation.py)
        d["allocatedGpus"] = [a.gpu_index for a in GpuAllocation.for_task(self.id)] if self.id else []
        pol = TaskRestartPolicy.for_task(self.id) if self.id else None
        d["maxRestarts"] = pol.max_restarts if pol else 0  # additive: restart policy (th-run)
        d["restarts"] = pol.restarts if pol else 0
        return d

    @property
    def max_restarts(self) -> int:
        pol = TaskRestartPolicy.for_task(self.id) if self.id else None
        return pol.max_restarts if pol else 0

    def set_max_restarts(self, n: int) -> None:
        assert isinstance(n, int) and not isinstance(n, bool) and 0 <= n <= 100, \
            "maxRestarts must be an integer in [0, 100]"
        pol = TaskRestartPolicy.for_task(self.id)
        if pol is None:
            pol = TaskRestartPolicy(task_id=self.id, max_restarts=n, restarts=0)
        pol.max_restarts = n
        pol.save()

    def record_restarts(self, restarts: int, last_exit_code=None) -> None:
        pol = TaskRestartPolicy.for_task(self.id)
        if pol is not None and (pol.restarts != restarts or pol.last_exit_code != last_exit_code):
            pol.restarts = restarts
            pol.last_exit_code = last_exit_code
            pol.save()


class Job(CRUDModel, Base):
    __tablename__ = "jobs"
    __table_args__ = {"sqlite_autoincrement": True}
    __public__ = ["id", "name", "description", "user_id", "start_at", "stop_at"]
    id = Column(Integer, primary_key=True, autoincrement=True)
    name = Column(String(40), nullable=False)
    description = Column(Text)
    user_id = Column(Integer, ForeignKey("users.id", ondelete="CASCADE"))
    user = relationship("User", back_populates="_jobs")
    _status = Column(Enum(JobStatus), default=JobStatus.not_running, nullable=False)
    _start_at = Column(DateTime)
    _stop_at = Column(DateTime)
    is_queued = Column(Boolean)
    _tasks = relationship("Task", back_populates="job", cascade="all, delete-orphan", passive_deletes=True,
                          order_by="Task.id")

    def __init__(self, start_at=None, stop_at=None, status=None, **kw):
        super().__init__(**kw)
        self._status = status or JobStatus.not_running
        self.start_at = start_at
        self.stop_at = stop_at

    def __repr__(self):
        return f"<Job id={self.id}, name={self.name}, user={self.user_id}, status={self._status.name}>"

    def check_assertions(self):
        if self.stop_at is not None and self.start_at is not None:
            assert self.stop_at >= self.start_at, "Time of the end must happen after the start!"

    @property
    def tasks(self):
        return self._tasks

    @property
    def number_of_tasks(self):
        return len(self._tasks)

    @property
    def status(self):
        return self._status

    def add_task(self, task):
        if task in self._tasks:
            raise InvalidRequestException(f"Task {task} is already assigned to job {self}!")
        self._tasks.append(task)
        self.synchronize_status()
        self.save()

    def remove_task(self, task):
        if task not in self._tasks:
            raise InvalidRequestException(f"Task {task} is not assigned to job {self}!")
        self._tasks.remove(task)
        self.save()

    def synchronize_status(self):
        """Derive the job status from its tasks (reference ``models/Job.py:81-99``)."""
        before = self._status
        statuses = [t.status for t in self._tasks]
        if TaskStatus.unsynchronized in statuses and self._status is not JobStatus.pending:
            self._status = JobStatus.unsynchronized
        elif TaskStatus.running in statuses:
            self._status = JobStatus.running
        elif TaskStatus.terminated in statuses:
            self._status = JobStatus.terminated
        elif TaskStatus.not_running in statuses and self._status is not JobStatus.pending:
            self._status = JobStatus.not_running
        if before is JobStatus.running and self._status is not JobStatus.running:
            self.is_queued = False
        self.save()

    def enqueue(self):
        assert self._status is not JobStatus.pending, "Cannot enqueue job that is already pending"
        assert TaskStatus.running not in [t.status for t in self._tasks], \
            "Cannot enqueue job that contains running tasks"
        self.is_queued = True
        self._status = JobStatus.pending
        self.save()

    def dequeue(self):
        assert self._status == JobStatus.pending, "Only pending jobs can be dequeued"
        self.is_queued = False
        self._status = JobStatus.not_running
        self.save()

    @property
    def start_at(self):
        return self._start_at

    @start_at.setter
    def start_at(self, value):
        d = dates.try_parse(value) if value is not None else None
        if d is not None and d < dates.utcnow():
            d = dates.utcnow()  # fork behaviour: a start in the past means "now"
        self._start_at = d

    @property
    def stop_at(self):
        return self._stop_at

    @stop_at.setter
    def stop_at(self, value):
        self._stop_at = dates.try_parse(value) if value is not None else None

    def as_dict(self, include_private=None):
        d = super().as_dict(bool(include_private))
        d["status"] = self._status.name
        d["isQueued"] = bool(self.is_queued)  # additive (dashboard queue badge)
        return d

    @staticmethod
    def get_job_queue():
        return Job.query.filter(Job.is_queued.is_(True)).filter(Job._status != JobStatus.running).all()

    @staticmethod
    def get_jobs_running_from_queue():
        return Job.query.filter(Job.is_queued.is_(True)).filter(Job._status == JobStatus.running).all()


# ----------------------------------------------------------------------------- allocations
class GpuAllocation(CRUDModel, Base):
    """One GPU held by one task while it is launching or running (daemon-owned, additive table).

    The reference kept no record of which GPU a task held: the scheduler re-derived it from
    ``CUDA_VISIBLE_DEVICES`` each tick and deduplicated within one round only
    (``core/services/JobSchedulingService.py:140-168``).  Here every launch inserts one row per
    device; the UNIQUE (hostname, gpu_index) constraint makes a double allocation impossible at
    the database level, whatever thread or request tries it (see :mod:`..core.allocation`).
    The table lives outside the alembic revision chain (created idempotently next to it), so a
    database stays readable by TensorHive 1.1."""

    __tablename__ = "gpu_allocations"
    __table_args__ = (UniqueConstraint("hostname", "gpu_index", name="uq_gpu_allocations_host_gpu"),
                      {"sqlite_autoincrement": True})
    __public__ = ["id", "task_id", "job_id", "hostname", "gpu_index", "gpu_uuid", "created_at"]
    id = Column(Integer, primary_key=True, autoincrement=True)
    task_id = Column(Integer, ForeignKey("tasks.id", ondelete="CASCADE"), nullable=False, index=True)
    job_id = Column(Integer, ForeignKey("jobs.id", ondelete="CASCADE"), nullable=True)
    hostname = Column(String(40), nullable=False)
    gpu_index = Column(Integer, nullable=False)
    gpu_uuid = Column(String(64), nullable=True)
    created_at = Column(DateTime, default=_utcnow, nullable=False)

    def __repr__(self):
        return f"<GpuAllocation task={self.task_id} {self.hostname}:{self.gpu_index}>"

    @classmethod
    def for_task(cls, task_id: int):
        return cls.query.filter(cls.task_id == task_id).order_by(cls.id).all()

    @classmethod
    def held(cls) -> set[tuple[str, int]]:
        return {(a.hostname, a.gpu_index) for a in cls.query.all()}


class TaskRestartPolicy(CRUDModel, Base):
    """Restart policy of one task (daemon-owned, additive table, like ``gpu_allocations``).

    The reference only detects a failed task (``core/services/JobSchedulingService.py:210-252``);
    here ``max_restarts`` is passed to ``th-run spawn --max-restarts`` and the supervisor starts a
    run that exited non-zero again, unless the stop was requested.  ``restarts`` and
    ``last_exit_code`` mirror the supervisor's session state at each synchronisation."""

    __tablename__ = "task_restart_policies"
    __public__ = ["task_id", "max_restarts", "restarts", "last_exit_code"]
    task_id = Column(Integer, ForeignKey("tasks.id", ondelete="CASCADE"), primary_key=True)
    max_restarts = Column(Integer, default=0, nullable=False)
    restarts = Column(Integer, default=0, nullable=False)
    last_exit_code = Column(Integer, nullable=True)

    @classmethod
    def for_task(cls, task_id: int):
        return cls.query.filter(cls.task_id == task_id).first()
