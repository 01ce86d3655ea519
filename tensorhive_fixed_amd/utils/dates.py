"""API date formats (part of the wire contract; reference ``utils/DateUtils.py:8-69``).

Input: ``%Y-%m-%dT%H:%M:%S.%fZ``; output: ``%Y-%m-%dT%H:%M:%S+00:00``.  Everything is naive UTC.
"""
from __future__ import annotations

import datetime as _dt

INPUT_FORMAT = "%Y-%m-%dT%H:%M:%S.%fZ"
OUTPUT_FORMAT = "%Y-%m-%dT%H:%M:%S"
SERVER_TZ = "+00:00"


def utcnow() -> _dt.datetime:
    """Naive UTC now (the DB stores naive UTC datetimes)."""
    return _dt.datetime.now(_dt.timezone.utc).replace(tzinfo=None)


def parse(value: str) -> _dt.datetime:
    """Parse an API datetime; also accepts the output format and plain ISO strings."""
    for fmt in (INPUT_FORMAT, "%Y-%m-%dT%H:%M:%SZ", "%Y-%m-%dT%H:%M:%S"):
        try:
            return _dt.datetime.strptime(value, fmt)
        except ValueError:
            pass
    v = value.strip()
    if v.endswith("Z"):
        v = v[:-1] + "+00:00"
    d = _dt.datetime.fromisoformat(v)
    if d.tzinfo is not None:
        d = d.astimezone(_dt.timezone.utc).replace(tzinfo=None)
    return d


def try_parse(value) -> _dt.datetime | None:
    if isinstance(value, str):
        return parse(value)
    if isinstance(value, _dt.datetime):
        return value
    return None


def stringify(value: _dt.datetime) -> str:
    return value.strftime(OUTPUT_FORMAT) + SERVER_TZ


def to_api_input(value: _dt.datetime) -> str:
    return value.strftime(INPUT_FORMAT)


def try_stringify(value: _dt.datetime | None) -> str | None:
    return None if value is None else stringify(value)


def utc2local(value: _dt.datetime) -> _dt.datetime:
    """UTC naive -> local naive (used in e-mail text; reference ``core/utils/time.py:5-9``)."""
    return value.replace(tzinfo=_dt.timezone.utc).astimezone().replace(tzinfo=None)
