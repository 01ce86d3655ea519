"""Reservation permission check (reference ``core/utils/ReservationVerifier.py:6-109``).

A reservation ``[start, end)`` on resource R is allowed iff the union of the owner's restrictions
(own + groups', non-expired, global or covering R) covers the whole interval, honouring weekly
schedules -- including windows that wrap past midnight (``hour_start > hour_end``) and the
``23:59`` "until end of day" convention.  The algorithm advances a cursor from ``start``: any
restriction active at the cursor pushes it to the end of the window it grants; the reservation
is allowed once the cursor reaches ``end``.  Pure and deterministic -> unit tested heavily.
"""
from __future__ import annotations

from datetime import datetime, time, timedelta

from sqlalchemy.exc import NoResultFound

from ..utils import dates

_END_OF_DAY = time(hour=23, minute=59)


def _advance_by_schedules(cursor: datetime, end: datetime, schedules) -> datetime:
    """Latest instant >= cursor reachable through back-to-back schedule windows."""
    while True:
        moved = False
        for sch in schedules:
            day = cursor.weekday() + 1
            days = sch.schedule_days
            if str(day) in days and sch.hour_start <= cursor.time():
                if sch.hour_end == _END_OF_DAY:
                    cursor = cursor.replace(hour=0, minute=0, second=0, microsecond=0) + timedelta(days=1)
                elif sch.hour_start > sch.hour_end:  # window wraps past midnight
                    cursor = cursor.replace(hour=sch.hour_end.hour, minute=sch.hour_end.minute,
                                            second=0, microsecond=0) + timedelta(days=1)
                elif cursor.time() < sch.hour_end:
                    cursor = cursor.replace(hour=sch.hour_end.hour, minute=sch.hour_end.minute,
                                            second=0, microsecond=0)
                else:
                    continue
                moved = True
            elif str(((day - 2) % 7) + 1) in days and cursor.time() < sch.hour_end < sch.hour_start:
                # a window that started the previous day and has not ended yet
                cursor = cursor.replace(hour=sch.hour_end.hour, minute=sch.hour_end.minute, second=0, microsecond=0)
                moved = True
            if cursor.minute == 59:
                cursor = cursor + timedelta(minutes=1)
            if cursor >= end:
                return cursor
        if not moved:
            return cursor


def is_reservation_allowed(user, reservation) -> bool:
    from ..models.orm import Resource

    try:
        resource = Resource.get(reservation.resource_id)
    except NoResultFound:
        return False
    candidates = [r for r in user.get_restrictions(include_group=True)
                  if r.is_global or resource in r.resources]
    cursor, end = reservation.start, reservation.end
    while True:
        moved = False
        for r in candidates:
            if r.starts_at <= cursor and (r.ends_at is None or cursor < r.ends_at):
                if not r.schedules:
                    if r.ends_at is None:
                        return True
                    cursor = r.ends_at
                    moved = True
                else:
                    nxt = _advance_by_schedules(cursor, end, r.schedules)
                    if r.ends_at is not None:
                        nxt = min(nxt, max(cursor, r.ends_at))
                    if nxt > cursor:
                        cursor = nxt
                        moved = True
                if cursor >= end:
                    return True
        if not moved:
            return False


def update_user_reservations_statuses(user, have_users_permissions_increased: bool) -> None:
    """Re-evaluate ``is_cancelled`` of the user's future reservations after a permission change."""
    now = dates.utcnow()
    for res in user.get_reservations(include_cancelled=True):
        if res.end <= now:
            continue
        if have_users_permissions_increased:
            if res.is_cancelled and is_reservation_allowed(user, res) and not res.would_interfere():
                res.is_cancelled = False
                res.save()
        elif not res.is_cancelled and not is_reservation_allowed(user, res):
            res.is_cancelled = True
            res.save()


class ReservationVerifier:
    """Class-style facade kept for API parity with the reference."""

    is_reservation_allowed = staticmethod(is_reservation_allowed)
    update_user_reservations_statuses = staticmethod(update_user_reservations_statuses)
