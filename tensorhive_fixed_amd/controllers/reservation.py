"""GPU reservations (reference ``controllers/reservation.py``).

Fork behaviour kept (and tested): reservations may start in the past (the reference's past-start
check is commented out, ``reservation.py:89-90``).  Creation runs the permission verifier;
owners may delete only future reservations, admins any.
"""
from __future__ import annotations

from ..core.verifier import is_reservation_allowed
from ..models.orm import Reservation, User
from ..utils import dates
from ..utils.exceptions import ForbiddenException
from ._common import M, guarded, is_admin, me, snake


def get(resources_ids: list | None = None, start: str | None = None, end: str | None = None):
    if resources_ids is None and start is None and end is None:
        return [r.as_dict() for r in Reservation.all()], 200
    if not (resources_ids and start and end):
        return {"msg": M("general.bad_request")}, 400
    try:
        s, e = dates.parse(start), dates.parse(end)
        found = Reservation.filter_by_uuids_and_time_range(resources_ids, s, e)
    except (ValueError, AssertionError) as err:
        return {"msg": f"{M('general.bad_request')}. {err}"}, 400
    return [r.as_dict() for r in found], 200


@guarded(forbidden="reservation.create.failure.forbidden", assertion="reservation.create.failure.invalid")
def create(reservation: dict):
    r = Reservation(title=reservation["title"], description=reservation["description"],
                    resource_id=reservation["resourceId"], user_id=reservation["userId"],
                    start=reservation["start"], end=reservation["end"])
    if not is_admin() and r.user_id != me():
        raise ForbiddenException("Cannot reserve resources in another user's name")
    owner = User.get(r.user_id if is_admin() else me())
    if not is_reservation_allowed(owner, r):
        raise ForbiddenException("Reservation not allowed")
    r.save()
    _notify_scheduler()
    return {"msg": M("reservation.create.success"), "reservation": r.as_dict()}, 201


@guarded(not_found="reservation.not_found", forbidden="reservation.update.failure.forbidden",
         assertion="reservation.update.failure.assertions")
def update(id: int, newValues: dict):
    r = Reservation.get(id)
    now = dates.utcnow()
    if r.end < now and not is_admin():
        raise ForbiddenException("reservation already finished")
    allowed = {"title", "description", "resourceId", "end"}
    if r.start > now or is_admin():
        allowed.add("start")
    if not set(newValues).issubset(allowed):
        raise ForbiddenException("invalid field is present")
    for k, v in newValues.items():
        setattr(r, snake(k), v)
    owner = User.get(r.user_id)
    if not (is_admin() or r.user_id == me()) or not is_reservation_allowed(owner, r):
        raise ForbiddenException("reservation not allowed")
    r.is_cancelled = False
    r.save()
    _notify_scheduler()
    return {"msg": M("reservation.update.success"), "reservation": r.as_dict()}, 201


@guarded(not_found="reservation.not_found", assertion_status=403)
def delete(id: int):
    r = Reservation.get(id)
    assert (r.start > dates.utcnow() and r.user_id == me()) or is_admin(), M("general.unprivileged")
    r.destroy()
    _notify_scheduler()
    return {"msg": M("reservation.delete.success")}, 200


def _notify_scheduler() -> None:
    """Reservation changes can free or block GPUs: wake the job scheduler (event-driven)."""
    from ..api.app import daemon

    d = daemon()
    if d is not None:
        d.wake("reservation")
