"""Weekly restriction schedules (reference ``controllers/schedule.py``)."""
from __future__ import annotations

from datetime import datetime

from ..core.verifier import update_user_reservations_statuses
from ..models.orm import RestrictionSchedule
from ..utils.weekday import Weekday
from ._common import Abort, M, check_fields, guarded


def _days(names):
    try:
        return [Weekday[d] for d in names]
    except KeyError:
        raise Abort(422, M("general.bad_request"))


def _hour(s: str):
    try:
        return datetime.strptime(s, "%H:%M").time()
    except ValueError:
        raise Abort(422, M("general.bad_request"))


def get():
    return [s.as_dict() for s in RestrictionSchedule.all()], 200


@guarded(not_found="schedule.not_found")
def get_by_id(id: int):
    return {"msg": M("schedule.get.success"), "schedule": RestrictionSchedule.get(id).as_dict()}, 200


@guarded(assertion="schedule.create.failure.invalid")
def create(schedule: dict):
    s = RestrictionSchedule(schedule_days=_days(schedule["scheduleDays"]), hour_start=_hour(schedule["hourStart"]),
                            hour_end=_hour(schedule["hourEnd"]))
    s.save()
    return {"msg": M("schedule.create.success"), "schedule": s.as_dict()}, 201


def _recheck_all(restrictions, increased=None):
    for r in restrictions:
        for u in r.get_all_affected_users():
            if increased is None:
                update_user_reservations_statuses(u, True)
                update_user_reservations_statuses(u, False)
            else:
                update_user_reservations_statuses(u, increased)


@guarded(not_found="schedule.not_found", assertion="schedule.update.failure.assertions")
def update(id: int, newValues: dict):
    check_fields(newValues, {"scheduleDays", "hourStart", "hourEnd"})
    s = RestrictionSchedule.get(id)
    if "scheduleDays" in newValues:
        s.schedule_days = _days(newValues["scheduleDays"])
    if "hourStart" in newValues:
        s.hour_start = _hour(newValues["hourStart"])
    if "hourEnd" in newValues:
        s.hour_end = _hour(newValues["hourEnd"])
    s.save()
    _recheck_all(s.restrictions)
    return {"msg": M("schedule.update.success"), "schedule": s.as_dict()}, 200


@guarded(not_found="schedule.not_found", assertion_status=403)
def delete(id: int):
    s = RestrictionSchedule.get(id)
    restrictions = list(s.restrictions)
    s.destroy()
    for r in restrictions:
        from ..database import db_session

        db_session.refresh(r)
        _recheck_all([r], increased=len(r.schedules) == 0)
    return {"msg": M("schedule.delete.success")}, 200
