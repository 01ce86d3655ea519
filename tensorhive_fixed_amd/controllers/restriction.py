"""Restrictions (permissions) and their assignment to users/groups/resources/hosts/schedules
(reference ``controllers/restriction.py``).  Every change that widens or narrows someone's
permissions re-evaluates the ``is_cancelled`` flag of their future reservations."""
from __future__ import annotations

from sqlalchemy.exc import NoResultFound

from ..core.verifier import update_user_reservations_statuses
from ..models.orm import Group, Resource, Restriction, RestrictionSchedule, User
from ..utils import dates
from ._common import Abort, M, check_fields, guarded, snake

FULL = dict(include_groups=True, include_users=True, include_resources=True)


def _recheck(users, increased: bool | None) -> None:
    for u in users:
        if increased is None:
            update_user_reservations_statuses(u, True)
            update_user_reservations_statuses(u, False)
        else:
            update_user_reservations_statuses(u, increased)


@guarded(assertion_status=400)
def get(user_id: int | None = None, group_id: int | None = None, resource_id: str | None = None,
        schedule_id: int | None = None, include_user_groups: bool | None = None):
    if all(v is None for v in (user_id, group_id, resource_id, schedule_id, include_user_groups)):
        return [r.as_dict(**FULL) for r in Restriction.all()], 200
    found = []
    try:
        if user_id is not None:
            found += User.get(user_id).get_restrictions(include_group=bool(include_user_groups))
        if group_id is not None:
            found += Group.get(group_id).get_restrictions()
        if resource_id is not None:
            found += Resource.get(resource_id).get_restrictions()
        if schedule_id is not None:
            found += list(RestrictionSchedule.get(schedule_id).restrictions)
    except NoResultFound:
        return {"msg": M("general.bad_request")}, 400
    opts = dict(include_groups=group_id is None, include_users=user_id is None,
                include_resources=schedule_id is None)
    return [r.as_dict(**opts) for r in dict.fromkeys(found)], 200


@guarded(assertion="restriction.create.failure.invalid")
def create(restriction: dict):
    r = Restriction(name=restriction.get("name"), starts_at=restriction["startsAt"],
                    ends_at=dates.try_parse(restriction.get("endsAt")), is_global=restriction["isGlobal"])
    r.save()
    return {"msg": M("restriction.create.success"), "restriction": r.as_dict(**FULL)}, 201


@guarded(not_found="restriction.not_found", assertion="restriction.update.failure.assertions")
def update(id: int, newValues: dict):
    check_fields(newValues, {"name", "startsAt", "endsAt", "isGlobal"})
    r = Restriction.get(id)
    for k, v in newValues.items():
        setattr(r, snake(k), v)
    r.save()
    _recheck(r.get_all_affected_users(), None)
    return {"msg": M("restriction.update.success"), "restriction": r.as_dict(**FULL)}, 200


@guarded(not_found="restriction.not_found", assertion_status=403)
def delete(id: int):
    r = Restriction.get(id)
    users = r.get_all_affected_users()
    r.destroy()
    _recheck(users, False)
    return {"msg": M("restriction.delete.success")}, 200


def _restriction(rid: int) -> Restriction:
    try:
        return Restriction.get(rid)
    except NoResultFound:
        raise Abort(404, M("restriction.not_found"))


def _target(cls, key, not_found: str):
    try:
        return cls.get(key)
    except NoResultFound:
        raise Abort(404, M(not_found))


def _ok(path: str, r: Restriction):
    return {"msg": M(path), "restriction": r.as_dict(**FULL)}, 200


@guarded(invalid="restriction.users.apply.failure.duplicate", assertion="restriction.users.apply.failure.assertions")
def apply_to_user(restriction_id: int, user_id: int):
    r = _restriction(restriction_id)
    u = _target(User, user_id, "user.not_found")
    r.apply_to_user(u)
    _recheck([u], True)
    return _ok("restriction.users.apply.success", r)


@guarded(invalid="restriction.users.remove.failure.not_found", invalid_status=404,
         assertion="restriction.users.remove.failure.assertions")
def remove_from_user(restriction_id: int, user_id: int):
    r = _restriction(restriction_id)
    u = _target(User, user_id, "user.not_found")
    r.remove_from_user(u)
    _recheck([u], False)
    return _ok("restriction.users.remove.success", r)


@guarded(invalid="restriction.groups.apply.failure.duplicate", assertion="restriction.groups.apply.failure.assertions")
def apply_to_group(restriction_id: int, group_id: int):
    r = _restriction(restriction_id)
    g = _target(Group, group_id, "group.not_found")
    r.apply_to_group(g)
    _recheck(g.users, True)
    return _ok("restriction.groups.apply.success", r)


@guarded(invalid="restriction.groups.remove.failure.not_found", invalid_status=404,
         assertion="restriction.groups.remove.failure.assertions")
def remove_from_group(restriction_id: int, group_id: int):
    r = _restriction(restriction_id)
    g = _target(Group, group_id, "group.not_found")
    r.remove_from_group(g)
    _recheck(g.users, False)
    return _ok("restriction.groups.remove.success", r)


@guarded(invalid="restriction.resources.apply.failure.duplicate",
         assertion="restriction.resources.apply.failure.assertions")
def apply_to_resource(restriction_id: int, resource_uuid: str):
    r = _restriction(restriction_id)
    res = _target(Resource, resource_uuid, "resource.not_found")
    r.apply_to_resource(res)
    _recheck(r.get_all_affected_users(), True)
    return _ok("restriction.resources.apply.success", r)


@guarded(invalid="restriction.resources.remove.failure.not_found", invalid_status=404,
         assertion="restriction.resources.remove.failure.assertions")
def remove_from_resource(restriction_id: int, resource_uuid: str):
    r = _restriction(restriction_id)
    res = _target(Resource, resource_uuid, "resource.not_found")
    r.remove_from_resource(res)
    _recheck(r.get_all_affected_users(), False)
    return _ok("restriction.resources.remove.success", r)


def _host_resources(hostname: str):
    from .nodes import register_resources_from_snapshot

    register_resources_from_snapshot()
    res = Resource.get_by_hostname(hostname)
    if not res:
        raise Abort(404, M("nodes.hostname.not_found"))
    return res


@guarded(assertion="restriction.hosts.apply.failure.assertions")
def apply_to_resources_by_hostname(restriction_id: int, hostname: str):
    r = _restriction(restriction_id)
    r.apply_to_resources(_host_resources(hostname))
    _recheck(r.get_all_affected_users(), True)
    return _ok("restriction.hosts.apply.success", r)


@guarded(assertion="restriction.hosts.remove.failure.assertions")
def remove_from_resources_by_hostname(restriction_id: int, hostname: str):
    r = _restriction(restriction_id)
    r.remove_from_resources(_host_resources(hostname))
    _recheck(r.get_all_affected_users(), False)
    return _ok("restriction.hosts.remove.success", r)


@guarded(invalid="restriction.schedules.add.failure.duplicate", assertion="restriction.schedules.add.failure.assertions")
def add_schedule(restriction_id: int, schedule_id: int):
    r = _restriction(restriction_id)
    s = _target(RestrictionSchedule, schedule_id, "schedule.not_found")
    first = not r.schedules
    r.add_schedule(s)
    # the first schedule narrows an always-on restriction; further ones widen it
    _recheck(r.get_all_affected_users(), not first)
    return _ok("restriction.schedules.add.success", r)


@guarded(invalid="restriction.schedules.remove.failure.not_found", invalid_status=404,
         assertion="restriction.schedules.remove.failure.assertions")
def remove_schedule(restriction_id: int, schedule_id: int):
    r = _restriction(restriction_id)
    s = _target(RestrictionSchedule, schedule_id, "schedule.not_found")
    r.remove_schedule(s)
    _recheck(r.get_all_affected_users(), not r.schedules)
    return _ok("restriction.schedules.remove.success", r)
