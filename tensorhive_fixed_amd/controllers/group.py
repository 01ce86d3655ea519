"""Groups and memberships (reference ``controllers/group.py``)."""
from __future__ import annotations

from ..core.verifier import update_user_reservations_statuses
from ..models.orm import Group, User
from ._common import Abort, M, check_fields, guarded, snake


def get(only_default: bool = False):
    groups = Group.get_default_groups() if only_default else Group.all()
    return [g.as_dict() for g in groups], 200


@guarded(not_found="group.not_found")
def get_by_id(id: int):
    return {"msg": M("group.get.success"), "group": Group.get(id).as_dict()}, 200


@guarded(assertion="group.create.failure.invalid")
def create(group: dict):
    g = Group(name=group["name"], is_default=bool(group.get("isDefault", False)))
    g.save()
    return {"msg": M("group.create.success"), "group": g.as_dict()}, 201


@guarded(not_found="group.not_found", assertion="group.update.failure.assertions")
def update(id: int, newValues: dict):
    check_fields(newValues, {"name", "isDefault"})
    g = Group.get(id)
    for k, v in newValues.items():
        setattr(g, snake(k), v)
    g.save()
    return {"msg": M("group.update.success"), "group": g.as_dict()}, 200


@guarded(not_found="group.not_found", assertion_status=403)
def delete(id: int):
    g = Group.get(id)
    members = list(g.users)
    g.destroy()
    for u in members:
        update_user_reservations_statuses(u, have_users_permissions_increased=False)
    return {"msg": M("group.delete.success")}, 200


def _get_pair(group_id: int, user_id: int):
    from sqlalchemy.exc import NoResultFound

    try:
        g = Group.get(group_id)
    except NoResultFound:
        raise Abort(404, M("group.not_found"))
    try:
        u = User.get(user_id)
    except NoResultFound:
        raise Abort(404, M("user.not_found"))
    return g, u


@guarded(invalid="group.users.add.failure.duplicate", assertion="group.users.add.failure.assertions")
def add_user(group_id: int, user_id: int):
    g, u = _get_pair(group_id, user_id)
    g.add_user(u)
    update_user_reservations_statuses(u, have_users_permissions_increased=True)
    return {"msg": M("group.users.add.success"), "group": g.as_dict()}, 200


@guarded(invalid="group.users.remove.failure.not_found", invalid_status=404,
         assertion="group.users.remove.failure.assertions")
def remove_user(group_id: int, user_id: int):
    g, u = _get_pair(group_id, user_id)
    g.remove_user(u)
    update_user_reservations_statuses(u, have_users_permissions_increased=False)
    return {"msg": M("group.users.remove.success"), "group": g.as_dict()}, 200
