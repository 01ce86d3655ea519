"""Users, login/logout, token refresh, SSH self-signup (reference ``controllers/user.py``)."""
from __future__ import annotations

import logging

from sqlalchemy.exc import IntegrityError

from ..api import auth
from ..api.app import daemon
from ..config import get_config
from ..models.orm import Group, RevokedToken, Role, User
from ._common import Abort, M, guarded, is_admin, me

log = logging.getLogger(__name__)


def get():
    priv = is_admin()
    return [u.as_dict(include_private=priv) for u in User.all()], 200


@guarded(not_found="user.not_found")
def get_by_id(id: int):
    user = User.get(id)
    priv = is_admin() or id == me()
    return {"msg": M("user.get.success"), "user": user.as_dict(include_private=priv)}, 200


def do_create(form: dict):
    try:
        user = User(username=form["username"], email=form["email"], password=form["password"],
                    roles=[Role(name="user")])
        user.save()
    except AssertionError as e:
        from ..database import db_session

        db_session.rollback()
        return {"msg": M("user.create.failure.invalid", reason=e)}, 422
    except IntegrityError:
        from ..database import db_session

        db_session.rollback()
        return {"msg": M("user.create.failure.duplicate")}, 409
    for group in Group.get_default_groups():
        try:
            group.add_user(user)
        except Exception:  # noqa: BLE001 - membership is best effort
            log.warning("user %s created but not added to default group %s", user.username, group.name)
    return {"msg": M("user.create.success"), "user": user.as_dict(include_private=True)}, 201


def create(newUser: dict):
    return do_create(newUser)


def ssh_signup(user: dict):
    """Self-signup: prove UNIX identity by logging into the first node AS the claimed user with
    the TensorHive key (the user must have authorised it first)."""
    d = daemon()
    nodes = get_config().ssh.available_nodes
    if not nodes:
        return {"msg": M("general.unprivileged")}, 403
    host = next(iter(nodes))
    from ..core import ssh

    try:
        ok = ssh.verify_login_as(host, user["username"], d.ssh_key_path if d else get_config().ssh.key_file)
    except Exception as e:  # noqa: BLE001
        return {"msg": f"An error occurred while authenticating: {e}"}, 500
    if not ok:
        return {"msg": M("general.unprivileged")}, 403
    return do_create(user)


def authorized_keys_entry():
    from ..core import ssh

    key = get_config().ssh.key_file
    return ssh.authorized_keys_entry(key, get_config().app_server.host), 200


@guarded(not_found="user.not_found", assertion="user.update.failure.invalid")
def update(newValues: dict):
    if newValues.get("id") is None:
        return {"msg": M("general.bad_request")}, 400
    user = User.get(newValues["id"])
    for f in ("username", "password", "email", "roles"):
        v = newValues.get(f)
        if v is None:
            continue
        if f == "roles":
            v = [Role(name=r) for r in v]
        setattr(user, f, v)
    user.save()
    d = user.as_dict(include_private=True)
    # 'reservation' is the key the reference answers with (kept for clients); 'user' is additive
    return {"msg": M("user.update.success"), "reservation": d, "user": d}, 201


@guarded(not_found="user.not_found", assertion="user.update.failure.invalid")
def change_password(form: dict):
    """Self-service password change (new; ``PUT /user`` is admin-only in TensorHive 1.1, which left
    non-admin users without a way to change their own password).  The old password must match."""
    user = User.get(me())
    if not User.verify_hash(form["oldPassword"], user.password):
        return {"msg": M("user.login.failure.credentials")}, 403
    user.password = form["newPassword"]
    user.save()
    return {"msg": M("user.update.success")}, 200


@guarded(not_found="user.not_found")
def delete(id: int):
    if id == me():
        raise Abort(403, M("user.delete.self"))
    User.get(id).destroy()
    return {"msg": M("user.delete.success")}, 200


def login(user: dict):
    from sqlalchemy.exc import NoResultFound

    try:
        found = User.find_by_username(user["username"])
    except NoResultFound:
        return {"msg": M("user.not_found")}, 404
    if not User.verify_hash(user["password"], found.password):
        return {"msg": M("user.login.failure.credentials")}, 401
    return {"msg": M("user.login.success", username=found.username),
            "access_token": auth.create_access_token(found.id, found.role_names, fresh=True),
            "refresh_token": auth.create_refresh_token(found.id)}, 200


def _logout(kind: str):
    try:
        RevokedToken(jti=auth.current().jti).save()
    except Exception:  # noqa: BLE001
        log.error(M("token.revoke.failure", token_type=kind))
        return {"msg": M("general.internal_error")}, 500
    return {"msg": M("user.logout.success")}, 200


def logout_with_access_token():
    return _logout("Access")


def logout_with_refresh_token():
    return _logout("Refresh")


def generate():
    uid = auth.get_jwt_identity()
    try:
        roles = User.get(uid).role_names
    except Exception:  # noqa: BLE001
        return {"msg": M("token.refresh.failure")}, 401
    return {"msg": M("token.refresh.success"), "access_token": auth.create_access_token(uid, roles, fresh=False)}, 200
