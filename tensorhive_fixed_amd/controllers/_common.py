"""Shared controller plumbing: message lookup and exception -> (content, status) mapping."""
from __future__ import annotations

import functools
import logging
import re

from sqlalchemy.exc import IntegrityError, NoResultFound

from ..api import auth
from ..config import get_config
from ..database import db_session
from ..utils.exceptions import ForbiddenException, InvalidRequestException

log = logging.getLogger(__name__)


def M(path: str, **fmt) -> str:
    """Message from the responses catalogue by dotted path, formatted with ``fmt``."""
    node = get_config().api.responses
    for part in path.split("."):
        node = node[part]
    return node.format(**fmt) if fmt else node


def snake(name: str) -> str:
    return re.sub(r"(?<!^)([A-Z])", r"_\1", name).lower()


class Abort(Exception):
    """Raise inside a controller to answer ``(msg, status)`` immediately."""

    def __init__(self, status: int, msg: str, **extra):
        super().__init__(msg)
        self.status, self.msg, self.extra = status, msg, extra


def guarded(not_found: str | None = None, assertion: str | None = None, invalid: str | None = None,
            invalid_status: int = 409, forbidden: str | None = None, integrity: str | None = None,
            assertion_status: int = 422):
    """Map domain exceptions to responses. Message args are catalogue paths; ``{reason}`` gets
    the exception text."""

    def deco(fn):
        @functools.wraps(fn)
        def wrapper(*a, **kw):
            try:
                return fn(*a, **kw)
            except Abort as e:
                db_session.rollback()
                return {"msg": e.msg, **e.extra}, e.status
            except NoResultFound as e:
                db_session.rollback()
                return {"msg": M(not_found) if not_found else str(e)}, 404
            except ForbiddenException as e:
                db_session.rollback()
                return {"msg": M(forbidden, reason=e) if forbidden else str(e)}, 403
            except InvalidRequestException as e:
                db_session.rollback()
                return {"msg": M(invalid, reason=e) if invalid else str(e)}, invalid_status
            except IntegrityError as e:
                db_session.rollback()
                return {"msg": M(integrity) if integrity else str(e.orig)}, 409
            except AssertionError as e:
                db_session.rollback()
                return {"msg": M(assertion, reason=e) if assertion else str(e)}, assertion_status
            except auth.AuthError:
                raise
            except Exception as e:  # noqa: BLE001
                db_session.rollback()
                log.exception("controller %s failed", fn.__qualname__)
                return {"msg": M("general.internal_error") + f" {e}"}, 500
        return wrapper
    return deco


def me() -> int:
    return auth.get_jwt_identity()


def is_admin() -> bool:
    return auth.is_admin()


def check_fields(values: dict, allowed: set[str]) -> None:
    extra = set(values) - allowed
    assert not extra, f"invalid field is present: {sorted(extra)}"
