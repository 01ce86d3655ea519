"""Authentication/authorisation for the REST API (replaces flask_jwt_extended; reference
``authorization.py:11-45`` + ``config.py:262-298``).

* HS256 Bearer tokens with the flask_jwt_extended 3.x claims (``utils/jwt.py``);
  access tokens carry ``user_claims.roles``.
* Denylist: the ``jti`` of every checked token type is looked up in ``revoked_tokens``.
* Status semantics the web UI relies on: missing header -> 401, expired -> 401 (the SPA then
  refreshes and retries), revoked -> 401, malformed/wrong type -> 422, non-admin on an admin
  operation -> 403 ``{"msg": "Unprivileged"}``.
* Tokens whose signature does not verify or that carry no ``exp`` are 401 (a key rotation then
  sends the SPA through refresh -> login instead of showing an error).
* No token is signed or accepted while ``[auth] secret_key`` is empty or a public default such
  as the reference's ``jwt-some-secret`` (``tensorhive/config.py:289``), unless
  ``TENSORHIVE_ALLOW_INSECURE_SECRET=1`` (tests only): anyone could forge an admin token.
"""
from __future__ import annotations

from dataclasses import dataclass

from flask import g, request

from ..config import get_config, insecure_secret_allowed, secret_is_insecure
from ..utils import jwt


class InsecureSecret(RuntimeError):
    """The configured signing key is empty or publicly known."""


def signing_key() -> str:
    key = get_config().auth.secret_key
    if secret_is_insecure(key) and not insecure_secret_allowed():
        raise InsecureSecret("[auth] secret_key is empty or a public default; run `tensorhive init` "
                             "or set a random secret_key in main_config.ini")
    return key


class AuthError(Exception):
    def __init__(self, status: int, msg: str):
        super().__init__(msg)
        self.status = status
        self.msg = msg


@dataclass
class Identity:
    user_id: int
    roles: list[str]
    token_type: str
    jti: str
    fresh: bool = False

    @property
    def is_admin(self) -> bool:
        return "admin" in self.roles


def _responses():
    return get_config().api.responses


def create_access_token(user_id: int, roles: list[str], fresh: bool = False) -> str:
    a = get_config().auth
    return jwt.create_token(user_id, "access", signing_key(), a.access_token_expires, fresh=fresh,
                            user_claims={"roles": list(roles)})


def create_refresh_token(user_id: int) -> str:
    a = get_config().auth
    return jwt.create_token(user_id, "refresh", signing_key(), a.refresh_token_expires)


def decode_token(token: str) -> dict:
    return jwt.decode(token, signing_key())


def _bearer() -> str:
    h = request.headers.get("Authorization")
    if not h:
        raise AuthError(401, _responses()["token"]["missing_auth_header"])
    parts = h.split()
    if len(parts) != 2 or parts[0] != "Bearer":
        raise AuthError(422, "Bad Authorization header. Expected value 'Bearer <JWT>'")
    return parts[1]


def verify(required_type: str = "access") -> Identity:
    """Verify the request's bearer token; store and return the identity."""
    from ..models.orm import RevokedToken

    cfg = get_config().auth
    try:
        claims = decode_token(_bearer())
    except jwt.ExpiredSignature:
        raise AuthError(401, _responses()["token"]["expired"])
    except (jwt.InvalidSignature, jwt.MissingClaim) as e:
        raise AuthError(401, str(e))
    except InsecureSecret as e:
        raise AuthError(401, str(e))
    except jwt.JWTError as e:
        raise AuthError(422, str(e))
    ttype = claims.get("type")
    if ttype != required_type:
        raise AuthError(422, _responses()["token"]["refresh" if required_type == "refresh" else "access"]["required"])
    if cfg.blacklist_enabled and ttype in cfg.blacklist_token_checks and RevokedToken.is_jti_blacklisted(claims["jti"]):
        raise AuthError(401, _responses()["token"]["revoked"])
    roles = (claims.get("user_claims") or {}).get("roles", [])
    ident = Identity(int(claims["identity"]), list(roles), ttype, claims["jti"], bool(claims.get("fresh")))
    g.th_identity = ident
    return ident


def current() -> Identity:
    ident = getattr(g, "th_identity", None)
    if ident is None:
        raise AuthError(401, _responses()["general"]["unauthorized"])
    return ident


def get_jwt_identity() -> int:
    return current().user_id


def get_jwt_claims() -> dict:
    return {"roles": current().roles}


def is_admin() -> bool:
    ident = getattr(g, "th_identity", None)
    return bool(ident and ident.is_admin)


def enforce(mode: str | None) -> None:
    """``mode``: None (public), 'jwt', 'admin', 'refresh', 'scrape' (the handler authenticates:
    a static scrape token or a JWT, see ``controllers/nodes.py:_prometheus_scope``)."""
    if mode is None or mode == "scrape":
        return
    if mode == "refresh":
        verify("refresh")
        return
    ident = verify("access")
    if mode == "admin" and not ident.is_admin:
        raise AuthError(403, _responses()["general"]["unprivileged"])
