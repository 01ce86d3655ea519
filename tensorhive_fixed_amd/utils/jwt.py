"""Minimal HS256 JSON Web Tokens (stdlib only) with flask_jwt_extended 3.x claim names.

Claims: ``iat, nbf, jti, exp, identity, fresh, type ('access'|'refresh'), user_claims``
(reference ``authorization.py:26-34``).  Tokens are not byte-compatible with the reference's
(they live at most a day), the claim semantics are.
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import json
import time
import uuid
from datetime import timedelta


class JWTError(Exception):
    pass


class ExpiredSignature(JWTError):
    pass


class InvalidSignature(JWTError):
    pass


class MissingClaim(JWTError):
    pass


def _b64(b: bytes) -> str:
    return base64.urlsafe_b64encode(b).decode("ascii").rstrip("=")


def _unb64(s: str) -> bytes:
    return base64.urlsafe_b64decode(s + "=" * (-len(s) % 4))


def encode(payload: dict, secret: str) -> str:
    header = {"typ": "JWT", "alg": "HS256"}
    h = _b64(json.dumps(header, separators=(",", ":")).encode())
    p = _b64(json.dumps(payload, separators=(",", ":"), default=str).encode())
    sig = hmac.new(secret.encode(), f"{h}.{p}".encode(), hashlib.sha256).digest()
    return f"{h}.{p}.{_b64(sig)}"


def decode(token: str, secret: str, leeway: float = 0.0, now: float | None = None) -> dict:
    """Verify and return the claims. A bad signature raises :class:`InvalidSignature`, a token
    without a numeric ``exp`` :class:`MissingClaim`, an expired one :class:`ExpiredSignature`."""
    try:
        h, p, s = token.split(".")
        header = json.loads(_unb64(h))
        payload = json.loads(_unb64(p))
        sig = _unb64(s)
    except (ValueError, json.JSONDecodeError) as e:
        raise JWTError("malformed token") from e
    if header.get("alg") != "HS256":
        raise JWTError("unsupported algorithm")
    want = hmac.new(secret.encode(), f"{h}.{p}".encode(), hashlib.sha256).digest()
    if not hmac.compare_digest(sig, want):
        raise InvalidSignature("signature verification failed")
    t = time.time() if now is None else now
    # every token this server issues expires; one without ``exp`` was minted elsewhere and would
    # otherwise be valid forever
    if not isinstance(payload.get("exp"), (int, float)):
        raise MissingClaim("token has no expiry")
    if t > payload["exp"] + leeway:
        raise ExpiredSignature("token has expired")
    if "nbf" in payload and t + leeway < payload["nbf"]:
        raise JWTError("token not yet valid")
    return payload


def create_token(identity, token_type: str, secret: str, expires: timedelta, fresh: bool = False,
                 user_claims: dict | None = None, now: float | None = None) -> str:
    t = int(time.time() if now is None else now)
    payload = {"iat": t, "nbf": t, "jti": str(uuid.uuid4()), "exp": t + int(expires.total_seconds()),
               "identity": identity, "type": token_type}
    if token_type == "access":
        payload["fresh"] = fresh
        payload["user_claims"] = user_claims or {}
    return encode(payload, secret)
