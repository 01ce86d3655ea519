"""passlib-compatible ``pbkdf2_sha256`` hashes with the standard library.

Format (passlib modular crypt): ``$pbkdf2-sha256$<rounds>$<ab64 salt>$<ab64 digest>``, where ab64 is
base64 with ``.`` instead of ``+`` and no padding; 16-byte salt, 32-byte digest, 29000 rounds by
default.  Existing TensorHive databases (passlib 1.7, ``models/User.py:92-96``) verify unchanged.
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import os

DEFAULT_ROUNDS = 29000
SALT_BYTES = 16
PREFIX = "$pbkdf2-sha256$"


def ab64_encode(b: bytes) -> str:
    return base64.b64encode(b).decode("ascii").rstrip("=").replace("+", ".")


def ab64_decode(s: str) -> bytes:
    s = s.replace(".", "+")
    return base64.b64decode(s + "=" * (-len(s) % 4))


def hash_password(password: str, rounds: int = DEFAULT_ROUNDS, salt: bytes | None = None) -> str:
    salt = os.urandom(SALT_BYTES) if salt is None else salt
    dk = hashlib.pbkdf2_hmac("sha256", password.encode("utf-8"), salt, rounds, 32)
    return f"{PREFIX}{rounds}${ab64_encode(salt)}${ab64_encode(dk)}"


def verify_password(password: str, hashed: str) -> bool:
    try:
        if not hashed.startswith(PREFIX):
            return False
        rounds_s, salt_s, dk_s = hashed[len(PREFIX):].split("$")
        salt, want = ab64_decode(salt_s), ab64_decode(dk_s)
        got = hashlib.pbkdf2_hmac("sha256", password.encode("utf-8"), salt, int(rounds_s), len(want))
        return hmac.compare_digest(got, want)
    except (ValueError, TypeError):
        return False
