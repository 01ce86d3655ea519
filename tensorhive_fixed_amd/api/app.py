"""Flask application: spec-driven router + strict validator + JWT enforcement.

Replaces connexion (``api/APIServer.py:16-49``).  For every :class:`~.spec.Op`:
path parameters are typed by the URL converter, query parameters are coerced and validated
(unknown ones -> 400, like connexion's ``strict_validation=True``), the JSON body is checked
against its schema (required fields and types) and passed to the controller under its
``x-body-name``.  Validation errors use the problem+json shape connexion produced.  The
controller returns ``(content, status)``.

The running daemon (telemetry snapshots, transports, services) is reachable from controllers
through :func:`daemon` -- explicit dependency injection instead of the reference's
``TensorHiveManager`` metaclass singleton.
"""
from __future__ import annotations

import importlib
import json
import logging
import time
from typing import Any

from flask import Flask, Response, current_app, jsonify, request

from .. import __version__
from ..config import get_config
from ..database import db_session
from . import auth
from .spec import EXTRA_OPERATIONS, OPERATIONS, RESPONSES, SCHEMAS, Op, SchemaError, openapi_document, validate

log = logging.getLogger(__name__)
_EXT = "tensorhive_fixed_amd"


class ValidationError(Exception):
    pass


def daemon():
    """The Daemon bound to the current app (None when running the API alone, e.g. tests)."""
    try:
        return current_app.extensions.get(_EXT, {}).get("daemon")
    except RuntimeError:
        return None


def problem(status: int, detail: str, title: str | None = None):
    titles = {400: "Bad Request", 401: "Unauthorized", 403: "Forbidden", 404: "Not Found", 405: "Method Not Allowed",
              422: "Unprocessable Entity", 500: "Internal Server Error"}
    body = {"detail": detail, "status": status, "title": title or titles.get(status, "Error"), "type": "about:blank"}
    return Response(json.dumps(body), status=status, mimetype="application/problem+json")


def _coerce(value: str, t: str, name: str):
    if t == "integer":
        try:
            return int(value)
        except ValueError:
            raise ValidationError(f"Wrong type, expected 'integer' for query parameter '{name}'")
    if t == "number":
        try:
            return float(value)
        except ValueError:
            raise ValidationError(f"Wrong type, expected 'number' for query parameter '{name}'")
    if t == "boolean":
        v = value.strip().lower()
        if v in ("true", "1", "yes"):
            return True
        if v in ("false", "0", "no"):
            return False
        raise ValidationError(f"Wrong type, expected 'boolean' for query parameter '{name}'")
    return value


def _query_args(op: Op) -> dict:
    allowed = {p.name: p for p in op.params if p.where == "query"}
    unknown = [k for k in request.args.keys() if k not in allowed]
    if unknown:
        raise ValidationError(f"Extra query parameter(s) {','.join(unknown)} not in spec")
    out: dict[str, Any] = {}
    for name, p in allowed.items():
        if name not in request.args:
            if p.required:
                raise ValidationError(f"Missing query parameter '{name}'")
            continue
        if p.type == "array":
            vals = request.args.getlist(name)
            items: list[str] = []
            for v in vals:
                items.extend(x for x in v.split(",") if x != "")
            out[name] = [_coerce(x, p.items, name) for x in items]
            continue
        raw = request.args.get(name)
        if p.nullable and raw in ("", "null"):
            out[name] = None
            continue
        v = _coerce(raw, p.type, name)
        if p.enum and v not in p.enum:
            raise ValidationError(f"'{v}' is not one of {p.enum}")
        out[name] = v
    return out


def _validate_body(schema_name: str):
    """The JSON body against its spec schema, nested objects included (``cmdsegments`` entries,
    ``scheduleDays`` names, date-time strings, bounds): a violation is a 400 problem, as
    connexion's validator answered, before any controller runs."""
    body = request.get_json(silent=True)
    if body is None:
        raise ValidationError("Request body is not valid JSON" if request.data else "Request body is required")
    if not isinstance(body, dict):
        raise ValidationError(f"{body!r} is not of type 'object'")
    try:
        validate(body, SCHEMAS[schema_name], "body")
    except SchemaError as e:
        raise ValidationError(str(e))
    return body


def _resolve(handler: str):
    mod, fn = handler.rsplit(".", 1)
    return getattr(importlib.import_module(f"{__package__.rsplit('.', 1)[0]}.controllers.{mod}"), fn)


def _flask_path(op: Op) -> str:
    p = op.path
    for prm in op.params:
        if prm.where == "path":
            conv = "int:" if prm.type == "integer" else ""
            p = p.replace("{" + prm.name + "}", f"<{conv}{prm.name}>")
    return p


class ResponseContractError(AssertionError):
    pass


def check_response(op: Op, content, status: int) -> None:
    """A controller's answer against the document: the status must be one the operation
    declares and the body must match that status's schema (tests turn this on for every
    request: ``TH_VALIDATE_RESPONSES``)."""
    ok, body, errors = RESPONSES[op.handler]
    if status != ok and status not in errors:
        raise ResponseContractError(f"{op.method} {op.path}: undeclared status {status}")
    sch = body if status == ok else SCHEMAS["Message"]
    if sch is None:
        return
    try:
        validate(json.loads(json.dumps(content, default=str)), sch, f"{op.handler}[{status}]")
    except SchemaError as e:
        raise ResponseContractError(str(e))


def _make_view(op: Op):
    func = _resolve(op.handler)

    def view(**path_kwargs):
        t0 = time.perf_counter()
        try:
            auth.enforce(op.auth)
            kwargs = dict(path_kwargs)
            kwargs.update(_query_args(op))
            if op.body:
                kwargs[op.body_name] = _validate_body(op.body)
            result = func(**kwargs)
        except ValidationError as e:
            return problem(400, str(e))
        except auth.AuthError as e:
            return jsonify({"msg": e.msg}), e.status
        finally:
            stats = current_app.extensions.get(_EXT, {}).get("latency")
            if stats is not None:
                stats.observe(op.handler, time.perf_counter() - t0)
        if isinstance(result, Response):
            return result
        if isinstance(result, tuple):
            content, status = result[0], result[1]
        else:
            content, status = result, 200
        if current_app.config.get("TH_VALIDATE_RESPONSES"):
            check_response(op, content, status)
        return Response(json.dumps(content, default=str), status=status, mimetype="application/json")

    view.__name__ = f"{op.method.lower()}_{op.handler.replace('.', '_')}"
    return view


class LatencyStats:
    """Per-operation request latency reservoir (exposed at /metrics/internal)."""

    def __init__(self, cap: int = 4096):
        import collections
        import threading

        self._lock = threading.Lock()
        self._data: dict[str, collections.deque] = {}
        self._cap = cap
        self._deque = collections.deque

    def observe(self, key: str, seconds: float) -> None:
        with self._lock:
            d = self._data.get(key)
            if d is None:
                d = self._data[key] = self._deque(maxlen=self._cap)
            d.append(seconds)

    def summary(self) -> dict:
        with self._lock:
            out = {}
            for k, d in self._data.items():
                xs = sorted(d)
                if not xs:
                    continue
                out[k] = {"n": len(xs), "p50_ms": 1000 * xs[len(xs) // 2],
                          "p99_ms": 1000 * xs[min(len(xs) - 1, int(0.99 * len(xs)))]}
            return out


def create_app(daemon_obj=None) -> Flask:
    cfg = get_config()
    prefix = "/" + cfg.api.url_prefix.strip("/")
    app = Flask(__name__)
    app.extensions[_EXT] = {"daemon": daemon_obj, "latency": LatencyStats()}
    for op in OPERATIONS + EXTRA_OPERATIONS:
        app.add_url_rule(prefix + _flask_path(op), endpoint=f"{op.method}:{op.path}", view_func=_make_view(op),
                         methods=[op.method])

    @app.route(prefix + "/openapi.json")
    def openapi_json():
        return jsonify(openapi_document(cfg.api.title, cfg.api.url_prefix, __version__, cfg.api.responses))

    @app.route(prefix + "/ui/")
    def api_ui():
        from pathlib import Path

        html = (Path(__file__).with_name("explorer.html")).read_text()
        return Response(html, mimetype="text/html")

    @app.after_request
    def cors(resp):
        resp.headers["Access-Control-Allow-Origin"] = "*"
        resp.headers["Access-Control-Allow-Headers"] = "Authorization, Content-Type"
        resp.headers["Access-Control-Allow-Methods"] = "GET, POST, PUT, DELETE, OPTIONS"
        return resp

    @app.before_request
    def preflight():
        if request.method == "OPTIONS":
            return Response(status=200)
        return None

    @app.errorhandler(404)
    def not_found(_e):
        return problem(404, "The requested URL was not found on the server.")

    @app.errorhandler(405)
    def bad_method(_e):
        return problem(405, "The method is not allowed for the requested URL.")

    @app.errorhandler(Exception)
    def internal(e):
        log.exception("unhandled error in API: %s", e)
        db_session.rollback()
        return jsonify({"msg": cfg.api.responses["general"]["internal_error"]}), 500

    app.config.setdefault("TH_REMOVE_SESSION", True)

    @app.teardown_appcontext
    def remove_session(_exc=None):
        # one session per request thread; in-process test clients share the caller's thread
        # and keep it (TH_REMOVE_SESSION=False) so fixtures stay attached
        if app.config["TH_REMOVE_SESSION"]:
            db_session.remove()
        else:
            db_session.rollback() if _exc is not None else None

    return app
