"""Monitoring endpoints ``/nodes/*`` (reference ``controllers/nodes.py``).

Served straight from the daemon's current immutable telemetry snapshot: no SSH, no lock.
Every read auto-registers newly seen GPUs as ``Resource`` rows (as the reference does) but only
when the snapshot version changed since the last registration (the reference inserted on every
read path).  Non-admins see only GPUs their restrictions allow.  Responses carry the sample age
(``X-Sample-Age-Ms`` header / ``sampleAgeMs`` in topology) so dashboards can show staleness.
"""
from __future__ import annotations

import datetime
import threading

from flask import Response
from sqlalchemy import event
from sqlalchemy.orm import Session

from .. import database
from ..api.app import daemon
from ..database import db_session
from ..models.orm import Group, Resource, Restriction, RestrictionAssignee, User
from ..utils import dates
from ._common import M, is_admin, me

_reg_lock = threading.Lock()

# ------------------------------------------------------------------ permitted-GPU cache
# A non-admin poll needs the set of GPUs the caller's restrictions cover: 4-6 queries (user,
# restrictions, groups, their restrictions, resources), most of a restricted user's poll time.
# The set is cached per (database, user) and dropped when (a) any flush touches a user, group,
# restriction or resource (their association collections mark the owners dirty), or (b) one of
# the user's restrictions starts or ends -- the set changes with the clock, without a write.
_perm_epoch = [0]
_perm_cache: dict = {}
_perm_lock = threading.Lock()
_PERM_TYPES = (User, Group, Restriction, RestrictionAssignee, Resource)


@event.listens_for(Session, "after_flush")
def _perm_invalidate(session, _ctx):
    if any(isinstance(o, _PERM_TYPES) for o in (*session.new, *session.dirty, *session.deleted)):
        with _perm_lock:
            _perm_epoch[0] += 1
            _perm_cache.clear()


def allowed_gpus_cached(user_id: int) -> set[str] | None:
    key = (id(database.engine()), user_id)
    now = dates.utcnow()
    with _perm_lock:
        epoch = _perm_epoch[0]
        hit = _perm_cache.get(key)
    if hit is not None and hit[0] == epoch and now < hit[2]:
        return hit[1]
    user = User.get(user_id)
    allowed = user.allowed_gpu_uuids()
    bounds = [t for r in user.get_restrictions(include_expired=True, include_group=True)
              for t in (r.starts_at, r.ends_at) if t is not None and t > now]
    with _perm_lock:
        if _perm_epoch[0] == epoch:  # nothing changed while we read
            _perm_cache[key] = (epoch, allowed, min(bounds, default=datetime.datetime.max))
    return allowed


def _snapshot():
    d = daemon()
    if d is None:
        return None
    return d.infrastructure.snapshot()


def register_resources_from_snapshot(snap=None) -> None:
    snap = snap or _snapshot()
    d = daemon()
    if snap is None or d is None:
        return
    with _reg_lock:
        _registered_version = d.__dict__.setdefault("_resource_registration", {"v": -1, "ids": set()})
        if snap.version == _registered_version["v"]:
            return
        known = _registered_version["ids"]
        new = []
        for host, entry in snap.data.items():
            for uuid, g in ((entry or {}).get("GPU") or {}).items():
                if uuid not in known:
                    new.append((uuid, g.get("name"), host))
        if new:
            existing = {r.id for r in Resource.query.filter(Resource.id.in_([u for u, _, _ in new])).all()}
            for uuid, name, host in new:
                if uuid not in existing:
                    db_session.add(Resource(id=uuid, name=(name or "")[:40], hostname=host))
                known.add(uuid)
            db_session.commit()
        _registered_version["v"] = snap.version


def filtered_view(data: dict, allowed: set[str] | None) -> dict:
    """The snapshot restricted to ``allowed`` GPU UUIDs (``None`` = everything), hosts left
    without GPUs dropped (reference ``models/User.py:166-186``).  A shallow view: host and GPU
    entries are shared with the immutable snapshot, never copied -- the reference deep-copied
    the whole infrastructure on every poll (``controllers/nodes.py:15``)."""
    if allowed is None:
        return data
    out = {}
    for host, entry in data.items():
        gpus = (entry or {}).get("GPU")
        if gpus is None:
            continue
        keep = {u: g for u, g in gpus.items() if u in allowed}
        if keep:
            out[host] = {**entry, "GPU": keep}
    return out


def _allowed() -> set[str] | None:
    return None if is_admin() else allowed_gpus_cached(me())


def get_infrastructure() -> dict:
    """Read-only view of the current snapshot as the caller may see it (do not mutate)."""
    snap = _snapshot()
    if snap is None:
        return {}
    register_resources_from_snapshot(snap)
    return filtered_view(snap.data, _allowed())


class _JsonCache:
    """Serialised ``/nodes/metrics`` bodies keyed by (snapshot version, permitted GPU set): every
    dashboard of the same permission class shares one ``json.dumps`` per sample."""

    def __init__(self, size: int = 64):
        self.size = size
        self._d: dict = {}
        self._lock = threading.Lock()

    def get(self, key, build):
        with self._lock:
            hit = self._d.get(key)
        if hit is not None:
            return hit
        body = build()
        with self._lock:
            if len(self._d) >= self.size:
                self._d.pop(next(iter(self._d)))
            self._d[key] = body
        return body


_metrics_cache = _JsonCache()


def _with_age(content, status=200, body: str | None = None, snap=None):
    import json
    import time

    snap = snap or _snapshot()
    resp = Response(body if body is not None else json.dumps(content, default=str), status=status,
                    mimetype="application/json")
    if snap is not None and snap.sampled_at:
        now = time.time()
        resp.headers["X-Sample-Age-Ms"] = str(int(1000 * (now - min(snap.sampled_at.values()))))
        # per host, so the dashboard can flag one stale node (heartbeat freshness)
        resp.headers["X-Host-Sample-Age-Ms"] = ",".join(f"{h}={int(1000 * (now - t))}"
                                                        for h, t in sorted(snap.sampled_at.items()))
    return resp


def get_all_data():
    import json

    snap = _snapshot()
    if snap is None:
        return _with_age({})
    register_resources_from_snapshot(snap)
    allowed = _allowed()
    key = (id(daemon()), snap.version, None if allowed is None else frozenset(allowed))
    body = _metrics_cache.get(key, lambda: json.dumps(filtered_view(snap.data, allowed), default=str))
    return _with_age(None, body=body, snap=snap)


def get_hostnames():
    return list(get_infrastructure().keys()), 200


def _host(hostname: str):
    infra = get_infrastructure()
    if hostname not in infra:
        return None
    return infra[hostname]


def _not_found():
    return {"msg": M("nodes.hostname.not_found")}, 404


def get_gpu_info(hostname: str):
    h = _host(hostname)
    if h is None:
        return _not_found()
    gpus = h.get("GPU") or {}
    return {u: {"name": g.get("name"), "index": g.get("index"), "bdf": g.get("bdf"),
                "numa_node": g.get("numa_node")} for u, g in gpus.items()}, 200


def get_gpu_metrics(hostname: str, metric_type: str | None = None):
    h = _host(hostname)
    if h is None:
        return _not_found()
    gpus = h.get("GPU") or {}
    if metric_type is None:
        return _with_age({u: g.get("metrics") for u, g in gpus.items()})
    return _with_age({u: (g.get("metrics") or {}).get(metric_type, {"value": None, "unit": None})
                      for u, g in gpus.items()})


def get_cpu_metrics(hostname: str, metric_type: str | None = None):
    h = _host(hostname)
    if h is None:
        return _not_found()
    cpus = h.get("CPU") or {}
    if metric_type is None:
        return {k: c.get("metrics") for k, c in cpus.items()}, 200
    return {k: (c.get("metrics") or {}).get(metric_type, {"value": None, "unit": None}) for k, c in cpus.items()}, 200


def get_gpu_processes(hostname: str):
    h = _host(hostname)
    if h is None:
        return _not_found()
    gpus = h.get("GPU") or {}
    return {u: g.get("processes") for u, g in gpus.items()}, 200


def get_topology():
    """xGMI link matrix + NUMA + BDF per host (new; feeds rank->device placement)."""
    d = daemon()
    if d is None:
        return {}, 200
    return d.topology(), 200


def _prom_escape(v) -> str:
    return str(v).replace("\\", "\\\\").replace('"', '\\"')


def _prometheus_scope() -> set[str] | None:
    """Who may scrape, and what they see (the reference kept every ``/nodes/*`` read behind a JWT
    and the per-user filter, ``tensorhive/controllers/nodes.py:13-50``).

    * ``Authorization: Bearer <[api] prometheus_token>`` (constant-time compare): full view;
    * an admin JWT access token: full view;
    * a non-admin JWT: 403 unless ``[api] prometheus_allow_users``; then only permitted GPUs;
    * no or bad credentials: 401 / 422 (as every JWT endpoint)."""
    import hmac

    from flask import request

    from ..api.auth import AuthError, verify
    from ..config import get_config

    cfg = get_config().api
    h = request.headers.get("Authorization", "")
    token = h[7:] if h.startswith("Bearer ") else ""
    if cfg.prometheus_token and token and hmac.compare_digest(token.encode(), cfg.prometheus_token.encode()):
        return None
    ident = verify("access")  # raises AuthError 401 (missing/expired/revoked) or 422 (malformed)
    if ident.is_admin:
        return None
    if not cfg.prometheus_allow_users:
        raise AuthError(403, M("general.unprivileged"))
    return allowed_gpus_cached(ident.user_id)


def get_prometheus():
    """Prometheus text exposition of the latest snapshot: numeric GPU/CPU metrics per host and GPU,
    snapshot age per host, service loop timings.  No user names or process lists.  Authenticated
    (see :func:`_prometheus_scope`); a non-admin scrape is filtered like ``/nodes/metrics``."""
    import time

    allowed = _prometheus_scope()
    d = daemon()
    lines = ["# TYPE tensorhive_gpu_metric gauge", "# TYPE tensorhive_sample_age_seconds gauge"]
    if d is not None:
        snap = d.infrastructure.snapshot()
        now = time.time()
        for host, entry in sorted(filtered_view(snap.data, allowed).items()):
            h = _prom_escape(host)
            if host in snap.sampled_at:
                lines.append(f'tensorhive_sample_age_seconds{{host="{h}"}} {now - snap.sampled_at[host]:.3f}')
            for uuid, g in sorted(((entry or {}).get("GPU") or {}).items()):
                for name, m in sorted((g.get("metrics") or {}).items()):
                    v = (m or {}).get("value")
                    if isinstance(v, (int, float)):
                        lines.append(f'tensorhive_gpu_metric{{host="{h}",gpu="{g.get("index")}",uuid="{uuid}",'
                                     f'metric="{_prom_escape(name)}",unit="{_prom_escape(m.get("unit", ""))}"}} {v}')
                lines.append(f'tensorhive_gpu_processes{{host="{h}",gpu="{g.get("index")}",uuid="{uuid}"}} '
                             f'{len(g.get("processes") or [])}')
            for cpu in (((entry or {}).get("CPU") or {}) if allowed is None else {}).values():
                for name, m in sorted((cpu.get("metrics") or {}).items()):
                    v = (m or {}).get("value")
                    if isinstance(v, (int, float)):
                        lines.append(f'tensorhive_cpu_metric{{host="{h}",metric="{_prom_escape(name)}"}} {v}')
        for svc, st in (d.service_stats() if allowed is None else {}).items():
            for k in ("p50_ms", "p99_ms"):
                if isinstance(st.get(k), (int, float)):
                    lines.append(f'tensorhive_service_loop_ms{{service="{svc}",quantile="{k[:3]}"}} {st[k]}')
            lines.append(f'tensorhive_service_ticks_total{{service="{svc}"}} {st.get("ticks", 0)}')
    return Response("\n".join(lines) + "\n", status=200, mimetype="text/plain; version=0.0.4")


def get_internal_metrics():
    """Service loop timings and API latency percentiles (observability, new)."""
    from flask import current_app

    d = daemon()
    out = {"api": current_app.extensions["tensorhive_fixed_amd"]["latency"].summary()}
    if d is not None:
        out["services"] = d.service_stats()
        snap = d.infrastructure.snapshot()
        out["snapshot_version"] = snap.version
    return out, 200
