"""Task attribution that cannot be forged (round-4 verdict item 1).

A GPU process *claims* a TensorHive task through ``TENSORHIVE_TASK_ID`` in its environment, which
anybody can set.  The claim is accepted only when the process really belongs to that task's
``th-run`` session on that node:

* its uid is the uid the task runs as (``uid``/``user`` in th-run's state file), **and**
* its session id is the task's session (``sid``: th-run's first child called ``setsid``; every
  process the task forks stays in it), **or** its parent chain reaches the task's ``th-run``
  monitor (a rank that called ``setsid`` itself).

A process started outside the session cannot join it (``setsid``/``setpgid`` only leave or move
within a session), and a user cannot take another uid, so the check holds against a process that
copies a victim's task id.  A claim that fails is dropped: the process keeps ``claimed_task_id``
and is judged by its UNIX owner, exactly like the reference, whose enforcer knew no tasks at all
(``tensorhive/core/services/ProtectionService.py:97-99``, owner from ``ps -o user`` in
``tensorhive/core/monitors/GPUMonitor.py:94-107``).

The session facts come from th-run itself: the spawn command prints the new session's state in the
same round trip (``task_nursery.spawn``), every ``th-run ls`` refreshes them
(``task_nursery.running``), and a claim for a task the registry has not seen (a daemon restarted
under a running task) triggers one rate-limited ``th-run ls`` of that task's owner on that node
before it is judged.

:meth:`Attestor.attest_entry` runs in the monitoring service before a sample is published, so every
consumer -- :class:`~.services.ProtectionService`, the queue's eviction check
(``JobSchedulingService.sync_running_from_queue``), the in-task HBM counters (``core/hbm.py``) and
the ``/nodes`` API -- sees attested task ids only.
"""
from __future__ import annotations

import logging
import threading
import time

from . import hbm

log = logging.getLogger(__name__)

SESSION_PREFIX = "tensorhive_task_"


def _int(v) -> int | None:
    try:
        return int(v)
    except (TypeError, ValueError):
        return None


def task_id_of_session(name: str) -> str | None:
    name = str(name or "")
    return name[len(SESSION_PREFIX):] if name.startswith(SESSION_PREFIX) else None


class SessionRegistry:
    """``(host, task id) -> th-run session facts`` (sid, uid, user, monitor pid, pids), fed by
    every th-run listing the daemon reads."""

    def __init__(self):
        self._lock = threading.Lock()
        self._d: dict[tuple[str, str], dict] = {}

    def record(self, host: str, sess: dict, listed_as: str | None = None) -> None:
        """``listed_as``: the login whose th-run state this session came from."""
        tid = task_id_of_session(sess.get("name"))
        if tid is None:
            return
        rec = {"sid": _int(sess.get("sid")), "uid": _int(sess.get("uid")), "user": sess.get("user") or None,
               "monitor_pid": _int(sess.get("monitor_pid")), "pid": _int(sess.get("pid")),
               "listed_as": listed_as, "seen": time.monotonic()}
        with self._lock:
            self._d[(host, tid)] = rec

    def replace_listing(self, host: str, user: str | None, sessions: list[dict]) -> None:
        """A complete live listing of the sessions ``user`` sees on ``host``: record them and forget
        the sessions of that listing that are no longer live (their sid may be reused later)."""
        live = set()
        for s in sessions:
            self.record(host, s, listed_as=user)
            tid = task_id_of_session(s.get("name"))
            if tid is not None:
                live.add(tid)
        if user is None:
            return
        with self._lock:
            for (h, tid), rec in list(self._d.items()):
                if h == host and rec.get("listed_as") == user and tid not in live:
                    del self._d[(h, tid)]

    def get(self, host: str, task_id) -> dict | None:
        with self._lock:
            r = self._d.get((host, str(task_id)))
            return dict(r) if r else None

    def forget(self, host: str, task_id) -> None:
        with self._lock:
            self._d.pop((host, str(task_id)), None)

    def clear(self) -> None:
        with self._lock:
            self._d.clear()


REGISTRY = SessionRegistry()


def check(proc: dict, sess: dict | None) -> str | None:
    """Why ``proc``'s task claim does not hold against the task's session ``sess`` (None = holds)."""
    if sess is None:
        return "no th-run session of that task on this node"
    puid, suid = _int(proc.get("uid")), sess.get("uid")
    if puid is not None and puid >= 0 and suid is not None:
        if puid != suid:
            return f"uid {puid} is not the task's uid {suid}"
    elif proc.get("owner") and sess.get("user"):
        if proc["owner"] != sess["user"]:
            return f"owner {proc['owner']} is not the task's user {sess['user']}"
    else:
        return "the process's uid is unknown"
    psid, ssid = _int(proc.get("sid")), sess.get("sid")
    if psid is not None and psid > 0 and ssid is not None and psid == ssid:
        return None
    mon = sess.get("monitor_pid")
    if mon is not None and mon in {_int(a) for a in (proc.get("ancestors") or [])}:
        return None
    return "not in the task's th-run session"


class Attestor:
    """Replaces every unverifiable ``task_id`` of an infrastructure entry before it is published.

    ``lookup(host, task_id)`` (optional) refreshes the registry for a task it has not seen, at most
    once per ``refetch_s`` per (host, task): the daemon's implementation lists the task owner's
    sessions on that node (``task_nursery.running``, an SSH round trip for a remote node), which also
    records them.

    ``background=True`` (the daemon) never runs a lookup on the caller's thread: ``publish`` is called
    from the monitoring pool, the task-event listener and the node agents' stream readers, and an
    unreachable node's SSH timeout must not stall any of them.  An unseen claim is queued for one
    worker thread; until its lookup has run the process is published with the claim unattested (marked
    ``attestation_pending`` for the API, but judged by every consumer exactly like a rejected claim, i.e.
    by its UNIX owner: an unverified claim never exempts a process), and the next sample after the
    lookup attests it from the registry.

    The bookkeeping (rate limit, warnings, queue) is shared by those threads and guarded by one lock,
    which is never held across a lookup."""

    # at most this many session lookups per second over all claims: claims are free to forge, so many
    # distinct forged task ids must not turn into as many th-run listings
    MAX_LOOKUPS_PER_S = 2.0
    _MAX_TRACKED = 4096  # rate-limit / warning bookkeeping entries kept before old ones are pruned

    def __init__(self, registry: SessionRegistry = REGISTRY, lookup=None, refetch_s: float = 5.0,
                 background: bool = False):
        self.registry = registry
        self.lookup = lookup
        self.refetch_s = refetch_s
        self.background = background
        self._lock = threading.Lock()
        self._fetched: dict[tuple[str, str], float] = {}
        self._warned: dict[tuple[str, int, str], float] = {}
        self._fallback_warned: dict[tuple[str, str], float] = {}
        self._lookup_times: list[float] = []
        self._pending: set[tuple[str, str]] = set()  # background lookups queued or running
        self._queue = None
        self._worker = None
        self.rejected = 0
        self.lookups = 0

    @classmethod
    def _prune(cls, d: dict, now: float, keep_s: float) -> None:
        if len(d) > cls._MAX_TRACKED:
            for k in [k for k, t in list(d.items()) if now - t > keep_s]:
                d.pop(k, None)
            while len(d) > cls._MAX_TRACKED:  # still too many recent ones: drop the oldest
                d.pop(min(d, key=d.get), None)

    def _lookup_allowed(self, now: float) -> bool:
        """Caller holds ``_lock``."""
        self._lookup_times = [t for t in self._lookup_times if now - t < 1.0]
        if len(self._lookup_times) >= self.MAX_LOOKUPS_PER_S:
            return False
        self._lookup_times.append(now)
        return True

    def _claim_lookup(self, k: tuple[str, str]) -> bool:
        """Reserve a lookup of ``k`` under the rate limit and the per-task refetch interval."""
        now = time.monotonic()
        with self._lock:
            if k in self._pending:
                return False
            if now - self._fetched.get(k, -1e9) < self.refetch_s or not self._lookup_allowed(now):
                return False
            self._fetched[k] = now
            self._prune(self._fetched, now, self.refetch_s)
            return True

    def _run_lookup(self, host: str, tid: str) -> None:
        self.lookups += 1
        try:
            self.lookup(host, tid)
        except Exception as e:  # noqa: BLE001 -- unreachable node: the claim stays unverified
            log.debug("attribution: session lookup of task %s on %s failed: %s", tid, host, e)

    def _worker_loop(self) -> None:
        while True:
            k = self._queue.get()
            if k is None:
                return
            try:
                self._run_lookup(*k)
            finally:
                with self._lock:
                    self._pending.discard(k)

    def _enqueue(self, k: tuple[str, str]) -> None:
        import queue

        with self._lock:
            self._pending.add(k)
            if self._worker is None:
                self._queue = queue.Queue()
                self._worker = threading.Thread(target=self._worker_loop, name="th-attest-lookup", daemon=True)
                self._worker.start()
            q = self._queue
        q.put(k)

    def close(self) -> None:
        with self._lock:
            w, q, self._worker = self._worker, self._queue, None
        if w is not None:
            q.put(None)
            w.join(2.0)

    def drain(self, timeout: float = 5.0) -> bool:
        """Wait until no background lookup is queued or running (tests, shutdown); True if drained."""
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            with self._lock:
                if not self._pending:
                    return True
            time.sleep(0.005)
        return False

    def pending(self, host: str, tid: str) -> bool:
        with self._lock:
            return (host, str(tid)) in self._pending

    def _session(self, host: str, tid: str) -> tuple[dict | None, bool]:
        """(session facts, lookup still pending)."""
        sess = self.registry.get(host, tid)
        if sess is not None or self.lookup is None:
            return sess, False
        k = (host, tid)
        if self.background:
            if self.pending(host, tid):
                return None, True
            if self._claim_lookup(k):
                self._enqueue(k)
                return None, True
            return None, False
        if self._claim_lookup(k):
            self._run_lookup(host, tid)
            sess = self.registry.get(host, tid)
        return sess, False

    def _warn_fallback(self, host: str, tid: str, sess: dict) -> None:
        """A session th-run did not start (the setsid shell fallback records no sid / uid): none of its
        processes can be attested, which costs the task its in-task HBM counters and, when its UNIX
        account is not the TensorHive user, its protection exemption.  Said once per task."""
        if sess.get("sid") is not None or sess.get("uid") is not None:
            return
        now = time.monotonic()
        with self._lock:
            if (host, tid) in self._fallback_warned:
                return
            self._fallback_warned[(host, tid)] = now
            self._prune(self._fallback_warned, now, 3600.0)
        log.warning("attribution: task %s on %s was not started by th-run (no session id / uid recorded): its "
                    "processes cannot be attested and are judged by their UNIX owner", tid, host)

    def verify(self, host: str, proc: dict) -> bool:
        return self._verify(host, proc)[0]

    def _verify(self, host: str, proc: dict) -> tuple[bool, bool]:
        """(attested, lookup pending)."""
        tid = proc.get("task_id")
        if tid in (None, ""):
            return False, False
        sess, pending = self._session(host, str(tid))
        if sess is not None:
            self._warn_fallback(host, str(tid), sess)
        why = check(proc, sess)
        if why is None:
            return True, False
        if pending:
            return False, True
        k = (host, _int(proc.get("pid")) or 0, str(tid))
        now = time.monotonic()
        with self._lock:
            self.rejected += 1
            warn = now - self._warned.get(k, -1e9) > 60.0
            if warn:
                self._warned[k] = now
                self._prune(self._warned, now, 60.0)
        if warn:
            log.warning("attribution: pid %s on %s (owner %s) claims task %s: rejected, %s", proc.get("pid"), host,
                        proc.get("owner"), tid, why)
        return False, False

    def attest_entry(self, host: str, entry: dict | None) -> dict | None:
        """In place: keep each process's ``task_id`` only if it verifies (else move it to
        ``claimed_task_id``; ``attestation_pending`` while its background lookup has not run), then
        derive the in-task HBM metrics from the attested processes."""
        if not entry:
            return entry
        for g in (entry.get("GPU") or {}).values():
            if not g:
                continue
            for p in g.get("processes") or []:
                tid = p.get("task_id")
                if tid in (None, ""):
                    continue
                ok, pending = self._verify(host, p)
                if not ok:
                    p["claimed_task_id"] = str(tid)
                    p["task_id"] = None
                    if pending:
                        p["attestation_pending"] = True
        hbm.finalize_entry(entry)
        return entry
