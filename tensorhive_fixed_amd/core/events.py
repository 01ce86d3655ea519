"""Task exit as an event (round-4 verdict item 5; BASELINE config 4).

The reference discovers that a task ended only through its 30 s scheduling tick
(``tensorhive/core/services/JobSchedulingService.py:286-297``), and round 4 still found a local
exit by polling (monitoring sees the device freed, then the scheduler re-lists th-run sessions
every 0.5 s).  Here the th-run monitor of every task sends ONE datagram when the task has exited
and its state file says so (``th-run spawn --notify SOCK``, ``native/th_run.cpp``):

* the daemon's own node: :class:`EventListener` owns a unix datagram socket in a private
  ``mkdtemp`` directory; tasks of any user can send to it (the message is only a hint: a forged
  one costs one scheduler tick, never a state change -- the scheduler re-reads th-run's state);
* remote nodes: the node agent (``agent.py --events SOCK``) listens on the node, samples the node
  at once and forwards the event as a line of its telemetry stream (``RemoteBackend``).

On an event the daemon takes a fresh telemetry sample of that host (the device shows the exited
task's process no more) and wakes the job scheduler, which then releases the task's devices and
starts the next queued job in the same tick (``Daemon.on_task_event``).
"""
from __future__ import annotations

import json
import logging
import os
import select
import socket
import tempfile
import threading
import time

log = logging.getLogger(__name__)


def parse_event(data: bytes) -> dict | None:
    try:
        ev = json.loads(data.decode("utf-8", "replace"))
    except ValueError:
        return None
    if not isinstance(ev, dict) or ev.get("event") != "task_exit":
        return None
    return ev


def open_event_socket(path: str | None = None) -> tuple[socket.socket, str, str | None]:
    """A bound unix datagram socket any local user may send to.  Without ``path`` (or ``"auto"``) it
    lives in a fresh private directory under ``$XDG_RUNTIME_DIR`` or the temp dir (mode 0711: nobody
    can pre-create or replace the socket; returned third, to remove on close); with ``path`` an
    existing socket file of ours is replaced, anything else is refused."""
    tmpdir = None
    if path in (None, "", "auto"):
        base = os.environ.get("XDG_RUNTIME_DIR")
        base = base if base and os.path.isdir(base) and os.access(base, os.W_OK) else None
        tmpdir = tempfile.mkdtemp(prefix="tensorhive-events-", dir=base)
        os.chmod(tmpdir, 0o711)  # others may reach the socket by its name, not list the directory
        path = os.path.join(tmpdir, "events.sock")
    else:
        try:
            st = os.lstat(path)
            import stat as _st

            if _st.S_ISSOCK(st.st_mode) and st.st_uid == os.getuid():
                os.unlink(path)
            else:
                raise OSError(f"{path} exists and is not our socket")
        except FileNotFoundError:
            pass
    s = socket.socket(socket.AF_UNIX, socket.SOCK_DGRAM)
    try:
        s.bind(path)
        os.chmod(path, 0o666)
    except OSError:
        s.close()
        raise
    return s, path, tmpdir


class EventListener:
    """Reads task-exit datagrams on the daemon's node and calls ``on_event(event)`` per event."""

    def __init__(self, on_event, path: str | None = None):
        self.on_event = on_event
        self.sock, self.path, self._tmpdir = open_event_socket(path)
        self._stop = threading.Event()
        self.received = 0
        self.last_at: float | None = None
        self._thread = threading.Thread(target=self._run, name="th-task-events", daemon=True)
        self._thread.start()

    def _run(self) -> None:
        while not self._stop.is_set():
            try:
                r, _, _ = select.select([self.sock], [], [], 0.5)
                if not r:
                    continue
                data = self.sock.recv(65536)
            except OSError:
                if self._stop.is_set():
                    return
                time.sleep(0.05)
                continue
            ev = parse_event(data)
            if ev is None:
                continue
            self.received += 1
            self.last_at = time.time()
            try:
                self.on_event(ev)
            except Exception:  # noqa: BLE001 -- a failing handler must not stop the listener
                log.exception("task event handler failed")

    def close(self) -> None:
        self._stop.set()
        try:
            self.sock.close()
        except OSError:
            pass
        self._thread.join(2.0)
        for p in (self.path,):
            try:
                os.unlink(p)
            except OSError:
                pass
        if self._tmpdir:
            try:
                os.rmdir(self._tmpdir)
            except OSError:
                pass
