"""Helpers for the daemon's long-lived helper processes (``th-probe``, ``th-counters``)."""
from __future__ import annotations

import threading
from collections import deque


class StderrTail:
    """Drains a child's stderr pipe on a thread of its own, keeping the last ``lines`` lines.

    A helper that writes more than a pipe buffer (64 KiB) to an unread stderr blocks in
    ``write`` and stops producing samples; draining keeps it running while the tail stays
    available for the error message when it exits."""

    def __init__(self, stream, lines: int = 50, name: str = "stderr"):
        self._tail: deque = deque(maxlen=lines)
        self._stream = stream
        self._thread = threading.Thread(target=self._run, name=f"{name}-stderr", daemon=True)
        self._thread.start()

    def _run(self) -> None:
        try:
            for line in self._stream:
                self._tail.append(line.rstrip("\n"))
        except (OSError, ValueError):  # pipe closed under us
            pass

    def text(self, wait: float = 1.0, limit: int = 500) -> str:
        """The retained tail (waits up to ``wait`` s for the drain to reach EOF)."""
        self._thread.join(wait)
        return "\n".join(self._tail).strip()[-limit:]
