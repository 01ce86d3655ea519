"""Node agent: the full MI355X telemetry of ONE node as a JSON-lines stream.

``python3 -m tensorhive_fixed_amd.agent --stream 250 [--probe] [--task-hbm] [--counters]``

The reference monitored every configured host the same way -- one ``nvidia-smi --query-gpu`` over
a parallel SSH client of all hosts (``tensorhive/core/monitors/GPUMonitor.py:20-48``,
``core/managers/SSHConnectionManager.py:21-30``).  Here a remote node runs this agent inside ONE
multiplexed SSH channel (``core/telemetry.py:RemoteBackend``, agent mode), and it samples the node
with exactly the code the daemon uses for its own node (:class:`AmdSmiBackend`):

* libthsmi (amdsmi + KFD/DRM process attribution, owners, ``TENSORHIVE_TASK_ID``);
* the ``th-probe`` agent on every GPU of the node (the probe's MFMA / HBM contention metrics), a
  child of this process, so neither it nor the agent is ever listed as a tenant;
* the node's in-task HBM counter files (``/dev/shm/th-hbm-*.json``, written by tasks th-run
  started with ``[launcher] hbm_tool``), authenticated and merged per GPU (``core/hbm.py``);
* optionally the device-wide counter sampler (``th-counters``).

With ``--events SOCK`` the agent also listens for th-run's task-exit datagrams (``core/events.py``):
on one it samples the node at once and sends ``{"v": 1, ..., "event": {...}}`` after that entry.

Every line is ``{"v": 1, "ts": <unix s>, "host": <node>, "entry": <infrastructure entry>}``; the
entry is the same per-host document the local backend publishes, so the API, protection,
allocation and usage logging see remote GPUs exactly like local ones.  The agent exits (and stops
its probe) when the SSH channel closes (EPIPE on stdout), on SIGTERM/SIGHUP, or after ``--once``.

``--backend stub`` samples a scripted fake node instead (CPU tests: ``--stub-process`` injects
``GPU:PID:OWNER[:TASK]`` tenants and ``--hbm-glob`` points at test counter files).
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import sys
import time

EVENT_MIN_GAP_S = 0.02  # minimum time between an event-triggered sample and the previous sample
MAX_EVENTS_PER_SAMPLE = 64  # task-exit events forwarded with one sample (a flood's excess is dropped)


def _stub_backend(args):
    from .core.telemetry import StubBackend

    be = StubBackend(gpus_per_host=args.stub_gpus)
    for spec in args.stub_process or []:
        parts = spec.split(":")
        gpu, pid, owner = int(parts[0]), int(parts[1]), parts[2]
        be.add_process(args.host, gpu, pid, owner, task_id=parts[3] if len(parts) > 3 and parts[3] else None)
    return be


def build_backend(args):
    if args.backend == "stub":
        return _stub_backend(args)
    from .core.telemetry import AmdSmiBackend

    return AmdSmiBackend(probe=args.probe, probe_period=args.probe_period, counters=args.counters,
                         counters_period_ms=args.counters_period_ms, task_hbm=args.task_hbm)


def sample(backend, args) -> dict | None:
    entry = backend.sample(args.host)
    if entry is not None and args.backend == "stub" and args.task_hbm:
        from .core.telemetry import apply_task_hbm

        apply_task_hbm(entry, args.hbm_glob)
    return entry


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(prog="tensorhive-agent", description=__doc__.split("\n\n")[0])
    ap.add_argument("--stream", type=int, default=0, metavar="MS", help="emit one line every MS ms (0 = once)")
    ap.add_argument("--once", action="store_true")
    ap.add_argument("--host", default=socket.gethostname())
    ap.add_argument("--backend", choices=("amdsmi", "stub"), default="amdsmi")
    ap.add_argument("--probe", dest="probe", action="store_true", default=True)
    ap.add_argument("--no-probe", dest="probe", action="store_false")
    ap.add_argument("--probe-period", type=float, default=1.0)
    ap.add_argument("--task-hbm", dest="task_hbm", action="store_true", default=True)
    ap.add_argument("--no-task-hbm", dest="task_hbm", action="store_false")
    ap.add_argument("--counters", action="store_true")
    ap.add_argument("--counters-period-ms", type=int, default=1000)
    ap.add_argument("--stub-gpus", type=int, default=8)
    ap.add_argument("--stub-process", action="append", metavar="GPU:PID:OWNER[:TASK]")
    ap.add_argument("--hbm-glob", default=None, help="counter files to merge (default /dev/shm/th-hbm-*.json)")
    ap.add_argument("--events", default=None, metavar="SOCK",
                    help="unix datagram socket th-run notifies on task exit (core/events.py): the agent "
                         "samples the node at once and forwards the event.  'auto': a socket in a fresh "
                         "private directory; the bound path is reported as the stream's first line")
    args = ap.parse_args(argv)

    stop = {"flag": False}

    def _stop(*_):
        stop["flag"] = True

    for sig in (signal.SIGTERM, signal.SIGHUP, signal.SIGINT):
        signal.signal(sig, _stop)
    backend = build_backend(args)
    period = max(0.02, args.stream / 1000.0) if args.stream > 0 else 0.0
    ev_sock = ev_path = ev_tmp = None
    if args.events and period > 0:
        from .core.events import open_event_socket

        try:
            ev_sock, ev_path, ev_tmp = open_event_socket(args.events)
            # the daemon hands th-run --notify only the path an agent reports having bound (a
            # fixed world-writable path can be squatted by another local user)
            print(json.dumps({"v": 1, "host": args.host, "events_socket": ev_path}), flush=True)
        except OSError as e:  # another agent's socket, a squatted path: exits are found by polling
            print(json.dumps({"v": 1, "warning": f"task events unavailable: {e}"[:300]}), flush=True)
    rc = 0

    def emit(doc) -> bool:
        try:
            sys.stdout.write(json.dumps(doc, separators=(",", ":")) + "\n")
            sys.stdout.flush()
            return True
        except BrokenPipeError:  # the SSH channel is gone: stop the probe with us
            return False

    try:
        events: list[dict] = []
        while not stop["flag"]:
            t0 = time.monotonic()
            entry = sample(backend, args)
            if not emit({"v": 1, "ts": round(time.time(), 3), "host": args.host, "entry": entry}):
                break
            # task exits that arrived: forwarded AFTER a sample taken once they had happened
            if events and not all(emit({"v": 1, "ts": round(time.time(), 3), "host": args.host, "event": ev})
                                  for ev in events):
                break
            events = []
            if args.once or period == 0.0:
                break
            left = period - (time.monotonic() - t0)
            while left > 0 and not stop["flag"]:
                if ev_sock is not None:
                    import select

                    from .core.events import parse_event

                    # an event samples the node at once, but not sooner than EVENT_MIN_GAP_S after the last
                    # sample: any local user can send to the socket, so a flood coalesces into one sample
                    since = time.monotonic() - t0
                    wait = min(left, 0.05) if not events else max(0.0, EVENT_MIN_GAP_S - since)
                    if events and wait == 0.0:
                        break  # sample now
                    r, _, _ = select.select([ev_sock], [], [], wait)
                    if r:
                        ev = parse_event(ev_sock.recv(65536))
                        if ev is not None and len(events) < MAX_EVENTS_PER_SAMPLE:
                            events.append(ev)
                else:
                    time.sleep(min(left, 0.05))
                left = period - (time.monotonic() - t0)
    except Exception as e:  # noqa: BLE001 -- report and exit non-zero; the daemon restarts us
        print(json.dumps({"v": 1, "error": f"{type(e).__name__}: {e}"[:300]}), flush=True)
        rc = 1
    finally:
        if ev_sock is not None:
            try:
                ev_sock.close()
                os.unlink(ev_path)
                if ev_tmp:
                    os.rmdir(ev_tmp)
            except OSError:
                pass
        try:
            backend.close()
        except Exception:  # noqa: BLE001
            pass
        try:  # no "Exception ignored ... BrokenPipeError" noise on a closed channel
            sys.stdout = open(os.devnull, "w")
        except OSError:
            pass
    return rc


if __name__ == "__main__":
    sys.exit(main())
