"""Remote task lifecycle on top of the native ``th-run`` supervisor (reference
``core/task_nursery.py:1-315``, which drove GNU ``screen`` over SSH).

Public functions keep the reference's shape:
  * :func:`spawn` -> pid of the task's process group leader (the command itself, not a screen
    wrapper, so GPU process lists and task PIDs can be matched);
  * :func:`terminate` -- ``gracefully=True`` SIGINT, ``None`` SIGTERM (was ``screen -X quit``),
    ``False`` SIGKILL, always to the whole process group (torchrun + every rank);
  * :func:`running` -- live sessions of a user on a host, ONE round trip per host (``th-run ls``);
  * restart policy: ``max_restarts`` > 0 makes ``th-run`` start a failed run again (new pid, same
    log and session name); :func:`running_sessions` maps the spawn-time pid to the current one;
  * :func:`fetch_log` -- ``~/TensorHiveLogs/task_<id>.log`` (whole file or tail).
Names (``tensorhive_task_<id>``) and log paths are unchanged.  Every task gets
``TENSORHIVE_TASK_ID=<id>`` in its environment, which the telemetry uses to attribute GPU
processes to tasks -- a claim the daemon accepts only for processes of that task's th-run session
running as its uid (``core/attribution.py``, fed by the session state :func:`spawn` and
:func:`running` read).  If ``th-run`` is not installed on a remote node, a ``setsid`` +
``tee`` shell fallback keeps spawn/kill/log working.
"""
from __future__ import annotations

import json
import logging
import shlex

from ..config import get_config
from . import attribution, ssh
from .transport import Result, TransportManager

log = logging.getLogger(__name__)

SESSION_PREFIX = "tensorhive_task_"


class SpawnError(Exception):
    pass


class ExitCodeError(Exception):
    pass


def session_name(task_id) -> str:
    return f"{SESSION_PREFIX}{task_id}"


def log_path(task_id) -> str:
    d = get_config().launcher.log_dir.rstrip("/")
    return f"{d}/task_{task_id}.log"


def _th_run(host: str) -> str:
    spec = get_config().ssh.available_nodes.get(host, {})
    if spec.get("transport") == "local":
        from ..native.build import th_run_binary

        return th_run_binary()
    return get_config().launcher.supervisor


_transports: TransportManager | None = None


def use_transports(tm: TransportManager | None) -> None:
    """Route task operations through the daemon's transports (set by :class:`Daemon`)."""
    global _transports
    _transports = tm


_event_socket_for = None  # host -> th-run --notify socket (core/events.py), set by the Daemon


def use_event_sockets(fn) -> None:
    global _event_socket_for
    _event_socket_for = fn


def _notify_path(host: str) -> str | None:
    fn = _event_socket_for
    try:
        return fn(host) if fn is not None else None
    except Exception:  # noqa: BLE001 -- events are an optimisation; spawning must not fail on them
        return None


def _client(host: str, user: str) -> TransportManager:
    return ssh.get_client(*ssh.build_dedicated_config_for(host, user))


def _run(host: str, user: str, cmd: str, timeout: float | None = None) -> Result:
    timeout = timeout or get_config().ssh.timeout + 20
    tm = _transports
    if tm is not None and host in tm.transports:
        return tm.get(host).run(cmd, timeout=timeout, user=user)
    return _client(host, user).run(host, cmd, timeout=timeout)


def build_spawn_command(command: str, task_id, th_run: str, extra_env: dict | None = None,
                        max_restarts: int = 0, notify: str | None = None) -> str:
    name = session_name(task_id)
    logf = log_path(task_id)
    # the task's exit is an event: th-run sends one datagram to this socket (core/events.py)
    note = f" --notify {shlex.quote(notify)}" if notify else ""
    env = {"TENSORHIVE_TASK_ID": str(task_id), **(extra_env or {})}
    env_args = " ".join(f"--env {shlex.quote(f'{k}={v}')}" for k, v in env.items())
    th = shlex.quote(th_run)
    policy = ""
    if max_restarts and int(max_restarts) > 0:  # th-run restarts a failed run (the fallback cannot)
        policy = f" --max-restarts {int(max_restarts)} --restart-delay {get_config().launcher.restart_delay:g}"
    # th-run prints the task's pid; `status` then prints the new session's state (sid, uid, monitor
    # pid) in the same round trip, for core/attribution.py
    primary = (f"{th} spawn --name {name} --log {logf}{note} {env_args}{policy} -- bash -lc {shlex.quote(command)}"
               f" && {th} status --name {name}")
    envs = " ".join(f"{k}={shlex.quote(str(v))}" for k, v in env.items())
    fallback = (f"mkdir -p $(dirname {logf}) && ( {envs} setsid bash -lc {shlex.quote(command)} "
                f"> >(tee -a {logf} >/dev/null) 2>&1 < /dev/null & echo $! )")
    return f"if command -v {th} >/dev/null 2>&1 || [ -x {th} ]; then {primary}; else {fallback}; fi"


# profilers that open their own counter sessions: a task running one must not also carry the
# in-task counter tool (one device-counting session per GPU; the profiler's would lose)
_PROFILERS = ("rocprofv3", "rocprofv2", "rocprof", "rocprof-compute", "rocprof-sys-run", "omniperf")


def runs_profiler(command: str) -> bool:
    """Whether ``command`` runs a rocprofiler-based profiler, or opts out of the counter tool with
    ``TENSORHIVE_HBM_COUNTERS=0``."""
    try:
        words = shlex.split(command)
    except ValueError:
        words = command.split()
    for w in words:
        if w in ("TENSORHIVE_HBM_COUNTERS=0", "TENSORHIVE_HBM_COUNTERS=no"):
            return True
        if w.rsplit("/", 1)[-1] in _PROFILERS:
            return True
    return False


def spawn_env(hostname: str, command: str = "") -> dict[str, str]:
    """Environment th-run gives every task on ``hostname`` besides ``TENSORHIVE_TASK_ID``: the
    in-task HBM counter tool (``[amd_monitor] task_hbm_counters``, ``core/hbm.py``) -- this
    install's ``libthhbm`` on the daemon's own node, ``[launcher] hbm_tool`` (a path on the node)
    on remote nodes, whose node agent publishes the files (``agent.py``).  Left out when the
    command runs a profiler (``tensorhive profile --pmc``) or says ``TENSORHIVE_HBM_COUNTERS=0``."""
    cfg = get_config()
    if not getattr(cfg.amd_monitor, "task_hbm_counters", False) or runs_profiler(command):
        return {}
    spec = cfg.ssh.available_nodes.get(hostname, {})
    if spec.get("transport") == "local":
        from .hbm import task_env

        return task_env()
    remote_tool = getattr(cfg.launcher, "hbm_tool", "")
    if remote_tool and spec.get("transport", "ssh") == "ssh":
        return {"ROCP_TOOL_LIBRARIES": remote_tool}
    return {}


def spawn(command: str, hostname: str, user: str, name_appendix: str = "", extra_env: dict | None = None,
          max_restarts: int = 0) -> int:
    env = {**spawn_env(hostname, command), **(extra_env or {})}
    r = _run(hostname, user, build_spawn_command(command, name_appendix, _th_run(hostname), env,
                                                 max_restarts, _notify_path(hostname)))
    if r.exception is not None:
        raise SpawnError(f"connection failed: {r.exception}")
    pid = None
    for line in r.stdout.strip().splitlines():
        line = line.strip()
        if line.isdigit() and pid is None:
            pid = int(line)
        elif line.startswith("{"):
            try:
                attribution.REGISTRY.record(hostname, json.loads(line), listed_as=user)
            except json.JSONDecodeError:
                pass
    if pid is None:
        raise SpawnError(f"unable to parse pid from {r.stdout!r} / {r.stderr.strip()!r}")
    return pid


def terminate(pid: int, hostname: str, user: str, gracefully: bool | None = True) -> int:
    verb = {True: "interrupt", None: "terminate", False: "kill"}[gracefully]
    sig = {True: "INT", None: "TERM", False: "KILL"}[gracefully]
    th = shlex.quote(_th_run(hostname))
    cmd = (f"if command -v {th} >/dev/null 2>&1 || [ -x {th} ]; then {th} {verb} --pid {int(pid)}; "
           f"else kill -{sig} -- -{int(pid)} 2>/dev/null || kill -{sig} {int(pid)}; fi")
    r = _run(hostname, user, cmd)
    if r.exception is not None:
        raise ConnectionError(str(r.exception))
    return r.exit_code


def running(hostname: str, user: str) -> list[dict]:
    """Live th-run sessions of ``user`` on ``hostname`` (dicts: name, pid, pgid, started, ...)."""
    th = shlex.quote(_th_run(hostname))
    r = _run(hostname, user, f"if command -v {th} >/dev/null 2>&1 || [ -x {th} ]; then {th} ls; fi")
    if r.exception is not None:
        raise ConnectionError(str(r.exception))
    out = []
    for line in r.stdout.splitlines():
        line = line.strip()
        if not line.startswith("{"):
            continue
        try:
            d = json.loads(line)
        except json.JSONDecodeError:
            continue
        if str(d.get("name", "")).startswith(SESSION_PREFIX):
            out.append(d)
    if r.exit_code == 0:  # a complete listing: the attestation registry follows it
        attribution.REGISTRY.replace_listing(hostname, user, out)
    return out


def running_pids(hostname: str, user: str) -> list[int]:
    return [int(d["pid"]) for d in running(hostname, user)]


def _pid_history(d: dict) -> list[int]:
    pids = [int(d["pid"])]
    for k in ("first_pid", "pgid"):
        if d.get(k) not in (None, ""):
            pids.append(int(d[k]))
    for p in str(d.get("pids") or "").split(","):
        if p.strip().isdigit():
            pids.append(int(p))
    return pids


def running_sessions(hostname: str, user: str) -> dict:
    """Live sessions keyed by their session name (``tensorhive_task_<id>``) and by every pid the
    task has run as: the spawn-time pid, each restart's pid (th-run's ``pids`` history) and the
    current one.  A daemon that stored any of them -- or none, after a restart -- finds the session."""
    out: dict = {}
    for d in running(hostname, user):
        out[str(d.get("name"))] = d
        cur = int(d["pid"])
        out[cur] = d
        for p in _pid_history(d):
            out.setdefault(p, d)
    return out


def fetch_log(hostname: str, user: str, task_id, tail: bool = False, tail_lines: int = 10) -> tuple[list[str], str]:
    path = log_path(task_id)
    cmd = f"tail -n {int(tail_lines)} {path}" if tail else f"cat {path}"
    r = _run(hostname, user, cmd)
    if r.exception is not None:
        raise ConnectionError(str(r.exception))
    if r.exit_code != 0:
        raise FileNotFoundError(path)
    return r.stdout.splitlines(), path
