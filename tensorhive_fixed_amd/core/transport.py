"""Node transports: how the daemon runs commands on a node (replaces parallel-ssh/libssh2).

Reference: ``core/managers/SSHConnectionManager.py`` (one ParallelSSHClient over all hosts +
cached per-host clients, optional proxy jump) and ``core/ssh.py`` (``run_command`` with
``stop_on_errors=False``).  Here:

* :class:`LocalTransport` -- fork/exec on the node the daemon runs on (no sshd needed); can run
  as another UNIX user through ``runuser`` when the daemon is root.
* :class:`SSHTransport` -- the OpenSSH client with **ControlMaster multiplexing** (one TCP/SSH
  session per host and user, reused by every command: no per-command handshake), optional
  ProxyJump, BatchMode, TensorHive's dedicated key.
* :class:`FakeTransport` -- scripted replies + fault injection (drop host, hang, fail) for tests.
* :class:`SimulatedNode` -- a node that understands the ``th-run`` protocol in-process (spawn,
  ls, signals, logs) and shows spawned tasks as GPU processes in a :class:`StubBackend`; used by
  the CPU test-suite, demos and the daemon benchmarks (``transport = simulated``).
* :class:`TransportManager` -- per-host transports from ``hosts_config.ini`` and a thread-pool
  fan-out (``run_all``) whose per-host failures never abort the others.
"""
from __future__ import annotations

import concurrent.futures as cf
import getpass
import json
import logging
import os
import re
import shlex
import subprocess
import threading
import time
from dataclasses import dataclass, field
from pathlib import Path
from typing import Callable

log = logging.getLogger(__name__)


@dataclass
class Result:
    host: str
    stdout: str
    stderr: str
    exit_code: int
    exception: BaseException | None = None

    @property
    def ok(self) -> bool:
        return self.exception is None and self.exit_code == 0

    @property
    def lines(self) -> list[str]:
        return self.stdout.splitlines()


class Transport:
    host: str = "localhost"
    user: str | None = None

    def run(self, command: str, timeout: float | None = None, user: str | None = None,
            env: dict | None = None) -> Result:
        raise NotImplementedError

    def close(self) -> None:
        pass


class LocalTransport(Transport):
    def __init__(self, host: str = "localhost", user: str | None = None):
        self.host = host
        self.user = user

    def _argv(self, command: str, user: str | None) -> list[str]:
        me = getpass.getuser()
        if user and user != me:
            if os.geteuid() == 0:
                return ["runuser", "-u", user, "--", "bash", "-lc", command]
            log.debug("local transport cannot switch to %s (not root); running as %s", user, me)
        return ["bash", "-c", command]

    def stream_argv(self, command: str, user: str | None = None) -> list[str]:
        """argv of a long-running command whose stdout the caller reads (telemetry streams)."""
        return self._argv(command, user or self.user)

    def run(self, command, timeout=None, user=None, env=None) -> Result:
        try:
            p = subprocess.run(self._argv(command, user or self.user), capture_output=True, text=True,
                               timeout=timeout, env={**os.environ, **(env or {})})
            return Result(self.host, p.stdout, p.stderr, p.returncode)
        except subprocess.TimeoutExpired as e:
            return Result(self.host, e.stdout or "", e.stderr or "", 124, e)
        except OSError as e:
            return Result(self.host, "", str(e), 127, e)


class SSHTransport(Transport):
    """OpenSSH with a persistent ControlMaster per (host, user)."""

    def __init__(self, host: str, user: str, port: int = 22, key_file: str | None = None,
                 proxy: dict | None = None, timeout: float = 10.0, control_dir: str | None = None):
        self.host, self.user, self.port = host, user, port
        self.key_file, self.proxy, self.timeout = key_file, proxy, timeout
        self.control_dir = Path(control_dir or os.path.expanduser("~/.cache/tensorhive/ssh"))
        self.control_dir.mkdir(parents=True, exist_ok=True, mode=0o700)

    def base_argv(self, user: str | None = None) -> list[str]:
        u = user or self.user
        argv = ["ssh", "-p", str(self.port), "-o", "BatchMode=yes", "-o", "StrictHostKeyChecking=accept-new",
                "-o", f"ConnectTimeout={int(max(1, self.timeout))}", "-o", "ControlMaster=auto",
                "-o", f"ControlPath={self.control_dir}/%r@%h:%p", "-o", "ControlPersist=600",
                "-o", "ServerAliveInterval=15"]
        if self.key_file:
            argv += ["-i", self.key_file, "-o", "IdentitiesOnly=yes"]
        if self.proxy:
            argv += ["-J", f"{self.proxy['proxy_user']}@{self.proxy['proxy_host']}:{self.proxy.get('proxy_port', 22)}"]
        return argv + [f"{u}@{self.host}"]

    def stream_argv(self, command: str, user: str | None = None) -> list[str]:
        """argv of a long-running remote command over the ControlMaster channel (telemetry streams)."""
        return self.base_argv(user) + [command]

    def run(self, command, timeout=None, user=None, env=None) -> Result:
        if env:
            command = " ".join(f"{k}={shlex.quote(str(v))}" for k, v in env.items()) + " " + command
        argv = self.base_argv(user) + [command]
        try:
            p = subprocess.run(argv, capture_output=True, text=True, timeout=timeout or (self.timeout + 60))
            exc = None
            if p.returncode == 255:  # ssh itself failed (connection/auth)
                exc = ConnectionError(p.stderr.strip() or "ssh connection failed")
            return Result(self.host, p.stdout, p.stderr, p.returncode, exc)
        except subprocess.TimeoutExpired as e:
            return Result(self.host, "", "timeout", 124, e)
        except OSError as e:
            return Result(self.host, "", str(e), 127, e)

    def close(self) -> None:
        subprocess.run(self.base_argv()[:-1] + ["-O", "exit", f"{self.user}@{self.host}"], capture_output=True)


class FakeTransport(Transport):
    """Scripted transport for tests: ``rules`` are (regex, handler|Result-like tuple)."""

    def __init__(self, host: str, user: str = "tensorhive"):
        self.host, self.user = host, user
        self.rules: list[tuple[re.Pattern, Callable[[str, str | None], tuple[str, str, int]]]] = []
        self.calls: list[tuple[str, str | None]] = []
        self.down = False
        self.hang = 0.0
        self._lock = threading.Lock()

    def on(self, pattern: str, reply) -> "FakeTransport":
        fn = reply if callable(reply) else (lambda _c, _u, r=reply: r)
        self.rules.append((re.compile(pattern), fn))
        return self

    def run(self, command, timeout=None, user=None, env=None) -> Result:
        with self._lock:
            self.calls.append((command, user))
        if self.down:
            return Result(self.host, "", "host unreachable", 255, ConnectionError("host unreachable"))
        if self.hang:
            time.sleep(min(self.hang, timeout or self.hang))
            return Result(self.host, "", "timeout", 124, TimeoutError("hang"))
        for pat, fn in self.rules:
            if pat.search(command):
                out, err, rc = fn(command, user)
                return Result(self.host, out, err, rc)
        return Result(self.host, "", f"no rule for: {command}", 127)


class SimulatedNode(FakeTransport):
    """In-process node speaking the ``th-run`` protocol (see ``native/th_run.cpp``).

    Spawned tasks get a fresh pid; when ``telemetry`` (a StubBackend) is given they appear on the
    GPUs named by ``HIP_VISIBLE_DEVICES`` with their owner and ``TENSORHIVE_TASK_ID``, exactly as
    the amdsmi backend would report them.  ``exit_task(pid)`` simulates a task finishing."""

    _SPAWN = re.compile(r"spawn --name (\S+) --log (\S+)(?: --notify \S+)?((?: --env \S+)*)(?: --max-restarts (\d+) --restart-delay \S+)?"
                        r" -- bash -lc (.*?)(?: && \S+ status --name \S+)?; else")
    _SIG = re.compile(r"then \S+ (interrupt|terminate|kill) --pid (\d+)")

    def __init__(self, host: str, telemetry=None, first_pid: int = 40000):
        super().__init__(host)
        self.telemetry = telemetry
        self.sessions: dict[int, dict] = {}
        self.logs: dict[str, list[str]] = {}
        self.ttys: list[tuple[str, str]] = []  # (user, tty) pairs reported by `who`
        self.tty_messages: list[tuple[str, str]] = []  # (tty, text) written by warnings
        self.killed: list[tuple[int, str | None, bool]] = []  # (pid, as user, via sudo)
        self._next = first_pid
        self.on_event = None  # th-run's task-exit notification (the Daemon's on_task_event)

    def run(self, command, timeout=None, user=None, env=None) -> Result:
        with self._lock:
            self.calls.append((command, user))
        if self.down:
            return Result(self.host, "", "host unreachable", 255, ConnectionError("host unreachable"))
        for pat, fn in self.rules:  # explicit rules win (fault injection)
            if pat.search(command):
                out, err, rc = fn(command, user)
                return Result(self.host, out, err, rc)
        m = self._SPAWN.search(command)
        if m:
            return self._spawn(m, user)
        m = self._SIG.search(command)
        if m:
            return self._signal(int(m.group(2)), m.group(1), user)
        if re.search(r"then \S+ ls; fi", command):
            with self._lock:
                lines = [json.dumps({k: v for k, v in s.items() if k not in ("gpus", "env")})
                         for s in self.sessions.values() if s["user"] == user]
            return Result(self.host, "\n".join(lines) + ("\n" if lines else ""), "", 0)
        m = re.match(r"(?:tail -n (\d+)|cat) (\S+)$", command.strip())
        if m:
            lines = self.logs.get(m.group(2))
            if lines is None:
                return Result(self.host, "", "No such file", 1)
            lines = lines[-int(m.group(1)):] if m.group(1) else lines
            return Result(self.host, "".join(l + "\n" for l in lines), "", 0)
        if command.strip() == "uname":
            return Result(self.host, "Linux\n", "", 0)
        if command.strip() == "who":
            return Result(self.host, "".join(f"{u} {t} 2026-01-01 00:00\n" for u, t in self.ttys), "", 0)
        if "| tee /dev/" in command:
            for text, tty in re.findall(r"echo -e (.*?) \| tee /dev/(\S+) >/dev/null", command, re.S):
                self.tty_messages.append((tty, shlex.split(text)[0] if text.startswith("'") else text))
            return Result(self.host, "", "", 0)
        m = re.match(r"(sudo -n )?kill ((?:\d+ ?)+)$", command.strip())
        if m:
            for pid in map(int, m.group(2).split()):
                self.killed.append((pid, user, bool(m.group(1))))
                self._drop_gpu_process(pid)
                with self._lock:
                    self.sessions.pop(pid, None)
            return Result(self.host, "", "", 0)
        return Result(self.host, "", f"simulated node: unsupported command {command[:80]}", 127)

    def _drop_gpu_process(self, pid: int) -> None:
        if self.telemetry is None:
            return
        with self.telemetry._lock:
            for k, procs in list(self.telemetry.processes.items()):
                if k[0] == self.host:
                    self.telemetry.processes[k] = [p for p in procs if p["pid"] != pid]

    def _spawn(self, m, user) -> Result:
        name, logf, envs, cmd = m.group(1), m.group(2), m.group(3), m.group(5)
        max_restarts = int(m.group(4) or 0)
        env = dict(shlex.split(e)[0].split("=", 1) for e in re.findall(r"--env (\S+)", envs))
        cmd = shlex.split(cmd)[0] if cmd.startswith("'") else cmd
        gpus = []
        mv = re.search(r"(?:HIP|ROCR)_VISIBLE_DEVICES=([0-9,]+)", cmd)
        if mv:
            gpus = [int(x) for x in mv.group(1).split(",") if x]
        with self._lock:
            pid = self._next
            self._next += 1
            # th-run's session facts: the first child's setsid gives the session id, the monitor
            # is its child (pids of their own, disjoint from task pids)
            sid, mon = 900000 + pid, 800000 + pid
            self.sessions[pid] = {"name": name, "pid": pid, "pgid": pid, "started": time.time(), "user": user,
                                  "command": cmd, "log": logf, "gpus": gpus, "first_pid": pid, "pids": str(pid), "restarts": 0,
                                  "max_restarts": max_restarts, "env": env, "sid": sid, "monitor_pid": mon,
                                  "status": "running"}
            self.logs[logf] = [f"[simulated] {cmd}"]
            status = json.dumps({k: v for k, v in self.sessions[pid].items() if k not in ("gpus", "env")})
        if self.telemetry is not None:
            for g in gpus:
                self.telemetry.add_process(self.host, g, pid, user or "", cmd[:80], env.get("TENSORHIVE_TASK_ID"),
                                           sid=sid, ancestors=[mon])
        return Result(self.host, f"{pid}\n{status}\n", "", 0)

    def crash_task(self, pid: int, code: int = 1) -> int | None:
        """Simulate a run exiting with ``code``: like th-run, a session with restarts left is
        started again under a new pid (returned); otherwise it ends (None)."""
        with self._lock:
            s = self.sessions.get(pid)
        if s is None:
            return None
        if s["restarts"] >= s["max_restarts"]:
            self.exit_task(pid, f"[simulated] exit code {code}", code=code)
            return None
        self._drop_gpu_process(pid)
        with self._lock:
            self.sessions.pop(pid, None)
            new = self._next
            self._next += 1
            s = dict(s, pid=new, pgid=new, restarts=s["restarts"] + 1, last_exit_code=code,
                     pids=f"{s['pids']},{new}")
            self.sessions[new] = s
            self.logs.setdefault(s["log"], []).append(
                f"[th-run] exit code {code}; restart {s['restarts']}/{s['max_restarts']}")
        if self.telemetry is not None:
            for g in s["gpus"]:
                self.telemetry.add_process(self.host, g, new, s["user"] or "", s["command"][:80],
                                           s["env"].get("TENSORHIVE_TASK_ID"), sid=s["sid"],
                                           ancestors=[s["monitor_pid"]])
        return new

    def exit_task(self, pid: int, line: str = "[simulated] done", code: int = 0) -> None:
        with self._lock:
            s = self.sessions.pop(pid, None)
        if s is None:
            return
        self.logs.setdefault(s["log"], []).append(line)
        self._drop_gpu_process(pid)
        if self.on_event is not None:  # like th-run: after the state says exited
            self.on_event({"event": "task_exit", "name": s["name"], "pid": pid, "exit_code": code,
                           "ended_ms": int(time.time() * 1000)})

    def _signal(self, pid: int, verb: str, user) -> Result:
        with self._lock:
            s = self.sessions.get(pid) or next(
                (x for x in self.sessions.values() if str(pid) in str(x.get("pids", "")).split(",")), None)
            pid = s["pid"] if s else pid
        if s is None or (user and s["user"] != user):
            return Result(self.host, "", f"no such session {pid}", 1)
        self.exit_task(pid, f"[simulated] {verb}")
        return Result(self.host, "", "", 0)


@dataclass
class TransportManager:
    """Per-host transports + parallel fan-out (``stop_on_errors=False`` semantics)."""

    transports: dict[str, Transport] = field(default_factory=dict)
    max_workers: int = 32

    @classmethod
    def from_config(cls, nodes: dict[str, dict], key_file: str | None, proxy: dict | None,
                    timeout: float = 10.0) -> "TransportManager":
        tm = cls()
        for host, spec in nodes.items():
            kind = spec.get("transport", "ssh")
            if kind == "local" or (kind == "auto" and host in ("localhost", "127.0.0.1")):
                tm.transports[host] = LocalTransport(host, spec.get("user"))
            elif kind == "simulated":
                tm.transports[host] = SimulatedNode(host)
            else:
                tm.transports[host] = SSHTransport(host, spec.get("user") or getpass.getuser(),
                                                   int(spec.get("port", 22)), key_file, proxy, timeout)
        return tm

    def hosts(self) -> list[str]:
        return list(self.transports)

    def get(self, host: str) -> Transport:
        t = self.transports.get(host)
        if t is None:
            raise KeyError(f"unknown host {host}")
        return t

    def run(self, host: str, command: str, **kw) -> Result:
        return self.get(host).run(command, **kw)

    def run_all(self, command: str | Callable[[str], str], hosts: list[str] | None = None,
                timeout: float | None = None) -> dict[str, Result]:
        hosts = hosts or self.hosts()
        if not hosts:
            return {}
        with cf.ThreadPoolExecutor(max_workers=min(self.max_workers, len(hosts))) as ex:
            futs = {h: ex.submit(self.transports[h].run, command(h) if callable(command) else command,
                                 timeout=timeout) for h in hosts}
            out = {}
            for h, f in futs.items():
                try:
                    out[h] = f.result()
                except Exception as e:  # noqa: BLE001
                    out[h] = Result(h, "", str(e), 1, e)
            return out

    def test_all(self, timeout: float = 10.0) -> dict[str, bool]:
        """``uname`` on every host (reference ``test_all_connections``)."""
        return {h: r.ok for h, r in self.run_all("uname", timeout=timeout).items()}

    def close(self) -> None:
        for t in self.transports.values():
            try:
                t.close()
            except Exception:  # noqa: BLE001
                pass
