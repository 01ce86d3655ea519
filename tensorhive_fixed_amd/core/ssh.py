"""Stateless SSH helpers with the reference's API shape (``core/ssh.py:32-177``) on top of
:mod:`.transport` (OpenSSH + ControlMaster instead of parallel-ssh/paramiko).

``build_dedicated_config_for(host, user)`` -> transport config to act AS ``user`` on ``host``
with TensorHive's key; ``get_client`` is memoised; ``run_command``/``get_stdout`` keep the
"one failed host does not stop the others" semantics; keys are ed25519 made by ``ssh-keygen``
(mode 0600, never overwritten unless ``replace``).
"""
from __future__ import annotations

import logging
import os
import socket
import subprocess
from pathlib import Path

from ..config import get_config
from ..utils.decorators import memoize
from .transport import LocalTransport, Result, SSHTransport, Transport, TransportManager

log = logging.getLogger(__name__)


def build_dedicated_config_for(host: str, user: str) -> tuple[dict, dict | None]:
    assert host and user, "Arguments must not be None!"
    nodes = get_config().ssh.available_nodes
    assert host in nodes, f"unknown host {host}"
    spec = nodes[host]
    cfg = {host: {"user": user, "pkey": get_config().ssh.key_file, "port": spec.get("port", 22),
                  "transport": spec.get("transport", "ssh")}}
    return cfg, get_config().ssh.proxy


def _freeze(d):
    if isinstance(d, dict):
        return tuple(sorted((k, _freeze(v)) for k, v in d.items()))
    return d


@memoize
def _client(frozen_cfg, frozen_proxy) -> TransportManager:
    cfg = {h: dict(v) for h, v in frozen_cfg}
    proxy = dict(frozen_proxy) if frozen_proxy else None
    tm = TransportManager()
    for host, spec in cfg.items():
        if spec.get("transport") == "local":
            tm.transports[host] = LocalTransport(host, spec["user"])
        else:
            tm.transports[host] = SSHTransport(host, spec["user"], int(spec.get("port", 22)), spec.get("pkey"),
                                               proxy, get_config().ssh.timeout)
    return tm


def get_client(config: dict, pconfig: dict | None = None) -> TransportManager:
    return _client(_freeze(config), _freeze(pconfig) if pconfig else None)


def run_command(client: TransportManager, command: str, timeout: float | None = None) -> dict[str, Result]:
    return client.run_all(command, timeout=timeout)


def get_stdout(host: str, output: dict[str, Result]) -> str | None:
    r = output[host]
    if r.exception is not None:
        raise r.exception
    return r.stdout.rstrip("\n")


def succeeded(host: str, output: dict[str, Result]) -> bool:
    return output[host].ok


def generate_key(path: Path, replace: bool = False) -> Path:
    path = Path(path).expanduser()
    if path.exists() and not replace:
        raise FileExistsError(str(path))
    path.parent.mkdir(parents=True, exist_ok=True)
    for p in (path, path.with_suffix(path.suffix + ".pub")):
        if p.exists():
            p.unlink()
    subprocess.run(["ssh-keygen", "-q", "-t", "ed25519", "-N", "", "-C", f"tensorhive@{socket.gethostname()}",
                    "-f", str(path)], check=True, capture_output=True)
    os.chmod(path, 0o600)
    return path


def init_ssh_key(path: Path | str) -> Path:
    path = Path(path).expanduser()
    if path.exists():
        log.info("using existing SSH key %s", path)
        return path
    log.info("generating SSH key %s", path)
    return generate_key(path)


def public_key(path: Path | str) -> str:
    path = Path(path).expanduser()
    pub = path.with_suffix(path.suffix + ".pub")
    if pub.exists():
        return pub.read_text().strip()
    out = subprocess.run(["ssh-keygen", "-y", "-f", str(path)], capture_output=True, text=True, check=True)
    return out.stdout.strip()


def authorized_keys_entry(key_path: Path | str, host: str | None = None) -> str:
    """The line a user appends to ~/.ssh/authorized_keys (reference ``user.authorized_keys_entry``)."""
    parts = public_key(init_ssh_key(key_path)).split()
    return f"{parts[0]} {parts[1]} tensorhive@{host or socket.gethostname()}"


def verify_login_as(host: str, username: str, key_path: str) -> bool:
    """Self-signup proof: can TensorHive's key log into ``host`` as ``username``?"""
    spec = get_config().ssh.available_nodes.get(host, {})
    if spec.get("transport") == "local":
        import pwd

        try:
            pwd.getpwnam(username)
        except KeyError:
            return False
        ak = Path(pwd.getpwnam(username).pw_dir) / ".ssh" / "authorized_keys"
        try:
            key = public_key(key_path).split()[1]
            return ak.exists() and key in ak.read_text()
        except (OSError, subprocess.CalledProcessError, IndexError):
            return False
    t = SSHTransport(host, username, int(spec.get("port", 22)), key_path, get_config().ssh.proxy,
                     get_config().ssh.timeout)
    return t.run("true", timeout=get_config().ssh.timeout + 5).ok


def node_tty_sessions(transport: Transport) -> list[dict]:
    """Active terminal sessions on a node: ``[{'USER': ..., 'TTY': ...}]`` from ``who``."""
    r = transport.run("who")
    if not r.ok:
        return []
    return parse_who(r.stdout)


def parse_who(stdout: str) -> list[dict]:
    out = []
    for line in stdout.splitlines():
        cols = line.split()
        if len(cols) >= 2:
            out.append({"USER": cols[0], "TTY": cols[1]})
    return out
