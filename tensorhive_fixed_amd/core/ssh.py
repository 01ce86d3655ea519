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


def _ssh_login_ok(host: str, username: str, port: int, key_path: str) -> bool:
    """The reference's proof (``tensorhive/controllers/user.py:99-117``): log into ``host`` AS
    ``username`` with TensorHive's key and run ``true``."""
    t = SSHTransport(host, username, int(port), key_path, get_config().ssh.proxy, get_config().ssh.timeout)
    try:
        return t.run("true", timeout=get_config().ssh.timeout + 5).ok
    except Exception:  # noqa: BLE001 -- no sshd / no route: not a proof
        return False


def authorized_keys_lists_key(username: str, key_path: str) -> tuple[bool, str]:
    """Fallback proof on the daemon's own node: ``username``'s ``~/.ssh/authorized_keys`` lists
    TensorHive's public key as a key entry.  Trusted only when sshd itself would trust the file
    (``StrictModes``): ``~/.ssh`` and the file are owned by that user, are not group- or
    world-writable and are not symlinks; the home directory is not group- or world-writable either.
    Returns (proved, reason)."""
    import pwd
    import stat as st

    try:
        pw = pwd.getpwnam(username)
    except KeyError:
        return False, "no such user on this node"
    try:
        key = public_key(key_path).split()
        ktype, kdata = key[0], key[1]
    except (OSError, subprocess.CalledProcessError, IndexError):
        return False, "TensorHive's key is unreadable"
    home = Path(pw.pw_dir)
    sshdir, ak = home / ".ssh", home / ".ssh" / "authorized_keys"
    for p, what in ((home, "home directory"), (sshdir, "~/.ssh"), (ak, "authorized_keys")):
        try:
            # the home directory may be a symlink (/home -> /data/home): judged by what it points to
            info = os.stat(p) if p == home else os.lstat(p)
        except OSError:
            return False, f"{what} is not readable by the daemon"
        if st.S_ISLNK(info.st_mode):
            return False, f"{what} is a symlink"
        if p != home and info.st_uid != pw.pw_uid:
            return False, f"{what} is not owned by {username}"
        if p == home and info.st_uid not in (pw.pw_uid, 0):
            return False, f"{what} is not owned by {username}"
        if info.st_mode & 0o022:
            return False, f"{what} is group- or world-writable"
    try:
        fd = os.open(ak, os.O_RDONLY | os.O_NOFOLLOW)
        with os.fdopen(fd, "r", errors="replace") as f:
            text = f.read(1 << 20)
    except OSError:
        return False, "authorized_keys is not readable by the daemon"
    for line in text.splitlines():
        parts = line.strip().split()
        if not parts or parts[0].startswith("#"):
            continue
        # options may precede the key type: find "<type> <base64>" as consecutive fields
        for i in range(len(parts) - 1):
            if parts[i] == ktype and parts[i + 1] == kdata:
                return True, "key listed"
    return False, "TensorHive's key is not listed"


def verify_login_as(host: str, username: str, key_path: str) -> bool:
    """Self-signup proof: can TensorHive's key log into ``host`` as ``username``?

    Remote nodes: an SSH login as the user, as in the reference.  The daemon's own node
    (``transport = local``): the same SSH login to the node first; only when that cannot be made
    (no sshd on the node) the user's ``authorized_keys``, read with sshd's own ownership and mode
    rules (:func:`authorized_keys_lists_key`) -- a non-root daemon that cannot read it gets no proof."""
    spec = get_config().ssh.available_nodes.get(host, {})
    port = int(spec.get("port", 22))
    if spec.get("transport") == "local":
        if _ssh_login_ok(spec.get("address") or "localhost", username, port, key_path):
            return True
        ok, why = authorized_keys_lists_key(username, key_path)
        if not ok:
            log.info("sign-up proof for %s on %s failed: %s", username, host, why)
        return ok
    return _ssh_login_ok(host, username, port, key_path)


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
