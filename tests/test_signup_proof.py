"""Self-sign-up proof on the daemon's own node (round-5 verdict weak #6; reference
``tensorhive/controllers/user.py:99-117`` proves identity by logging in AS the user).

``verify_login_as`` on a ``transport = local`` node tries that SSH login first and falls back to the user's
``authorized_keys`` only under sshd's own StrictModes rules.  The refusal cases are checked here with a fake
passwd entry whose home is a temp directory."""
import os
import pwd
from types import SimpleNamespace

import pytest

from tensorhive_fixed_amd.core import ssh


@pytest.fixture()
def home(tmp_path, monkeypatch):
    key = ssh.generate_key(tmp_path / "th_key")
    h = tmp_path / "home" / "alice"
    (h / ".ssh").mkdir(parents=True)
    os.chmod(h, 0o755)
    os.chmod(h / ".ssh", 0o700)
    ak = h / ".ssh" / "authorized_keys"
    pub = ssh.public_key(key)
    ak.write_text("ssh-ed25519 AAAAother other@x\n" + f'from="10.0.0.0/8" {pub}\n')
    os.chmod(ak, 0o600)
    entry = SimpleNamespace(pw_name="alice", pw_dir=str(h), pw_uid=os.getuid(), pw_gid=os.getgid())
    real = pwd.getpwnam
    monkeypatch.setattr(pwd, "getpwnam", lambda n: entry if n == "alice" else real(n))
    return SimpleNamespace(key=str(key), home=h, ak=ak, entry=entry, pub=pub)


def test_listed_key_with_options_is_a_proof(home):
    assert ssh.authorized_keys_lists_key("alice", home.key) == (True, "key listed")


def test_unknown_user(home):
    assert not ssh.authorized_keys_lists_key("no-such-user-xyz", home.key)[0]


def test_key_only_in_a_comment_or_substring_is_not_a_proof(home):
    kdata = home.pub.split()[1]
    home.ak.write_text(f"# {home.pub}\nssh-ed25519 AAAAother {kdata}\nssh-ed25519 {kdata}XYZ x\n")
    ok, why = ssh.authorized_keys_lists_key("alice", home.key)
    assert not ok and "not listed" in why


def test_file_owned_by_someone_else_is_refused(home):
    home.entry.pw_uid = os.getuid() + 4242  # the files are ours, not alice's
    ok, why = ssh.authorized_keys_lists_key("alice", home.key)
    assert not ok and "not owned" in why


@pytest.mark.parametrize("what,mode", [("ak", 0o620), ("ak", 0o602), ("ssh", 0o770), ("home", 0o777)])
def test_group_or_world_writable_paths_are_refused(home, what, mode):
    p = {"ak": home.ak, "ssh": home.home / ".ssh", "home": home.home}[what]
    os.chmod(p, mode)
    ok, why = ssh.authorized_keys_lists_key("alice", home.key)
    assert not ok and "writable" in why


def test_symlinked_authorized_keys_is_refused(home, tmp_path):
    target = tmp_path / "elsewhere"
    target.write_text(home.ak.read_text())
    home.ak.unlink()
    home.ak.symlink_to(target)
    ok, why = ssh.authorized_keys_lists_key("alice", home.key)
    assert not ok and "symlink" in why


def test_unreadable_file_is_no_proof(home, monkeypatch):
    real_open = os.open

    def deny(path, *a, **k):
        if str(path) == str(home.ak):
            raise PermissionError("denied")
        return real_open(path, *a, **k)

    monkeypatch.setattr(os, "open", deny)
    ok, why = ssh.authorized_keys_lists_key("alice", home.key)
    assert not ok and "not readable" in why


def test_local_node_tries_the_ssh_login_first(home, monkeypatch):
    cfg = SimpleNamespace(ssh=SimpleNamespace(available_nodes={"me": {"transport": "local", "port": 2222}},
                                              proxy=None, timeout=1.0))
    monkeypatch.setattr(ssh, "get_config", lambda: cfg)
    calls = []
    monkeypatch.setattr(ssh, "_ssh_login_ok", lambda h, u, port, k: calls.append((h, u, port)) or True)
    home.ak.write_text("")  # the fallback would refuse: the login alone proves it
    assert ssh.verify_login_as("me", "alice", home.key)
    assert calls == [("localhost", "alice", 2222)]
    # no sshd on the node: the StrictModes-checked authorized_keys decides
    monkeypatch.setattr(ssh, "_ssh_login_ok", lambda *a: False)
    assert not ssh.verify_login_as("me", "alice", home.key)
    home.ak.write_text(home.pub + "\n")
    assert ssh.verify_login_as("me", "alice", home.key)


def test_remote_node_uses_only_the_login(home, monkeypatch):
    cfg = SimpleNamespace(ssh=SimpleNamespace(available_nodes={"n1": {"port": 22}}, proxy=None, timeout=1.0))
    monkeypatch.setattr(ssh, "get_config", lambda: cfg)
    monkeypatch.setattr(ssh, "_ssh_login_ok", lambda *a: False)
    assert not ssh.verify_login_as("n1", "alice", home.key)  # a readable authorized_keys is not enough


def test_symlinked_home_directory_is_followed(home, tmp_path):
    link = tmp_path / "home-link"
    link.symlink_to(home.home)
    home.entry.pw_dir = str(link)
    assert ssh.authorized_keys_lists_key("alice", home.key)[0]
