"""Task lifecycle on the daemon's own node through the native ``th-run`` supervisor (BASELINE
config 0: "job queue runs `sleep 1` via local SSH/screen").  Runs as the current UNIX user, so
the local transport executes commands directly (no user switch)."""
import getpass
import os
import shutil
import signal
import subprocess
import time

import pytest

from tensorhive_fixed_amd.native.build import build_all, path_of

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="needs a C++ compiler for th-run")


@pytest.fixture(scope="module", autouse=True)
def _native():
    build_all(strict=False)
    assert path_of("th-run").exists()


@pytest.fixture()
def local(tmp_path, monkeypatch):
    from tensorhive_fixed_amd import config as C
    from tensorhive_fixed_amd.core import task_nursery
    from tensorhive_fixed_amd.core.transport import LocalTransport, TransportManager

    monkeypatch.setenv("TH_RUN_STATE_DIR", str(tmp_path / "state"))
    C.init_config_files(tmp_path)
    (tmp_path / "hosts_config.ini").write_text(f"[localhost]\nuser = {getpass.getuser()}\ntransport = local\n")
    main = (tmp_path / "main_config.ini").read_text().replace("~/TensorHiveLogs", str(tmp_path / "logs"))
    main = main.replace("~/.config/TensorHive/hosts_config.ini", str(tmp_path / "hosts_config.ini"))
    (tmp_path / "main_config.ini").write_text(main)
    C.set_config(C.load_config(tmp_path))
    tm = TransportManager({"localhost": LocalTransport("localhost")})
    task_nursery.use_transports(tm)
    yield task_nursery
    task_nursery.use_transports(None)
    C.set_config(None)


def _alive(pid):
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    # a zombie awaiting its reaper counts as gone
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().split()[2] != "Z"
    except FileNotFoundError:
        return False


def _wait(cond, timeout=10.0):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if cond():
            return True
        time.sleep(0.05)
    return False


def test_spawn_log_and_exit(local):
    me = getpass.getuser()
    pid = local.spawn("echo hello from $TENSORHIVE_TASK_ID; sleep 1", "localhost", me, name_appendix="11")
    assert pid > 0
    names = [s["name"] for s in local.running("localhost", me)]
    assert "tensorhive_task_11" in names
    assert _wait(lambda: not _alive(pid), 15)
    assert _wait(lambda: "tensorhive_task_11" not in [s["name"] for s in local.running("localhost", me)])
    lines, path = local.fetch_log("localhost", me, 11)
    assert lines[0] == "hello from 11" and path.endswith("task_11.log")
    tail, _ = local.fetch_log("localhost", me, 11, tail=True, tail_lines=1)
    assert len(tail) == 1


def _log_or_empty(local, user, name):
    try:
        return local.fetch_log("localhost", user, name)[0]
    except FileNotFoundError:
        return []


def test_interrupt_foreground_task(local):
    me = getpass.getuser()
    pid = local.spawn("echo started; sleep 300; echo not reached", "localhost", me, name_appendix="int")
    assert _wait(lambda: _alive(pid))
    # interrupt once the command runs: a SIGINT that lands while `bash -l` still sources profile
    # scripts can be swallowed by one of their children, and bash then goes on to `sleep 300`
    assert _wait(lambda: "started" in _log_or_empty(local, me, "int"))
    assert local.terminate(pid, "localhost", me, gracefully=True) == 0
    assert _wait(lambda: not _alive(pid), 15)
    lines, _ = local.fetch_log("localhost", me, "int")
    assert "not reached" not in lines


# bash starts background jobs with SIGINT ignored, so group-wide SIGINT is not tested here
@pytest.mark.parametrize("graceful,code", [(None, 0), (False, 0)])
def test_terminate_whole_process_group(local, graceful, code):
    me = getpass.getuser()
    # a launcher with two children, like torchrun with ranks
    pid = local.spawn("sleep 300 & sleep 300 & wait", "localhost", me, name_appendix=f"g{graceful}")
    assert _wait(lambda: len(subprocess.run(["pgrep", "-g", str(pid)], capture_output=True, text=True)
                             .stdout.split()) >= 3)
    kids = [int(x) for x in subprocess.run(["pgrep", "-g", str(pid)], capture_output=True, text=True).stdout.split()]
    assert local.terminate(pid, "localhost", me, gracefully=graceful) == code
    assert _wait(lambda: not any(_alive(k) for k in kids), 15)


def test_terminate_unknown_pid_fails(local):
    assert local.terminate(999_999, "localhost", getpass.getuser(), gracefully=False) != 0


def test_missing_log_raises(local):
    with pytest.raises(FileNotFoundError):
        local.fetch_log("localhost", getpass.getuser(), 424242)


def test_th_run_status_and_wait(tmp_path, monkeypatch):
    th = str(path_of("th-run"))
    env = {**os.environ, "TH_RUN_STATE_DIR": str(tmp_path)}
    out = subprocess.run([th, "spawn", "--name", "tensorhive_task_w", "--log", str(tmp_path / "w.log"), "--",
                          "bash", "-c", "exit 7"], capture_output=True, text=True, env=env)
    assert out.returncode == 0 and int(out.stdout.strip()) > 0
    w = subprocess.run([th, "wait", "--name", "tensorhive_task_w", "--timeout", "10"], capture_output=True,
                       text=True, env=env)
    assert w.returncode == 7
    st = subprocess.run([th, "status", "--name", "tensorhive_task_w"], capture_output=True, text=True, env=env)
    assert '"exit_code":7' in st.stdout.replace(" ", "")
