"""Sanitizer runs of the native host tools (SURVEY §5 race / memory-error detection):
AddressSanitizer + UBSan and ThreadSanitizer builds of the th-run supervisor's whole spawn / ls /
status / wait / signal cycle (including its forked monitor process), of th-smi's start-up path,
and of libthsmi driven from four threads at once (``native/thsmi_stress.cpp``), with every
sanitizer report written to a file and asserted absent.  The GPU-side TSan runs (full amdsmi
sample, the th-counters reader) are in tests/gpu/test_native_gpu.py."""
import os
import shutil
import subprocess
import time

import pytest

from tensorhive_fixed_amd.native.build import _build_one, path_of, sanitizer_env, tsan_argv, tsan_env

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++ with libasan")


def _build(name):
    _, err = _build_one(name, False)
    if err and ("libasan" in err or "libtsan" in err):
        pytest.skip("sanitizer runtime not available")
    assert err is None, err
    return str(path_of(name))


def _reports(d):
    return {p: open(os.path.join(d, p)).read()[-2000:] for p in os.listdir(d)}


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_th_run_under_sanitizers(tmp_path, kind):
    th = _build(f"th-run-{kind}")
    rep = tmp_path / "reports"
    rep.mkdir()
    san = sanitizer_env(str(rep)) if kind == "asan" else tsan_env(str(rep))
    env = {**os.environ, "TH_RUN_STATE_DIR": str(tmp_path / "state"), **san}

    def run(*a, timeout=30):
        argv = tsan_argv(th, *a) if kind == "tsan" else [th, *a]
        return subprocess.run(argv, capture_output=True, text=True, env=env, timeout=timeout)

    # the task-exit datagram path (--notify) runs under the sanitizer too
    import socket

    ev_path = str(tmp_path / "ev.sock")
    ev = socket.socket(socket.AF_UNIX, socket.SOCK_DGRAM)
    ev.bind(ev_path)
    ev.settimeout(20)
    r = run("spawn", "--name", "tensorhive_task_a", "--log", str(tmp_path / "a.log"), "--env", "X=1",
            "--notify", ev_path, "--", "bash", "-c", "echo $X; exit 3")
    assert r.returncode == 0, r.stderr
    assert run("wait", "--name", "tensorhive_task_a", "--timeout", "20").returncode == 3
    import json as _json

    msg = _json.loads(ev.recv(4096))
    ev.close()
    assert msg["event"] == "task_exit" and msg["name"] == "tensorhive_task_a" and msg["exit_code"] == 3
    r = run("spawn", "--name", "tensorhive_task_b", "--log", str(tmp_path / "b.log"), "--", "sleep", "60")
    pid = int(r.stdout.strip())
    ls = run("ls")
    assert "tensorhive_task_b" in ls.stdout
    assert '"running"' in run("status", "--name", "tensorhive_task_b").stdout.replace(" ", "")
    assert run("terminate", "--name", "tensorhive_task_b").returncode == 0
    assert run("wait", "--name", "tensorhive_task_b", "--timeout", "20").returncode != 0
    assert run("kill", "--name", "tensorhive_task_nope").returncode != 0
    assert run("bogus-subcommand").returncode != 0
    # monitors write their reports when they exit
    t0 = time.time()
    while time.time() - t0 < 10 and os.path.exists(f"/proc/{pid}"):
        time.sleep(0.1)
    time.sleep(0.5)
    assert (tmp_path / "a.log").read_text().strip() == "1"
    assert _reports(rep) == {}


def test_th_smi_startup_under_asan(tmp_path):
    smi = _build("th-smi-asan")
    rep = tmp_path / "reports"
    rep.mkdir()
    r = subprocess.run([smi], capture_output=True, text=True, timeout=60,
                       env={**os.environ, **sanitizer_env(str(rep))})
    # no GPU here: amdsmi init fails cleanly; on a GPU node it prints one JSON sample
    assert r.returncode in (0, 1) and (r.returncode == 1 or r.stdout.startswith("{"))
    assert _reports(rep) == {}


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_libthsmi_from_four_threads(tmp_path, kind):
    """Two threads sampling the host half (CPU + KFD/DRM process scan), one the full sample and
    topology (when amdsmi is up), one rewriting the ignore list -- no race, no memory error."""
    exe = _build(f"thsmi-stress-{kind}")
    rep = tmp_path / "reports"
    rep.mkdir()
    san = sanitizer_env(str(rep)) if kind == "asan" else tsan_env(str(rep))
    argv = tsan_argv(exe, "--iters", "120") if kind == "tsan" else [exe, "--iters", "120"]
    r = subprocess.run(argv, capture_output=True, text=True, timeout=300, env={**os.environ, **san})
    assert r.returncode == 0, (r.stdout, r.stderr[-2000:], _reports(rep))
    assert '"bad":0' in r.stdout
    assert _reports(rep) == {}
