"""Telemetry beyond the daemon's own process on a real MI355X (round-3 verdict items 2 and 4).

* The node agent reached through a transport (``bash -c`` here, ``ssh node`` in production)
  delivers the same per-GPU fields as the local AmdSmiBackend: probe metrics, HBM source label.
* A GPU shared by a counted th-run task and a foreign process reports ``hbm_bw_source =
  partial`` with a total that covers both streams.
* A ``tensorhive profile --pmc`` task spawned through th-run (with ``task_hbm_counters`` on)
  still produces its counter CSV: the counter tool is left out of profiler commands.
"""
import getpass
import json
import os
import subprocess
import sys
import time
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[2]


def _first_gpu(entry):
    return sorted(entry["GPU"].values(), key=lambda g: g["index"])[0]


def test_remote_agent_over_a_transport_matches_the_local_backend():
    from tensorhive_fixed_amd.core.telemetry import AmdSmiBackend, RemoteBackend
    from tensorhive_fixed_amd.core.transport import LocalTransport, TransportManager

    tm = TransportManager({"thisbox": LocalTransport("thisbox")})
    agent = f"env PYTHONPATH={ROOT} {sys.executable} -m tensorhive_fixed_amd.agent"
    be = RemoteBackend(tm, stream_ms=250, mode="agent", agent_cmd=agent,
                       agent_args="--probe --probe-period 0.25 --task-hbm")
    remote = None
    try:
        t0 = time.time()
        while time.time() - t0 < 90:
            e = be.sample("thisbox")
            if e and all((g["metrics"].get("mfma_contention") or {}).get("value") is not None
                         for g in e["GPU"].values()):
                remote = e
                break
            time.sleep(0.25)
        assert remote is not None, be.errors
        assert be.node_mode("thisbox") == "agent"
        agent_pid = be._procs["thisbox"].pid
    finally:
        be.close()
    local_be = AmdSmiBackend(probe=True, probe_period=0.25, task_hbm=True)
    try:
        assert local_be.probe.wait_first(60), local_be.probe.error
        time.sleep(0.6)
        local = local_be.sample("localhost")
    finally:
        local_be.close()
    assert set(remote["GPU"]) == set(local["GPU"])  # same UUIDs
    for uuid, g in local["GPU"].items():
        r = remote["GPU"][uuid]
        assert r["index"] == g["index"] and r["bdf"] == g["bdf"]
        missing = set(g["metrics"]) - set(r["metrics"])
        assert not missing, (uuid, missing)
        assert r["metrics"]["hbm_bw_source"]["value"] in ("umc_activity", "counters", "partial")
        # neither the agent nor its probe is a tenant of the GPUs it watches
        assert all(p["pid"] != agent_pid for p in r["processes"])
    print("remote fields:", sorted(_first_gpu(remote)["metrics"]))


def _stream(env, secs, kind="add"):
    return subprocess.Popen([sys.executable, str(ROOT / "scripts" / "hbm_stream.py"), str(secs), kind],
                            stdout=subprocess.PIPE, text=True, cwd=ROOT, env={**os.environ, **env})


def test_counted_task_beside_a_foreign_stream_is_partial():
    from tensorhive_fixed_amd.core import hbm
    from tensorhive_fixed_amd.core.telemetry import AmdSmiBackend
    from tensorhive_fixed_amd.native.build import _build_one

    _build_one("libthhbm", False)
    tool = hbm.tool_path()
    assert tool
    be = AmdSmiBackend(task_hbm=True)
    secs = 8
    start = {"HBM_STREAM_START_AT": f"{time.time() + 25:.3f}"}  # both streams over the same window
    counted = _stream({**hbm.task_env(), "TH_HBM_PERIOD_MS": "500", "TENSORHIVE_TASK_ID": "77", **start},
                      secs)
    foreign = _stream(start, secs)
    try:
        assert json.loads(counted.stdout.readline()) == {"ready": True}
        assert json.loads(foreign.stdout.readline()) == {"ready": True}
        t0 = float(start["HBM_STREAM_START_AT"])
        time.sleep(max(0.0, t0 + 2.0 - time.time()))  # > a tool period and an amdsmi rate window in
        vals, counted_part, sources = [], [], set()
        t_end = t0 + secs - 1.5
        while time.time() < t_end:
            m = _first_gpu(be.sample("localhost"))["metrics"]
            sources.add(m["hbm_bw_source"]["value"])
            if m["hbm_bw_source"]["value"] == "partial":
                vals.append(m["hbm_bw"]["value"])
                counted_part.append(m["hbm_counted"]["value"])
            time.sleep(0.25)
        a = json.loads(counted.communicate(timeout=120)[0].strip().splitlines()[-1])
        b = json.loads(foreign.communicate(timeout=120)[0].strip().splitlines()[-1])
    finally:
        for p in (counted, foreign):
            if p.poll() is None:
                p.kill()
        be.close()
    assert vals, f"never partial: {sources}"
    total = a["GBps"] + b["GBps"]
    got = sorted(vals)[len(vals) // 2]
    part = sorted(counted_part)[len(counted_part) // 2]
    print(f"partial hbm_bw {got:.0f} GB/s (counted part {part:.0f}) vs streams {a['GBps']:.0f} + {b['GBps']:.0f}")
    assert abs(got - total) <= 0.2 * total, (vals, a, b)
    assert part < got  # the foreign stream is not hidden behind the counted bytes
    assert "counters" not in sources  # never labelled fully counted while a tenant is uncounted


def test_profile_pmc_task_through_th_run_writes_its_csv(tmp_path, monkeypatch):
    import shutil

    if shutil.which("rocprofv3") is None:
        pytest.skip("rocprofv3 not available")
    from tensorhive_fixed_amd import config as C
    from tensorhive_fixed_amd.core import hbm, task_nursery
    from tensorhive_fixed_amd.native.build import _build_one

    _build_one("libthhbm", False)
    assert hbm.tool_path()
    monkeypatch.setenv("TENSORHIVE_CONFIG_DIR", str(tmp_path))
    monkeypatch.setenv("TH_RUN_STATE_DIR", str(tmp_path / "th-run"))
    C.init_config_files(tmp_path)
    (tmp_path / "hosts_config.ini").write_text(f"[localhost]\nuser = {getpass.getuser()}\ntransport = local\n")
    main = (tmp_path / "main_config.ini").read_text().replace("~/TensorHiveLogs", str(tmp_path / "logs"))
    (tmp_path / "main_config.ini").write_text(main)
    cfg = C.load_config(tmp_path)
    assert cfg.amd_monitor.task_hbm_counters
    C.set_config(cfg)
    task_nursery.use_transports(None)
    try:
        out = tmp_path / "pmc"
        cmd = (f"cd /tmp && TMPDIR=/tmp {shutil.which('rocprofv3')} --pmc SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d {out} -o run "
               f"-- {sys.executable} {ROOT}/scripts/mfma_load.py gemm 1")
        assert task_nursery.spawn_env("localhost", cmd) == {}  # no in-task counter session beside rocprofv3
        user = getpass.getuser()
        pid = task_nursery.spawn(cmd, "localhost", user, name_appendix="4711")
        t0 = time.time()
        while time.time() - t0 < 180 and pid in task_nursery.running_pids("localhost", user):
            time.sleep(1.0)
        log_text = Path(task_nursery.log_path(4711)).read_text()
        csvs = list(out.rglob("*counter_collection.csv"))
        assert csvs, log_text[-3000:]
        assert any("SQ_WAVES" in f.read_text() for f in csvs)
        assert '"kind": "gemm"' in log_text
    finally:
        C.set_config(None)
