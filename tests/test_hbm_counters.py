"""In-task HBM counters (core/hbm.py): per-GPU rates from the tool's per-process files, stale and
dead-process files ignored (dead ones removed), and th-run tasks on the local node carry the tool."""
import json
import os
import time

import pytest

from tensorhive_fixed_amd.core import hbm


def _doc(tmp_path, pid, bdf, rd, wr, window_ms=500.0, age_s=0.0, name=None):
    f = tmp_path / (name or f"th-hbm-{pid}.json")
    f.write_text(json.dumps({"pid": pid, "ts_ns": int((time.time() - age_s) * 1e9), "window_ms": window_ms,
                             "gpus": [{"bdf": bdf, "rd_bytes": rd, "wr_bytes": wr, "counters": {}}]}))
    return f


def test_rates_sum_processes_per_gpu_and_drop_stale_or_dead(tmp_path):
    me = os.getpid()
    _doc(tmp_path, me, "0000:05:00.0", 1.0e12, 0.5e12, name="th-hbm-a.json")         # 2.0 / 1.0 TB/s
    _doc(tmp_path, os.getppid(), "0000:05:00.0", 0.5e12, 0.0, name="th-hbm-b.json")  # + 1.0 TB/s read
    _doc(tmp_path, me, "0000:15:00.0", 1e9, 1e9, age_s=60, name="th-hbm-c.json")     # stale: ignored
    dead = _doc(tmp_path, 2 ** 22 + 12345, "0000:25:00.0", 1e12, 1e12, name="th-hbm-d.json")
    r = hbm.read_rates(str(tmp_path / "th-hbm-*.json"))
    assert set(r) == {"0000:05:00.0"}
    assert abs(r["0000:05:00.0"]["hbm_read"] - 3000.0) < 1e-6 and abs(r["0000:05:00.0"]["hbm_write"] - 1000.0) < 1e-6
    assert not dead.exists()  # a dead process's file is cleaned up
    m = hbm.metrics_for([{"index": 0, "bdf": "0000:05:00.0"}, {"index": 1, "bdf": "0000:15:00.0"}], r)
    assert m[0]["hbm_bw"]["value"] == 4000.0 and m[0]["hbm_bw_source"]["value"] == "counters" and 1 not in m


def test_local_tasks_get_the_counter_tool(cfg, monkeypatch):
    from tensorhive_fixed_amd.core import task_nursery

    monkeypatch.setattr(hbm, "tool_path", lambda: "/opt/th/libthhbm.so")
    cfg.ssh.available_nodes["localnode"] = {"transport": "local"}
    assert task_nursery.spawn_env("localnode") == {"ROCP_TOOL_LIBRARIES": "/opt/th/libthhbm.so"}
    assert task_nursery.spawn_env("node-a") == {}  # remote / simulated nodes: no local monitor reads the files
    cfg.amd_monitor.task_hbm_counters = False
    assert task_nursery.spawn_env("localnode") == {}
    cmd = task_nursery.build_spawn_command("python t.py", 7, "th-run", {"ROCP_TOOL_LIBRARIES": "/x.so"})
    assert "--env ROCP_TOOL_LIBRARIES=/x.so" in cmd and "--env TENSORHIVE_TASK_ID=7" in cmd


def test_task_tool_does_not_link_the_profiler_sdk():
    """libthhbm must not carry a DT_NEEDED entry on librocprofiler-sdk: a tool that links it makes
    rocprofiler-sdk ELF-parse every library loaded in the task at HIP initialisation (+3.3 s per task
    under torch, profiles/r05_daemon/README.md); the tool resolves the SDK's entry points with dlsym."""
    import shutil
    import subprocess

    from tensorhive_fixed_amd.native.build import _build_one, path_of

    if shutil.which("readelf") is None:
        pytest.skip("readelf not available")
    name, err = _build_one("libthhbm", False)
    if err:
        pytest.skip(f"libthhbm not buildable here: {err[:200]}")
    out = subprocess.run(["readelf", "-d", str(path_of("libthhbm"))], capture_output=True, text=True, check=True).stdout
    needed = [ln for ln in out.splitlines() if "(NEEDED)" in ln]
    assert needed, out
    assert not any("rocprofiler" in ln for ln in needed), needed
