"""GpuProbe / ProbeBaseline logic on CPU (the th-probe agent replaced by a scripted stand-in that
speaks its line protocol): per-GPU matching by BDF, idle re-baselining, duty cycle, and the
backend's self-pid filter."""
import json
import sys
import textwrap
import time

from tensorhive_fixed_amd.core.telemetry import GpuProbe, ProbeBaseline

FAKE = textwrap.dedent("""
    import json, sys, time
    # per line: {hip: mfma_us}; every GPU gets 8 workgroups on 4 XCDs
    script = json.loads(sys.argv[1])
    for i, step in enumerate(script):
        gpus = [{"hip": int(h), "bdf": "0000:%02x:00.0" % (5 + 16 * int(h)), "latency_us": 40.0,
                 "wg": [[w %% 4, us, 20.0, 50.0] for w in range(8)]} for h, us in step.items()]
        print(json.dumps({"ts_ns": i + 1, "period_ms": 100, "gpus": gpus}), flush=True)
        time.sleep(0.15)
    time.sleep(30)
""")


def _fake(tmp_path, script):
    f = tmp_path / "fake_probe.py"
    f.write_text(FAKE.replace("%%", "%"))
    return [sys.executable, str(f), json.dumps(script)]


def _gpus(util=(0.0, 0.0), procs=([], [])):
    return [{"index": i, "bdf": "0000:%02x:00.0" % (5 + 16 * i), "metrics": {"utilization": {"value": util[i]}},
             "processes": procs[i]} for i in range(2)]


def test_baseline_relearns_while_idle_and_ignores_outliers():
    b = ProbeBaseline(window=4, min_idle=3)
    b.observe(5.0, 30.0, 99.0, is_idle=False)  # one anomalously fast sample under load
    assert not b.learned and b.reference()[0] == 5.0  # provisional: best seen
    for us in (10.0, 10.2, 9.9):
        b.observe(us, 40.0, 50.0, is_idle=True)
    assert b.learned and b.reference() == (10.0, 40.0, 50.0)  # median of idle samples, not the outlier
    for us in (12.0, 12.1, 12.2, 12.0):  # clocks changed: the window re-learns
        b.observe(us, 40.0, 50.0, is_idle=True)
    assert b.reference()[0] == 12.1


def test_probe_stream_derives_per_gpu_metrics(tmp_path):
    idle = [{"0": 10.0, "1": 10.0}] * 4
    loaded = [{"0": 10.0, "1": 25.0}] * 40  # GPU 1's MFMA chain is 2.5x slower
    probe = GpuProbe(period=0.1, cmd=_fake(tmp_path, idle + loaded))
    try:
        assert probe.wait_first(10)
        seen = {}
        t0 = time.time()
        while time.time() - t0 < 10:
            doc = probe.latest()
            m = probe.metrics_for(_gpus(util=(0.0, 0.0) if doc["ts_ns"] <= 4 else (0.0, 95.0),
                                        procs=([], []) if doc["ts_ns"] <= 4 else ([], [{"pid": 7}])))
            seen[doc["ts_ns"]] = m
            if doc["ts_ns"] >= 8:
                break
            time.sleep(0.05)
        last = seen[max(seen)]
        assert set(last) == {0, 1}
        assert last[0]["mfma_contention"]["value"] == 0.0
        assert abs(last[1]["mfma_contention"]["value"] - 60.0) < 0.5  # 1 - 10/25
        assert last[1]["probe_baseline"]["value"] == "idle"
        assert last[0]["probe_xcds"]["value"] == 4
        assert last[0]["probe_duty"]["value"] == round(100 * 30e-6 / 0.1, 4)  # (10+20) us per 100 ms
    finally:
        probe.close()


FLOOD = textwrap.dedent("""
    import json, sys, time
    sys.stderr.write("x" * 1023 + "\\n" * 1)
    for _ in range(400):  # 400 KiB of stderr: a pipe nobody reads would block the agent here
        sys.stderr.write("w" * 1023 + "\\n")
    sys.stderr.flush()
    print(json.dumps({"ts_ns": 1, "period_ms": 100, "gpus": []}), flush=True)
    time.sleep(30)
""")


def test_agent_stderr_is_drained(tmp_path):
    f = tmp_path / "flood.py"
    f.write_text(FLOOD)
    probe = GpuProbe(period=0.1, cmd=[sys.executable, str(f)])
    try:
        assert probe.wait_first(15), "agent blocked on a full stderr pipe"
    finally:
        probe.close()


def test_dead_agent_is_restarted_with_backoff(tmp_path):
    f = tmp_path / "crash.py"
    f.write_text("import sys\nsys.stderr.write('device lost\\n')\nsys.exit(3)\n")
    probe = GpuProbe(period=0.1, cmd=[sys.executable, str(f)])
    try:
        probe._proc.wait(10)
        probe._thread.join(10)
        assert probe.error.startswith("th-probe exited (3)") and "device lost" in probe.error
        first = probe.pid
        assert probe.ensure_running(backoff_s=3600) is False  # within the backoff window
        assert probe.ensure_running(backoff_s=0.0) is True
        assert probe.restarts == 1 and probe.pid != first
    finally:
        probe.close()
    assert probe.ensure_running(backoff_s=0.0) is False  # closed: never restarted
