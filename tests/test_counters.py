"""Device-wide counter plumbing: derived metrics and the streaming reader, with a
stand-in for the native ``th-counters`` binary (the real one is exercised in tests/gpu)."""
import json
import os
import stat

from tensorhive_fixed_amd.core.counters import CounterStream, derive


def test_derive_units():
    g = {"counters": {"GRBM_GUI_ACTIVE": 750, "GRBM_COUNT": 1000, "SQ_INSTS_VALU_MFMA_MOPS_BF16": 1e9,
                      "TCC_EA0_RDREQ_sum": 1e9, "TCC_EA0_RDREQ_32B_sum": 0, "TCC_EA0_WRREQ_sum": 5e8,
                      "TCC_EA0_WRREQ_64B_sum": 5e8}}
    m = derive(g, 100.0)
    assert m["gpu_busy"] == {"value": 75.0, "unit": "%"}
    assert m["mfma_tflops"]["value"] == round(1e9 * 512 / 0.1 / 1e12, 1)
    assert m["hbm_read"]["value"] == round(64e9 / 0.1 / 1e9, 1)
    assert m["hbm_write"]["value"] == round(32e9 / 0.1 / 1e9, 1)
    assert derive({"counters": {}}, 100.0) == {}


def test_derive_mfma_busy_from_sq_cycles():
    # 100 k elapsed cycles per XCD (GRBM sums the 8 XCDs), every one of 1024 SIMDs busy 52 % of them
    g = {"counters": {"GRBM_GUI_ACTIVE": 8e5, "GRBM_COUNT": 8e5, "SQ_VALU_MFMA_BUSY_CYCLES": 0.52 * 1e5 * 1024}}
    assert derive(g, 50.0)["mfma_busy"] == {"value": 52.0, "unit": "%"}
    g["counters"]["SQ_VALU_MFMA_BUSY_CYCLES"] = 3e9  # clamped: never above 100 %
    assert derive(g, 50.0)["mfma_busy"]["value"] == 100.0
    assert "mfma_busy" not in derive({"counters": {"GRBM_COUNT": 10, "GRBM_GUI_ACTIVE": 5}}, 50.0)


def test_counter_stream_reads_lines(tmp_path):
    line = json.dumps({"ts_ns": 1, "window_ms": 100, "gpus": [
        {"kfd_id": 1234, "bdf": "0000:05:00.0", "counters": {"GRBM_GUI_ACTIVE": 5, "GRBM_COUNT": 10}}]})
    fake = tmp_path / "th-counters"
    fake.write_text(f"#!/bin/sh\necho '{line}'\nsleep 5\n")
    fake.chmod(fake.stat().st_mode | stat.S_IEXEC)
    cs = CounterStream(binary=str(fake))
    try:
        assert cs.wait_first(5)
        assert cs.latest() == {1234: {"gpu_busy": {"value": 50.0, "unit": "%"}}}
    finally:
        cs.close()


def test_counter_stream_reports_errors(tmp_path):
    fake = tmp_path / "th-counters"
    fake.write_text('#!/bin/sh\necho \'{"error": "no GPU agent"}\'\n')
    fake.chmod(fake.stat().st_mode | stat.S_IEXEC)
    cs = CounterStream(binary=str(fake))
    try:
        assert cs.wait_first(5) is False and cs.error == "no GPU agent"
    finally:
        cs.close()


def test_counter_stream_exposes_its_pid_for_the_ignore_list(tmp_path):
    fake = tmp_path / "th-counters"
    fake.write_text("#!/bin/sh\nexec sleep 5\n")
    fake.chmod(fake.stat().st_mode | stat.S_IEXEC)
    cs = CounterStream(binary=str(fake))
    try:
        for _ in range(100):
            if cs.pid:
                break
            import time
            time.sleep(0.05)
        assert cs.pid and os.path.exists(f"/proc/{cs.pid}")
    finally:
        cs.close()
