"""BASELINE config 4 on the real node (real time): three users' GPU jobs go through the queue, the
daemon's telemetry and gang placement start them as real processes, and a foreign process on a
reserved GPU is detected afterwards (benchmarks.multitenant_node)."""
import getpass

import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.skipif(getpass.getuser() == "root", reason="th-run jobs run as an ordinary user")
def test_real_node_queue_runs_every_job_and_flags_the_intruder():
    from tensorhive_fixed_amd import benchmarks

    r = benchmarks.multitenant_node(jobs_per_user=1, duration_s=(2.0, 3.0), arrival_s=0.5, timeout_s=100.0)
    assert r["jobs"] == 3 and r["launched"] == 3, r
    assert set(r["job_status"]) <= {"terminated", "not_running"}, r
    assert r["telemetry_samples"] > 10 and r["node_gpu_util"] > 0, r
    assert r["violation"] and r["violation"]["reserved_by"] == ["bob"], r
    assert r["violation"]["intruder"] == getpass.getuser(), r
    # the scheduler ticks every 30 s: queued jobs were started by the "device freed" wake-up
    if r["gpus_on_node"] == 1:  # three jobs on one device: two of them waited for it
        assert r["handoff_p50_ms"] is not None, r
    assert r["handoff_p50_ms"] is None or r["handoff_p50_ms"] < 3000, r
