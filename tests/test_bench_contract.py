"""bench.py contract (driver): ``torchrun --nproc-per-node N bench.py --gpus N --steps K --warmup W``
prints ONE JSON line from rank 0 with the whole-job value.  Rehearsed here with 2 gloo ranks on the
CPU and the tiny model (the 8-GPU RCCL run is the driver's)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 8])
def test_multi_rank_bench_prints_one_json_line(tmp_path, world):
    """world 8 rehearses the driver's 8-GPU launch (ZeRO-1 over 8 ranks, small buckets) on gloo."""
    env = {**os.environ, "TH_DIST_BACKEND": "gloo", "OMP_NUM_THREADS": "1" if world > 2 else "2"}
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
                        "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
                        "--gpus", str(world), "--steps", "2", "--warmup", "1", "--model", "tiny", "--seq-len", "64",
                        "--micro-batch", "2", "--bucket-mb", "0.25"], capture_output=True, text=True, env=env,
                       timeout=300, cwd=tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert KEYS <= set(d)
    assert d["n_gpus"] == world and d["steps"] == 2 and d["warmup"] == 1 and d["scaling"] == "weak"
    assert d["config"]["parallelism"] == f"dp{world}" and d["config"]["global_batch"] == 2 * world
    assert d["config"]["zero"] == 1  # sharded optimizer is the multi-rank default
    # whole-job aggregate: tokens of both ranks over the (max-over-ranks) step time
    assert abs(d["value"] - world * 2 * 64 / (d["ms_per_step"] / 1e3)) / d["value"] < 0.01
    # self-verification (round-2 verdict item 2): the process group the ranks really formed
    census = d["dist"]
    assert census["world_size"] == world and census["backend"] == "gloo"
    assert [r["rank"] for r in census["ranks"]] == list(range(world))
    assert sorted(r["local_rank"] for r in census["ranks"]) == list(range(world))
    assert all(r["cpus"] for r in census["ranks"]) and "bound" in census["ranks"][0]
    assert census["comm_env"].get("TORCH_NCCL_ASYNC_ERROR_HANDLING") == "1"
    assert census["distinct_devices"] == 0  # CPU ranks have no GPU; on MI355X it must equal world_size
    # self-diagnosis of the first multi-GPU run (round-3 verdict item 7): per-rank stalls on
    # communication, max over ranks per step, and every rank's row
    for k in ("exposed_comm_ms_per_step", "allgather_wait_ms", "opt_wait_ms"):
        assert isinstance(d[k], (int, float)) and 0.0 <= d[k] <= d["ms_per_step"], (k, d[k])
    comm = census["comm"]
    assert [r["rank"] for r in comm["per_rank"]] == list(range(world))
    for row in comm["per_rank"]:
        assert row["grad_sync_ms_per_step"] > 0.0  # gloo: the bucket waits block the host
        assert {"allgather_ms_per_step", "opt_wait_ms_per_step", "step_ms"} <= set(row)
    assert d["exposed_comm_ms_per_step"] >= max(r["grad_sync_ms_per_step"] for r in comm["per_rank"]) - 1e-6
    assert comm["rccl"] is None  # gloo: no RCCL communicator


def test_bench_refuses_a_hipblaslt_workspace_that_faults(tmp_path):
    env = {**os.environ, "HIPBLASLT_WORKSPACE_SIZE": "8192"}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "0", "--model",
                        "tiny"], capture_output=True, text=True, env=env, timeout=120, cwd=tmp_path)
    assert r.returncode == 2 and "HIPBLASLT_WORKSPACE_SIZE=8192" in r.stderr and not r.stdout.strip()
    r = subprocess.run([sys.executable, "-m", "tensorhive_fixed_amd.workloads.llama3_ddp", "--steps", "1"],
                       capture_output=True, text=True, env={**env, "PYTHONPATH": ROOT}, timeout=120, cwd=tmp_path)
    assert r.returncode == 2 and "refusing to start" in r.stderr


def test_blas_workspace_rules():
    from tensorhive_fixed_amd.utils.blas_env import UnsafeBlasWorkspace, check_blas_workspace

    check_blas_workspace({})
    check_blas_workspace({"HIPBLASLT_WORKSPACE_SIZE": str(128 * 1024)})
    for bad in ("8192", "0", "lots"):
        with pytest.raises(UnsafeBlasWorkspace):
            check_blas_workspace({"HIPBLASLT_WORKSPACE_SIZE": bad})


def test_parse_rccl_init_log():
    from tensorhive_fixed_amd.parallel.comm_diag import parse_rccl_init

    log = """host:1:1 [0] NCCL INFO RCCL version 2.22.3+hip7.0 HEAD:abc
host:1:1 [0] NCCL INFO comm 0x55 rank 0 nRanks 8 nNodes 1 localRanks 8 localRank 0 MNNVL 0
host:1:1 [0] NCCL INFO Channel 00/32 :    0   1   2   3   4   5   6   7
host:1:1 [0] NCCL INFO Channel 31/32 :    0   7   6   5   4   3   2   1
host:1:1 [0] NCCL INFO Trees [0] 1/-1/-1->0->-1 [1] 1/-1/-1->0->-1
host:1:1 [0] NCCL INFO P2P Chunksize set to 524288
host:1:1 [0] NCCL INFO Channel 00/0 : 0[0] -> 1[1] via P2P/IPC
host:1:1 [0] NCCL INFO Channel 01/0 : 0[0] -> 1[1] via P2P/IPC
host:1:1 [0] NCCL INFO threadThresholds 8/8/64 | 64/8/64 | 512 | 512
host:1:1 [0] NCCL INFO 32 coll channels, 32 collnet channels, 0 nvls channels, 32 p2p channels, 32 p2p channels per peer
host:1:1 [0] NCCL WARN something odd
[2026-10-17 12:58:03] host:1:2 [0] /src/init.cc:161 NCCL WARN something odd
"""
    d = parse_rccl_init(log)
    assert d["library"] == "RCCL" and d["version"] == "2.22.3+hip7.0" and d["nranks"] == 8
    assert d["channels"] == 32 and d["coll_channels"] == 32 and d["p2p_channels"] == 32 and d["trees"] == 1
    assert d["transports"] == {"P2P/IPC": 2} and d["p2p_chunksize"] == 524288
    assert d["thread_thresholds"].startswith("8/8/64") and d["warnings"] == ["something odd"]  # deduplicated


def test_prepare_rccl_log_respects_user_settings(monkeypatch, tmp_path):
    from tensorhive_fixed_amd.parallel import comm_diag

    monkeypatch.setenv("TMPDIR", str(tmp_path))
    for k in ("NCCL_DEBUG", "NCCL_DEBUG_SUBSYS", "NCCL_DEBUG_FILE", "TH_RCCL_INIT_LOG"):
        monkeypatch.delenv(k, raising=False)
    import tempfile
    monkeypatch.setattr(tempfile, "tempdir", str(tmp_path))
    assert comm_diag.prepare_rccl_log(3) is None  # a training job: RCCL logs stay on stderr
    assert "NCCL_DEBUG_FILE" not in os.environ
    monkeypatch.setenv("TH_RCCL_INIT_LOG", "1")  # bench.py opts in
    p = comm_diag.prepare_rccl_log(3)
    assert p and p.endswith("-r3.log") and os.environ["NCCL_DEBUG"] == "INFO" and os.environ["NCCL_DEBUG_SUBSYS"] == "INIT"
    monkeypatch.delenv("NCCL_DEBUG_FILE")
    monkeypatch.setenv("NCCL_DEBUG", "TRACE")
    assert comm_diag.prepare_rccl_log(0) is None  # the user's own debugging wins
    monkeypatch.setenv("NCCL_DEBUG", "WARN")
    monkeypatch.setenv("NCCL_DEBUG_FILE", "/x/y")
    assert comm_diag.prepare_rccl_log(0) is None

