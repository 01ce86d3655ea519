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
