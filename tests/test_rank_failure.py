"""Failure behaviour of the multi-rank payload (round-5 verdict weak #3): one of 4 ranks dies in the middle
of a training step -- after its forward and backward, before its gradient collectives complete -- and the
torchrun job must end non-zero within a bounded time instead of leaving the other ranks blocked in a
collective.  gloo on the CPU; the RCCL run has the same shape (torchrun tears the group down when a worker
exits, and TORCH_NCCL_ASYNC_ERROR_HANDLING=1 / the process-group timeout bound a peer lost on another node)."""
import os
import socket
import subprocess
import sys
import textwrap
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = textwrap.dedent("""
    import os, sys
    sys.path.insert(0, {root!r})
    import torch
    from tensorhive_fixed_amd.models.llama3 import LlamaConfig
    from tensorhive_fixed_amd.parallel.dist import init_distributed
    from tensorhive_fixed_amd.workloads.llama3_ddp import Trainer

    torch.set_num_threads(1)
    info = init_distributed("cpu")
    tr = Trainer(LlamaConfig.tiny(), info, micro_batch=2, seq_len=32, bucket_mb=0.05)
    if info.rank == 2:
        real = tr.store.finish_grad_sync
        def dying():
            if tr.opt.step_count == 2:
                print("rank 2: dying inside step 3", flush=True)
                os._exit(7)
            real()
        tr.store.finish_grad_sync = dying
    for _ in range(10000):
        tr.step()
""")


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_a_rank_dying_mid_step_ends_the_job_nonzero(tmp_path):
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(root=ROOT))
    env = {**os.environ, "OMP_NUM_THREADS": "1", "TH_DIST_TIMEOUT_S": "60"}
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
                        "--master-addr", "127.0.0.1", "--master-port", str(_port()), "--max-restarts", "0",
                        str(script)], capture_output=True, text=True, env=env, timeout=240, cwd=tmp_path)
    dt = time.monotonic() - t0
    assert "rank 2: dying inside step 3" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
    assert r.returncode != 0
    assert "exitcode" in r.stderr and "7" in r.stderr, r.stderr[-3000:]
    assert dt < 150, f"the job took {dt:.0f} s to end after a rank died"


def test_process_group_timeout_from_env(monkeypatch):
    from tensorhive_fixed_amd.parallel.dist import pg_timeout

    monkeypatch.delenv("TH_DIST_TIMEOUT_S", raising=False)
    assert pg_timeout().total_seconds() == 900
    monkeypatch.setenv("TH_DIST_TIMEOUT_S", "45")
    assert pg_timeout().total_seconds() == 45
