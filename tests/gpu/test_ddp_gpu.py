"""Flat-buffer DDP on GPU tensors with several ranks (the box has one GPU: ranks share it over
gloo; RCCL over xGMI is exercised by the driver's multi-GPU bench) and the RCCL code path itself
in a one-rank group that still issues every collective (TH_FORCE_COLLECTIVES=1)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_ranks_stay_identical():
    env = {**os.environ, "TH_DIST_BACKEND": "gloo", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "scripts/ddp_check.py"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    doc = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert doc["world"] == 2 and doc["params_identical"] and doc["n_buckets"] > 1
    # ZeRO-1: replicas identical after the all-gathers, same trajectory as the replicated optimizer
    assert doc["params_identical_zero1"] and doc["zero1_vs_zero0_frac_off"] < 1e-3
    assert doc["opt_state_numel"][1] < doc["opt_state_numel"][0]


def test_rccl_collectives_path_one_rank():
    """backend nccl (= RCCL): bucketed reduce-scatter during backward, the norm all-reduce and the
    parameter all-gathers on the optimizer side stream -- the exact calls of the 8-GPU run."""
    env = {**os.environ, "TH_DIST_BACKEND": "nccl", "TH_FORCE_COLLECTIVES": "1", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "scripts/ddp_check.py"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    doc = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert doc["backend"] == "nccl" and doc["world"] == 1 and doc["n_buckets"] > 1
    assert doc["params_identical_zero1"] and doc["zero1_vs_zero0_frac_off"] < 1e-3
