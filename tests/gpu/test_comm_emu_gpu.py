"""The one-GPU RCCL channel-footprint rehearsal (parallel/comm_emu.py, ops/csrc/comm_emu.hip) on hardware:
launches always drain (stop marker, byte budget, time slice), hold one CU each, and a training step with the
emulation on stays numerically identical to one without it."""
import time

import pytest
import torch

from tensorhive_fixed_amd.ops import _lib
from tensorhive_fixed_amd.parallel.comm_emu import CommEmulator, parse

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _load():
    _lib.load()


def test_persist_launches_end_at_the_stop_marker():
    emu = CommEmulator(parse("cus=16,slice_ms=2000,buffer_mb=64"), torch.device("cuda"))
    a = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
    t0 = time.perf_counter()
    emu.bucket_ready(256 << 20)
    emu.bucket_ready(256 << 20)
    for _ in range(20):
        a = (a @ a).clamp_(-1, 1)
    emu.stop()
    torch.cuda.synchronize()
    emu.side.synchronize()
    dt = time.perf_counter() - t0
    r = emu.report()
    assert r["launches"] == 2 and r["workgroups"] == 32, r
    assert r["copied_gb"] > 0
    assert dt < 1.5, f"the stop marker did not end the launches ({dt:.2f} s; slice 2 s)"


def test_time_slice_drains_without_a_stop():
    emu = CommEmulator(parse("cus=8,slice_ms=30,buffer_mb=32"), torch.device("cuda"))
    t0 = time.perf_counter()
    emu.bucket_ready(1 << 20)
    emu.side.synchronize()
    dt = time.perf_counter() - t0
    assert 0.025 < dt < 1.0, dt
    r = emu.report()
    assert r["workgroups"] == 8 and 25 <= r["ms_per_workgroup"] <= 200, r


def test_bucket_mode_moves_its_budget_and_ends():
    emu = CommEmulator(parse("cus=16,mode=bucket,world=8,busbw=300,copy=450,buffer_mb=64"), torch.device("cuda"))
    nbytes = 256 << 20
    emu.bucket_ready(nbytes)
    emu.side.synchronize()
    r = emu.report()
    want = emu.cfg.bucket_seconds(nbytes) * 450e9  # bytes copied at the modelled rate
    assert r["workgroups"] == 16
    assert 0.9 * want <= r["copied_gb"] * 1e9 <= 1.2 * want + 16 * 65536 * 16, (r, want)


def test_one_workgroup_per_cu():
    """Two 128-workgroup launches on two streams: each workgroup reserves 96 KB of LDS, so at most 256 are
    resident and both finish within one slice of each other (no CU holds two)."""
    e1 = CommEmulator(parse("cus=128,slice_ms=20,buffer_mb=64"), torch.device("cuda"))
    e2 = CommEmulator(parse("cus=128,slice_ms=20,buffer_mb=64"), torch.device("cuda"))
    e1.bucket_ready(1 << 20)
    e2.bucket_ready(1 << 20)
    torch.cuda.synchronize()
    e1.side.synchronize()
    e2.side.synchronize()
    assert e1.report()["workgroups"] == 128 and e2.report()["workgroups"] == 128


def test_training_step_with_emulation_matches_without(monkeypatch):
    from tensorhive_fixed_amd.models.llama3 import LlamaConfig
    from tensorhive_fixed_amd.parallel.dist import DistInfo
    from tensorhive_fixed_amd.workloads.llama3_ddp import Trainer

    info = DistInfo(0, 0, 1, torch.device("cuda", 0), None)
    losses = {}
    for spec in ("", "cus=32,slice_ms=20,buffer_mb=64"):
        monkeypatch.setenv("TH_COMM_EMU", spec)
        tr = Trainer(LlamaConfig.tiny(), info, micro_batch=2, seq_len=256, seed=0)
        assert (tr.store.comm_emu is not None) == bool(spec)
        assert tr.bwd_cus == (224 if spec else None)
        losses[spec] = [float(tr.step()) for _ in range(3)]
        torch.cuda.synchronize()
        if spec:
            r = tr.store.comm_emu.report()
            assert r["launches"] >= 3 and r["workgroups"] == 32 * r["launches"], r
    assert losses[""] == losses["cus=32,slice_ms=20,buffer_mb=64"]


def test_bucket_mode_emulates_reduce_scatter_and_all_gather(monkeypatch):
    """Bucket mode: one launch per bucket for its reduce-scatter (backward) and one for its all-gather (after
    its optimizer update); persist mode launches at bucket-ready points only."""
    from tensorhive_fixed_amd.models.llama3 import LlamaConfig
    from tensorhive_fixed_amd.parallel.dist import DistInfo
    from tensorhive_fixed_amd.workloads.llama3_ddp import Trainer

    info = DistInfo(0, 0, 1, torch.device("cuda", 0), None)
    monkeypatch.setenv("TH_COMM_EMU", "cus=8,mode=bucket,buffer_mb=32")
    tr = Trainer(LlamaConfig.tiny(), info, micro_batch=2, seq_len=256, seed=0, bucket_mb=0.25)
    nb = len(tr.store.buckets)
    for _ in range(2):
        tr.step()
    torch.cuda.synchronize()
    r = tr.store.comm_emu.report()
    assert r["launches"] == 2 * 2 * nb, (r, nb)


def test_bucket_mode_dependencies_keep_numerics_and_order(monkeypatch):
    """deps=1: the optimizer waits for every modelled reduce-scatter and each forward layer for its modelled
    all-gather (events on the emulator's stream); the trajectory equals the run without emulation."""
    from tensorhive_fixed_amd.models.llama3 import LlamaConfig
    from tensorhive_fixed_amd.parallel.dist import DistInfo
    from tensorhive_fixed_amd.workloads.llama3_ddp import Trainer

    info = DistInfo(0, 0, 1, torch.device("cuda", 0), None)
    losses = {}
    for spec in ("", "cus=16,mode=bucket,busbw=5,buffer_mb=32,deps=1"):  # 5 GB/s: collectives far longer than compute
        monkeypatch.setenv("TH_COMM_EMU", spec)
        tr = Trainer(LlamaConfig.tiny(), info, micro_batch=2, seq_len=256, seed=0, bucket_mb=0.25)
        losses[spec] = [float(tr.step()) for _ in range(3)]
        torch.cuda.synchronize()
        if spec:
            assert all(b.emu_done is None for b in tr.store.buckets)  # every reduce-scatter was waited on
            r = tr.store.comm_emu.report()
            assert r["launches"] == 2 * 3 * len(tr.store.buckets), r
    assert losses[""] == losses["cus=16,mode=bucket,busbw=5,buffer_mb=32,deps=1"]
