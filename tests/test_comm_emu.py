"""CPU checks of the one-GPU RCCL channel-footprint rehearsal's configuration (parallel/comm_emu.py) and of the
trainer's backward CU budget; the kernel itself runs in tests/gpu/test_comm_emu_gpu.py."""
import pytest
import torch

from tensorhive_fixed_amd.parallel.comm_emu import CommEmulator, EmuConfig, parse


def test_parse_spec():
    assert parse(None) is None and parse("") is None and parse("cus=0") is None
    c = parse("cus=32, mode=bucket,world=8,busbw=250,copy=0,slice_ms=20,buffer_mb=64")
    assert (c.cus, c.mode, c.world, c.busbw, c.copy, c.slice_ms, c.buffer_mb) == (32, "bucket", 8, 250.0, 0.0, 20.0, 64.0)
    assert parse("cus=8,mode=bucket,deps=1").deps == 1 and parse("cus=8").deps == 0
    for bad in ("cus=300", "mode=ring", "cus=8,world=1", "cus=8,busbw=0", "nope=1", "cus=", "cus=8,deps=1",
                "cus=8,mode=bucket,deps=2"):
        with pytest.raises(ValueError):
            parse(bad)


def test_bucket_time_is_the_ring_reduce_scatter():
    c = EmuConfig(cus=16, mode="bucket", world=8, busbw=300.0)
    assert abs(c.bucket_seconds(256 << 20) - (256 << 20) * 7 / 8 / 300e9) < 1e-12
    assert abs(c.bucket_seconds(256 << 20) * 1e3 - 0.7829) < 1e-3  # ~0.78 ms per 256 MB bucket


def test_no_emulator_on_cpu(monkeypatch):
    monkeypatch.setenv("TH_COMM_EMU", "cus=16")
    assert CommEmulator.from_env(torch.device("cpu")) is None


def test_backward_cu_budget_policy(monkeypatch):
    """Rehearsal: the emulated channel count; otherwise only an explicit TH_COMM_CUS changes the 256-CU plan
    (profiles/r06_comm/: the re-plan costs more on the idle chip than it saves in the modelled 8-rank schedule),
    a channel cap included."""
    from types import SimpleNamespace

    from tensorhive_fixed_amd.workloads.llama3_ddp import backward_cu_budget

    for k in ("TH_COMM_CUS", "NCCL_MAX_NCHANNELS"):
        monkeypatch.delenv(k, raising=False)
    one = SimpleNamespace(comm_emu=None, collectives=False, world=1)
    multi = SimpleNamespace(comm_emu=None, collectives=True, world=8)
    emu = SimpleNamespace(comm_emu=SimpleNamespace(cfg=EmuConfig(cus=32)), collectives=False, world=1)
    assert backward_cu_budget(one) is None and backward_cu_budget(multi) is None
    assert backward_cu_budget(emu) == 224
    monkeypatch.setenv("NCCL_MAX_NCHANNELS", "16")
    assert backward_cu_budget(multi) is None and backward_cu_budget(one) is None
    monkeypatch.setenv("TH_COMM_CUS", "16")
    assert backward_cu_budget(multi) == 240
    monkeypatch.setenv("TH_COMM_CUS", "0")
    assert backward_cu_budget(multi) is None and backward_cu_budget(emu) is None
    monkeypatch.setenv("TH_COMM_CUS", "250")
    assert backward_cu_budget(one) == 64  # never below 64 CUs


def test_streamk_data_parallel_preset(monkeypatch):
    """profiles/r06_comm/skdp: hipBLASLt's stream-K kernels tiled data-parallel -- free on an idle chip, +9 % on
    the step with 16 CUs held; preset for every run before hipBLASLt initialises, never over a user's value."""
    from tensorhive_fixed_amd.parallel.dist import apply_env_defaults, comm_env, rccl_env_defaults

    assert rccl_env_defaults()["TENSILE_STREAMK_DATA_PARALLEL"] == "1"
    monkeypatch.delenv("TENSILE_STREAMK_DATA_PARALLEL", raising=False)
    apply_env_defaults()
    import os

    assert os.environ["TENSILE_STREAMK_DATA_PARALLEL"] == "1"
    assert comm_env()["TENSILE_STREAMK_DATA_PARALLEL"] == "1"  # recorded in the bench census
    monkeypatch.setenv("TENSILE_STREAMK_DATA_PARALLEL", "0")
    apply_env_defaults()
    assert os.environ["TENSILE_STREAMK_DATA_PARALLEL"] == "0"


def test_launcher_template_carries_the_payload_presets():
    from tensorhive_fixed_amd.core.launcher import RCCL_ENV
    from tensorhive_fixed_amd.parallel.dist import rccl_env_defaults

    assert RCCL_ENV == rccl_env_defaults()
