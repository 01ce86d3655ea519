"""CPU checks of the TN weight-gradient GEMM wrapper (ops/gemm_tn.py): the reference path, the
accumulate flag, the split-K choice that fills the 256 CUs, and the shape gate (the HIP kernel
itself is checked against fp32 on the GPU in tests/gpu/test_gemm_tn_gpu.py)."""
import pytest
import torch

from tensorhive_fixed_amd.ops.gemm_tn import default_splitk, gemm_tn_, supported


@pytest.mark.parametrize("accumulate", [False, True])
def test_cpu_reference_path(accumulate):
    g = torch.Generator().manual_seed(0)
    a = torch.randn(64, 24, generator=g).to(torch.bfloat16)
    b = torch.randn(64, 40, generator=g).to(torch.bfloat16)
    out = torch.randn(24, 40, generator=g).to(torch.bfloat16)
    ref = a.float().t() @ b.float() + (out.float() if accumulate else 0)
    gemm_tn_(a, b, out, accumulate=accumulate)
    assert (out.float() - ref).abs().max() <= 0.02 * ref.abs().max() + 1e-2


def test_shape_gate():
    assert supported(4096, 4096, 32768)
    assert supported(128256, 4096, 4096)  # the LM head: 501 row tiles
    assert not supported(4096 + 128, 4096, 32768)
    assert not supported(4096, 4096, 32768 + 32)
    assert not supported(4096, 4096, 64 * 3, splitk=2)


def test_splitk_fills_the_chip(monkeypatch):
    monkeypatch.delenv("TH_GEMM_TN_SPLITK", raising=False)
    # Llama-3-8B weight grads at 32768 tokens (measured choices: profiles/r01_gemm_tn/)
    assert default_splitk(4096, 4096, 32768) == 1   # 256 tiles: exactly one round
    assert default_splitk(6144, 4096, 32768) == 2   # 384 tiles: 1.5 rounds -> 768 = 3 rounds
    assert default_splitk(4096, 14336, 32768) == 2  # 896 tiles: 3.5 rounds -> 7 rounds
    assert default_splitk(28672, 4096, 32768) == 1  # 1792 tiles: 7 full rounds
    monkeypatch.setenv("TH_GEMM_TN_SPLITK", "3")
    assert default_splitk(4096, 4096, 32768) == 3


def test_mismatched_shapes_are_rejected():
    a = torch.zeros(64, 24, dtype=torch.bfloat16)
    b = torch.zeros(32, 40, dtype=torch.bfloat16)
    with pytest.raises(ValueError):
        gemm_tn_(a, b, torch.zeros(24, 40, dtype=torch.bfloat16))


@pytest.mark.parametrize("mode", [0, 6, 8, 11])
def test_retired_launch_modes_are_rejected(mode):
    """Only the hb schedule's launch modes 9 / 10 exist since round 5 (profiles/r05_gemm/)."""
    a = torch.zeros(64, 24, dtype=torch.bfloat16)
    b = torch.zeros(64, 40, dtype=torch.bfloat16)
    with pytest.raises(ValueError):
        gemm_tn_(a, b, torch.zeros(24, 40, dtype=torch.bfloat16), pingpong=mode)
