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


def test_band_policy_and_range():
    """Per-shape XCD band heights (profiles/r05_gemm/tn_band2.jsonl) and the 4-bit launch field's range."""
    from tensorhive_fixed_amd.ops import gemm_tn as g

    if g._BAND_POLICY:
        assert g.default_band(28672, 4096, 32768) == 1  # gate|up weight gradient
        assert g.default_band(128256, 4096, 4096) == 4  # LM-head chunk
    for m, n in ((6144, 4096), (4096, 4096), (4096, 14336)):  # wqkv, wo, w2: the compiled default
        assert g.default_band(m, n, 32768) == 0
    a, b, out = torch.zeros(64, 256), torch.zeros(64, 256), torch.zeros(256, 256)
    for bad in (-1, 16):
        with pytest.raises(ValueError):
            g.gemm_tn_(a, b, out, band=bad)
