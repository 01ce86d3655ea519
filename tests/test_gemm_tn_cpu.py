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
    monkeypatch.setenv("TH_GEMM_TN_SPLITK", "4")
    assert default_splitk(4096, 4096, 32768) == 4


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


LLAMA_WGRAD = {"wqkv": (6144, 4096, 32768), "wo": (4096, 4096, 32768), "w13": (28672, 4096, 32768),
               "w2": (4096, 14336, 32768), "lm_head_chunk": (128256, 4096, 4096)}


def test_plan_at_256_cus_keeps_round5_choices(monkeypatch):
    """The CU-aware planner reproduces the round-5 launches on an idle chip: wqkv / w2 whole rounds with a
    2-way split remainder, wo / w13 / the LM-head chunk whole tiles."""
    from tensorhive_fixed_amd.ops.gemm_tn import tn_plan

    monkeypatch.delenv("TH_GEMM_TN_SPLITK", raising=False)
    got = {k: tn_plan(*v, cus=256) for k, v in LLAMA_WGRAD.items()}
    assert got == {"wqkv": (2, 256), "wo": (1, 256), "w13": (1, 1792), "w2": (2, 768), "lm_head_chunk": (1, 8016)}


@pytest.mark.parametrize("cus", [248, 240, 232, 224, 208, 192, 160, 128])
def test_plan_for_fewer_cus_stays_near_the_ideal(monkeypatch, cus):
    """Round-6 verdict item 1: with RCCL's channels holding 256 - cus CUs, a round sized for 256 spills the
    few tiles that do not fit into a second full round (wo: 256 tiles -> 2 rounds on 255 CUs).  The plan
    for the CUs actually available stays within 15 % of tiles / cus on every Llama weight-gradient shape and
    never loses to the 256-CU plan run on the same CUs, while on the idle chip it stays within 12 % of the
    256-CU plan."""
    from tensorhive_fixed_amd.ops.gemm_tn import plan_time, tn_plan

    monkeypatch.delenv("TH_GEMM_TN_SPLITK", raising=False)
    for name, (m, n, k) in LLAMA_WGRAD.items():
        tiles = (m // 256) * (n // 256)
        sk, full = tn_plan(m, n, k, cus=cus)
        t = plan_time(tiles, sk, full, cus)
        naive = plan_time(tiles, *tn_plan(m, n, k, cus=256), cus)
        assert t <= naive + 1e-9, (name, cus, t, naive)
        assert t <= 1.15 * tiles / cus + 0.06, (name, cus, sk, full, t, tiles / cus)
        idle = plan_time(tiles, sk, full, 256)
        assert idle <= 1.12 * plan_time(tiles, *tn_plan(m, n, k, cus=256), 256), (name, cus, idle)
        assert k % (64 * sk) == 0 and k // sk >= 2048 and 0 <= full <= tiles


def test_wo_gradient_no_longer_doubles_when_a_few_cus_are_busy(monkeypatch):
    from tensorhive_fixed_amd.ops.gemm_tn import plan_time, tn_plan

    monkeypatch.delenv("TH_GEMM_TN_SPLITK", raising=False)
    assert plan_time(256, 1, 256, 240) == 2.0  # the 256-CU plan on 240 CUs: a second full round
    sk, full = tn_plan(4096, 4096, 32768, cus=240)
    assert sk > 1 and full < 256 and plan_time(256, sk, full, 240) < 1.2
    assert plan_time(256, sk, full, 256) < 1.12  # the pieces fill the CUs the whole tiles leave idle


def test_list_schedule_model():
    from tensorhive_fixed_amd.ops.gemm_tn import plan_time

    assert plan_time(512, 1, 512, 256) == 2.0
    assert plan_time(257, 1, 257, 256) == 2.0
    # 240 whole tiles + 16 tiles x 8 pieces on 256 CUs: the 16 free CUs run 8 pieces each during the round
    assert abs(plan_time(256, 8, 240, 256) - (8 * (1 / 8 + 0.01) + 0.02)) < 1e-9


def test_workspace_covers_only_the_split_tiles():
    """Round-5 verdict weak #7: the slab holds split tiles only (w2 at 256 CUs: 128 remainder tiles x 2)."""
    from tensorhive_fixed_amd.ops.gemm_tn import workspace_floats

    assert workspace_floats(4096, 14336, 2, 768) == 128 * 2 * 65536  # 64 MiB, was 470 MB (sk * M * N)
    assert workspace_floats(4096, 14336, 2, 0) == 896 * 2 * 65536
    assert workspace_floats(4096, 4096, 1, 256) == 0
    assert workspace_floats(4096, 4096, 4, 224) == 32 * 4 * 65536


def test_cu_budget_context(monkeypatch):
    from tensorhive_fixed_amd.ops import gemm_tn as g

    base = g.compute_cus()
    with g.cu_budget(224):
        assert g.compute_cus() == 224
        with g.cu_budget(None):
            assert g.compute_cus() == 224
    assert g.compute_cus() == base
    with pytest.raises(ValueError):
        with g.cu_budget(0):
            pass
