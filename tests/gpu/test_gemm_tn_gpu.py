"""gfx950 weight-gradient GEMM (C (+)= Aᵀ B, operands [tokens, features]) against an fp32 reference."""
import pytest
import torch

from tensorhive_fixed_amd.ops import _lib
from tensorhive_fixed_amd.ops.gemm_tn import gemm_tn_

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _load():
    _lib.load()


@pytest.mark.parametrize("M,N,K,splitk", [(256, 256, 64, 1), (512, 768, 1024, 1), (768, 512, 4096, 2),
                                          (1024, 256, 2048, 4), (256, 1280, 640, 1),
                                          (512, 256, 192, 1), (256, 512, 1344, 1)])  # odd k-tile counts 3, 21
@pytest.mark.parametrize("accumulate", [False, True])
@pytest.mark.parametrize("pingpong", [9, 10])
def test_gemm_tn_matches_fp32(M, N, K, splitk, accumulate, pingpong):
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N + K)
    a = torch.randn(K, M, device="cuda", dtype=torch.bfloat16, generator=g)
    b = torch.randn(K, N, device="cuda", dtype=torch.bfloat16, generator=g)
    out = torch.randn(M, N, device="cuda", dtype=torch.bfloat16, generator=g)
    ref = a.float().t() @ b.float() + (out.float() if accumulate else 0)
    gemm_tn_(a, b, out, accumulate=accumulate, splitk=splitk, pingpong=pingpong)
    torch.cuda.synchronize()
    err = (out.float() - ref).abs().max().item()
    assert err <= 0.02 * ref.abs().max().item() + 1e-2, err


@pytest.mark.parametrize("pingpong", [9, 10])
def test_gemm_tn_strided_operands_and_asymmetry(pingpong):
    """Row-strided views (a slice of a wider activation) and an asymmetric operand pair catch a
    swapped row/column map."""
    K, M, N = 512, 256, 512
    big_a = torch.randn(K, M + 128, device="cuda", dtype=torch.bfloat16)
    a = big_a[:, 64:64 + M]
    b = (torch.arange(K * N, device="cuda").reshape(K, N) % 7 - 3).to(torch.bfloat16)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    gemm_tn_(a, b, out, splitk=1, pingpong=pingpong)
    ref = a.float().t() @ b.float()
    assert (out.float() - ref).abs().max().item() <= 0.02 * ref.abs().max().item() + 1e-2


@pytest.mark.parametrize("band", [0, 1, 4, 15])
@pytest.mark.parametrize("accumulate", [False, True])
def test_gemm_tn_data_parallel_plus_remainder_split(accumulate, band):
    """Mode 10: 272 tiles = one data-parallel round of 256 whole tiles + 16 remainder tiles split 2 ways
    (slab + per-tile reduce); every tile of both parts must match fp32, for several XCD band heights
    (the remainder tiles and the reduce kernel follow the same band map)."""
    K, M, N = 256, 4096, 4352
    g = torch.Generator(device="cuda").manual_seed(5)
    a = torch.randn(K, M, device="cuda", dtype=torch.bfloat16, generator=g)
    b = torch.randn(K, N, device="cuda", dtype=torch.bfloat16, generator=g)
    out = torch.randn(M, N, device="cuda", dtype=torch.bfloat16, generator=g)
    ref = a.float().t() @ b.float() + (out.float() if accumulate else 0)
    gemm_tn_(a, b, out, accumulate=accumulate, splitk=2, pingpong=10, band=band)
    torch.cuda.synchronize()
    err = (out.float() - ref).abs().max().item()
    assert err <= 0.02 * ref.abs().max().item() + 1e-2, err


@pytest.mark.parametrize("name,M,N,K,accumulate", [
    ("wqkv", 6144, 4096, 32768, False),
    ("wo", 4096, 4096, 32768, False),
    ("w13", 28672, 4096, 32768, False),
    ("w2", 4096, 14336, 32768, False),
    ("lm_head_chunk", 128256 // 256 * 256, 4096, 4096, True),
])
def test_gemm_tn_llama_wgrad_shapes_match_fp32(name, M, N, K, accumulate):
    """Every weight-gradient shape of the Llama-3-8B step (32768 tokens; the LM head per 4096-token chunk,
    accumulating) with the default launch (mode 10, default split-K) against an fp32 reference."""
    g = torch.Generator(device="cuda").manual_seed(M + N)
    a = torch.randn(K, M, device="cuda", dtype=torch.bfloat16, generator=g)
    b = torch.randn(K, N, device="cuda", dtype=torch.bfloat16, generator=g)
    out = torch.randn(M, N, device="cuda", dtype=torch.bfloat16, generator=g) if accumulate else \
        torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ref = a.float().t() @ b.float()
    if accumulate:
        ref += out.float()
    gemm_tn_(a, b, out, accumulate=accumulate)
    torch.cuda.synchronize()
    rel = ((out.float() - ref).norm() / ref.norm()).item()
    assert rel < 5e-3, (name, rel)
    del a, b, out, ref
    torch.cuda.empty_cache()


@pytest.mark.parametrize("cus", [255, 240, 224, 200])
@pytest.mark.parametrize("accumulate", [False, True])
def test_gemm_tn_cu_budget_launches_match_fp32(cus, accumulate):
    """CU-aware launches (round 6): a budget below 256 moves the whole-tile / split-K boundary of the mixed
    grid and the tile-local split-K slab; 272 tiles over K 8192 exercise both parts for several remainders."""
    from tensorhive_fixed_amd.ops.gemm_tn import cu_budget, tn_plan

    K, M, N = 2048 * 4, 4096, 4352
    g = torch.Generator(device="cuda").manual_seed(cus)
    a = torch.randn(K, M, device="cuda", dtype=torch.bfloat16, generator=g)
    b = torch.randn(K, N, device="cuda", dtype=torch.bfloat16, generator=g)
    out = torch.randn(M, N, device="cuda", dtype=torch.bfloat16, generator=g)
    ref = a.float().t() @ b.float() + (out.float() if accumulate else 0)
    with cu_budget(cus):
        sk, full = tn_plan(M, N, K)
        assert sk > 1 and 0 < full < 272
        gemm_tn_(a, b, out, accumulate=accumulate)
    torch.cuda.synchronize()
    err = (out.float() - ref).abs().max().item()
    assert err <= 0.02 * ref.abs().max().item() + 1e-2, err


@pytest.mark.parametrize("name,M,N,K", [("wqkv", 6144, 4096, 32768), ("wo", 4096, 4096, 32768)])
def test_gemm_tn_llama_shapes_at_224_cus(name, M, N, K):
    from tensorhive_fixed_amd.ops.gemm_tn import cu_budget

    g = torch.Generator(device="cuda").manual_seed(M)
    a = torch.randn(K, M, device="cuda", dtype=torch.bfloat16, generator=g)
    b = torch.randn(K, N, device="cuda", dtype=torch.bfloat16, generator=g)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ref = a.float().t() @ b.float()
    with cu_budget(224):
        gemm_tn_(a, b, out)
    torch.cuda.synchronize()
    rel = ((out.float() - ref).norm() / ref.norm()).item()
    assert rel < 5e-3, (name, rel)
