"""gfx950 NT GEMM (ops/csrc/gemm_nt.hip) against an fp32 PyTorch reference: the Llama forward /
input-gradient layout, beta = 0 and 1, non-contiguous row strides, every Llama-3-8B shape at a
reduced token count, and an asymmetric operand that would catch a transposed output."""
import pytest
import torch

pytestmark = pytest.mark.gpu

D, F, HQKV, V = 4096, 14336, 6144, 128256


def _run(M, N, K, beta, stride_pad=0, seed=0, variant=None):
    from tensorhive_fixed_amd.ops import _lib
    from tensorhive_fixed_amd.ops.gemm_nt import gemm_nt_, usable

    _lib.load()
    g = torch.Generator(device="cuda").manual_seed(seed + M + N + K)
    a = torch.randn(M, K + stride_pad, device="cuda", dtype=torch.bfloat16, generator=g)[:, :K]
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16, generator=g)
    c = torch.randn(M, N, device="cuda", dtype=torch.bfloat16, generator=g)
    assert usable(a, b, c)  # the HIP kernel runs, not the fallback
    c0 = c.float().clone()
    gemm_nt_(a, b, c, accumulate=bool(beta), variant=variant)
    torch.cuda.synchronize()
    ref = a.float() @ b.float().t() + (c0 if beta else 0)
    return ((c.float() - ref).norm() / ref.norm()).item()


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 4096), (1024, 512, 14336), (256, 6144, 4096),
                                   (768, 256, 128)])
@pytest.mark.parametrize("beta", [0, 1])
def test_gemm_nt_matches_fp32(M, N, K, beta):
    assert _run(M, N, K, beta, stride_pad=64) < 5e-3


@pytest.mark.parametrize("name,N,K", [("wqkv.fwd", HQKV, D), ("wo.fwd", D, D), ("w13.fwd", 2 * F, D), ("w2.fwd", D, F),
                                      ("wqkv.dgrad", D, HQKV), ("w13.dgrad", D, 2 * F), ("w2.dgrad", F, D),
                                      ("head.fwd", V, D), ("head.dgrad", D, V)])
def test_gemm_nt_llama_shapes(name, N, K):
    M = 512 if N * K > 200_000_000 else 1024
    assert _run(M, N, K, 0) < 5e-3, name


@pytest.mark.parametrize("variant", [0, 1, 8, 16, 17, 20])
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 512, 128), (256, 512, 4096)])
def test_gemm_nt_schedule_variants_match_fp32(M, N, K, variant):
    """Every compiled schedule variant (A/B aids) is exact too: a variant that read a stale
    accumulator returned inf here before the accumulators were pinned ahead of the loop."""
    assert _run(M, N, K, 0, variant=variant) < 5e-3


def test_gemm_nt_output_orientation():
    """A = I (rows of the identity), asymmetric B: C must equal B^T exactly."""
    from tensorhive_fixed_amd.ops import _lib
    from tensorhive_fixed_amd.ops.gemm_nt import gemm_nt_

    _lib.load()
    M = N = K = 256
    a = torch.eye(M, K, device="cuda", dtype=torch.bfloat16)
    b = (torch.arange(N * K, device="cuda", dtype=torch.float32).view(N, K) % 251 - 125).to(torch.bfloat16)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    gemm_nt_(a, b, c)
    torch.cuda.synchronize()
    assert torch.equal(c, b.t().contiguous())
