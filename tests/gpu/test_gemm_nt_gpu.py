"""gfx950 NT GEMM (ops/csrc/gemm_nt.hip) against an fp32 PyTorch reference: the Llama forward /
input-gradient layout, beta = 0 and 1, non-contiguous row strides."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,N,K", [(256, 256, 32), (512, 768, 4096), (1024, 512, 14336), (256, 6144, 4096)])
@pytest.mark.parametrize("beta", [0, 1])
@pytest.mark.parametrize("mfma16", [False, True], ids=["mfma32x32x16", "mfma16x16x32"])
def test_gemm_nt_matches_fp32(M, N, K, beta, mfma16):
    from tensorhive_fixed_amd.ops import _lib
    from tensorhive_fixed_amd.ops.gemm_nt import gemm_nt_

    _lib.load()
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    a = torch.randn(M, K + 64, device="cuda", dtype=torch.bfloat16, generator=g)[:, :K]  # row stride K + 64
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16, generator=g)
    c = torch.randn(M, N, device="cuda", dtype=torch.bfloat16, generator=g)
    c0 = c.float().clone()
    gemm_nt_(a, b, c, accumulate=bool(beta), mfma16=mfma16)
    ref = a.float() @ b.float().t() + (c0 if beta else 0)
    rel = ((c.float() - ref).norm() / ref.norm()).item()
    assert rel < 5e-3, rel
