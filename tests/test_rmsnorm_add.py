"""Fused residual-add RMSNorm (ops/rmsnorm.py: rmsnorm_add_fork) against the unfused composition."""
import torch

from tensorhive_fixed_amd.ops.rmsnorm import rmsnorm_add_fork, rmsnorm_fork


def test_rmsnorm_add_fork_matches_add_then_fork_cpu():
    torch.manual_seed(0)
    T, D = 12, 64
    y = torch.randn(T, D, dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn(T, D, dtype=torch.bfloat16, requires_grad=True)
    w = (1 + 0.1 * torch.randn(D)).to(torch.bfloat16).requires_grad_(True)
    h, x = rmsnorm_add_fork(y, r, w)
    dh, dx = torch.randn_like(h), torch.randn_like(x)
    (h.float() * dh.float()).sum().add((x.float() * dx.float()).sum()).backward()
    y2, r2, w2 = (t.detach().clone().requires_grad_(True) for t in (y, r, w))
    s = (y2.float() + r2.float()).to(torch.bfloat16)
    h2, x2 = rmsnorm_fork(s, w2)
    (h2.float() * dh.float()).sum().add((x2.float() * dx.float()).sum()).backward()
    assert torch.equal(x, x2) and torch.allclose(h.float(), h2.float(), atol=1e-2)
    for a, b in ((y.grad, y2.grad), (r.grad, r2.grad), (w.grad, w2.grad)):
        assert torch.allclose(a.float(), b.float(), atol=3e-2, rtol=3e-2)
