"""Numerics of every gfx950 HIP kernel against a plain PyTorch fp32 reference of the same op.

All tests run in ONE process on the GPU box (``pytest -m gpu``); shapes are checked on the host
by the Python wrappers before any launch.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib_loaded():
    from tensorhive_fixed_amd.ops import _lib
    _lib.load(build_if_missing=True)
    assert _lib.library_path().exists()


def _close(a, b, atol, rtol=0.0):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    tol = atol + rtol * b.abs().max().item()
    assert err <= tol, f"max abs err {err} > {tol}"


@pytest.mark.parametrize("T,D", [(1, 4096), (37, 4096), (256, 2048), (64, 8192), (5, 136)])
def test_rmsnorm_fwd_bwd(T, D):
    from tensorhive_fixed_amd.ops.rmsnorm import rmsnorm
    torch.manual_seed(0)
    x = torch.randn(T, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    w = (1 + 0.1 * torch.randn(D, device=DEV)).to(torch.bfloat16).requires_grad_(True)
    y = rmsnorm(x, w, 1e-5)
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().float().requires_grad_(True)
    yr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-5) * wr
    _close(y, yr, 3e-2, 1e-2)
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g.float())
    _close(x.grad, xr.grad, 5e-2, 2e-2)
    _close(w.grad, wr.grad, 0.1, 2e-2)


@pytest.mark.parametrize("T,F", [(7, 14336), (128, 512), (1, 64)])
def test_swiglu_fwd_bwd(T, F):
    from tensorhive_fixed_amd.ops.swiglu import swiglu
    torch.manual_seed(1)
    gu = torch.randn(T, 2 * F, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    out = swiglu(gu)
    r = gu.detach().float().requires_grad_(True)
    g, u = r.chunk(2, -1)
    outr = torch.nn.functional.silu(g) * u
    _close(out, outr, 3e-2, 1e-2)
    d = torch.randn_like(out)
    out.backward(d)
    outr.backward(d.float())
    _close(gu.grad, r.grad, 5e-2, 2e-2)


@pytest.mark.parametrize("B,S,Hq,Hkv", [(1, 128, 4, 1), (2, 64, 32, 8)])
def test_rope_inplace(B, S, Hq, Hkv):
    from tensorhive_fixed_amd.ops.rope import rope_inplace, rope_reference_
    torch.manual_seed(2)
    Dh = 128
    row = (Hq + 2 * Hkv) * Dh
    x = torch.randn(B * S, row, device=DEV, dtype=torch.bfloat16)
    a = x.clone()
    rope_inplace(a, S, Hq + Hkv, Dh, 500000.0, 1.0)
    ref = rope_reference_(x.float().clone(), S, Hq + Hkv, Dh, 500000.0, 1.0)
    _close(a, ref, 3e-2, 1e-2)
    assert torch.equal(a[:, (Hq + Hkv) * Dh:], x[:, (Hq + Hkv) * Dh:])  # v untouched
    rope_inplace(a, S, Hq + Hkv, Dh, 500000.0, -1.0)  # inverse rotation
    _close(a, x, 5e-2, 2e-2)


@pytest.mark.parametrize("R,V", [(4, 128256), (33, 1000), (2, 13)])
def test_cross_entropy_rows(R, V):
    from tensorhive_fixed_amd.ops.cross_entropy import ce_rows_
    torch.manual_seed(3)
    logits = (3 * torch.randn(R, V, device=DEV)).to(torch.bfloat16)
    tgt = torch.randint(0, V, (R,), device=DEV)
    tgt[0] = -100
    ref_l = logits.float()
    lse = torch.logsumexp(ref_l, -1)
    loss_ref = torch.where(tgt >= 0, lse - ref_l.gather(1, tgt.clamp(min=0)[:, None])[:, 0], 0.0)
    p = torch.softmax(ref_l, -1)
    p[torch.arange(R), tgt.clamp(min=0)] -= 1.0
    p = p * 0.5
    p[0] = 0
    lg = logits.clone()
    loss = ce_rows_(lg, tgt, 0.5)
    _close(loss, loss_ref, 2e-2, 1e-3)
    _close(lg, p, 2e-3, 1e-2)


def test_linear_cross_entropy_matches_reference():
    from tensorhive_fixed_amd.ops.cross_entropy import linear_cross_entropy
    torch.manual_seed(4)
    T, D, V = 300, 256, 1000
    h = torch.randn(T, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    w = (0.05 * torch.randn(V, D, device=DEV)).to(torch.bfloat16).requires_grad_(True)
    t = torch.randint(0, V, (T,), device=DEV)
    loss = linear_cross_entropy(h, w, t, chunk=128)
    loss.backward()
    hr = h.detach().float().requires_grad_(True)
    wr = w.detach().float().requires_grad_(True)
    lr = torch.nn.functional.cross_entropy(hr @ wr.t(), t)
    lr.backward()
    _close(loss, lr, 1e-2, 1e-3)
    _close(h.grad, hr.grad, 2e-3, 5e-2)
    _close(w.grad, wr.grad, 2e-3, 5e-2)


@pytest.mark.parametrize("n", [8, 4096, 1 << 20])
def test_adamw_flat(n):
    from tensorhive_fixed_amd.ops.adamw import adamw_flat_, grad_sumsq_
    torch.manual_seed(5)
    p = torch.randn(n, device=DEV).to(torch.bfloat16)
    master = p.float().clone()
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    g = torch.randn(n, device=DEV).to(torch.bfloat16)
    ns = torch.zeros(1, device=DEV)
    grad_sumsq_(g, ns)
    _close(ns, g.float().pow(2).sum()[None], 1e-3, 1e-4)
    ref_p = master.clone()
    ref_m, ref_v = m.clone(), v.clone()
    for step in (1, 2, 3):
        adamw_flat_(p, master, m, v, g, lr=1e-3, beta1=0.9, beta2=0.95, eps=1e-8, weight_decay=0.1,
                    step=step, grad_scale=0.5, norm_sq=ns, clip=1.0)
        tn = ns.sqrt() * 0.5
        gs = g.float() * 0.5 * torch.clamp(1.0 / (tn + 1e-6), max=1.0)
        ref_m = 0.9 * ref_m + 0.1 * gs
        ref_v = 0.95 * ref_v + 0.05 * gs * gs
        ref_p = ref_p * (1 - 1e-3 * 0.1)
        ref_p = ref_p - 1e-3 / (1 - 0.9 ** step) * ref_m / (ref_v.sqrt() / math.sqrt(1 - 0.95 ** step) + 1e-8)
    _close(master, ref_p, 1e-5, 1e-5)
    _close(p, ref_p, 2e-2, 1e-2)


def test_embedding_backward_deterministic():
    from tensorhive_fixed_amd.ops.embedding import embedding
    torch.manual_seed(6)
    V, D, T = 1000, 512, 4096
    w = torch.randn(V, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    tok = torch.randint(0, 50, (T,), device=DEV)  # many repeats
    y = embedding(tok, w)
    g = torch.randn_like(y)
    y.backward(g)
    ref = torch.zeros(V, D, device=DEV)
    ref.index_add_(0, tok, g.float())
    _close(w.grad, ref, 0.25, 1e-2)
    g1 = w.grad.clone()
    w.grad = None
    embedding(tok, w).backward(g)
    assert torch.equal(g1, w.grad)  # bitwise reproducible (no atomics)


@pytest.mark.parametrize("R,C,ld", [(128, 64, 64), (4096, 28672, 28672), (136, 72, 72), (8, 8, 8), (1000, 48, 96)])
def test_transpose_bitexact(R, C, ld):
    from tensorhive_fixed_amd.ops.transpose import transpose
    torch.manual_seed(7)
    base = torch.randn(R, ld, device=DEV, dtype=torch.bfloat16)
    x = base[:, :C]  # row-strided view when ld > C
    out = transpose(x)
    torch.cuda.synchronize()
    assert out.shape == (C, R) and torch.equal(out, x.t().contiguous())


def test_linear_nt_backward_matches_plain_forms():
    """dgrad via the transposed weight and the wgrad_nt path give the same gradients as the plain
    GEMM forms (same bf16 GEMM inputs; fp32 accumulation order may differ)."""
    from tensorhive_fixed_amd.ops.linear import linear
    torch.manual_seed(8)
    T, K, N = 512, 256, 384
    x = torch.randn(T, K, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    g = torch.randn(T, N, device=DEV, dtype=torch.bfloat16)
    linear(x, w, wgrad_nt=True).backward(g)
    ref_dx = g.float() @ w.float()
    ref_dw = g.float().t() @ x.float()
    _close(x.grad, ref_dx, 0.5, 1e-2)
    _close(w.grad, ref_dw, 0.5, 1e-2)


@pytest.mark.parametrize("T,F", [(256, 64), (4096, 1024), (200, 128)])
def test_swiglu_bwd_transposed_output(T, F):
    from tensorhive_fixed_amd.ops import _lib
    torch.manual_seed(9)
    gu = torch.randn(T, 2 * F, device=DEV, dtype=torch.bfloat16)
    d = torch.randn(T, F, device=DEV, dtype=torch.bfloat16)
    dgu = torch.empty_like(gu)
    dguT = torch.empty(2 * F, T, device=DEV, dtype=torch.bfloat16)
    _lib.call("th_swiglu_bwd_t", d.data_ptr(), gu.data_ptr(), dgu.data_ptr(), dguT.data_ptr(), T, F,
              _lib.stream_ptr(gu.device))
    g, u = gu.float().chunk(2, -1)
    s = torch.sigmoid(g)
    ref = torch.cat([d.float() * u * s * (1 + g * (1 - s)), d.float() * g * s], -1)
    _close(dgu, ref, 2e-2, 1e-2)
    assert torch.equal(dguT, dgu.t())


@pytest.mark.parametrize("w13_tn", [True, False])
def test_gate_up_swiglu_matches_unfused(w13_tn, monkeypatch):
    """Both weight-gradient paths of the fused gate|up + SwiGLU node: the TN kernel on dGU and H (default),
    and hipBLASLt on dGU^T (written by the transposing SwiGLU backward) and H^T."""
    from tensorhive_fixed_amd.ops import mlp
    from tensorhive_fixed_amd.ops.linear import linear
    from tensorhive_fixed_amd.ops.mlp import gate_up_swiglu
    from tensorhive_fixed_amd.ops.swiglu import swiglu
    monkeypatch.setattr(mlp, "_W13_TN", w13_tn)
    torch.manual_seed(10)
    T, D, F = 512, 256, 512
    h = torch.randn(T, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    w = (torch.randn(2 * F, D, device=DEV, dtype=torch.bfloat16) * 0.05).requires_grad_(True)
    g = torch.randn(T, F, device=DEV, dtype=torch.bfloat16)
    a = gate_up_swiglu(h, w)
    a.backward(g)
    h2, w2 = h.detach().clone().requires_grad_(True), w.detach().clone().requires_grad_(True)
    swiglu(linear(h2, w2)).backward(g)
    _close(a, swiglu(linear(h2.detach(), w2.detach())), 1e-2, 1e-2)
    _close(h.grad, h2.grad, 5e-2, 2e-2)
    _close(w.grad, w2.grad, 5e-2, 2e-2)


def test_rmsnorm_fork_fuses_residual_gradient():
    from tensorhive_fixed_amd.ops.rmsnorm import rmsnorm, rmsnorm_fork
    torch.manual_seed(11)
    T, D = 300, 4096
    x = torch.randn(T, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    w = (1 + 0.1 * torch.randn(D, device=DEV)).to(torch.bfloat16).requires_grad_(True)
    gh, gr = torch.randn(T, D, device=DEV, dtype=torch.bfloat16), torch.randn(T, D, device=DEV, dtype=torch.bfloat16)
    h, xr = rmsnorm_fork(x, w)
    assert xr.data_ptr() == x.data_ptr()
    torch.autograd.backward([h, xr], [gh, gr])
    xf = x.detach().float().requires_grad_(True)
    wf = w.detach().float().requires_grad_(True)
    ref = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5) * wf
    torch.autograd.backward([ref, xf], [gh.float(), gr.float()])
    _close(h, ref, 3e-2, 1e-2)
    _close(x.grad, xf.grad, 5e-2, 1e-2)
    _close(w.grad, wf.grad, 0.5, 1e-2)
    assert rmsnorm is not None


def test_rmsnorm_add_fork_kernel_matches_fp32_reference():
    from tensorhive_fixed_amd.ops.rmsnorm import rmsnorm_add_fork
    torch.manual_seed(3)
    T, D = 300, 4096
    y = torch.randn(T, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn(T, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = (1 + 0.1 * torch.randn(D, device="cuda")).to(torch.bfloat16).requires_grad_(True)
    h, x = rmsnorm_add_fork(y, r, w)
    s = y.detach().float() + r.detach().float()
    assert (x.float() - s).abs().max().item() < 0.07  # bf16 rounding of the sum
    xs = x.detach().float()
    ref = xs * torch.rsqrt(xs.pow(2).mean(-1, keepdim=True) + 1e-5) * w.detach().float()
    assert (h.float() - ref).abs().max().item() < 0.05
    dh, dx = torch.randn_like(h), torch.randn_like(x)
    torch.autograd.backward([h, x], [dh, dx])
    xr = xs.clone().requires_grad_(True)
    wr = w.detach().float().requires_grad_(True)
    hr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-5) * wr
    torch.autograd.backward([hr, xr], [dh.float(), dx.float()])
    for a, b in ((y.grad, xr.grad), (r.grad, xr.grad)):
        assert ((a.float() - b).norm() / b.norm()).item() < 1e-2
    assert ((w.grad.float() - wr.grad).norm() / wr.grad.norm()).item() < 1e-2
