"""CPU checks of the payload model built from the custom autograd ops (reference paths):
loss and every weight gradient must match a plain-PyTorch fp32 implementation of Llama."""
import math

import torch
import torch.nn.functional as F

from tensorhive_fixed_amd.models.llama3 import Llama, LlamaConfig


def _reference_loss(model: Llama, tok, tgt):
    cfg = model.cfg
    B, S = tok.shape
    hd = cfg.head_dim
    P = {n: p.detach().float().requires_grad_(True) for n, p in model.named_parameters()}

    def norm(x, w):
        return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + cfg.norm_eps) * w

    inv = 1.0 / (cfg.rope_theta ** (torch.arange(0, hd, 2, dtype=torch.float64) / hd))
    ang = (torch.arange(S, dtype=torch.float64)[:, None] * inv[None]).float()
    cos, sin = ang.cos()[None, :, None, :], ang.sin()[None, :, None, :]

    def rope(x):
        x1, x2 = x[..., : hd // 2], x[..., hd // 2:]
        return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], -1)

    x = P["tok_emb"][tok]
    for i in range(cfg.n_layers):
        pre = f"layers.{i}."
        h = norm(x, P[pre + "attn_norm"])
        qkv = h @ P[pre + "wqkv"].t()
        q = qkv[..., : cfg.n_heads * hd].view(B, S, cfg.n_heads, hd)
        k = qkv[..., cfg.n_heads * hd: (cfg.n_heads + cfg.n_kv_heads) * hd].view(B, S, cfg.n_kv_heads, hd)
        v = qkv[..., (cfg.n_heads + cfg.n_kv_heads) * hd:].view(B, S, cfg.n_kv_heads, hd)
        q, k = rope(q), rope(k)
        rep = cfg.n_heads // cfg.n_kv_heads
        qh = q.transpose(1, 2)
        kh = k.transpose(1, 2).repeat_interleave(rep, 1)
        vh = v.transpose(1, 2).repeat_interleave(rep, 1)
        s = qh @ kh.transpose(-1, -2) / math.sqrt(hd)
        s = s.masked_fill(torch.ones(S, S, dtype=torch.bool).triu(1), float("-inf"))
        o = (s.softmax(-1) @ vh).transpose(1, 2).reshape(B, S, -1)
        x = x + o @ P[pre + "wo"].t()
        h = norm(x, P[pre + "ffn_norm"])
        g, u = (h @ P[pre + "w13"].t()).chunk(2, -1)
        x = x + (F.silu(g) * u) @ P[pre + "w2"].t()
    h = norm(x, P["norm"])
    loss = F.cross_entropy((h @ P["lm_head"].t()).view(B * S, -1), tgt.reshape(-1))
    loss.backward()
    return loss, {n: p.grad for n, p in P.items()}


def test_custom_op_model_matches_reference_cpu():
    torch.manual_seed(0)
    cfg = LlamaConfig.tiny()
    model = Llama(cfg, device="cpu", dtype=torch.bfloat16, seed=3)
    tok = torch.randint(0, cfg.vocab_size, (2, 64))
    tgt = torch.randint(0, cfg.vocab_size, (2, 64))
    loss = model(tok, tgt)
    loss.backward()
    ref_loss, ref_grads = _reference_loss(model, tok, tgt)
    assert abs(float(loss.detach()) - float(ref_loss.detach())) < 2e-2
    for n, p in model.named_parameters():
        a, b = p.grad.float(), ref_grads[n]
        rel = float((a - b).norm() / (b.norm() + 1e-8))
        assert rel < 6e-2, (n, rel)


def test_param_count_llama3_8b():
    assert LlamaConfig.llama3_8b().num_params() == 8_030_261_248


def test_gate_up_swiglu_cpu_matches_unfused():
    import torch

    from tensorhive_fixed_amd.ops.linear import linear
    from tensorhive_fixed_amd.ops.mlp import gate_up_swiglu
    from tensorhive_fixed_amd.ops.swiglu import swiglu

    torch.manual_seed(0)
    h = torch.randn(64, 32, dtype=torch.bfloat16, requires_grad=True)
    w = (torch.randn(128, 32, dtype=torch.bfloat16) * 0.1).requires_grad_(True)
    g = torch.randn(64, 64, dtype=torch.bfloat16)
    gate_up_swiglu(h, w).backward(g)
    h2, w2 = h.detach().clone().requires_grad_(True), w.detach().clone().requires_grad_(True)
    swiglu(linear(h2, w2)).backward(g)
    assert torch.allclose(h.grad.float(), h2.grad.float(), atol=3e-2, rtol=2e-2)
    assert torch.allclose(w.grad.float(), w2.grad.float(), atol=3e-2, rtol=2e-2)


def test_add_norm_flow_matches_addmm_epilogue_flow_cpu(monkeypatch):
    """The default flow (residual adds fused into the next RMSNorm) and the TH_ADD_NORM=0 flow
    (residual added in the GEMM epilogue) give the same loss and gradients within bf16 noise."""
    from tensorhive_fixed_amd.models import llama3

    cfg = LlamaConfig.tiny()
    tok = torch.randint(0, cfg.vocab_size, (2, 48), generator=torch.Generator().manual_seed(1))
    tgt = torch.randint(0, cfg.vocab_size, (2, 48), generator=torch.Generator().manual_seed(2))
    out = {}
    for flag in (True, False):
        monkeypatch.setattr(llama3, "ADD_NORM", flag)
        model = Llama(cfg, device="cpu", dtype=torch.bfloat16, seed=5)
        loss = model(tok, tgt)
        loss.backward()
        out[flag] = (float(loss.detach()), {n: p.grad.float().clone() for n, p in model.named_parameters()})
    assert abs(out[True][0] - out[False][0]) < 1e-2
    for n, a in out[True][1].items():
        b = out[False][1][n]
        rel = float((a - b).norm() / (b.norm() + 1e-8))
        assert rel < 3e-2, (n, rel)


def test_lm_head_grad_is_f32_accumulated_over_chunks():
    """ADVICE r2 (cross_entropy.py:67): with an f32 main_grad (TH_GRAD_FP32) the LM-head weight
    gradient is summed over CE chunks in f32 -- each chunk's bf16 product is added as produced."""
    import types

    import torch

    from tensorhive_fixed_amd.ops.cross_entropy import linear_cross_entropy

    torch.manual_seed(0)
    T, D, V, chunk = 512, 64, 96, 16  # 32 chunks: a bf16 running sum would round 32 times
    h = torch.randn(T, D).bfloat16().requires_grad_()
    w = (torch.randn(V, D) * 0.05).bfloat16()
    tgt = torch.randint(0, V, (T,))
    ready = []
    w.main_grad = torch.zeros(V * D, dtype=torch.float32)
    w.th_store = types.SimpleNamespace(accumulating=False, mark_ready=lambda p: ready.append(p))
    linear_cross_entropy(h, w, tgt, chunk=chunk).backward()
    assert ready, "the store was told the gradient is final"
    hd, wd = h.detach().double(), w.double()
    p = torch.softmax(hd @ wd.t(), -1)
    p[torch.arange(T), tgt] -= 1
    ref = (p / T).t() @ hd
    got = w.main_grad.view(V, D).double()
    err = ((got - ref).norm() / ref.norm()).item()
    assert err < 4e-3, err  # f32 sum of bf16 chunk products: 2.0e-3; the old bf16 running sum: 6.9e-3
