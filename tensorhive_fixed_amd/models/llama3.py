"""Llama-3 decoder (8B configuration by default) built on the gfx950 kernels of ``ops/``.

This is the N07 payload model of SURVEY §2.12 (the reference has no model code at all; it only
*launches* user trainings -- ``examples/PyTorch/README.md:30-64``).  Architecture facts:
L = 32, d = 4096, 32 query / 8 kv heads of 128, FFN 14336 (SwiGLU), vocab 128256,
RoPE theta = 5e5, RMSNorm eps = 1e-5, untied LM head.

Per block the data flow is chosen for MI355X:
  x -> RMSNorm (HIP) -> ONE fused QKV GEMM [4096 -> 6144] -> RoPE in place + causal GQA flash
  attention straight out of the packed qkv buffer (HIP, MFMA) -> O-proj GEMM -> residual add
  fused INTO the next RMSNorm (``rmsnorm_add_fork``: one kernel reads the projection and the
  residual stream, writes their bf16 sum and the normalised row) -> ONE fused gate|up GEMM
  [4096 -> 28672] -> SwiGLU (HIP) -> down GEMM, whose residual add is again taken by the next
  block's (or the final) RMSNorm.  ``TH_ADD_NORM=0`` selects the older flow, where the O-proj and
  down GEMMs add the residual in an ``addmm`` beta = 1 epilogue; both flows are checked against
  each other in ``tests/test_rmsnorm_add.py``.
The LM head is fused with the cross-entropy (chunked, logits never materialised whole).
Every weight gradient is written by its producing GEMM/kernel into the flat DDP buffer.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

import torch
from torch import nn

from ..ops.attention import qkv_attention
from ..ops.cross_entropy import linear_cross_entropy
from ..ops.embedding import embedding
from ..ops.linear import linear
from ..ops.mlp import gate_up_swiglu
from ..ops.rmsnorm import rmsnorm, rmsnorm_add_fork, rmsnorm_fork
from ..ops.swiglu import swiglu


@dataclass
class LlamaConfig:
    vocab_size: int = 128256
    dim: int = 4096
    n_layers: int = 32
    n_heads: int = 32
    n_kv_heads: int = 8
    ffn_dim: int = 14336
    rope_theta: float = 500000.0
    norm_eps: float = 1e-5
    max_seq_len: int = 8192
    ce_chunk: int = 4096

    @property
    def head_dim(self) -> int:
        return self.dim // self.n_heads

    @classmethod
    def llama3_8b(cls) -> "LlamaConfig":
        # TH_CE_CHUNK: tokens per LM-head + cross-entropy chunk (logits of one chunk: chunk x 128256 bf16)
        return cls(ce_chunk=int(os.environ.get("TH_CE_CHUNK", "4096")))

    @classmethod
    def tiny(cls) -> "LlamaConfig":
        """Test-size model with the same head geometry (head_dim 128, GQA 4:1)."""
        return cls(vocab_size=512, dim=256, n_layers=2, n_heads=2, n_kv_heads=1, ffn_dim=512,
                   max_seq_len=512, ce_chunk=64)

    @classmethod
    def named(cls, name: str) -> "LlamaConfig":
        table = {"llama3-8b": cls.llama3_8b, "llama3_8b": cls.llama3_8b, "tiny": cls.tiny,
                 "llama3-1b-shape": lambda: cls(dim=2048, n_layers=16, n_heads=16, n_kv_heads=4,
                                                ffn_dim=8192)}
        return table[name.lower()]()

    def num_params(self) -> int:
        d, f, v, L = self.dim, self.ffn_dim, self.vocab_size, self.n_layers
        kv = self.n_kv_heads * self.head_dim
        per_layer = d * (d + 2 * kv) + d * d + 2 * f * d + f * d + 2 * d
        return v * d * 2 + L * per_layer + d

    def flops_per_token(self, seq_len: int) -> float:
        """Training FLOPs per token (fwd + bwd = 3x fwd), causal attention counted at half."""
        n_mat = self.num_params() - self.vocab_size * self.dim  # embedding is a gather
        attn = 2 * 2 * self.n_layers * seq_len * self.dim / 2  # QK^T + PV, causal half
        return 6 * n_mat + 3 * attn


# projections whose weight grad runs on transposed operand copies (ops/linear.py): where the GEMM
# speed-up outweighs the transposes (measured: profiles/r01_gemm/)
WGRAD_NT = set(filter(None, os.environ.get("TH_WGRAD_NT_LAYERS", "w13").split(",")))
# projections whose weight grad runs on the gfx950 TN kernel (ops/gemm_tn.py), measured faster than
# hipBLASLt there (scripts/bench_gemm_tn.py)
WGRAD_TN = set(filter(None, os.environ.get("TH_WGRAD_TN_LAYERS", "wqkv,wo,w2").split(",")))
_FORK = os.environ.get("TH_RMSNORM_FORK", "1") == "1"


# residual adds fused into the following RMSNorm (rmsnorm_add_fork) instead of beta=1 GEMM epilogues
ADD_NORM = _FORK and os.environ.get("TH_ADD_NORM", "1") == "1"


def _norm(x, w, eps):
    if _FORK:
        return rmsnorm_fork(x, w, eps)
    return rmsnorm(x, w, eps), x


class LlamaBlock(nn.Module):
    def __init__(self, cfg: LlamaConfig, device, dtype):
        super().__init__()
        d, hd = cfg.dim, cfg.head_dim
        qkv_out = (cfg.n_heads + 2 * cfg.n_kv_heads) * hd
        self.cfg = cfg
        self.attn_norm = nn.Parameter(torch.ones(d, device=device, dtype=dtype))
        self.wqkv = nn.Parameter(torch.empty(qkv_out, d, device=device, dtype=dtype))
        self.wo = nn.Parameter(torch.empty(d, cfg.n_heads * hd, device=device, dtype=dtype))
        self.ffn_norm = nn.Parameter(torch.ones(d, device=device, dtype=dtype))
        self.w13 = nn.Parameter(torch.empty(2 * cfg.ffn_dim, d, device=device, dtype=dtype))
        self.w2 = nn.Parameter(torch.empty(d, cfg.ffn_dim, device=device, dtype=dtype))

    def forward(self, x: torch.Tensor, B: int, S: int, pending: torch.Tensor | None = None):
        """Without ADD_NORM: returns the block output.  With it: returns ``(y, x)``, the MLP-down
        projection and the residual stream, whose sum the next norm forms (``pending`` of the next
        block / the final norm)."""
        c = self.cfg
        # rmsnorm_fork: the residual gradient is added inside the RMSNorm backward kernel
        if pending is not None:
            h, x = rmsnorm_add_fork(pending, x, self.attn_norm, c.norm_eps)
        else:
            h, x = _norm(x, self.attn_norm, c.norm_eps)
        qkv = linear(h, self.wqkv, wgrad_nt="wqkv" in WGRAD_NT, wgrad_tn="wqkv" in WGRAD_TN)
        o = qkv_attention(qkv, B, S, c.n_heads, c.n_kv_heads, c.head_dim, c.rope_theta)
        if ADD_NORM:
            y = linear(o, self.wo, wgrad_nt="wo" in WGRAD_NT, wgrad_tn="wo" in WGRAD_TN)
            h, x = rmsnorm_add_fork(y, x, self.ffn_norm, c.norm_eps)
        else:
            x = linear(o, self.wo, residual=x, wgrad_nt="wo" in WGRAD_NT, wgrad_tn="wo" in WGRAD_TN)
            h, x = _norm(x, self.ffn_norm, c.norm_eps)
        if "w13" in WGRAD_NT:  # fused gate|up + SwiGLU node: transposed dGU from the SwiGLU kernel
            a = gate_up_swiglu(h, self.w13)
        else:
            a = swiglu(linear(h, self.w13))
        if ADD_NORM:
            return linear(a, self.w2, wgrad_nt="w2" in WGRAD_NT, wgrad_tn="w2" in WGRAD_TN), x
        return linear(a, self.w2, residual=x, wgrad_nt="w2" in WGRAD_NT, wgrad_tn="w2" in WGRAD_TN)


class Llama(nn.Module):
    def __init__(self, cfg: LlamaConfig, device="cpu", dtype=torch.bfloat16, seed: int = 0):
        super().__init__()
        self.cfg = cfg
        self.tok_emb = nn.Parameter(torch.empty(cfg.vocab_size, cfg.dim, device=device, dtype=dtype))
        self.layers = nn.ModuleList([LlamaBlock(cfg, device, dtype) for _ in range(cfg.n_layers)])
        self.norm = nn.Parameter(torch.ones(cfg.dim, device=device, dtype=dtype))
        self.lm_head = nn.Parameter(torch.empty(cfg.vocab_size, cfg.dim, device=device, dtype=dtype))
        # ZeRO-1 hook: called with the parameters about to be read, so a sharded store can make the
        # stream wait for exactly the all-gather buckets holding them (parallel/flat.py)
        self.param_gate = None
        self.reset_parameters(seed)

    @torch.no_grad()
    def reset_parameters(self, seed: int = 0) -> None:
        g = torch.Generator(device=self.tok_emb.device)
        g.manual_seed(seed)
        std = 0.02
        out_std = std / math.sqrt(2 * self.cfg.n_layers)
        self.tok_emb.normal_(0, std, generator=g)
        self.lm_head.normal_(0, std, generator=g)
        for blk in self.layers:
            blk.wqkv.normal_(0, std, generator=g)
            blk.w13.normal_(0, std, generator=g)
            blk.wo.normal_(0, out_std, generator=g)
            blk.w2.normal_(0, out_std, generator=g)

    def params_in_backward_order(self) -> list[tuple[str, nn.Parameter, bool]]:
        """(name, param, weight_decay?) in the order backward produces their gradients."""
        out = [("lm_head", self.lm_head, True), ("norm", self.norm, False)]
        for i in reversed(range(len(self.layers))):
            b = self.layers[i]
            out += [(f"layers.{i}.w2", b.w2, True), (f"layers.{i}.w13", b.w13, True),
                    (f"layers.{i}.ffn_norm", b.ffn_norm, False), (f"layers.{i}.wo", b.wo, True),
                    (f"layers.{i}.wqkv", b.wqkv, True), (f"layers.{i}.attn_norm", b.attn_norm, False)]
        out.append(("tok_emb", self.tok_emb, True))
        return out

    def hidden(self, tokens: torch.Tensor) -> torch.Tensor:
        B, S = tokens.shape
        gate = self.param_gate
        if gate is not None:
            gate(self.tok_emb)
        x = embedding(tokens, self.tok_emb).view(B * S, self.cfg.dim)
        pending = None
        for blk in self.layers:
            if gate is not None:
                gate(blk.attn_norm, blk.wqkv, blk.wo, blk.ffn_norm, blk.w13, blk.w2)
            if ADD_NORM:
                pending, x = blk(x, B, S, pending)
            else:
                x = blk(x, B, S)
        if gate is not None:
            gate(self.norm, self.lm_head)
        if pending is not None:
            return rmsnorm_add_fork(pending, x, self.norm, self.cfg.norm_eps)[0]
        return rmsnorm(x, self.norm, self.cfg.norm_eps)

    def forward(self, tokens: torch.Tensor, targets: torch.Tensor | None = None,
                n_valid: int | None = None) -> torch.Tensor:
        """Returns the mean CE loss when ``targets`` is given, else the final hidden states."""
        h = self.hidden(tokens)
        if targets is None:
            return h
        return linear_cross_entropy(h, self.lm_head, targets.reshape(-1), self.cfg.ce_chunk,
                                    n_valid=n_valid)

    @torch.no_grad()
    def logits(self, tokens: torch.Tensor) -> torch.Tensor:
        return torch.mm(self.hidden(tokens), self.lm_head.t()).view(*tokens.shape, -1)
