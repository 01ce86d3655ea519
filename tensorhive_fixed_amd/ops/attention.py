"""Causal GQA attention on the packed qkv projection (RoPE fused into the same autograd node).

``qkv_attention(qkv, B, S, Hq, Hkv, Dh, theta)`` takes the raw ``[B*S, (Hq + 2*Hkv) * Dh]`` output
of the fused QKV GEMM, rotates q/k in place (``csrc/rope.hip``), runs causal flash attention
straight out of that packed buffer (no transposes, no q/k/v copies) and returns
``o[B*S, Hq*Dh]`` ready for the output projection.  Backward produces ``dqkv`` in the same packed
layout and applies the inverse rotation in place.

Backends:
  * ``hip``  -- ``csrc/flash_attn.hip``: MFMA (v_mfma_f32_32x32x16_bf16) flash attention fwd/bwd
               for gfx950, LSE saved for the backward recompute.  Default on device.
  * ``sdpa`` -- torch's scaled_dot_product_attention, kept ONLY as an explicitly selected
               comparison point (``TH_ATTN_BACKEND=sdpa``); never chosen silently.
  * CPU tensors always use the fp32 math reference.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn.functional as Fn

from . import _lib
from .rope import rope_inplace, rope_tables


def attention_backend() -> str:
    """``TH_ATTN_BACKEND`` if set, else ``hip``.  On a GPU the flash kernel must be in
    libthk.so: a missing or stale library raises instead of falling back to SDPA (a silent
    fallback would measure torch's attention and report it as ours).  Without a GPU the answer
    is ``hip`` too -- CPU tensors take the fp32 reference path inside :func:`qkv_attention`."""
    env = os.environ.get("TH_ATTN_BACKEND")
    if env:
        return env
    if not torch.cuda.is_available():
        return "hip"
    lib = _lib.load()  # raises with the build hint when libthk.so is missing
    if not hasattr(lib, "th_flash_attn_fwd"):
        raise RuntimeError("libthk.so has no th_flash_attn_fwd: rebuild it (python -m tensorhive_fixed_amd.ops.build) "
                           "or select TH_ATTN_BACKEND=sdpa explicitly")
    return "hip"


def attention_reference(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = True) -> torch.Tensor:
    """fp32 math reference. q [B,S,Hq,D], k/v [B,S,Hkv,D] -> [B,S,Hq,D]."""
    B, S, Hq, D = q.shape
    Hkv = k.shape[2]
    rep = Hq // Hkv
    qf = q.float().transpose(1, 2)
    kf = k.float().transpose(1, 2).repeat_interleave(rep, dim=1)
    vf = v.float().transpose(1, 2).repeat_interleave(rep, dim=1)
    s = qf @ kf.transpose(-1, -2) / math.sqrt(D)
    if causal:
        m = torch.ones(S, S, dtype=torch.bool, device=q.device).triu(1)
        s = s.masked_fill(m, float("-inf"))
    p = s.softmax(-1)
    return (p @ vf).transpose(1, 2).to(q.dtype)


def _split(qkv: torch.Tensor, B: int, S: int, Hq: int, Hkv: int, Dh: int):
    q = qkv[:, : Hq * Dh].view(B, S, Hq, Dh)
    k = qkv[:, Hq * Dh: (Hq + Hkv) * Dh].view(B, S, Hkv, Dh)
    v = qkv[:, (Hq + Hkv) * Dh:].view(B, S, Hkv, Dh)
    return q, k, v


def _sdpa(q, k, v):
    o = Fn.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                                        is_causal=True, enable_gqa=True)
    return o.transpose(1, 2)


def flash_fwd(qkv: torch.Tensor, B: int, S: int, Hq: int, Hkv: int, Dh: int,
              causal: bool = True, variant: int | None = None) -> tuple[torch.Tensor, torch.Tensor]:
    """HIP flash attention forward on the packed layout -> (o [B*S, Hq*Dh], lse [B, Hq, S] f32).

    ``variant`` (0-31, experiments only) selects a kernel variant: bit0 Q pre-scaling, bit1
    deferred rescale, bit2 double-buffered K/V tiles, bit3 KV-major block order, bit4 (with all of
    0-3) the tile DMA spread over the S chain; ``None`` = the built-in default."""
    row = qkv.shape[1]
    if qkv.dtype != torch.bfloat16 or not qkv.is_contiguous() or Dh != 128:
        raise ValueError("flash kernel needs contiguous bf16 packed qkv and head_dim 128")
    if Hq % Hkv or row != (Hq + 2 * Hkv) * Dh or qkv.shape[0] != B * S:
        raise ValueError("flash kernel: inconsistent packed-qkv geometry")
    o = torch.empty((B * S, Hq * Dh), device=qkv.device, dtype=qkv.dtype)
    lse = torch.empty((B, Hq, S), device=qkv.device, dtype=torch.float32)
    q = qkv.data_ptr()
    k = q + Hq * Dh * 2
    v = k + Hkv * Dh * 2
    _lib.call("th_flash_attn_fwd", q, k, v, o.data_ptr(), lse.data_ptr(), B, S, Hq, Hkv, Dh,
              int(causal), row, S * row, Hq * Dh, S * Hq * Dh, 1.0 / math.sqrt(Dh),
              0 if variant is None else (64 if variant == 64 else
                                         16 + (int(variant) & 15) + 32 * ((int(variant) >> 4) & 1)),
              _lib.stream_ptr(qkv.device))
    return o, lse


# launch flags of the backward (th_flash_attn_bwd), A/B aids: bit0 q-major dQ order; bit19 dQ tile DMA
# spread over the first S|dP chain; bit1 / bit2
# fused dK/dV order / priority; bit3 the fused register-staged dK/dV kernel instead of the paired
# half-width one; bit4 the one-wave-per-SIMD fused dK|dV kernel with AGPR-pinned accumulators (kf,
# S % 64 == 0; other lengths keep kh); bit5 register-staged K/V tiles in dQ and the fused dK/dV kernel (the path
# sequences whose LDS-DMA offsets overflow 32 bits take by themselves).  The 8-wave paired kernels
# of rounds 2-3 (old bits 6-8) are retired: profiles/r03_flash/retired_kc_kernels.patch
# Default: kf variant 3439 (flash_attn.hip VAR bits 0-3, 5, 6, 8, 10, 11: lse prefetch, mask in the
# initial C applied only on diagonal tiles, per-gap DMA pieces, selective pads, paired key blocks,
# barrier at the tile start, negated V, one block-code copy): whole backward 1.801 vs 1.938 ms for kh
# at B4 S4096 (profiles/r04_flash/).  Bit 19: the dQ kernel's tile DMA spread over its first S|dP
# chain (708 vs 722 us, 63.4 vs 60.5 % MFMA busy).  0 selects kh and the plain dQ kernel.
# VAR 7535 = 3439 + bit12: the S' chain starts from -lse * log2(e) written by the dQ kernel (no
# multiply per element in kf): 1023.6 vs 1048.4 us (profiles/r04_flash/kf21_*).
KF_DEFAULT_FLAGS = 16 | (7535 << 6) | (1 << 19)
_BWD_FLAGS = int(os.environ.get("TH_FA_BWD_FLAGS", str(KF_DEFAULT_FLAGS)))


# TH_FA_ROPE_FUSED=0: the rotary backward of dq / dk as its own in-place pass after the attention
# backward instead of inside the dQ and dK|dV kernels' epilogues
_ROPE_FUSED = os.environ.get("TH_FA_ROPE_FUSED", "1") == "1"


def flash_bwd(do: torch.Tensor, qkv: torch.Tensor, o: torch.Tensor, lse: torch.Tensor, B: int,
              S: int, Hq: int, Hkv: int, Dh: int, causal: bool = True, flags: int | None = None,
              rope: tuple[torch.Tensor, torch.Tensor] | None = None) -> torch.Tensor:
    """HIP flash attention backward -> dqkv in the packed layout.  ``rope`` = the (cos, sin) tables of
    ``ops/rope.py``: dq and dk come out with the rotary backward already applied (default dK|dV
    kernels: ``flags`` without bits 3 and 5)."""
    row = qkv.shape[1]
    if flags is None:
        flags = _BWD_FLAGS  # kf (flash_attn.hip falls back to kh when S % 64 != 0)
    if not do.is_contiguous():
        do = do.contiguous()
    dqkv = torch.empty_like(qkv)
    # delta = rowsum(dO * O) scratch (dQ is computed by its own query-centric kernel: no f32
    # accumulator, no atomics)
    # [0]: delta, [1]: -lse * log2(e) (written by the dQ kernel for the kf variants that read it)
    delta = torch.empty((2, B, Hq, S), device=qkv.device, dtype=torch.float32)
    q = qkv.data_ptr()
    k = q + Hq * Dh * 2
    v = k + Hkv * Dh * 2
    dq = dqkv.data_ptr()
    dk = dq + Hq * Dh * 2
    dv = dk + Hkv * Dh * 2
    if rope is not None:
        cos, sin = rope
        if cos.shape != (S, Dh // 2) or cos.dtype != torch.float32 or not cos.is_contiguous():
            raise ValueError("flash_bwd: rope tables must be contiguous f32 [S, Dh/2]")
        _lib.call("th_flash_attn_bwd_rope", q, k, v, o.data_ptr(), do.data_ptr(), lse.data_ptr(),
                  delta.data_ptr(), dq, dk, dv, B, S, Hq, Hkv, Dh, int(causal), row,
                  S * row, Hq * Dh, S * Hq * Dh, 1.0 / math.sqrt(Dh), cos.data_ptr(), sin.data_ptr(), int(flags),
                  _lib.stream_ptr(qkv.device))
        return dqkv
    _lib.call("th_flash_attn_bwd", q, k, v, o.data_ptr(), do.data_ptr(), lse.data_ptr(),
              delta.data_ptr(), None, dq, dk, dv, B, S, Hq, Hkv, Dh, int(causal), row,
              S * row, Hq * Dh, S * Hq * Dh, 1.0 / math.sqrt(Dh), int(flags), _lib.stream_ptr(qkv.device))
    return dqkv


class _QKVAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, B, S, Hq, Hkv, Dh, theta, backend):
        qkv = qkv if qkv.is_contiguous() else qkv.contiguous()
        rope_inplace(qkv, S, Hq + Hkv, Dh, theta, 1.0)
        ctx.dims = (B, S, Hq, Hkv, Dh, theta)
        ctx.backend = backend
        if qkv.is_cuda and backend == "hip":
            o, lse = flash_fwd(qkv, B, S, Hq, Hkv, Dh)
            ctx.save_for_backward(qkv, o, lse)
            return o
        q, k, v = _split(qkv, B, S, Hq, Hkv, Dh)
        if qkv.is_cuda:
            o = _sdpa(q, k, v)
        else:
            o = attention_reference(q, k, v)
        ctx.save_for_backward(qkv)
        return o.reshape(B * S, Hq * Dh)

    @staticmethod
    def backward(ctx, do):
        B, S, Hq, Hkv, Dh, theta = ctx.dims
        if ctx.backend == "hip" and do.is_cuda:
            qkv, o, lse = ctx.saved_tensors
            # rotary backward inside the kernels; the fused path needs 32-bit LDS-DMA offsets
            # (S * row * 2 B < 2^31, flash_attn.hip flash_bwd_impl), longer rows take the
            # register-staged kernels + a separate rotary pass
            row = qkv.shape[1]
            if _ROPE_FUSED and not (_BWD_FLAGS & (8 | 32)) and Dh == 128 and S * row * 2 < (1 << 31):
                tabs = rope_tables(S, Dh, theta, do.device)
                return (flash_bwd(do, qkv, o, lse, B, S, Hq, Hkv, Dh, flags=_BWD_FLAGS, rope=tabs),
                        None, None, None, None, None, None, None)
            dqkv = flash_bwd(do, qkv, o, lse, B, S, Hq, Hkv, Dh, flags=_BWD_FLAGS)
        else:
            (qkv,) = ctx.saved_tensors
            with torch.enable_grad():
                x = qkv.detach().requires_grad_(True)
                q, k, v = _split(x, B, S, Hq, Hkv, Dh)
                o = _sdpa(q, k, v) if x.is_cuda else attention_reference(q, k, v)
                (dqkv,) = torch.autograd.grad(o.reshape(B * S, Hq * Dh), x, do)
        rope_inplace(dqkv, S, Hq + Hkv, Dh, theta, -1.0)
        return dqkv, None, None, None, None, None, None, None


def qkv_attention(qkv: torch.Tensor, B: int, S: int, Hq: int, Hkv: int, Dh: int, theta: float,
                  backend: str | None = None) -> torch.Tensor:
    return _QKVAttention.apply(qkv, B, S, Hq, Hkv, Dh, theta, backend or attention_backend())
