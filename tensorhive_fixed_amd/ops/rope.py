"""Rotary embedding tables and the in-place RoPE op on the packed qkv projection.

The cos/sin table is computed once per (seq_len, head_dim, theta, device) in fp64 on the host
and cached as f32 on the device (``csrc/rope.hip`` reads it; no on-device trig).
Convention: rotate-half pairs ``(i, i + Dh/2)``, Llama-3 ``theta = 500000``.
"""
from __future__ import annotations

import threading

import torch

from . import _lib

_cache: dict[tuple, tuple[torch.Tensor, torch.Tensor]] = {}
_cache_lock = threading.Lock()


def rope_tables(S: int, Dh: int, theta: float, device: torch.device) -> tuple[torch.Tensor, torch.Tensor]:
    key = (S, Dh, float(theta), str(device))
    with _cache_lock:
        hit = _cache.get(key)
        if hit is not None:
            return hit
        inv = 1.0 / (theta ** (torch.arange(0, Dh, 2, dtype=torch.float64) / Dh))
        ang = torch.arange(S, dtype=torch.float64)[:, None] * inv[None, :]
        tabs = (ang.cos().float().contiguous().to(device), ang.sin().float().contiguous().to(device))
        _cache[key] = tabs
        return tabs


def rope_reference_(qkv: torch.Tensor, S: int, n_rot_heads: int, Dh: int, theta: float,
                    sign: float = 1.0) -> torch.Tensor:
    """In-place fp32 reference on a [T, row] tensor (used on CPU and as the test oracle)."""
    T = qkv.shape[0]
    cos, sin = rope_tables(S, Dh, theta, qkv.device)
    pos = torch.arange(T, device=qkv.device) % S
    c = cos[pos][:, None, :]
    s = sin[pos][:, None, :] * sign
    x = qkv[:, : n_rot_heads * Dh].view(T, n_rot_heads, Dh).float()
    x1, x2 = x[..., : Dh // 2], x[..., Dh // 2:]
    y = torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1)
    qkv[:, : n_rot_heads * Dh] = y.reshape(T, n_rot_heads * Dh).to(qkv.dtype)
    return qkv


def rope_inplace(qkv2d: torch.Tensor, S: int, n_rot_heads: int, Dh: int, theta: float,
                 sign: float = 1.0) -> torch.Tensor:
    """Rotate the first ``n_rot_heads`` heads of every row of ``qkv2d`` [T, row] in place."""
    if not qkv2d.is_cuda:
        return rope_reference_(qkv2d, S, n_rot_heads, Dh, theta, sign)
    if qkv2d.dtype != torch.bfloat16 or not qkv2d.is_contiguous() or Dh % 16:
        raise ValueError("rope kernel needs a contiguous bf16 [T, row] tensor and Dh % 16 == 0")
    T, row = qkv2d.shape
    if n_rot_heads * Dh > row:
        raise ValueError("rope: more rotated heads than the row holds")
    cos, sin = rope_tables(S, Dh, theta, qkv2d.device)
    _lib.call("th_rope_inplace", qkv2d.data_ptr(), cos.data_ptr(), sin.data_ptr(), T, S,
              n_rot_heads, row, Dh, float(sign), _lib.stream_ptr(qkv2d.device))
    return qkv2d
