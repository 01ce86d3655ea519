"""K-contiguous GEMM ``C (+)= A·Bᵀ`` (``csrc/gemm_nt.hip``): the forward ``x Wᵀ`` and input-gradient
``dY (Wᵀ)ᵀ`` form of every Llama linear layer -- one wave per SIMD, 256 x 256 x 64 tiles, the
accumulators pinned in the AGPR file by inline-asm MFMAs.  Shapes it does not tile fall back to
``torch.mm`` (hipBLASLt)."""
from __future__ import annotations

import os

import torch

from . import _lib

_TILE, _TK = 256, 64

# TH_GEMM_NT=1 routes the payload's forward / input-gradient GEMMs through this kernel
# (ops/linear.py, ops/mlp.py); the default keeps hipBLASLt until a same-box A/B says otherwise
ENABLED = os.environ.get("TH_GEMM_NT", "0") == "1"


def supported(m: int, n: int, k: int) -> bool:
    return m % _TILE == 0 and n % _TILE == 0 and k % _TK == 0


def usable(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor) -> bool:
    M, K = a.shape
    N = b.shape[0]
    return (a.is_cuda and a.dtype == b.dtype == out.dtype == torch.bfloat16 and supported(M, N, K)
            and a.stride(1) == 1 and b.stride(1) == 1 and out.stride(1) == 1
            and a.stride(0) % 8 == 0 and b.stride(0) % 8 == 0 and out.stride(0) % 8 == 0
            and a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0 and out.data_ptr() % 16 == 0
            and 16 * max(a.stride(0), b.stride(0)) < (1 << 31))


# schedule variant 8 (side work interleaved per MFMA) measured best on every shape (profiles/r04_gemm)
_VARIANT = int(os.environ.get("TH_GEMM_NT_VARIANT", "8"))


def gemm_nt_(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, accumulate: bool = False,
             variant: int | None = None) -> torch.Tensor:
    """``out[M, N] (+)= a[M, K] @ b[N, K]ᵀ`` (bf16 in / out, f32 accumulation).  ``variant`` (0, 1, 8,
    16, 17, 20; beta 0 only): schedule variants of ``csrc/gemm_nt.hip`` for A/B runs."""
    M, K = a.shape
    N, K2 = b.shape
    if K2 != K or tuple(out.shape) != (M, N):
        raise ValueError(f"gemm_nt_: shapes {tuple(a.shape)}, {tuple(b.shape)} -> {tuple(out.shape)}")
    if not usable(a, b, out):
        if accumulate:
            out.addmm_(a, b.t())
        else:
            torch.mm(a, b.t(), out=out)
        return out
    _lib.call("th_gemm_nt", a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), out.data_ptr(), out.stride(0),
              M, N, K, int(accumulate), _VARIANT if variant is None else int(variant) & 127, _lib.stream_ptr(a.device))
    return out


def mm_nt(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """``a @ b.t()`` into a new tensor (the kernel when it tiles the shape, else hipBLASLt)."""
    out = torch.empty((a.shape[0], b.shape[0]), device=a.device, dtype=a.dtype)
    return gemm_nt_(a, b, out)


def nt_mm(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """``a @ b.t()`` (into ``out`` when given) for the payload: this kernel when ``TH_GEMM_NT=1`` and
    it tiles the shape, else hipBLASLt."""
    if ENABLED and a.is_cuda:
        o = out if out is not None else torch.empty((a.shape[0], b.shape[0]), device=a.device, dtype=a.dtype)
        if usable(a, b, o):
            return gemm_nt_(a, b, o)
    if out is not None:
        return torch.mm(a, b.t(), out=out)
    return torch.mm(a, b.t())


def nt_into(a: torch.Tensor, b: torch.Tensor):
    """A weight-gradient ``write`` callback (``ops/_grad.deliver``) computing ``a @ b.t()``."""

    def _w(out: torch.Tensor, accumulate: bool) -> None:
        o2 = out.view(a.shape[0], b.shape[0])
        if ENABLED and usable(a, b, o2):
            gemm_nt_(a, b, o2, accumulate=accumulate)
        elif accumulate:
            o2.addmm_(a, b.t())
        else:
            torch.mm(a, b.t(), out=o2)

    return _w
