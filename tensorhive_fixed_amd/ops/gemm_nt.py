"""K-contiguous GEMM ``C (+)= A·Bᵀ`` (``csrc/gemm_nt.hip``): the forward ``x Wᵀ`` and input-gradient
``dY (Wᵀ)ᵀ`` form of every Llama linear layer, on the gfx950 machinery of the TN weight-grad
kernel.  Shapes it does not tile fall back to ``torch.mm``."""
from __future__ import annotations

import torch

from . import _lib

_TILE, _TK = 256, 32


def supported(m: int, n: int, k: int) -> bool:
    return m % _TILE == 0 and n % _TILE == 0 and k % _TK == 0


def gemm_nt_(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, accumulate: bool = False,
             mfma16: bool = False, variant: int = 0) -> torch.Tensor:
    """``out[M, N] (+)= a[M, K] @ b[N, K]ᵀ`` (bf16 in / out, f32 accumulation).

    ``variant`` (1-7, 16x16x32 kernel only) selects the round-3 probe variants of
    ``csrc/gemm_nt.hip``: bit 0 = 3-deep DMA in a 5-stage ring, bit 1 = s_setprio around the MFMA
    blocks, bit 2 = output through LDS as 16-B row stores."""
    M, K = a.shape
    N, K2 = b.shape
    if K2 != K or tuple(out.shape) != (M, N):
        raise ValueError(f"gemm_nt_: shapes {tuple(a.shape)}, {tuple(b.shape)} -> {tuple(out.shape)}")
    ok = (a.is_cuda and a.dtype == b.dtype == out.dtype == torch.bfloat16 and supported(M, N, K)
          and a.stride(1) == 1 and b.stride(1) == 1 and out.stride(1) == 1)
    if not ok:
        if accumulate:
            out.addmm_(a, b.t())
        else:
            torch.mm(a, b.t(), out=out)
        return out
    _lib.call("th_gemm_nt", a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), out.data_ptr(), out.stride(0),
              M, N, K, int(accumulate), int(mfma16) | ((int(variant) & 7) << 1) , _lib.stream_ptr(a.device))
    return out
