"""Weight-gradient GEMM ``C (+)= Aᵀ·B`` for operands stored [tokens, features] (``csrc/gemm_tn.hip``).

``dW = dYᵀ X`` sums over tokens, the slow dimension of both activation tensors.  hipBLASLt's kernel
for that operand layout reaches 1.0-1.2 PFLOP/s on the Llama-3-8B projection shapes; the
gfx950 kernel stages k-rows with LDS-DMA and reads MFMA operands with the hardware transpose read,
so no operand is transposed in memory.  Shapes it does not tile (M or N not a multiple of 256,
K not a multiple of 64 x split) fall back to ``torch.mm``.
"""
from __future__ import annotations

import os

import torch

from . import _lib

_TILE, _TK = 256, 64


def supported(m: int, n: int, k: int, splitk: int = 1) -> bool:
    return m % _TILE == 0 and n % _TILE == 0 and k % (_TK * splitk) == 0


def default_splitk(m: int, n: int, k: int, cus: int = 256) -> int:
    """Split K when the output tiles leave a ragged last round on the 256 CUs (1 workgroup/CU)."""
    env = os.environ.get("TH_GEMM_TN_SPLITK")
    if env:
        return int(env)
    tiles = (m // _TILE) * (n // _TILE)
    best, best_eff = 1, 0.0
    for s in (1, 2, 3, 4):
        if not supported(m, n, k, s):
            continue
        rounds = -(-tiles * s // cus)
        eff = tiles * s / (rounds * cus) - 0.03 * (s > 1)  # the slab round trip costs a few percent
        if eff > best_eff + 1e-9:
            best, best_eff = s, eff
    return best


# launch mode of the hb kernel (csrc/gemm_tn.hip, the only schedule since round 5; the round-1..4 modes 0-8
# were retired, profiles/r05_gemm/): 9 = whole-K tiles, or split-K for every tile when splitk > 1;
# 10 = whole tiles data-parallel on every CU, split-K only for the remainder tiles
_MODES = {9: 64, 10: 192}
_PP = int(os.environ.get("TH_GEMM_TN_PP", "10"))  # hb + data-parallel/remainder split: profiles/r05_gemm


_BAND_POLICY = os.environ.get("TH_GEMM_TN_BAND_POLICY", "1") == "1"


def default_band(m: int, n: int, k: int) -> int:
    """XCD band height (output-tile rows per band, 1-15; 0 = the compiled default, 8) measured per shape
    class (profiles/r05_gemm/tn_band2.jsonl, mode 10): the 8-row default is best or within 0.3 % on
    wqkv / wo / w2; the gate|up gradient (a tall 28672 x 4096 output over K 32768) runs 1.0 % faster in
    one-row bands, and the LM-head chunk (128256 x 4096 over K 4096) 0.9 % faster in 4-row bands."""
    if not _BAND_POLICY:
        return 0
    if m >= 16384 and n <= 4096 and k >= 16384:
        return 1
    if m >= 65536 and k <= 8192:
        return 4
    return 0


def gemm_tn_(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, accumulate: bool = False,
             splitk: int | None = None, pingpong: int | None = None, band: int | None = None) -> torch.Tensor:
    """``out[M, N] (+)= a[K, M]ᵀ @ b[K, N]`` (bf16 in / out, f32 accumulation).  ``band``: XCD band
    height in output-tile rows for the hb modes, 0-15 (0 = the compiled default; None = :func:`default_band`)."""
    K, M = a.shape
    K2, N = b.shape
    if K2 != K or tuple(out.shape) != (M, N):
        raise ValueError(f"gemm_tn_: shapes {tuple(a.shape)}, {tuple(b.shape)} -> {tuple(out.shape)}")
    mode = int(_PP if pingpong is None else pingpong)
    if mode not in _MODES:
        raise ValueError(f"gemm_tn_: launch mode {mode} not in {sorted(_MODES)}")
    if band is not None and not 0 <= int(band) <= 15:
        raise ValueError(f"gemm_tn_: band {band} not in 0..15")
    if not a.is_cuda:
        r = a.float().t() @ b.float()
        out.copy_((out.float() + r if accumulate else r).to(out.dtype))
        return out
    sk = default_splitk(M, N, K) if splitk is None else splitk
    ok = (a.dtype == b.dtype == out.dtype == torch.bfloat16 and supported(M, N, K, sk)
          and a.stride(1) == 1 and b.stride(1) == 1 and out.stride(1) == 1)
    if not ok:
        if accumulate:
            out.addmm_(a.t(), b)
        else:
            torch.mm(a.t(), b, out=out)
        return out
    if band is None:
        band = default_band(M, N, K)
    ws = torch.empty(sk * M * N, device=a.device, dtype=torch.float32) if sk > 1 else None
    _lib.call("th_gemm_tn", a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), out.data_ptr(), out.stride(0),
              M, N, K, int(accumulate), sk, None if ws is None else ws.data_ptr(),
              _MODES[mode] | (int(band) << 8), _lib.stream_ptr(a.device))
    return out
