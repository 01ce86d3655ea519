"""Weight-gradient GEMM ``C (+)= Aᵀ·B`` for operands stored [tokens, features] (``csrc/gemm_tn.hip``).

``dW = dYᵀ X`` sums over tokens, the slow dimension of both activation tensors.  hipBLASLt's kernel
for that operand layout reaches 1.0-1.2 PFLOP/s on the Llama-3-8B projection shapes; the
gfx950 kernel stages k-rows with LDS-DMA and reads MFMA operands with the hardware transpose read,
so no operand is transposed in memory.  Shapes it does not tile (M or N not a multiple of 256,
K not a multiple of 64 x split) fall back to ``torch.mm``.
"""
from __future__ import annotations

import os
from contextlib import contextmanager

import torch

from . import _lib

_TILE, _TK = 256, 64


def supported(m: int, n: int, k: int, splitk: int = 1) -> bool:
    return m % _TILE == 0 and n % _TILE == 0 and k % (_TK * splitk) == 0


# CUs a launch may count on.  256 on an idle chip; during an N > 1 backward RCCL's channel kernels hold
# some (one workgroup per channel per collective), and the trainer lowers the budget for backward with
# :func:`cu_budget` (parallel/comm_emu.py rehearses that footprint on one GPU, profiles/r06_comm/).
_CUS_DEFAULT = int(os.environ.get("TH_GEMM_CUS", "256"))
_cus = _CUS_DEFAULT


def compute_cus() -> int:
    return _cus


@contextmanager
def cu_budget(cus: int | None):
    """Plan TN launches for ``cus`` available CUs inside the block (None: leave the budget unchanged)."""
    global _cus
    if cus is None:
        yield
        return
    if not 1 <= int(cus) <= 511:
        raise ValueError(f"cu_budget: {cus} not in 1..511")
    prev, _cus = _cus, int(cus)
    try:
        yield
    finally:
        _cus = prev


_SPLIT_COST = 0.03  # per split launch, in tile times: the f32 slab round trip + the reduce (profiles/r05_gemm)


def plan_time(tiles: int, splitk: int, dp: bool, cus: int) -> float:
    """Modelled launch time in whole-tile times: equal-length workgroups dispatched in rounds over ``cus``
    CUs.  ``dp``: full rounds of whole tiles, then the remainder tiles split ``splitk`` ways."""
    if splitk == 1:
        return float(-(-tiles // cus))
    if dp:
        full = tiles // cus * cus
        rem = tiles - full
        rounds = full // cus
        return rounds + (-(-rem * splitk // cus) / splitk + _SPLIT_COST if rem else 0.0)
    return -(-tiles * splitk // cus) / splitk + _SPLIT_COST


def tn_plan(m: int, n: int, k: int, cus: int | None = None) -> tuple[int, bool]:
    """(splitk, data-parallel + split remainder) with the least modelled time on ``cus`` CUs.  A plan with
    more splits must win by 2 % (the model ignores per-piece prologue cost), and a piece keeps >= 2048
    k-rows.  ``TH_GEMM_TN_SPLITK`` forces the split factor.  At 256 CUs this reproduces the round-5 choices
    on every Llama-3-8B weight-gradient shape (tests/test_gemm_tn_cpu.py)."""
    cus = compute_cus() if cus is None else int(cus)
    env = os.environ.get("TH_GEMM_TN_SPLITK")
    tiles = (m // _TILE) * (n // _TILE)
    if env:
        return int(env), int(env) > 1
    best, best_t = (1, False), plan_time(tiles, 1, False, cus)
    for s in (2, 4, 8):
        if not supported(m, n, k, s) or k // s < 2048:
            continue
        for dp in (True, False):
            t = plan_time(tiles, s, dp, cus)
            if t < best_t * 0.98:
                best, best_t = (s, dp), t
    return best


def default_splitk(m: int, n: int, k: int, cus: int | None = None) -> int:
    return tn_plan(m, n, k, cus)[0]


def workspace_floats(m: int, n: int, splitk: int, dp: bool, cus: int) -> int:
    """f32 slab the launch needs: (split tiles) x splitk x 256 x 256 (csrc/gemm_tn.hip:th_gemm_tn)."""
    if splitk <= 1:
        return 0
    tiles = (m // _TILE) * (n // _TILE)
    split_tiles = tiles - (tiles // cus * cus if dp else 0)
    return split_tiles * splitk * _TILE * _TILE


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
    cus = compute_cus()
    if splitk is None:
        sk, dp = tn_plan(M, N, K, cus)
    else:
        sk, dp = int(splitk), int(splitk) > 1
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
    # mode 9 = every tile split (or none); mode 10 = data-parallel whole tiles, split-K remainder
    dp = dp and mode == 10
    nws = workspace_floats(M, N, sk, dp, cus)
    ws = torch.empty(nws, device=a.device, dtype=torch.float32) if nws else None
    flags = _MODES[10 if dp else 9] | (int(band) << 8) | ((cus & 511) << 12)
    _lib.call("th_gemm_tn", a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), out.data_ptr(), out.stride(0),
              M, N, K, int(accumulate), sk, None if ws is None else ws.data_ptr(), nws, flags,
              _lib.stream_ptr(a.device))
    return out
