"""Weight-gradient GEMM ``C (+)= Aᵀ·B`` for operands stored [tokens, features] (``csrc/gemm_tn.hip``).

``dW = dYᵀ X`` sums over tokens, the slow dimension of both activation tensors.  hipBLASLt's kernel
for that operand layout reaches 1.0-1.2 PFLOP/s on the Llama-3-8B projection shapes; the
gfx950 kernel stages k-rows with LDS-DMA and reads MFMA operands with the hardware transpose read,
so no operand is transposed in memory.  Shapes it does not tile (M or N not a multiple of 256,
K not a multiple of 64 x split) fall back to ``torch.mm``.
"""
from __future__ import annotations

import functools
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


_PIECE_COST = 0.01   # per split-K piece, in whole-tile times: its prologue and the f32 slab write
_REDUCE_COST = 0.02  # the per-tile reduce kernel after a launch with split tiles
_CHIP_CUS = 256


def plan_time(tiles: int, splitk: int, full: int, cus: int) -> float:
    """Modelled time of one launch in whole-tile times: ``full`` whole-K tiles, then ``tiles - full`` tiles
    split ``splitk`` ways, dispatched in grid order onto ``cus`` CUs, each workgroup to the CU that frees
    first (csrc/gemm_tn.hip: one grid holds both kinds)."""
    import heapq

    rem = tiles - full
    if rem and splitk == 1:
        full, rem = tiles, 0
    if cus >= full + rem * splitk:  # everything in one wave
        t = 1.0 if full else 0.0
        return max(t, (1.0 / splitk + _PIECE_COST) if rem else 0.0) + (_REDUCE_COST if rem else 0.0)
    whole_rounds, left = divmod(full, cus)
    t0 = float(whole_rounds)
    free = [t0] * (cus - left) + [t0 + 1.0] * left
    heapq.heapify(free)
    piece = 1.0 / splitk + _PIECE_COST
    end = max(free) if left else t0
    for _ in range(rem * splitk):
        t = heapq.heappop(free) + piece
        end = max(end, t)
        heapq.heappush(free, t)
    return end + (_REDUCE_COST if rem else 0.0)


def tn_plan(m: int, n: int, k: int, cus: int | None = None) -> tuple[int, int]:
    """(splitk, whole tiles) of the launch.  ``cus``: the CUs the launch may have to live with (default the
    :func:`cu_budget`); below 256 the plan weighs its time on ``cus`` CUs (RCCL's channels holding the rest)
    and on the idle chip equally, each against its ideal ``tiles / CUs``.  A plan with more splits must win by
    2 % (the model ignores everything but rounds), and a piece keeps >= 2048 k-rows.
    ``TH_GEMM_TN_SPLITK`` forces the split factor (every tile split).  At 256 CUs this reproduces the round-5
    choices on every Llama-3-8B weight-gradient shape (tests/test_gemm_tn_cpu.py)."""
    cmin = compute_cus() if cus is None else int(cus)
    env = os.environ.get("TH_GEMM_TN_SPLITK")
    if env:
        s = int(env)
        return s, ((m // _TILE) * (n // _TILE) if s == 1 else 0)
    return _tn_plan(m, n, k, cmin)


@functools.lru_cache(maxsize=1024)
def _tn_plan(m: int, n: int, k: int, cmin: int) -> tuple[int, int]:
    """Cached: the list-schedule model runs in Python and a launch must not wait for it (the step issues
    ~130 TN launches; planning each one again cost milliseconds of host time per launch)."""
    tiles = (m // _TILE) * (n // _TILE)
    cs = sorted({cmin, _CHIP_CUS}) if cmin < _CHIP_CUS else [cmin]
    if tiles > 2 * cmin:
        # measured (profiles/r06_comm/micro2): with 8-32 CUs held, the 256-CU plan of the gate|up (1792 tiles)
        # and down (896) gradients beats every re-plan (6.0 vs 6.1 ms, 2.9 vs 3.2 ms): their split pieces cost
        # more than the spilled round; only wo (256 tiles) and wqkv (384) gain (0.93 vs 1.25, 1.49 vs 1.63 ms)
        cs = [_CHIP_CUS]

    def cost(s: int, full: int) -> float:
        return sum(plan_time(tiles, s, full, c) / (tiles / c) for c in cs) / len(cs)

    best, best_c = (1, tiles), cost(1, tiles)
    for s in (2, 4, 8):
        if not supported(m, n, k, s) or k // s < 2048:
            continue
        fulls = {0} | {tiles - tiles % c for c in cs} | {max(0, tiles - tiles % c - c) for c in cs}
        for full in sorted(fulls, reverse=True):
            if full >= tiles:
                continue
            c = cost(s, full)
            if c < best_c * 0.98:
                best, best_c = (s, full), c
    return best


def default_splitk(m: int, n: int, k: int, cus: int | None = None) -> int:
    return tn_plan(m, n, k, cus)[0]


def workspace_floats(m: int, n: int, splitk: int, full: int) -> int:
    """f32 slab the launch needs: (split tiles) x splitk x 256 x 256 (csrc/gemm_tn.hip:th_gemm_tn)."""
    if splitk <= 1:
        return 0
    tiles = (m // _TILE) * (n // _TILE)
    return (tiles - full) * splitk * _TILE * _TILE


# launch mode of the hb kernel (csrc/gemm_tn.hip, the only schedule since round 5; the round-1..4 modes 0-8
# were retired, profiles/r05_gemm/): 9 = whole-K tiles, or split-K for every tile when splitk > 1;
# 10 = the planned mix: whole tiles first, split-K pieces of the remaining tiles in the same grid
_MODES = {9: 64, 10: 64}
_PP = int(os.environ.get("TH_GEMM_TN_PP", "10"))


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
    tiles = (M // _TILE) * (N // _TILE)
    if splitk is None and mode == 10:
        sk, full = tn_plan(M, N, K)
    elif splitk is None:
        sk, full = 1, tiles
    else:
        sk = int(splitk)
        full = tiles if sk == 1 else (tn_full_for(M, N, sk) if mode == 10 else 0)
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
    nws = workspace_floats(M, N, sk, full)
    ws = torch.empty(nws, device=a.device, dtype=torch.float32) if nws else None
    _lib.call("th_gemm_tn", a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), out.data_ptr(), out.stride(0),
              M, N, K, int(accumulate), sk, full, None if ws is None else ws.data_ptr(), nws,
              _MODES[mode] | (int(band) << 8), _lib.stream_ptr(a.device))
    return out


def tn_full_for(m: int, n: int, splitk: int, cus: int | None = None) -> int:
    """Whole tiles of a mode-10 launch with a forced split factor: the whole rounds that fit ``cus`` CUs."""
    c = compute_cus() if cus is None else int(cus)
    tiles = (m // _TILE) * (n // _TILE)
    return tiles - tiles % c if splitk > 1 else tiles
