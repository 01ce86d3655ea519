"""``transpose(x)``: contiguous ``x.T`` of a bf16 matrix -- HIP kernel on device (``csrc/transpose.hip``),
``x.t().contiguous()`` on the CPU.  Accepts a row-strided 2-D view (``x.stride(1) == 1``)."""
from __future__ import annotations

import torch

import os

from . import _lib

_TILE = int(os.environ.get("TH_TRANSPOSE_TILE", "0"))


def transpose(x: torch.Tensor, out: torch.Tensor | None = None, tile: int | None = None) -> torch.Tensor:
    if x.dim() != 2:
        raise ValueError("transpose expects a 2-D tensor")
    R, C = x.shape
    if out is None:
        out = torch.empty((C, R), device=x.device, dtype=x.dtype)
    if not x.is_cuda:
        out.copy_(x.t())
        return out
    if x.dtype != torch.bfloat16 or x.stride(1) != 1 or R % 8 or C % 8 or x.stride(0) % 8:
        raise ValueError(f"transpose kernel needs a bf16 [R, C] row-major view with R, C, ld % 8 == 0, got "
                         f"{tuple(x.shape)} {x.dtype} strides {x.stride()}")
    if not out.is_contiguous() or tuple(out.shape) != (C, R):
        raise ValueError("out must be a contiguous [C, R] tensor")
    _lib.call("th_transpose_bf16", x.data_ptr(), out.data_ptr(), R, C, x.stride(0), _TILE if tile is None else tile,
              _lib.stream_ptr(x.device))
    return out
