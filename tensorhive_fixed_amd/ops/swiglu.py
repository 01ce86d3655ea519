"""SwiGLU on the packed gate|up projection output -- HIP kernel on device, reference on CPU.

``swiglu(gu)`` with ``gu[..., 2F]`` = [gate | up] returns ``silu(gate) * up`` of shape ``[..., F]``.
Only ``gu`` is saved for backward (the F-wide product is recomputed inside the backward kernel).
Kernel: ``csrc/swiglu.hip``.
"""
from __future__ import annotations

import torch
import torch.nn.functional as Fn

from . import _lib


def swiglu_reference(gu: torch.Tensor) -> torch.Tensor:
    g, u = gu.float().chunk(2, dim=-1)
    return (Fn.silu(g) * u).to(gu.dtype)


class _SwiGLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu: torch.Tensor):
        F2 = gu.shape[-1]
        F = F2 // 2
        g2 = gu.reshape(-1, F2)
        if not g2.is_contiguous():
            g2 = g2.contiguous()
        T = g2.shape[0]
        if g2.is_cuda:
            if g2.dtype != torch.bfloat16 or F % 8:
                raise ValueError("swiglu kernel needs bf16 input with F % 8 == 0")
            out = torch.empty((T, F), device=g2.device, dtype=g2.dtype)
            _lib.call("th_swiglu_fwd", g2.data_ptr(), out.data_ptr(), T, F, _lib.stream_ptr(g2.device))
        else:
            out = swiglu_reference(g2)
        ctx.save_for_backward(g2)
        ctx.shape = gu.shape
        return out.view(*gu.shape[:-1], F)

    @staticmethod
    def backward(ctx, dout: torch.Tensor):
        (g2,) = ctx.saved_tensors
        T, F2 = g2.shape
        F = F2 // 2
        d2 = dout.reshape(T, F)
        if not d2.is_contiguous():
            d2 = d2.contiguous()
        if g2.is_cuda:
            dgu = torch.empty_like(g2)
            _lib.call("th_swiglu_bwd", d2.data_ptr(), g2.data_ptr(), dgu.data_ptr(), T, F,
                      _lib.stream_ptr(g2.device))
        else:
            g, u = g2.float().chunk(2, dim=-1)
            s = torch.sigmoid(g)
            df = d2.float()
            dgu = torch.cat([df * u * s * (1 + g * (1 - s)), df * g * s], dim=-1).to(g2.dtype)
        return dgu.view(ctx.shape)


def swiglu(gu: torch.Tensor) -> torch.Tensor:
    return _SwiGLU.apply(gu)
