"""Fused gate|up projection + SwiGLU: ``a = silu(h Wg^T) * (h Wu^T)`` with ``W13 = [Wg; Wu]``.

One autograd node instead of ``swiglu(linear(h, w13))``, so the backward can hand the SwiGLU
kernel's output straight to BOTH consumers in the layout each GEMM wants (``ops/linear.py``,
``profiles/r01_gemm/``):

* ``dH = dGU @ W13`` -- ``dGU`` row-major, W13 transposed once (K-contiguous "NT" form);
* ``dW13 = dGUᵀ @ H`` -- by default on the gfx950 TN kernel (``ops/gemm_tn.py``) straight from ``dGU`` and
  ``H`` as they are: 6.38 ms per layer with the plain SwiGLU backward against 6.60 for the previous path
  (``TH_W13_WGRAD_TN=0``: ``(dGUᵀ) @ (Hᵀ)ᵀ`` on hipBLASLt, with ``dGUᵀ`` written by the ``th_swiglu_bwd_t``
  kernel and ``Hᵀ`` from the transpose kernel; ``profiles/r05_gemm/w13_wgrad_paths.jsonl``).

On the CPU (unit tests) the same math runs in PyTorch.  ``F % 64 != 0`` falls back to the
unfused pair on the GPU.
"""
from __future__ import annotations

import os

import torch

from . import _lib
from ._grad import deliver, mm_into, nt_into, nt_mm
from .gemm_tn import gemm_tn_, supported as _tn_supported
from .linear import _DGRAD_NT, linear, tn_into
from .swiglu import swiglu, swiglu_reference
from .transpose import transpose


_W13_TN = os.environ.get("TH_W13_WGRAD_TN", "1") == "1"


class _GateUpSwiGLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h: torch.Tensor, w13: torch.Tensor):
        h2 = h.reshape(-1, h.shape[-1])
        if not h2.is_contiguous():
            h2 = h2.contiguous()
        gu = nt_mm(h2, w13) if h2.is_cuda else torch.mm(h2, w13.t())
        T, F2 = gu.shape
        F = F2 // 2
        if gu.is_cuda:
            a = torch.empty((T, F), device=gu.device, dtype=gu.dtype)
            _lib.call("th_swiglu_fwd", gu.data_ptr(), a.data_ptr(), T, F, _lib.stream_ptr(gu.device))
        else:
            a = swiglu_reference(gu)
        ctx.save_for_backward(h2, w13, gu)
        ctx.hshape = h.shape
        return a.view(*h.shape[:-1], F)

    @staticmethod
    def backward(ctx, da: torch.Tensor):
        h2, w13, gu = ctx.saved_tensors
        T, F2 = gu.shape
        F = F2 // 2
        d2 = da.reshape(T, F)
        if not d2.is_contiguous():
            d2 = d2.contiguous()
        if gu.is_cuda and _W13_TN and _tn_supported(F2, h2.shape[1], T):
            dgu = torch.empty_like(gu)
            _lib.call("th_swiglu_bwd", d2.data_ptr(), gu.data_ptr(), dgu.data_ptr(), T, F, _lib.stream_ptr(gu.device))
            dh = nt_mm(dgu, transpose(w13)) if _DGRAD_NT else torch.mm(dgu, w13)
            gw = deliver(w13, tn_into(dgu, h2),
                         lambda: gemm_tn_(dgu, h2, torch.empty(w13.shape, device=gu.device, dtype=gu.dtype)))
            del dgu
        elif gu.is_cuda:
            dgu = torch.empty_like(gu)
            dguT = torch.empty((F2, T), device=gu.device, dtype=gu.dtype)
            _lib.call("th_swiglu_bwd_t", d2.data_ptr(), gu.data_ptr(), dgu.data_ptr(), dguT.data_ptr(), T, F,
                      _lib.stream_ptr(gu.device))
            dh = nt_mm(dgu, transpose(w13)) if _DGRAD_NT else torch.mm(dgu, w13)
            del dgu
            hT = transpose(h2)
            gw = deliver(w13, nt_into(dguT, hT), lambda: torch.mm(dguT, hT.t()))
        else:
            g, u = gu.float().chunk(2, dim=-1)
            s = torch.sigmoid(g)
            df = d2.float()
            dgu = torch.cat([df * u * s * (1 + g * (1 - s)), df * g * s], dim=-1).to(gu.dtype)
            dh = torch.mm(dgu, w13)
            gw = deliver(w13, mm_into(dgu.t(), h2), lambda: torch.mm(dgu.t(), h2))
        return dh.view(ctx.hshape), gw


def gate_up_swiglu(h: torch.Tensor, w13: torch.Tensor) -> torch.Tensor:
    F = w13.shape[0] // 2
    if h.is_cuda and (F % 64 or h.numel() // h.shape[-1] % 8):
        return swiglu(linear(h, w13, wgrad_nt=True))
    return _GateUpSwiGLU.apply(h, w13)
