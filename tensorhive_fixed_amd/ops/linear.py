"""Linear layers whose weight gradient lands directly in the flat DDP gradient buffer.

GEMMs are plain library GEMMs (hipBLASLt through ``torch.mm``/``addmm``); what is custom is the
data flow: the residual add of the attention-out and MLP-down projections is fused into the
GEMM epilogue (``addmm`` with beta = 1), and ``dW = dYᵀ·X`` is written by the GEMM itself into
``weight.main_grad`` (see ``_grad.deliver``).
"""
from __future__ import annotations

import torch

from ._grad import deliver, mm_into


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: torch.Tensor, w: torch.Tensor, residual: torch.Tensor | None):
        x2 = x.reshape(-1, x.shape[-1])
        if residual is not None:
            y = torch.addmm(residual.reshape(-1, w.shape[0]), x2, w.t())
        else:
            y = torch.mm(x2, w.t())
        ctx.save_for_backward(x2, w)
        ctx.has_res = residual is not None
        ctx.xshape = x.shape
        return y if x.dim() == 2 else y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy: torch.Tensor):
        x2, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, w.shape[0])
        dx = torch.mm(dy2, w).view(ctx.xshape)
        gw = deliver(w, mm_into(dy2.t(), x2), lambda: torch.mm(dy2.t(), x2))
        return dx, gw, (dy if ctx.has_res else None)


def linear(x: torch.Tensor, w: torch.Tensor, residual: torch.Tensor | None = None) -> torch.Tensor:
    """``y = x @ w.T (+ residual)`` with weight-grad delivery into the flat buffer."""
    return _Linear.apply(x, w, residual)
