"""Linear layers whose weight gradient lands directly in the flat DDP gradient buffer.

GEMMs are hipBLASLt (``torch.mm``/``addmm``) or the gfx950 TN kernel for weight gradients; what is
custom is the data flow: ``dW = dYᵀ·X`` is written by the GEMM itself into ``weight.main_grad``
(see ``_grad.deliver``).  By default the residual adds of the attention-out and MLP-down
projections are NOT done here but in the next RMSNorm (``rmsnorm_add_fork``, ``models/llama3.py``);
with ``TH_ADD_NORM=0`` they run as an ``addmm`` beta = 1 epilogue of these GEMMs (``residual=``).

Operand layouts (measured, ``scripts/gemm_layouts.py`` -> ``profiles/r01_gemm/``): hipBLASLt on
gfx950 is fastest when both operands are contiguous along the reduction dim.  The forward
``x @ Wᵀ`` already is; the input grad ``dY @ W`` is not, so W is transposed once per backward by
a HIP kernel (``ops/transpose.py``, ~0.1 ms for the 235 MB gate|up weight) and the GEMM runs as
``dY @ (Wᵀ)ᵀ`` -- 8-13 % faster.  For ``wgrad_nt`` layers (the gate|up projection, whose weight
grad is the largest GEMM of the step) the weight grad runs as ``(dYᵀ) @ (Xᵀ)ᵀ`` on transposed
copies of both operands: 6.29 -> 4.74 ms on the GEMM for ~0.9 ms of transposes.
``TH_DGRAD_NT=0`` / ``TH_WGRAD_NT=0`` switch either back to the plain forms.

``wgrad_tn`` layers (attention qkv / out and the MLP down projection by default) compute
``dW = dYᵀ·X`` with the gfx950 TN kernel (``ops/gemm_tn.py``) straight from the [tokens, features]
activations -- no transposes, 3-19 % faster than hipBLASLt on those shapes
(``scripts/bench_gemm_tn.py``); ``TH_WGRAD_TN=0`` disables it.
"""
from __future__ import annotations

import os

import torch

from ._grad import deliver, mm_into, nt_into, nt_mm
from .gemm_tn import gemm_tn_, supported as _tn_supported
from .transpose import transpose

_DGRAD_NT = os.environ.get("TH_DGRAD_NT", "1") == "1"
_WGRAD_NT = os.environ.get("TH_WGRAD_NT", "1") == "1"
_WGRAD_TN = os.environ.get("TH_WGRAD_TN", "1") == "1"


def tn_into(a: torch.Tensor, b: torch.Tensor):
    """A ``write`` callback computing ``aᵀ @ b`` with the gfx950 TN kernel (beta = 1 when accumulating)."""

    def _w(out: torch.Tensor, accumulate: bool) -> None:
        gemm_tn_(a, b, out.view(a.shape[1], b.shape[1]), accumulate=accumulate)

    return _w


def _c(t: torch.Tensor) -> torch.Tensor:
    return t if t.is_contiguous() else t.contiguous()


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: torch.Tensor, w: torch.Tensor, residual: torch.Tensor | None, wgrad_nt: bool = False,
                wgrad_tn: bool = False):
        x2 = x.reshape(-1, x.shape[-1])
        if residual is not None:
            y = torch.addmm(residual.reshape(-1, w.shape[0]), x2, w.t())
        else:
            y = nt_mm(x2, w)
        ctx.save_for_backward(x2, w)
        ctx.has_res = residual is not None
        ctx.xshape = x.shape
        ctx.wgrad_nt = wgrad_nt
        ctx.wgrad_tn = wgrad_tn
        return y if x.dim() == 2 else y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy: torch.Tensor):
        x2, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, w.shape[0])
        if dy2.is_cuda and _DGRAD_NT:
            dx = nt_mm(dy2, transpose(w))
        else:
            dx = torch.mm(dy2, w)
        dx = dx.view(ctx.xshape)
        if ctx.wgrad_tn and dy2.is_cuda and _WGRAD_TN and _tn_supported(w.shape[0], w.shape[1], dy2.shape[0]):
            dyc, xc = _c(dy2), _c(x2)
            gw = deliver(w, tn_into(dyc, xc), lambda: torch.mm(dyc.t(), xc))
        elif ctx.wgrad_nt and dy2.is_cuda and _WGRAD_NT:
            dyT, xT = transpose(_c(dy2)), transpose(_c(x2))
            gw = deliver(w, nt_into(dyT, xT), lambda: torch.mm(dyT, xT.t()))
        else:
            gw = deliver(w, mm_into(dy2.t(), x2), lambda: torch.mm(dy2.t(), x2))
        return dx, gw, (dy if ctx.has_res else None), None, None


def linear(x: torch.Tensor, w: torch.Tensor, residual: torch.Tensor | None = None,
           wgrad_nt: bool = False, wgrad_tn: bool = False) -> torch.Tensor:
    """``y = x @ w.T (+ residual)`` with weight-grad delivery into the flat buffer."""
    return _Linear.apply(x, w, residual, wgrad_nt, wgrad_tn)
