"""Weight-gradient delivery into the flat DDP gradient buffer.

Every custom autograd function of the payload computes its weight gradient itself and writes it
straight into ``param.main_grad`` (a view of the flat bf16 gradient buffer owned by
:class:`tensorhive_fixed_amd.parallel.flat.FlatParamStore`) -- GEMM weight gradients via
``torch.mm(..., out=main_grad)`` (beta = 0) or ``addmm_`` (beta = 1 when accumulating
micro-batches).  There is no separate ``.grad`` tensor, no AccumulateGrad add, and no copy into a
communication bucket: the bucket IS the gradient.  After writing, the store is told that the
parameter is ready so it can launch that bucket's collective while backward continues.

Parameters that are not owned by a store (unit tests, plain use) get an ordinary returned
gradient instead.  With an f32 gradient buffer (``TH_GRAD_FP32=1``) the gradient is produced in
the compute dtype and added into the f32 ``main_grad`` (accumulation and reduction in f32).
"""
from __future__ import annotations

from typing import Callable

import torch


def deliver(weight: torch.Tensor, write: Callable[[torch.Tensor, bool], None],
            make: Callable[[], torch.Tensor]) -> torch.Tensor | None:
    """Route a weight gradient.

    ``write(out, accumulate)`` writes (or adds) the gradient into ``out``;
    ``make()`` returns a fresh gradient tensor when there is no flat buffer.
    Returns the value the autograd ``backward`` must return for this weight.
    """
    mg = getattr(weight, "main_grad", None)
    if mg is None:
        return make()
    store = weight.th_store
    if mg.dtype != weight.dtype:
        # f32 main gradients (TH_GRAD_FP32): the GEMM writes this micro-batch's gradient in the
        # compute dtype, the accumulation across micro-batches and the reduction run in f32
        g = make()
        if store.accumulating:
            mg.add_(g.view_as(mg))
        else:
            mg.copy_(g.view_as(mg))
        del g
    else:
        write(mg, store.accumulating)
    store.mark_ready(weight)
    return None


def mm_into(a: torch.Tensor, b: torch.Tensor) -> Callable[[torch.Tensor, bool], None]:
    """A ``write`` callback computing ``a @ b`` into ``out`` (accumulating with beta = 1)."""

    def _w(out: torch.Tensor, accumulate: bool) -> None:
        o2 = out.view(a.shape[0], b.shape[1])
        if accumulate:
            o2.addmm_(a, b)
        else:
            torch.mm(a, b, out=o2)

    return _w


def nt_mm(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """``a @ b.t()`` (into ``out`` when given): the K-contiguous ("NT") form of the forward and
    input-gradient GEMMs, on hipBLASLt.  (The hand-written NT kernel reached 0.93-0.96x of it at
    K = 4096 and 0.84x at large K and was removed: profiles/r05_gemm/.)"""
    if out is not None:
        return torch.mm(a, b.t(), out=out)
    return torch.mm(a, b.t())


def nt_into(a: torch.Tensor, b: torch.Tensor) -> Callable[[torch.Tensor, bool], None]:
    """A ``write`` callback computing ``a @ b.t()`` (hipBLASLt)."""
    return mm_into(a, b.t())
