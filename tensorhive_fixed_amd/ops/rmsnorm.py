"""RMSNorm (Llama) -- HIP kernel on device, fp32 PyTorch reference on CPU.

Kernel: ``csrc/rmsnorm.hip`` (one workgroup per row, row kept in registers, deterministic
slab-reduced weight gradient).  The weight gradient goes to the flat DDP buffer (``_grad``).
"""
from __future__ import annotations

import torch

from . import _lib
from ._grad import deliver


def rmsnorm_reference(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    r = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (xf * r * w.float()).to(x.dtype)


def _fwd(x: torch.Tensor, w: torch.Tensor, eps: float):
    D = x.shape[-1]
    x2 = x.reshape(-1, D)
    if not x2.is_contiguous():
        x2 = x2.contiguous()
    T = x2.shape[0]
    if x2.is_cuda:
        if x2.dtype != torch.bfloat16 or w.dtype != torch.bfloat16 or w.numel() != D or D % 8:
            raise ValueError("rmsnorm kernel needs bf16 [T, D] input, bf16 [D] weight, D % 8 == 0")
        y = torch.empty_like(x2)
        rstd = torch.empty(T, device=x2.device, dtype=torch.float32)
        _lib.call("th_rmsnorm_fwd", x2.data_ptr(), w.data_ptr(), y.data_ptr(), rstd.data_ptr(),
                  T, D, float(eps), _lib.stream_ptr(x2.device))
    else:
        xf = x2.float()
        rstd = torch.rsqrt(xf.pow(2).mean(-1) + eps)
        y = (xf * rstd[:, None] * w.float()).to(x2.dtype)
    return x2, y, rstd


def _fwd_add(y: torch.Tensor, r: torch.Tensor, w: torch.Tensor, eps: float):
    """xsum = y + r (bf16-rounded, as a beta=1 GEMM epilogue would produce), h = rmsnorm(xsum)."""
    D = y.shape[-1]
    y2, r2 = y.reshape(-1, D), r.reshape(-1, D)
    if not y2.is_contiguous():
        y2 = y2.contiguous()
    if not r2.is_contiguous():
        r2 = r2.contiguous()
    T = y2.shape[0]
    if y2.is_cuda:
        if (y2.dtype != torch.bfloat16 or r2.dtype != torch.bfloat16 or w.dtype != torch.bfloat16 or D % 8
                or w.numel() != D or r2.shape != y2.shape):
            raise ValueError("rmsnorm_add kernel needs bf16 [T, D] inputs, bf16 [D] weight, D % 8 == 0")
        xsum = torch.empty_like(y2)
        h = torch.empty_like(y2)
        rstd = torch.empty(T, device=y2.device, dtype=torch.float32)
        _lib.call("th_rmsnorm_add_fwd", y2.data_ptr(), r2.data_ptr(), w.data_ptr(), xsum.data_ptr(), h.data_ptr(),
                  rstd.data_ptr(), T, D, float(eps), _lib.stream_ptr(y2.device))
        return xsum, h, rstd
    xsum = (y2.float() + r2.float()).to(y2.dtype)
    x2, h, rstd = _fwd(xsum, w, eps)
    return x2, h, rstd


def _bwd(x2, w, rstd, dy: torch.Tensor, dres: torch.Tensor | None, shape):
    """dx (+ dres, fused on the GPU) and the routed weight gradient."""
    T, D = x2.shape
    dy2 = dy.reshape(T, D)
    if not dy2.is_contiguous():
        dy2 = dy2.contiguous()
    if dres is not None:
        dres = dres.reshape(T, D)
        if not dres.is_contiguous():
            dres = dres.contiguous()
    if x2.is_cuda:
        dx = torch.empty_like(x2)
        nblk = max(1, min(T, 512))
        ws = torch.empty(nblk * D, device=x2.device, dtype=torch.float32)

        def run(dw_out: torch.Tensor, accumulate: bool) -> None:
            _lib.call("th_rmsnorm_bwd", dy2.data_ptr(), x2.data_ptr(), w.data_ptr(),
                      rstd.data_ptr(), dx.data_ptr(), dw_out.data_ptr(), ws.data_ptr(), nblk, T,
                      D, int(accumulate), None if dres is None else dres.data_ptr(),
                      _lib.stream_ptr(x2.device))

        def make() -> torch.Tensor:
            out = torch.empty_like(w)
            run(out, False)
            return out

        gw = deliver(w, run, make)
        return dx.view(shape), gw
    xf, gf, wf = x2.float(), dy2.float(), w.float()
    r = rstd[:, None]
    dot = (gf * wf * xf).sum(-1, keepdim=True)
    dxf = r * gf * wf - xf * dot * r.pow(3) / D
    if dres is not None:
        dxf = dxf + dres.float()
    dwv = (gf * xf * r).sum(0)

    def write(out: torch.Tensor, accumulate: bool) -> None:
        if accumulate:
            out.copy_((out.float() + dwv).to(out.dtype))
        else:
            out.copy_(dwv.to(out.dtype))

    gw = deliver(w, write, lambda: dwv.to(w.dtype))
    return dxf.to(x2.dtype).view(shape), gw


class _RMSNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: torch.Tensor, w: torch.Tensor, eps: float):
        x2, y, rstd = _fwd(x, w, eps)
        ctx.save_for_backward(x2, w, rstd)
        ctx.shape = x.shape
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy: torch.Tensor):
        x2, w, rstd = ctx.saved_tensors
        dx, gw = _bwd(x2, w, rstd, dy, None, ctx.shape)
        return dx, gw, None


class _RMSNormFork(torch.autograd.Function):
    """``(rmsnorm(x), x)``: the second output carries x on to the residual add, so the two
    gradients of x (through the norm and through the residual branch) are summed inside the
    RMSNorm backward kernel instead of by autograd's separate elementwise add."""

    @staticmethod
    def forward(ctx, x: torch.Tensor, w: torch.Tensor, eps: float):
        x2, y, rstd = _fwd(x, w, eps)
        ctx.save_for_backward(x2, w, rstd)
        ctx.shape = x.shape
        return y.view(x.shape), x.view(x.shape)

    @staticmethod
    def backward(ctx, dy: torch.Tensor, dres: torch.Tensor | None):
        x2, w, rstd = ctx.saved_tensors
        dx, gw = _bwd(x2, w, rstd, dy, dres, ctx.shape)
        return dx, gw, None


class _RMSNormAddFork(torch.autograd.Function):
    """``(rmsnorm(y + r), y + r)``: the residual add of the previous sublayer fused into this norm
    (one kernel reads y and r, writes the residual stream and the normalised output), replacing the
    beta=1 GEMM epilogue whose input copy cost a full [T, D] read + write per residual.  Both
    inputs receive the same gradient: the norm backward with the residual-branch gradient added."""

    @staticmethod
    def forward(ctx, y: torch.Tensor, r: torch.Tensor, w: torch.Tensor, eps: float):
        xsum, h, rstd = _fwd_add(y, r, w, eps)
        ctx.save_for_backward(xsum, w, rstd)
        ctx.shape = y.shape
        return h.view(y.shape), xsum.view(y.shape)

    @staticmethod
    def backward(ctx, dh: torch.Tensor, dres: torch.Tensor | None):
        xsum, w, rstd = ctx.saved_tensors
        dx, gw = _bwd(xsum, w, rstd, dh, dres, ctx.shape)
        return dx, dx, gw, None


def rmsnorm_add_fork(y: torch.Tensor, r: torch.Tensor, w: torch.Tensor,
                     eps: float = 1e-5) -> tuple[torch.Tensor, torch.Tensor]:
    """``h, x = rmsnorm_add_fork(y, r, w)`` with ``x = y + r``: use ``h`` for the sublayer and ``x``
    as the residual stream."""
    return _RMSNormAddFork.apply(y, r, w, eps)


def rmsnorm_fork(x: torch.Tensor, w: torch.Tensor, eps: float = 1e-5) -> tuple[torch.Tensor, torch.Tensor]:
    """``h, x = rmsnorm_fork(x, w)``: use ``h`` for the sublayer and the returned ``x`` for the residual."""
    return _RMSNormFork.apply(x, w, eps)


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    return _RMSNorm.apply(x, w, eps)
