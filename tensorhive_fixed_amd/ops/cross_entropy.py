"""Fused LM-head + cross-entropy, chunked over tokens (the 128256-wide logits never exist whole).

Forward computes, chunk by chunk: ``logits_c = h_c @ Wᵀ`` (hipBLASLt) -> ``csrc/cross_entropy.hip``
turns the chunk into ``dlogits_c`` in place and emits per-row loss -> ``dh_c = dlogits_c @ W`` and
``dW += dlogits_cᵀ @ h_c`` (written straight into the flat gradient buffer).  The gradient work
is done inside forward because the loss is the graph's root: backward only scales ``dh``.

Contract: the returned mean loss must be back-propagated with an upstream gradient of 1
(``loss.backward()``), because the head weight gradient is already final when forward returns.
"""
from __future__ import annotations

import os

import torch

from . import _lib
from ._grad import nt_mm
from .gemm_tn import gemm_tn_, supported as gemm_tn_supported
from .linear import _DGRAD_NT
from .transpose import transpose

_HEAD_NT = os.environ.get("TH_HEAD_WGRAD_NT", "1") == "1"  # +0.3 % step (A/B in profiles/r01_gemm)
_HEAD_TN = os.environ.get("TH_HEAD_WGRAD_TN", "1") == "1"  # gfx950 TN kernel (hb) for dW += dlogitsᵀ h: no logits transpose, 3.44 vs 3.62 ms per 4096-token chunk (profiles/r05_step)


def ce_rows_(logits: torch.Tensor, target: torch.Tensor, grad_scale: float,
             ignore_index: int = -100) -> torch.Tensor:
    """In-place: logits[R, V] (bf16) -> dlogits; returns per-row loss (f32)."""
    R, V = logits.shape
    if logits.is_cuda:
        if logits.dtype != torch.bfloat16 or logits.stride(1) != 1 or target.dtype != torch.int64:
            raise ValueError("ce kernel needs row-major bf16 logits and int64 targets")
        loss = torch.empty(R, device=logits.device, dtype=torch.float32)
        lse = torch.empty(R, device=logits.device, dtype=torch.float32)
        _lib.call("th_ce_fwd_bwd", logits.data_ptr(), logits.stride(0), target.data_ptr(),
                  loss.data_ptr(), lse.data_ptr(), R, V, float(grad_scale), int(ignore_index),
                  _lib.stream_ptr(logits.device))
        return loss
    lf = logits.float()
    lse = torch.logsumexp(lf, dim=-1)
    valid = target != ignore_index
    tgt = target.clamp(min=0)
    loss = torch.where(valid, lse - lf.gather(1, tgt[:, None])[:, 0], torch.zeros_like(lse))
    p = torch.softmax(lf, dim=-1)
    p[torch.arange(R), tgt] -= 1.0
    p = p * torch.where(valid, grad_scale, 0.0)[:, None]
    logits.copy_(p.to(logits.dtype))
    return loss


class _LinearCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h: torch.Tensor, w: torch.Tensor, target: torch.Tensor, chunk: int,
                ignore_index: int, n_valid: int | None):
        D = h.shape[-1]
        h2 = h.reshape(-1, D)
        t = target.reshape(-1)
        T = h2.shape[0]
        if n_valid is None:  # one host sync; the trainer passes the count it already knows
            n_valid = int((t != ignore_index).sum().item())
        scale = 1.0 / max(1, n_valid)
        dh = torch.empty_like(h2)
        loss_sum = torch.zeros((), device=h2.device, dtype=torch.float32)
        mg = getattr(w, "main_grad", None)
        # TH_GRAD_FP32: each chunk's GEMM writes its bf16 product, which is added to the f32 main_grad
        # straight away -- the sum over chunks is an f32 accumulation, never a bf16 one.
        f32_main = mg is not None and mg.dtype != w.dtype
        if f32_main:
            acc = torch.empty(w.shape, device=w.device, dtype=w.dtype)
            mg_w = mg.view_as(w)
        else:
            acc = mg.view_as(w) if mg is not None else torch.zeros(w.shape, device=w.device, dtype=torch.float32)
        first_acc = mg is not None and (f32_main or not w.th_store.accumulating)
        # dh = dlogits @ W in the K-contiguous form (see ops/linear.py): one transpose of W per call
        w_kn = transpose(w).t() if (h2.is_cuda and _DGRAD_NT) else w
        for i, s0 in enumerate(range(0, T, chunk)):
            hc = h2[s0: s0 + chunk]
            logits = nt_mm(hc, w) if hc.is_cuda else torch.mm(hc, w.t())
            loss_sum += ce_rows_(logits, t[s0: s0 + chunk], scale, ignore_index).sum()
            if h2.is_cuda and _DGRAD_NT:
                nt_mm(logits, w_kn.t(), out=dh[s0: s0 + chunk])
            else:
                torch.mm(logits, w_kn, out=dh[s0: s0 + chunk])
            if mg is not None:
                # dW += dlogitsᵀ hc; with TH_HEAD_WGRAD_NT both operands are transposed first so the
                # GEMM runs in the K-contiguous form
                fresh = f32_main or (i == 0 and first_acc)  # overwrite acc instead of accumulating
                if _HEAD_TN and h2.is_cuda and gemm_tn_supported(w.shape[0], w.shape[1], hc.shape[0]):
                    # TN kernel straight from [tokens, V] logits and [tokens, D] hidden states
                    gemm_tn_(logits, hc, acc, accumulate=not fresh)
                else:
                    a_op, b_op = (transpose(logits), transpose(hc).t()) if (_HEAD_NT and h2.is_cuda) \
                        else (logits.t(), hc)
                    if fresh:
                        torch.mm(a_op, b_op, out=acc)
                    else:
                        acc.addmm_(a_op, b_op)
                    del a_op, b_op
                if f32_main:
                    (mg_w.copy_ if (i == 0 and not w.th_store.accumulating) else mg_w.add_)(acc)
            else:
                acc.addmm_(logits.t().float(), hc.float())
            del logits
        del w_kn
        if f32_main:
            del acc, mg_w
        if mg is not None:
            w.th_store.mark_ready(w)
            ctx.gw = None
        else:
            ctx.gw = acc.to(w.dtype)
        ctx.save_for_backward(dh)
        ctx.hshape = h.shape
        return loss_sum * scale

    @staticmethod
    def backward(ctx, g: torch.Tensor):
        (dh,) = ctx.saved_tensors
        dh = (dh * g.to(dh.dtype)).view(ctx.hshape)
        gw = ctx.gw * g.to(ctx.gw.dtype) if ctx.gw is not None else None
        return dh, gw, None, None, None, None


def linear_cross_entropy(h: torch.Tensor, w: torch.Tensor, target: torch.Tensor,
                         chunk: int = 4096, ignore_index: int = -100,
                         n_valid: int | None = None) -> torch.Tensor:
    """Mean token cross-entropy of ``h @ w.T`` against ``target`` (ignore_index masked).

    ``n_valid`` (number of non-ignored targets) avoids a device->host sync when known."""
    return _LinearCE.apply(h, w, target, chunk, ignore_index, n_valid)
