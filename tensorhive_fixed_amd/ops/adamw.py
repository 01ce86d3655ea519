"""Fused flat AdamW step (``csrc/adamw.hip``) with on-device global-norm clipping.

``adamw_flat_(param, master, exp_avg, exp_avg_sq, grad, ...)`` updates one contiguous range of the
flat parameter buffer in a single kernel.  With ``clip > 0`` a sum-of-squares pre-pass writes
``||g||^2`` into a device scalar that the step kernel reads (no host round trip).
"""
from __future__ import annotations

import torch

from . import _lib


def grad_sumsq_(grad: torch.Tensor, out: torch.Tensor, accumulate: bool = False) -> torch.Tensor:
    """out[0] (+)= sum(grad^2) for a flat bf16 gradient range (device, no sync)."""
    n = grad.numel()
    if grad.is_cuda:
        ws = torch.empty(2048, device=grad.device, dtype=torch.float32)
        fn = "th_sumsq_f32" if grad.dtype == torch.float32 else "th_sumsq_bf16"
        _lib.call(fn, grad.data_ptr(), n, ws.data_ptr(), out.data_ptr(), int(accumulate),
                  _lib.stream_ptr(grad.device))
    else:
        s = grad.float().pow(2).sum()
        out[0] = out[0] + s if accumulate else s
    return out


def adamw_flat_(param: torch.Tensor, master: torch.Tensor, exp_avg: torch.Tensor,
                exp_avg_sq: torch.Tensor, grad: torch.Tensor, *, lr: float, beta1: float,
                beta2: float, eps: float, weight_decay: float, step: int, grad_scale: float = 1.0,
                norm_sq: torch.Tensor | None = None, clip: float = 0.0) -> None:
    n = param.numel()
    for t in (master, exp_avg, exp_avg_sq, grad):
        if t.numel() != n:
            raise ValueError("adamw_flat_: all flat ranges must have the same length")
    if param.is_cuda:
        if n % 8 or param.dtype != torch.bfloat16 or grad.dtype not in (torch.bfloat16, torch.float32) \
                or master.dtype != torch.float32:
            raise ValueError("adamw kernel needs bf16 param, bf16/f32 grad, f32 state and n % 8 == 0")
        fn = "th_adamw_step_f32g" if grad.dtype == torch.float32 else "th_adamw_step"
        _lib.call(fn, param.data_ptr(), master.data_ptr(), exp_avg.data_ptr(),
                  exp_avg_sq.data_ptr(), grad.data_ptr(), n, float(lr), float(beta1), float(beta2),
                  float(eps), float(weight_decay), int(step), float(grad_scale),
                  None if norm_sq is None else norm_sq.data_ptr(), float(clip),
                  _lib.stream_ptr(param.device))
        return
    scale = grad_scale
    if norm_sq is not None and clip > 0:
        tn = float(norm_sq[0].sqrt()) * grad_scale
        scale *= min(1.0, clip / (tn + 1e-6))
    g = grad.float() * scale
    exp_avg.mul_(beta1).add_(g, alpha=1 - beta1)
    exp_avg_sq.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    master.mul_(1 - lr * weight_decay)
    denom = exp_avg_sq.sqrt() / (bc2 ** 0.5) + eps
    master.addcdiv_(exp_avg, denom, value=-lr / bc1)
    param.copy_(master.to(param.dtype))
