"""Token embedding whose backward is a deterministic sorted segment-sum kernel
(``csrc/embedding.hip``) writing straight into the flat gradient buffer."""
from __future__ import annotations

import torch
import torch.nn.functional as Fn

from . import _lib
from ._grad import deliver


class _Embedding(torch.autograd.Function):
    @staticmethod
    def forward(ctx, tokens: torch.Tensor, w: torch.Tensor):
        ctx.save_for_backward(tokens)
        ctx.wshape = w.shape
        ctx.w = w
        return Fn.embedding(tokens, w)

    @staticmethod
    def backward(ctx, dy: torch.Tensor):
        (tokens,) = ctx.saved_tensors
        w = ctx.w
        V, D = ctx.wshape
        ids = tokens.reshape(-1)
        dy2 = dy.reshape(-1, D)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        T = ids.shape[0]
        if dy2.is_cuda:
            if dy2.dtype != torch.bfloat16 or D % 8:
                raise ValueError("embedding backward kernel needs bf16 grads and D % 8 == 0")
            sorted_ids, perm = torch.sort(ids)

            def write(out: torch.Tensor, accumulate: bool) -> None:
                if not accumulate:
                    out.zero_()
                _lib.call("th_embedding_bwd", sorted_ids.data_ptr(), perm.data_ptr(),
                          dy2.data_ptr(), out.data_ptr(), T, D, int(accumulate),
                          _lib.stream_ptr(dy2.device))

            def make() -> torch.Tensor:
                out = torch.empty((V, D), device=dy2.device, dtype=dy2.dtype)
                write(out, False)
                return out
        else:
            def write(out: torch.Tensor, accumulate: bool) -> None:
                acc = torch.zeros((V, D), dtype=torch.float32)
                acc.index_add_(0, ids, dy2.float())
                if accumulate:
                    acc += out.view(V, D).float()
                out.copy_(acc.view_as(out).to(out.dtype))

            def make() -> torch.Tensor:
                out = torch.empty((V, D), dtype=dy2.dtype)
                write(out, False)
                return out

        gw = deliver(w, write, make)
        ctx.w = None
        return None, gw


def embedding(tokens: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    return _Embedding.apply(tokens, w)
