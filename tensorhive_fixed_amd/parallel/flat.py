"""Flat parameter / gradient storage with bucketed, backward-overlapped RCCL all-reduce.

MI355X-first data-parallel design (no torch DDP wrapper, no per-tensor grads):

* Every parameter of the model is re-homed into ONE contiguous bf16 buffer, laid out in
  *reverse forward order* (LM head first, embedding last), because that is the order in which
  backward produces the weight gradients.
* A matching flat bf16 gradient buffer holds ``param.main_grad`` views.  The payload's autograd
  functions write weight gradients straight into them with the GEMM itself (``ops/_grad.py``);
  nothing is zeroed (the first micro-batch overwrites, later ones accumulate with beta = 1).
* The gradient buffer is cut into buckets of ~``bucket_mb`` at parameter boundaries.  When the
  last parameter of a bucket reports ready, that bucket's ``all_reduce`` (RCCL over xGMI, SUM)
  is launched asynchronously while backward continues on the compute stream.  Buckets are
  large (default 256 MB) because xGMI is point-to-point: a ring is per-link bound, and fewer,
  larger collectives keep RCCL's channels busy.
* Averaging is folded into the optimizer (``grad_scale = 1/world``); the fused flat AdamW then
  updates the whole model with one kernel per parameter group.

The layout rules are validated on CPU with the gloo backend (tests/test_flat_ddp.py).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch
import torch.distributed as dist

from ..ops.adamw import adamw_flat_, grad_sumsq_

_ALIGN = 64  # elements; keeps every view 128-byte aligned and every range a multiple of 8


def _round_up(n: int, a: int) -> int:
    return (n + a - 1) // a * a


@dataclass
class _Bucket:
    index: int
    start: int
    end: int
    params: list = field(default_factory=list)
    pending: int = 0
    handle: object = None


class FlatParamStore:
    """Owns the flat parameter + gradient buffers and the bucketed gradient all-reduce."""

    def __init__(self, params_in_backward_order: list[tuple[str, torch.nn.Parameter, bool]],
                 device: torch.device, dtype: torch.dtype = torch.bfloat16,
                 process_group=None, bucket_mb: float = 256.0):
        self.device = torch.device(device)
        self.dtype = dtype
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_available() and dist.is_initialized() else 1
        # decayed (matrices) first, then non-decayed vectors: two contiguous optimizer groups
        ordered = [e for e in params_in_backward_order if e[2]] + [e for e in params_in_backward_order if not e[2]]
        offs, off = [], 0
        for _, p, _ in ordered:
            offs.append(off)
            off += _round_up(p.numel(), _ALIGN)
        self.numel = off
        self.decay_numel = sum(_round_up(p.numel(), _ALIGN) for _, p, d in ordered if d)
        self.param_buf = torch.zeros(self.numel, device=self.device, dtype=dtype)
        self.grad_buf = torch.zeros(self.numel, device=self.device, dtype=dtype)
        self.names: list[str] = []
        self.params: list[torch.nn.Parameter] = []
        self.offsets: dict[int, int] = {}
        for (name, p, _), o in zip(ordered, offs):
            n = p.numel()
            view = self.param_buf[o: o + n].view(p.shape)
            with torch.no_grad():
                view.copy_(p.data.to(device=self.device, dtype=dtype))
            p.data = view
            p.main_grad = self.grad_buf[o: o + n].view(p.shape)
            p.th_store = self
            self.names.append(name)
            self.params.append(p)
            self.offsets[id(p)] = o
        self._build_buckets(bucket_mb)
        self.accumulating = False
        self._sync_now = True
        self._ready_seen: set[int] = set()

    # ------------------------------------------------------------------ buckets
    def _build_buckets(self, bucket_mb: float) -> None:
        cap = max(_ALIGN, int(bucket_mb * 1024 * 1024 / self.grad_buf.element_size()))
        self.buckets: list[_Bucket] = []
        self.param_bucket: dict[int, _Bucket] = {}
        cur = None
        for p in self.params:
            o = self.offsets[id(p)]
            end = o + _round_up(p.numel(), _ALIGN)
            if cur is None or (end - cur.start > cap and cur.params):
                cur = _Bucket(len(self.buckets), o, end)
                self.buckets.append(cur)
            cur.end = end
            cur.params.append(p)
            self.param_bucket[id(p)] = cur

    def bucket_ranges(self) -> list[tuple[int, int]]:
        return [(b.start, b.end) for b in self.buckets]

    # ------------------------------------------------------------------ step protocol
    def begin_microbatch(self, accumulate: bool, sync: bool = True) -> None:
        """Call before each forward.

        ``accumulate``: this micro-batch adds to the existing gradients (beta = 1 GEMMs).
        ``sync``: buckets all-reduce as they complete (True only on the last micro-batch).
        """
        self.accumulating = accumulate
        self._ready_seen.clear()
        for b in self.buckets:
            b.pending = len(b.params)
            b.handle = None
        self._sync_now = sync

    def mark_ready(self, p: torch.Tensor) -> None:
        key = id(p)
        if key in self._ready_seen:
            raise RuntimeError("parameter gradient delivered twice in one micro-batch")
        self._ready_seen.add(key)
        b = self.param_bucket[key]
        b.pending -= 1
        if b.pending == 0 and self._sync_now and self.world > 1:
            b.handle = dist.all_reduce(self.grad_buf[b.start: b.end], op=dist.ReduceOp.SUM,
                                       group=self.pg, async_op=True)

    def finish_grad_sync(self) -> None:
        """Wait for every bucket; launch any bucket whose params did not all report."""
        if len(self._ready_seen) != len(self.params):
            missing = [n for n, p in zip(self.names, self.params) if id(p) not in self._ready_seen]
            raise RuntimeError(f"no gradient delivered for: {missing[:5]}...")
        if self.world == 1 or not self._sync_now:
            return
        for b in self.buckets:
            if b.handle is None:
                b.handle = dist.all_reduce(self.grad_buf[b.start: b.end], op=dist.ReduceOp.SUM,
                                           group=self.pg, async_op=True)
        for b in self.buckets:
            b.handle.wait()
            b.handle = None


class FlatAdamW:
    """AdamW over a :class:`FlatParamStore`: f32 master/m/v buffers, 2 fused launches per step."""

    def __init__(self, store: FlatParamStore, lr: float = 3e-4, betas=(0.9, 0.95), eps: float = 1e-8,
                 weight_decay: float = 0.1, clip: float = 1.0):
        self.store = store
        self.lr, self.betas, self.eps, self.wd, self.clip = lr, betas, eps, weight_decay, clip
        self.master = store.param_buf.float()
        self.exp_avg = torch.zeros_like(self.master)
        self.exp_avg_sq = torch.zeros_like(self.master)
        self.norm_sq = torch.zeros(1, device=store.device, dtype=torch.float32)
        self.step_count = 0

    def step(self, lr: float | None = None) -> None:
        st = self.store
        self.step_count += 1
        lr = self.lr if lr is None else lr
        scale = 1.0 / st.world
        if self.clip > 0:
            grad_sumsq_(st.grad_buf, self.norm_sq)
        groups = [(0, st.decay_numel, self.wd), (st.decay_numel, st.numel, 0.0)]
        for a, b, wd in groups:
            if b <= a:
                continue
            adamw_flat_(st.param_buf[a:b], self.master[a:b], self.exp_avg[a:b], self.exp_avg_sq[a:b],
                        st.grad_buf[a:b], lr=lr, beta1=self.betas[0], beta2=self.betas[1], eps=self.eps,
                        weight_decay=wd, step=self.step_count, grad_scale=scale,
                        norm_sq=self.norm_sq if self.clip > 0 else None, clip=self.clip)

    def grad_norm(self) -> float:
        """Global gradient norm of the last step (forces a host sync; for logging only)."""
        return math.sqrt(float(self.norm_sq[0])) / self.store.world
