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
* ``grad_dtype=float32`` (``TH_GRAD_FP32=1``): the gradient buffer, the micro-batch accumulation
  and the RCCL reduction are f32 (twice the gradient bytes on the wire; +16 GB for 8B params);
  the default keeps them bf16.  tests/test_flat_ddp.py bounds the bf16 path's error against the
  f32 path at world 8 with 4 accumulated micro-batches.

``shard=True`` (ZeRO-1, the default of the training payload when world > 1) keeps the same flat
buffers and buckets but distributes the optimizer:

* every bucket is padded to a multiple of ``world * 64`` elements and rank ``r`` owns the r-th
  contiguous slice of each bucket;
* a ready bucket is ``reduce_scatter``-ed in place (RCCL writes the summed slice straight into
  this rank's part of the gradient buffer) instead of all-reduced -- half the bytes on the
  critical path of backward;
* f32 master weights and Adam moments exist only for the owned slices (12 B/param / world: 12 GB
  instead of 96 GB per MI355X at 8 ranks), and the AdamW kernels stream 1/world of the model;
* the updated bf16 slices are ``all_gather``-ed back in place, bucket by bucket in FORWARD order,
  asynchronously: the next forward waits for a bucket only right before the first layer that
  reads it (``wait_params``), so the gather overlaps the embedding / first layers' compute.

Total traffic per step equals the all-reduce (reduce-scatter + all-gather), but the all-gather
leaves backward's critical path.  The layout rules and the numerical equivalence of the sharded
and replicated optimizers are validated on CPU with the gloo backend (tests/test_flat_ddp.py).
"""
from __future__ import annotations

import math
import os
import time
from collections import defaultdict
from contextlib import contextmanager
from dataclasses import dataclass, field

import torch
import torch.distributed as dist

from ..ops.adamw import adamw_flat_, grad_sumsq_
from .dist import forced_collectives

_ALIGN = 64  # elements; keeps every view 128-byte aligned and every range a multiple of 8


def _round_up(n: int, a: int) -> int:
    return (n + a - 1) // a * a


class WaitTimer:
    """Exposed-communication accounting: how long the compute stream stalls at each wait.

    A wait on an async collective (``work.wait()`` on RCCL) or on the side-stream optimizer makes
    the *current stream* wait; an event recorded just before and one just after the wait bound
    that stall on the device timeline, so ``elapsed(before, after)`` is exactly the part of the
    collective that was NOT hidden behind compute.  With gloo (CPU) the wait blocks the host and
    the span is host time.  Categories: ``grad_sync`` (gradient buckets at the end of backward),
    ``allgather`` (sharded parameters the next forward needs), ``opt_wait`` (the overlapped AdamW
    the next backward / forward layer waits for).  Event pairs are resolved lazily by
    :meth:`totals_ms` (one synchronize), so timing adds no host sync to a step."""

    CATEGORIES = ("grad_sync", "allgather", "opt_wait")

    def __init__(self, device: torch.device, enabled: bool = True):
        self.cuda = torch.device(device).type == "cuda"
        self.enabled = enabled
        self.reset()

    MAX_EVENTS = 4096  # pending event pairs before they are folded into totals (one sync)

    def reset(self) -> None:
        self._events: list[tuple[str, object, object]] = []
        self._host: dict[str, float] = defaultdict(float)  # seconds (host spans, folded events)
        self.counts: dict[str, int] = defaultdict(int)

    def _fold(self) -> None:
        """Resolve the pending event pairs into the totals and release them, so a long run that
        never reads the timer holds a bounded number of events."""
        if self._events:
            self._events[-1][2].synchronize()
            for cat, e0, e1 in self._events:
                self._host[cat] += float(e0.elapsed_time(e1)) / 1000.0
            self._events = []

    @contextmanager
    def span(self, cat: str):
        if not self.enabled:
            yield
            return
        if self.cuda:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
            yield
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            self._events.append((cat, e0, e1))
            if len(self._events) >= self.MAX_EVENTS:
                self._fold()
        else:
            t0 = time.perf_counter()
            yield
            self._host[cat] += time.perf_counter() - t0
        self.counts[cat] += 1

    def totals_ms(self) -> dict[str, float]:
        self._fold()
        return {c: 1000.0 * self._host.get(c, 0.0) for c in self.CATEGORIES}


@dataclass
class _Bucket:
    index: int
    start: int
    end: int
    params: list = field(default_factory=list)
    pending: int = 0
    handle: object = None  # gradient collective of this micro-batch
    gather: object = None  # parameter all-gather in flight (sharded mode)
    updated: object = None  # event: this bucket's optimizer update done (overlapped optimizer)
    emu_done: object = None  # rehearsal (TH_COMM_EMU deps=1): the modelled reduce-scatter's end
    emu_gathered: object = None  # rehearsal (TH_COMM_EMU deps=1): the modelled all-gather's end

    def shard(self, rank: int, world: int) -> tuple[int, int]:
        n = (self.end - self.start) // world
        return self.start + rank * n, self.start + (rank + 1) * n


class FlatParamStore:
    """Owns the flat parameter + gradient buffers and the bucketed gradient all-reduce."""

    def __init__(self, params_in_backward_order: list[tuple[str, torch.nn.Parameter, bool]],
                 device: torch.device, dtype: torch.dtype = torch.bfloat16,
                 process_group=None, bucket_mb: float = 256.0, shard: bool = False,
                 grad_dtype: torch.dtype | None = None):
        self.device = torch.device(device)
        self.dtype = dtype
        if grad_dtype is None:
            grad_dtype = torch.float32 if os.environ.get("TH_GRAD_FP32", "0") == "1" else dtype
        self.grad_dtype = grad_dtype
        self.pg = process_group
        initialized = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(process_group) if initialized else 1
        self.rank = dist.get_rank(process_group) if initialized else 0
        self.sharded = bool(shard)
        # collectives run when there is more than one rank -- or, with TH_FORCE_COLLECTIVES=1, in a
        # 1-rank group too, so the RCCL path (in-place reduce-scatter / all-gather on side streams)
        # can be exercised on a one-GPU box (tests/gpu/test_ddp_gpu.py)
        self.collectives = initialized and (self.world > 1 or forced_collectives())
        # decayed (matrices) first, then non-decayed vectors: two contiguous optimizer groups
        ordered = [e for e in params_in_backward_order if e[2]] + [e for e in params_in_backward_order if not e[2]]
        offs, self.buckets = self._layout([(p, d) for _, p, d in ordered], bucket_mb)
        self.numel = self.buckets[-1].end if self.buckets else 0
        self.decay_numel = max([o + p.numel() for (_, p, d), o in zip(ordered, offs) if d], default=0)
        self.decay_numel = _round_up(self.decay_numel, _ALIGN)
        self.param_buf = torch.zeros(self.numel, device=self.device, dtype=dtype)
        self.grad_buf = torch.zeros(self.numel, device=self.device, dtype=grad_dtype)
        self.names: list[str] = []
        self.params: list[torch.nn.Parameter] = []
        self.offsets: dict[int, int] = {}
        self.param_bucket: dict[int, _Bucket] = {}
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
        for b in self.buckets:
            for p in b.params:
                self.param_bucket[id(p)] = b
        self.accumulating = False
        self._sync_now = True
        self._ready_seen: set[int] = set()
        # called with each bucket whose (final micro-batch) gradients are complete and whose
        # collective, if any, is launched: FlatAdamW's early gradient-norm pass hooks in here
        self.ready_hook = None
        # exposed-communication spans: bench.py turns them on (TH_COMM_TIMING=1) and reports them
        # per rank; off for training jobs
        self.timer = WaitTimer(self.device, enabled=os.environ.get("TH_COMM_TIMING", "0") == "1")
        # one-GPU rehearsal of RCCL's channel CUs during backward (TH_COMM_EMU, parallel/comm_emu.py)
        from .comm_emu import CommEmulator

        self.comm_emu = CommEmulator.from_env(self.device)

    # ------------------------------------------------------------------ buckets
    def _layout(self, entries: list, bucket_mb: float) -> tuple[list[int], list[_Bucket]]:
        """Offsets of every parameter and the buckets: cut at parameter boundaries once a bucket
        reaches ``bucket_mb``; in sharded mode each bucket is padded to ``world * _ALIGN``."""
        cap = max(_ALIGN, int(bucket_mb * 1024 * 1024 / torch.empty((), dtype=self.dtype).element_size()))
        quantum = _ALIGN * (self.world if self.sharded else 1)
        offs: list[int] = []
        buckets: list[_Bucket] = []
        cur = None
        off = 0
        for p, _ in entries:
            size = _round_up(p.numel(), _ALIGN)
            if cur is None or (off + size - cur.start > cap and cur.params):
                if cur is not None:
                    off = cur.start + _round_up(off - cur.start, quantum)
                    cur.end = off
                cur = _Bucket(len(buckets), off, off)
                buckets.append(cur)
            offs.append(off)
            cur.params.append(p)
            off += size
        if cur is not None:
            cur.end = cur.start + _round_up(off - cur.start, quantum)
        return offs, buckets

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

    def _launch_grad_collective(self, b: _Bucket):
        full = self.grad_buf[b.start: b.end]
        if self.sharded:
            lo, hi = b.shard(self.rank, self.world)
            # in place: RCCL writes this rank's summed slice into its own part of the bucket
            return dist.reduce_scatter_tensor(self.grad_buf[lo:hi], full, op=dist.ReduceOp.SUM,
                                              group=self.pg, async_op=True)
        return dist.all_reduce(full, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)

    def mark_ready(self, p: torch.Tensor) -> None:
        key = id(p)
        if key in self._ready_seen:
            raise RuntimeError("parameter gradient delivered twice in one micro-batch")
        self._ready_seen.add(key)
        b = self.param_bucket[key]
        b.pending -= 1
        if b.pending == 0 and self._sync_now:
            if self.collectives:
                b.handle = self._launch_grad_collective(b)
            if self.comm_emu is not None:
                b.emu_done = self.comm_emu.bucket_ready((b.end - b.start) * self.grad_buf.element_size())
            if self.ready_hook is not None:
                self.ready_hook(b)

    def finish_grad_sync(self) -> None:
        """Wait for every bucket; launch any bucket whose params did not all report."""
        if len(self._ready_seen) != len(self.params):
            missing = [n for n, p in zip(self.names, self.params) if id(p) not in self._ready_seen]
            raise RuntimeError(f"no gradient delivered for: {missing[:5]}...")
        if self.comm_emu is not None and self._sync_now:
            self.comm_emu.stop()
        if not self.collectives or not self._sync_now:
            return
        for b in self.buckets:
            if b.handle is None:
                b.handle = self._launch_grad_collective(b)
        with self.timer.span("grad_sync"):
            for b in self.buckets:
                b.handle.wait()
                b.handle = None

    # ------------------------------------------------------------------ sharded (ZeRO-1) helpers
    def owned_ranges(self) -> list[tuple[int, int]]:
        """Per bucket, the flat range whose optimizer state this rank owns (the whole bucket when
        not sharded)."""
        if not self.sharded:
            return [(b.start, b.end) for b in self.buckets]
        return [b.shard(self.rank, self.world) for b in self.buckets]

    def mark_updated(self, index: int) -> None:
        """Record (on the current stream) that bucket ``index`` holds its new parameters."""
        ev = torch.cuda.Event()
        ev.record()
        self.buckets[index].updated = ev

    def gather_bucket(self, index: int) -> None:
        """All-gather bucket ``index`` in place, asynchronously (after its slice was updated)."""
        if not self.sharded or not self.collectives:
            return
        b = self.buckets[index]
        lo, hi = b.shard(self.rank, self.world)
        b.gather = dist.all_gather_into_tensor(self.param_buf[b.start: b.end], self.param_buf[lo:hi],
                                               group=self.pg, async_op=True)

    def start_param_gather(self) -> None:
        """All-gather every bucket, in forward order (the last bucket holds the embedding/norms)."""
        for b in reversed(self.buckets):
            self.gather_bucket(b.index)

    def wait_params(self, *params: torch.Tensor) -> None:
        """Make the current stream wait until the buckets holding ``params`` are up to date: their
        all-gather (sharded) or their overlapped optimizer update."""
        for p in params:
            b = self.param_bucket.get(id(p))
            if b is not None:
                self._wait_bucket(b)

    def wait_emu_reduced(self) -> None:
        """Rehearsal with ``deps=1``: the current stream waits for every bucket's modelled reduce-scatter."""
        for b in self.buckets:
            if b.emu_done is not None:
                torch.cuda.current_stream(self.device).wait_event(b.emu_done)
                b.emu_done = None

    def _wait_bucket(self, b: _Bucket) -> None:
        if b.emu_gathered is not None:
            torch.cuda.current_stream(self.device).wait_event(b.emu_gathered)
            b.emu_gathered = None
        if b.gather is not None:
            with self.timer.span("allgather"):
                b.gather.wait()
            b.gather = None
        if b.updated is not None:
            with self.timer.span("opt_wait"):
                torch.cuda.current_stream(self.device).wait_event(b.updated)
            b.updated = None

    def wait_all_params(self) -> None:
        for b in self.buckets:
            self._wait_bucket(b)


class FlatAdamW:
    """AdamW over a :class:`FlatParamStore`: f32 master/m/v for the owned ranges, fused launches
    per bucket (and per decay group).

    Replicated (DDP) store: the state covers every bucket.
    Sharded (ZeRO-1) store: the state covers this rank's slice of every bucket only; the global
    gradient norm is the all-reduced sum of the slices' squares, and after the update the store
    all-gathers the new bf16 parameters (overlapped with the next forward).

    ``overlap`` (GPU, default on; ``TH_OPT_OVERLAP=0`` disables): the step runs on a side stream,
    bucket by bucket in forward order, so the memory-bound AdamW sweep (≈38 ms for 8B parameters
    on one MI355X) can share the GPU with the next forward, which waits per layer for exactly the
    bucket it reads (``FlatParamStore.wait_params``).  Measured gain on one MI355X is small
    (23.85k vs 23.81k tokens/s, A/B/A/B on one box): the GEMMs leave the sweep few free CUs.  The next backward
    must not overwrite gradients the sweep still reads: the trainer calls :meth:`wait_done`
    before it (the LM-head gradient, written during the forward, is covered by the head's own
    bucket wait).  With ``TH_OPT_SUMSQ_EARLY=1`` the clip norm's sums of squares are also taken per
    bucket during backward (:meth:`_bucket_ready`), so after backward only the sweep itself stands
    between the last gradient and the next forward's first layer.
    """

    def __init__(self, store: FlatParamStore, lr: float = 3e-4, betas=(0.9, 0.95), eps: float = 1e-8,
                 weight_decay: float = 0.1, clip: float = 1.0, overlap: bool | None = None):
        self.store = store
        if overlap is None:
            overlap = os.environ.get("TH_OPT_OVERLAP", "1") == "1"
        self.overlap = bool(overlap) and store.device.type == "cuda"
        self.side = torch.cuda.Stream(device=store.device) if self.overlap else None
        self.done = None
        self.lr, self.betas, self.eps, self.wd, self.clip = lr, betas, eps, weight_decay, clip
        # (flat_lo, flat_hi, local_lo, weight_decay) segments: owned ranges split at the decay boundary
        self.segments: list[tuple[int, int, int, float]] = []
        local = 0
        # segment indices per bucket, so the sharded step can hand each bucket to its all-gather
        # as soon as its slice is updated
        self.bucket_segments: list[list[int]] = []
        self._owned = store.owned_ranges()
        for lo, hi in self._owned:
            mine = []
            for a, b, wd in ((lo, min(hi, store.decay_numel), weight_decay), (max(lo, store.decay_numel), hi, 0.0)):
                if b > a:
                    mine.append(len(self.segments))
                    self.segments.append((a, b, local, wd))
                    local += b - a
            self.bucket_segments.append(mine)
        self.local_numel = local
        self.master = torch.empty(local, device=store.device, dtype=torch.float32)
        for a, b, l0, _ in self.segments:
            self.master[l0: l0 + (b - a)].copy_(store.param_buf[a:b])
        self.exp_avg = torch.zeros_like(self.master)
        self.exp_avg_sq = torch.zeros_like(self.master)
        self.norm_sq = torch.zeros(1, device=store.device, dtype=torch.float32)
        self.step_count = 0
        # Early gradient norm (overlapped mode, opt-in TH_OPT_SUMSQ_EARLY=1): each bucket's sum of
        # squares runs on the side stream as soon as the bucket is complete (after its collective),
        # i.e. during the rest of backward, into its own slot; the step then only sums the slots.
        # It shortens the exposed optimizer wait (6.2 -> 3.9 ms) but not the one-GPU step, whose
        # backward has no idle CUs to absorb the sums (profiles/r05_step/README.md), so it is off.
        self.early_sumsq = self.overlap and clip > 0 and os.environ.get("TH_OPT_SUMSQ_EARLY", "0") == "1"
        self.norm_parts = None
        self._early_done: set[int] = set()
        self.early_steps = 0  # steps whose norm came from the early per-bucket sums
        if self.early_sumsq:
            self.norm_parts = torch.zeros(len(store.buckets), device=store.device, dtype=torch.float32)
            store.ready_hook = self._bucket_ready

    def step(self, lr: float | None = None) -> None:
        st = self.store
        self.step_count += 1
        lr = self.lr if lr is None else lr
        if self.overlap:
            self.side.wait_stream(torch.cuda.current_stream(st.device))  # gradients are complete
            with torch.cuda.stream(self.side):
                self._step(lr)
                self.done = torch.cuda.Event()
                self.done.record()
        else:
            self._step(lr)

    def _bucket_ready(self, b: _Bucket) -> None:
        """Store hook: ``||g||^2`` of bucket ``b``'s owned range into ``norm_parts[b.index]``, on the
        side stream, ordered after the gradient writes (an event on the current stream) and after
        the bucket's reduce-scatter / all-reduce (``work.wait()`` issued on the side stream)."""
        st = self.store
        ev = torch.cuda.Event()
        ev.record()
        self.side.wait_event(ev)
        lo, hi = self._owned[b.index]
        with torch.cuda.stream(self.side):
            if b.handle is not None:
                b.handle.wait()
            if hi > lo:
                grad_sumsq_(st.grad_buf[lo:hi], self.norm_parts[b.index: b.index + 1])
            else:
                self.norm_parts[b.index: b.index + 1].zero_()
        self._early_done.add(b.index)

    def wait_done(self) -> None:
        """Current stream waits for the whole (overlapped) optimizer step."""
        if self.done is not None:
            with self.store.timer.span("opt_wait"):
                torch.cuda.current_stream(self.store.device).wait_event(self.done)
            self.done = None

    @staticmethod
    def _merge(run: tuple | None, seg: tuple, same_wd: bool = True) -> tuple | None:
        """``run`` extended by ``seg`` when both are contiguous in the flat AND the local (state)
        index space (and share the weight decay), else None.  Segments are (flat_lo, flat_hi,
        local_lo, wd)."""
        if run is None:
            return seg
        a, b, l0, wd = run
        a2, b2, l2, wd2 = seg
        if same_wd and wd2 != wd:
            return None
        if a2 == b and l2 == l0 + (b - a):
            return (a, b2, l0, wd)
        if b2 == a and l2 + (b2 - a2) == l0:
            return (a2, b, l2, wd)
        return None

    def _launch_groups(self) -> list[tuple[tuple, list[int]]]:
        """AdamW launches in forward order: ``[(segment run, bucket indices it completes)]``.

        ``TH_OPT_GROUP_MPARAMS`` (millions of parameters, default 0 = one launch per bucket segment)
        lets launches cover several flat-contiguous buckets: the streaming kernel runs closer to the
        HBM ceiling on larger ranges (``profiles/r02_streaming/``), at the price of a coarser
        per-bucket hand-off to the next forward / all-gather."""
        limit = int(float(os.environ.get("TH_OPT_GROUP_MPARAMS", "0")) * 1e6)
        out: list[tuple[tuple, list[int]]] = []
        run, buckets = None, []
        for bi in reversed(range(len(self.bucket_segments))):
            for si in self.bucket_segments[bi]:
                seg = self.segments[si]
                merged = self._merge(run, seg) if limit > 0 else None
                if merged is not None and merged[1] - merged[0] <= limit:
                    run = merged
                else:
                    if run is not None:
                        out.append((run, buckets))
                    run, buckets = seg, []
            if run is None:  # a bucket this rank owns nothing of
                out.append((None, [bi]))
            else:
                buckets.append(bi)
        if run is not None:
            out.append((run, buckets))
        return out

    def _step(self, lr: float) -> None:
        st = self.store
        scale = 1.0 / st.world
        groups = self._launch_groups()
        st.wait_emu_reduced()  # rehearsal (deps=1): the norm and the update need every reduce-scatter
        early = self.early_sumsq and len(self._early_done) == len(st.buckets)
        self._early_done.clear()
        if self.clip > 0 and early:
            self.early_steps += 1
            torch.sum(self.norm_parts, dim=0, keepdim=True, out=self.norm_sq)
            if st.sharded and st.collectives:
                dist.all_reduce(self.norm_sq, op=dist.ReduceOp.SUM, group=st.pg)
        elif self.clip > 0:
            # ||g||^2 over maximal flat-contiguous runs (the sum does not care about decay groups)
            runs: list[tuple] = []
            merge = os.environ.get("TH_OPT_SUMSQ_RUNS", "1") == "1"  # 0: one pass per segment (old form)
            for seg in self.segments:
                m = self._merge(runs[-1], seg, same_wd=False) if runs and merge else None
                if m is not None and m[1] - m[0] <= (1 << 31) - 8:
                    runs[-1] = m
                else:
                    runs.append(seg)
            for i, (a, b, _, _) in enumerate(runs):
                grad_sumsq_(st.grad_buf[a:b], self.norm_sq, accumulate=i > 0)
            if not self.segments:
                self.norm_sq.zero_()
            if st.sharded and st.collectives:
                dist.all_reduce(self.norm_sq, op=dist.ReduceOp.SUM, group=st.pg)
        # forward order (last bucket first): in sharded mode each bucket's all-gather starts right after
        # its slice is updated, overlapping the remaining AdamW launches and then the next forward
        for run, buckets in groups:
            if run is not None:
                a, b, l0, wd = run
                l1 = l0 + (b - a)
                adamw_flat_(st.param_buf[a:b], self.master[l0:l1], self.exp_avg[l0:l1], self.exp_avg_sq[l0:l1],
                            st.grad_buf[a:b], lr=lr, beta1=self.betas[0], beta2=self.betas[1], eps=self.eps,
                            weight_decay=wd, step=self.step_count, grad_scale=scale,
                            norm_sq=self.norm_sq if self.clip > 0 else None, clip=self.clip)
            for bi in buckets:
                if st.sharded:
                    st.gather_bucket(bi)
                elif self.overlap:
                    st.mark_updated(bi)
                if st.comm_emu is not None:
                    # the rehearsal's ZeRO-1 parameter all-gather of this bucket (bucket mode only)
                    b = st.buckets[bi]
                    b.emu_gathered = st.comm_emu.bucket_gathered((b.end - b.start) * st.param_buf.element_size())

    def grad_norm(self) -> float:
        """Global gradient norm of the last step (forces a host sync; for logging only)."""
        if self.done is not None:
            self.done.synchronize()  # norm_sq is written on the side stream
        return math.sqrt(float(self.norm_sq[0])) / self.store.world
