"""Llama-3 bf16 data-parallel training payload (N07): synthetic tokens, random-init weights.

Launched one process per GPU (``torchrun --nproc_per_node N -m
tensorhive_fixed_amd.workloads.llama3_ddp``), typically by the tensorhive job queue through the
``torchrun`` task template with ``HIP_VISIBLE_DEVICES`` taken from the reservation.  It prints
``[th-train] step=… tokens/s=…`` lines; the daemon parses them from the task log tail
(``GET /api/tasks/{id}/training``, ``controllers/task.py:parse_training_lines``) and the dashboard
charts the series on the task's page.

One step = forward + backward (gradient buckets all-reduced -- or, with the ZeRO-1 sharded
optimizer that is the default for world > 1, reduce-scattered -- over RCCL while backward runs) +
fused flat AdamW with on-device global-norm clipping (+ the overlapped parameter all-gather when
sharded).  Nothing is skipped inside a step.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

from ..models.llama3 import Llama, LlamaConfig
from ..ops import gemm_tn
from ..parallel.dist import DistInfo, barrier, forced_collectives, init_distributed, max_over_ranks, shutdown
from ..parallel.flat import FlatAdamW, FlatParamStore


class SyntheticTokens:
    """Deterministic per-rank random token batches generated on the device."""

    def __init__(self, vocab: int, batch: int, seq: int, device: torch.device, rank: int, seed: int = 1234):
        self.vocab, self.batch, self.seq, self.device = vocab, batch, seq, device
        self.gen = torch.Generator(device=device)
        self.gen.manual_seed(seed + 7919 * rank)
        self.drawn = 0  # batches handed out: a resume replays this many draws on every rank

    def skip(self, n: int) -> None:
        for _ in range(n):
            self.next()

    def next(self) -> tuple[torch.Tensor, torch.Tensor]:
        self.drawn += 1
        buf = torch.randint(0, self.vocab, (self.batch, self.seq + 1), device=self.device,
                            generator=self.gen)
        return buf[:, :-1], buf[:, 1:]


class _Range:
    """roctx range (``TH_ROCTX=1``): shows steps / fwd / bwd / optimizer on rocprofv3 --marker-trace."""

    enabled = os.environ.get("TH_ROCTX") == "1"

    def __init__(self, name: str):
        self.name = name

    def __enter__(self):
        if self.enabled:
            torch.cuda.nvtx.range_push(self.name)  # roctx on ROCm builds

    def __exit__(self, *exc):
        if self.enabled:
            torch.cuda.nvtx.range_pop()


def backward_cu_budget(store: FlatParamStore) -> int | None:
    """CUs the TN weight-gradient launches may count on during a synchronising backward (ops/gemm_tn.py
    ``cu_budget``), or None for the whole chip.

    ``TH_COMM_CUS`` names the CUs the gradient collectives hold while they run (0 = plan for all 256).
    Unset, it is the emulated channel count when ``TH_COMM_EMU`` rehearses RCCL's footprint on one GPU, and
    0 otherwise: on a real multi-rank step the collectives hold CUs only while they run (~4 % of the step at
    300 GB/s), and the re-plan costs more on the idle rest than it saves (profiles/r06_comm/sweep2-5)."""
    env = os.environ.get("TH_COMM_CUS")
    if env is not None:
        reserved = int(env)
    elif store.comm_emu is not None:
        reserved = store.comm_emu.cfg.cus
    else:
        reserved = 0
    if reserved <= 0:
        return None
    return max(64, 256 - reserved)


def default_zero(world: int) -> int:
    """ZeRO stage of the payload: 1 (sharded optimizer) whenever there is more than one rank,
    unless ``TH_ZERO=0`` asks for the replicated DDP optimizer."""
    env = os.environ.get("TH_ZERO")
    if env is not None:
        return int(env)
    return 1 if world > 1 else 0


class Trainer:
    def __init__(self, cfg: LlamaConfig, info: DistInfo, micro_batch: int, seq_len: int,
                 grad_accum: int = 1, lr: float = 3e-4, bucket_mb: float = 256.0, seed: int = 0,
                 zero: int | None = None):
        self.cfg, self.info = cfg, info
        self.micro_batch, self.seq_len, self.grad_accum = micro_batch, seq_len, grad_accum
        dev = info.device
        if dev.type == "cuda":
            from ..ops.tuned import load_gemm_table

            from ..ops.tuned import table_path

            self.gemm_table = load_gemm_table()  # measured hipBLASLt / rocBLAS choices (TH_GEMM_TUNED)
            self.gemm_table_name = table_path().name if self.gemm_table else None
        self.zero = default_zero(info.world) if zero is None else zero
        self.model = Llama(cfg, device=dev, dtype=torch.bfloat16, seed=seed)
        self.store = FlatParamStore(self.model.params_in_backward_order(), dev, bucket_mb=bucket_mb,
                                    shard=self.zero >= 1 and (info.world > 1 or forced_collectives()))
        self.opt = FlatAdamW(self.store, lr=lr)
        if self.store.sharded or self.opt.overlap:
            self.model.param_gate = self.store.wait_params
        self.data = SyntheticTokens(cfg.vocab_size, micro_batch, seq_len, dev, info.rank)
        self.tokens_per_step = micro_batch * seq_len * grad_accum  # per rank
        self.bwd_cus = backward_cu_budget(self.store)  # TN launch geometry while collectives hold CUs
        self.last_loss: torch.Tensor | None = None

    def step(self) -> torch.Tensor:
        n_valid = self.micro_batch * self.seq_len
        loss_acc = None
        with _Range("train_step"):
            for mb in range(self.grad_accum):
                tokens, targets = self.data.next()
                self.store.begin_microbatch(accumulate=mb > 0, sync=mb == self.grad_accum - 1)
                with _Range("forward"):
                    loss = self.model(tokens, targets, n_valid=n_valid * self.grad_accum)
                if mb == 0:
                    self.opt.wait_done()  # the previous step's (overlapped) update read these gradients
                with _Range("backward"), gemm_tn.cu_budget(self.bwd_cus if mb == self.grad_accum - 1 else None):
                    loss.backward()
                loss_acc = loss.detach() if loss_acc is None else loss_acc + loss.detach()
            with _Range("grad_sync+adamw"):
                self.store.finish_grad_sync()
                self.opt.step()
        self.last_loss = loss_acc
        return loss_acc

    # ------------------------------------------------------------------ checkpoint / resume
    def _optim_state(self) -> dict:
        return {"master": self.opt.master, "exp_avg": self.opt.exp_avg, "exp_avg_sq": self.opt.exp_avg_sq}

    def state(self) -> dict:
        """Everything a bit-exact resume needs: flat params, f32 master / moments, step, data RNG.
        With a sharded optimizer the moments are this rank's slices (see :meth:`save`)."""
        self.store.wait_all_params()
        self.opt.wait_done()
        st = {"param_buf": self.store.param_buf, "step": torch.tensor(self.opt.step_count),
              "data_drawn": torch.tensor(self.data.drawn), "names": "\n".join(self.store.names),
              "zero_world": torch.tensor(self.info.world if self.store.sharded else 0)}
        if not self.store.sharded:
            st.update(self._optim_state())
        return st

    @staticmethod
    def shard_path(path: str, rank: int, world: int) -> str:
        return f"{path}.optim.{rank}-of-{world}"

    @staticmethod
    def _write(obj: dict, path: str) -> None:
        tmp = path + ".tmp"
        torch.save({k: (v.detach().cpu() if torch.is_tensor(v) else v) for k, v in obj.items()}, tmp)
        os.replace(tmp, path)

    def save(self, path: str) -> None:
        """Rank 0 writes the parameters (replicas are identical); with the sharded optimizer every
        rank also writes its own optimizer slices next to it.  Atomic renames."""
        st = self.state()
        if self.store.sharded:
            self._write(self._optim_state(), self.shard_path(path, self.info.rank, self.info.world))
        if self.info.rank == 0:
            self._write(st, path)

    def load(self, path: str) -> None:
        st = torch.load(path, map_location="cpu", weights_only=True)
        if st["names"] != "\n".join(self.store.names):
            raise ValueError("checkpoint does not match this model's parameter layout")
        zero_world = int(st.get("zero_world", torch.tensor(0)))
        want = self.info.world if self.store.sharded else 0
        if zero_world != want:
            raise ValueError(f"checkpoint optimizer sharding ({zero_world} ranks) does not match this run ({want})")
        opt = st if not self.store.sharded else torch.load(
            self.shard_path(path, self.info.rank, self.info.world), map_location="cpu", weights_only=True)
        with torch.no_grad():
            self.store.wait_all_params()
            self.store.param_buf.copy_(st["param_buf"])
            self.opt.master.copy_(opt["master"])
            self.opt.exp_avg.copy_(opt["exp_avg"])
            self.opt.exp_avg_sq.copy_(opt["exp_avg_sq"])
        self.opt.step_count = int(st["step"])
        # every rank has its own data stream: replay the same number of draws on each
        self.data.skip(int(st["data_drawn"]) - self.data.drawn)


def sync_device(info: DistInfo) -> None:
    if info.device.type == "cuda":
        torch.cuda.synchronize(info.device)


def run_timed(trainer: Trainer, steps: int, warmup: int) -> dict:
    info = trainer.info
    for _ in range(warmup):
        trainer.step()
    sync_device(info)
    barrier(info)
    sync_device(info)
    trainer.store.timer.reset()  # exposed-communication spans of the timed steps only
    t0 = time.perf_counter()
    for _ in range(steps):
        trainer.step()
    sync_device(info)
    barrier(info)
    sync_device(info)
    mine = time.perf_counter() - t0
    dt = max_over_ranks(mine, info)
    loss = float(trainer.last_loss) if trainer.last_loss is not None else float("nan")
    toks = trainer.tokens_per_step * info.world * steps
    waits = {f"{k}_ms_per_step": round(v / max(1, steps), 3) for k, v in trainer.store.timer.totals_ms().items()}
    waits["step_ms"] = round(1000.0 * mine / max(1, steps), 3)
    return {"seconds": dt, "ms_per_step": 1000.0 * dt / max(1, steps), "tokens_per_sec": toks / dt,
            "loss": loss, "waits": waits}


def _maybe_save(tr: Trainer, ckpt: str | None, args) -> None:
    if ckpt and args.ckpt_every and tr.opt.step_count % args.ckpt_every == 0:
        os.makedirs(os.path.dirname(ckpt), exist_ok=True)
        tr.save(ckpt)


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(description="Llama-3 bf16 DDP training on MI355X (synthetic data)")
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--seq-len", type=int, default=4096)
    ap.add_argument("--micro-batch", type=int, default=4)
    ap.add_argument("--grad-accum", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--log-every", type=int, default=1)
    ap.add_argument("--bucket-mb", type=float, default=256.0)
    ap.add_argument("--zero", type=int, default=None, help="1: shard the optimizer (default when world > 1)")
    ap.add_argument("--ckpt-dir", default=None, help="write <dir>/ckpt.pt every --ckpt-every steps (rank 0)")
    ap.add_argument("--ckpt-every", type=int, default=0)
    ap.add_argument("--resume", action="store_true", help="continue from <ckpt-dir>/ckpt.pt if present")
    args = ap.parse_args(argv)
    from ..utils.blas_env import refuse_unsafe_blas_workspace

    refuse_unsafe_blas_workspace("th-train")
    info = init_distributed()
    cfg = LlamaConfig.named(args.model)
    tr = Trainer(cfg, info, args.micro_batch, args.seq_len, args.grad_accum, bucket_mb=args.bucket_mb,
                 zero=args.zero)
    ckpt = os.path.join(args.ckpt_dir, "ckpt.pt") if args.ckpt_dir else None
    if ckpt and args.resume and os.path.exists(ckpt):
        tr.load(ckpt)
        if info.is_main:
            print(json.dumps({"event": "resumed", "step": tr.opt.step_count}), flush=True)
    # warm-up steps are real optimizer steps (excluded from the timing only); a resumed run continues
    # the same global step count up to warmup + steps
    total = args.warmup + args.steps
    while tr.opt.step_count < min(args.warmup, total):
        tr.step()
        _maybe_save(tr, ckpt, args)
    sync_device(info)
    t_last = time.perf_counter()
    while tr.opt.step_count < total:
        tr.step()
        s = tr.opt.step_count - args.warmup
        if s % args.log_every == 0:
            sync_device(info)
            now = time.perf_counter()
            dt = max_over_ranks(now - t_last, info)
            t_last = now
            tps = tr.tokens_per_step * info.world * args.log_every / dt
            if info.is_main:
                print(f"[th-train] step={s} loss={float(tr.last_loss):.4f} tokens/s={tps:.1f} "
                      f"world={info.world}", flush=True)
        _maybe_save(tr, ckpt, args)
    if info.is_main:
        print(json.dumps({"event": "done", "steps": tr.opt.step_count,
                          "loss": round(float(tr.last_loss), 6) if tr.last_loss is not None else None}), flush=True)
    shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
