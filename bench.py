#!/usr/bin/env python3
"""Headline benchmark: Llama-3-8B bf16 data-parallel training tokens/sec on N MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1 the driver starts
one rank per GPU with torchrun.  W untimed warm-up steps, then exactly K timed steps bracketed by
barrier + device synchronize on both sides; the time is the MAX over ranks; rank 0 prints ONE
JSON line.  ``value`` is the whole-job tokens/s (all ranks).  Weak scaling: per-GPU batch is
fixed (micro_batch x seq_len tokens per GPU per step).

Each timed step is the full training step: forward, backward with bucketed RCCL gradient
collectives over xGMI, and the fused AdamW update of all 8.03e9 parameters.  With N > 1 the
optimizer is ZeRO-1 sharded by default (gradient reduce-scatter during backward, each rank
updates 1/N of the parameters, bf16 all-gather overlapped with the next forward); ``--zero 0``
selects the replicated all-reduce optimizer.
Data: synthetic random tokens; weights: random init (no network, no checkpoints).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_TOKENS_PER_SEC = None  # the reference publishes no throughput


def daemon_poll_latency() -> dict | None:
    """The other half of the north-star metric (BASELINE.json): p50/p99 of ``GET /api/nodes/metrics``
    for a non-admin user with per-GPU restrictions, over HTTP to the daemon's threaded server
    (8 simulated nodes x 8 GPUs).  Runs in a child process AFTER the timed training steps, so it
    cannot touch the measured region; any failure reports null instead of failing the bench."""
    import subprocess

    code = ("import json; from tensorhive_fixed_amd import benchmarks as b; "
            "r = b.poll_latency(500); print(json.dumps({k: v['/api/nodes/metrics'] for k, v in r['results'].items()}))")
    try:
        out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, cwd=ROOT)
        res = json.loads(out.stdout.strip().splitlines()[-1])
        return {"poll_p50_ms_user_socket": res["user_socket"]["p50_ms"],
                "poll_p99_ms_user_socket": res["user_socket"]["p99_ms"],
                "poll_p50_ms_user_inprocess": res["user_inprocess"]["p50_ms"],
                "poll_p50_ms_admin_inprocess": res["admin_inprocess"]["p50_ms"],
                "setup": "8 simulated nodes x 8 GPUs, non-admin with per-GPU restrictions, HTTP keep-alive"}
    except Exception as e:  # noqa: BLE001
        return {"error": str(e)[:200]}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", default=os.environ.get("TH_BENCH_MODEL", "llama3-8b"))
    ap.add_argument("--seq-len", type=int, default=int(os.environ.get("TH_BENCH_SEQ", "4096")))
    # 8 x 4096 tokens per GPU: 258 GiB peak of the 288 GiB HBM3E (MB 4 reaches 4.8 % fewer tokens/s: the
    # per-step optimizer/all-reduce cost is amortized over twice the tokens and the GEMMs get M = 32768)
    ap.add_argument("--micro-batch", type=int, default=int(os.environ.get("TH_BENCH_MB", "8")))
    ap.add_argument("--bucket-mb", type=float, default=float(os.environ.get("TH_BENCH_BUCKET_MB", "256")))
    ap.add_argument("--grad-accum", type=int, default=int(os.environ.get("TH_BENCH_ACCUM", "1")))
    ap.add_argument("--zero", type=int, default=None, help="1 = sharded optimizer (default for N > 1), 0 = replicated")
    ap.add_argument("--daemon-bench", type=int, default=1,
                    help="rank 0 also measures the daemon's dashboard poll latency after the timed steps")
    args = ap.parse_args()
    # bench-only diagnostics: RCCL's INIT log to a per-rank file summarised in the JSON line, and
    # the exposed-communication wait spans (both off for ordinary training jobs)
    os.environ.setdefault("TH_RCCL_INIT_LOG", "1")
    os.environ.setdefault("TH_COMM_TIMING", "1")

    from tensorhive_fixed_amd.utils.blas_env import refuse_unsafe_blas_workspace

    refuse_unsafe_blas_workspace("bench")  # a known hipBLASLt fault; nothing touched the GPU yet

    import torch

    from tensorhive_fixed_amd.models.llama3 import LlamaConfig
    from tensorhive_fixed_amd.ops import _lib
    from tensorhive_fixed_amd.ops.attention import attention_backend
    from tensorhive_fixed_amd.parallel.comm_diag import comm_report
    from tensorhive_fixed_amd.parallel.dist import barrier, init_distributed, rank_census, shutdown
    from tensorhive_fixed_amd.workloads.llama3_ddp import Trainer, run_timed

    info = init_distributed()  # binds this rank to its GPU's NUMA CPUs before HIP starts any thread
    if torch.cuda.is_available():
        _lib.load(build_if_missing=True)  # the HIP kernels must be what runs; fail loudly otherwise
    if info.world != args.gpus and info.is_main:
        print(f"[bench] warning: --gpus {args.gpus} but WORLD_SIZE {info.world}", file=sys.stderr)
    cfg = LlamaConfig.named(args.model)
    tr = Trainer(cfg, info, args.micro_batch, args.seq_len, args.grad_accum, bucket_mb=args.bucket_mb,
                 zero=args.zero)
    res = run_timed(tr, args.steps, args.warmup)
    emu = tr.store.comm_emu.report() if tr.store.comm_emu is not None else None  # TH_COMM_EMU rehearsal
    census = rank_census(info)  # collective: every rank takes part, after the timed region
    comm = comm_report(res["waits"], info)  # collective too: per-rank exposed-communication spans
    n = info.world
    flops = cfg.flops_per_token(args.seq_len) * res["tokens_per_sec"]
    line = {
        "metric": "llama3_8b_bf16_ddp_train_tokens_per_sec",
        "value": round(res["tokens_per_sec"], 2),
        "unit": "tokens/s",
        "n_gpus": n,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(res["ms_per_step"], 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None if BASELINE_TOKENS_PER_SEC is None else res["tokens_per_sec"] / BASELINE_TOKENS_PER_SEC,
        "dtype": "bf16",
        "data": "synthetic",
        "config": {
            "model": "Llama-3-8B" if args.model in ("llama3-8b", "llama3_8b") else args.model,
            "global_batch": args.micro_batch * args.grad_accum * n,
            "micro_batch": args.micro_batch,
            "grad_accum": args.grad_accum,
            "seq_len": args.seq_len,
            "tokens_per_gpu_per_step": args.micro_batch * args.grad_accum * args.seq_len,
            "parallelism": f"dp{n}",
            "optimizer": "AdamW (fp32 master, fused flat kernel, clip 1.0)"
                         + (f", ZeRO-1 sharded over {n} ranks" if tr.store.sharded else ""),
            "zero": 1 if tr.store.sharded else 0,
            "attention": attention_backend(),
            "grad_bucket_mb": args.bucket_mb,
            "gemm_table": bool(getattr(tr, "gemm_table", False)),  # measured hipBLASLt/rocBLAS choices (ops/tuned)
            "gemm_table_kind": getattr(tr, "gemm_table_name", None),
        },
        "tflops_per_gpu": round(flops / n / 1e12, 1),
        "peak_mem_gib": round(torch.cuda.max_memory_allocated() / 2**30, 1) if torch.cuda.is_available() else None,
        "final_loss": round(res["loss"], 4),
        # where a step's time went besides compute (max over ranks, ms per step): the compute stream's
        # stalls on gradient buckets + parameter all-gathers, and on the overlapped optimizer
        "exposed_comm_ms_per_step": comm["exposed_comm_ms_per_step"],
        "allgather_wait_ms": comm["allgather_wait_ms"],
        "opt_wait_ms": comm["opt_wait_ms"],
        "dist": {**census, "comm": comm},
        # CUs the TN weight-gradient launches were planned for during backward (null = all 256) and the
        # one-GPU RCCL channel-footprint rehearsal, when TH_COMM_EMU asks for it (parallel/comm_emu.py)
        "tn_backward_cus": tr.bwd_cus,
        "comm_emu": emu,
    }
    if info.is_main:
        line["daemon"] = daemon_poll_latency() if args.daemon_bench else None
        print(json.dumps(line), flush=True)
    barrier(info)  # the other ranks keep their RCCL communicator until rank 0's daemon bench is done
    shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
