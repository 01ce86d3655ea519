"""Multi-rank correctness check of the flat-buffer DDP step on GPU tensors (torchrun launched).

Every rank trains the tiny Llama for 3 steps on its own synthetic batch, once with the replicated
all-reduce optimizer (ZeRO-0) and once with the sharded optimizer (ZeRO-1: reduce-scatter, 1/world
AdamW, all-gather overlapped with the next forward); afterwards all ranks must hold bit-identical
parameters in both modes and the two modes must agree to bf16 rounding.  Prints one JSON line on
rank 0.
Used by tests/gpu/test_ddp_gpu.py with TH_DIST_BACKEND=gloo (two ranks share the box's one GPU).
"""
import json
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, ".")
from tensorhive_fixed_amd.models.llama3 import LlamaConfig  # noqa: E402
from tensorhive_fixed_amd.parallel.dist import init_distributed, shutdown  # noqa: E402
from tensorhive_fixed_amd.workloads.llama3_ddp import Trainer  # noqa: E402


def _run(info, zero):
    cfg = LlamaConfig.named("tiny")
    tr = Trainer(cfg, info, micro_batch=2, seq_len=128, bucket_mb=0.25, zero=zero)
    for _ in range(3):
        tr.step()
    tr.store.wait_all_params()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    params = {n: p.detach().float().clone() for n, p in zip(tr.store.names, tr.store.params)}
    flat = torch.cat([params[n].reshape(-1) for n in sorted(params)])
    gathered = [torch.empty_like(flat) for _ in range(info.world)]
    dist.all_gather(gathered, flat)
    same = all(torch.equal(gathered[0], g) for g in gathered[1:])
    return tr, flat, same


def main():
    info = init_distributed()
    tr0, p0, same0 = _run(info, 0)
    tr1, p1, same1 = _run(info, 1)
    frac_off = float(((p0 - p1).abs() > 1e-2).float().mean())
    ok = same0 and same1 and tr1.store.sharded and frac_off < 1e-3
    if info.is_main:
        print(json.dumps({"world": info.world, "backend": info.backend, "params_identical": same0,
                          "params_identical_zero1": same1, "zero1_vs_zero0_frac_off": frac_off,
                          "n_buckets": len(tr0.store.buckets), "loss": float(tr0.last_loss),
                          "loss_zero1": float(tr1.last_loss),
                          "opt_state_numel": [tr0.opt.master.numel(), tr1.opt.master.numel()]}), flush=True)
    shutdown()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
