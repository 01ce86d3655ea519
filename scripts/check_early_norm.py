"""Llama-3-8B training step (bench shape): the early per-bucket gradient norm (TH_OPT_SUMSQ_EARLY=1)
against a fresh sum of squares over the same gradient buffer after the step, per bucket and total.
Prints one JSON line per step."""
import json
import os
import time

import torch

os.environ["TH_OPT_SUMSQ_EARLY"] = "1"  # the form under test (opt-in)

from tensorhive_fixed_amd.models.llama3 import LlamaConfig  # noqa: E402
from tensorhive_fixed_amd.ops.adamw import grad_sumsq_  # noqa: E402
from tensorhive_fixed_amd.parallel.dist import init_distributed  # noqa: E402
from tensorhive_fixed_amd.workloads.llama3_ddp import Trainer  # noqa: E402


def main():
    info = init_distributed("cuda")
    tr = Trainer(LlamaConfig.named("llama3-8b"), info, 8, 4096, 1)
    st, opt = tr.store, tr.opt
    assert opt.early_sumsq
    for s in range(3):
        t0 = time.time()
        tr.step()
        opt.wait_done()
        torch.cuda.synchronize()
        parts = opt.norm_parts.double().cpu()
        fresh = torch.zeros(len(st.buckets), device=st.device, dtype=torch.float32)
        for b in st.buckets:
            grad_sumsq_(st.grad_buf[b.start:b.end], fresh[b.index: b.index + 1])
        whole = torch.zeros(1, device=st.device, dtype=torch.float32)
        grad_sumsq_(st.grad_buf, whole)
        fresh = fresh.double().cpu()
        rel = ((parts - fresh).abs() / fresh.clamp_min(1e-30)).max().item()
        print(json.dumps({"step": s + 1, "early_steps": opt.early_steps, "buckets": len(st.buckets),
                          "norm_sq_used": float(opt.norm_sq[0]), "norm_sq_whole": float(whole[0]),
                          "max_rel_bucket_diff": rel, "loss": float(tr.last_loss),
                          "s": round(time.time() - t0, 2)}), flush=True)


if __name__ == "__main__":
    main()
