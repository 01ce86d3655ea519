"""LM-head weight gradient per CE chunk (round 5): dW[V, D] += dlogits[chunk, V]^T h[chunk, D].
The default path transposes both operands and runs hipBLASLt's K-contiguous GEMM (TH_HEAD_WGRAD_NT);
the TN path (TH_HEAD_WGRAD_TN) runs the gfx950 TN kernel (hb schedule, mode 10) straight on the
[tokens, V] logits.  Times both, transposes included, and checks TN against fp32 on a slice."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorhive_fixed_amd.ops import _lib  # noqa: E402
from tensorhive_fixed_amd.ops.gemm_tn import gemm_tn_  # noqa: E402
from tensorhive_fixed_amd.ops.transpose import transpose  # noqa: E402


def timed(fn, iters=10):
    ts = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    return statistics.median(ts)


def main():
    _lib.load()
    dev = torch.device("cuda:0")
    V, D = 128256, 4096
    for chunk in (4096, 8192):
        logits = torch.randn(chunk, V, device=dev, dtype=torch.bfloat16) * 0.01
        hc = torch.randn(chunk, D, device=dev, dtype=torch.bfloat16)
        acc = torch.zeros(V, D, device=dev, dtype=torch.bfloat16)

        def nt():
            a_op, b_op = transpose(logits), transpose(hc).t()
            acc.addmm_(a_op, b_op)

        def tn():
            gemm_tn_(logits, hc, acc, accumulate=True)

        acc.zero_()
        tn()
        ref = logits[:, :512].float().t() @ hc.float()
        err = ((acc[:512].float() - ref).norm() / ref.norm()).item()
        res = {"nt_T": [], "tn": []}
        for _ in range(3):
            res["nt_T"].append(timed(nt))
            res["tn"].append(timed(tn))
        fl = 2.0 * V * D * chunk
        out = {"chunk": chunk, "rel_err_tn_slice": err}
        for k, ts in res.items():
            out[k + "_ms"] = round(min(ts), 4)
            out[k + "_tflops"] = round(fl / min(ts) / 1e9)
        print(json.dumps(out), flush=True)
        del logits, hc, acc
    return 0


if __name__ == "__main__":
    sys.exit(main())
