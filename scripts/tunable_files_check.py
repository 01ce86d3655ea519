"""Does the lookup-only TunableOp table (ops/tuned) write any results file when a process exits?  Runs one
tuned-shape GEMM and one untuned one from /tmp, then the caller lists tunableop* files there and in the repo."""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from tensorhive_fixed_amd.ops.tuned import load_gemm_table  # noqa: E402

print("loaded", load_gemm_table(), "filename", torch.cuda.tunable.get_filename(), flush=True)
a = torch.randn(32768, 4096, device="cuda", dtype=torch.bfloat16)
w = torch.randn(28672, 4096, device="cuda", dtype=torch.bfloat16)
y = a @ w.t()
z = torch.randn(300, 200, device="cuda", dtype=torch.bfloat16) @ torch.randn(200, 100, device="cuda", dtype=torch.bfloat16)
torch.cuda.synchronize()
print("ok", flush=True)
