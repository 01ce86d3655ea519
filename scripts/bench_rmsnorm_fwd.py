"""RMSNorm forward with the fused residual add at the Llama-3-8B shape (T 32768, D 4096): bytes moved / time
(8 B per element: x, addend read; xsum, y written).  TH_RMS_WAVE=0|1 picks the kernel (per process)."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tensorhive_fixed_amd.ops import _lib  # noqa: E402

_lib.load()
T, D = 32768, 4096
dev = torch.device("cuda")
x = torch.randn(T, D, device=dev).to(torch.bfloat16)
a = torch.randn(T, D, device=dev).to(torch.bfloat16)
w = torch.rand(D, device=dev).to(torch.bfloat16)
xs, y = torch.empty_like(x), torch.empty_like(x)
rstd = torch.empty(T, device=dev)
fn = lambda: _lib.call("th_rmsnorm_add_fwd", x.data_ptr(), a.data_ptr(), w.data_ptr(), xs.data_ptr(),  # noqa: E731
                       y.data_ptr(), rstd.data_ptr(), T, D, 1e-5, _lib.stream_ptr(dev))
fn()
torch.cuda.synchronize()
s = x.float() + a.float()
ref = s * torch.rsqrt(s.pow(2).mean(-1, keepdim=True) + 1e-5) * w.float()
assert (y.float() - ref).abs().max().item() < 0.1
ts = []
for _ in range(9):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) / 10)
med = statistics.median(ts)
print(json.dumps({"kernel": "rmsnorm_add_fwd", "wave": os.environ.get("TH_RMS_WAVE", "1"), "us": round(med * 1e3, 1),
                  "tb_s": round(8 * T * D / 1e12 / (med / 1e3), 3)}))
