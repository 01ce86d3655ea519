"""RMSNorm backward at the Llama-3-8B shape (T 32768, D 4096, with the residual-gradient add) over
the number of workgroups (= dW partial slabs): bytes moved / time."""
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
dy = torch.randn(T, D, device=dev).to(torch.bfloat16)
dres = torch.randn(T, D, device=dev).to(torch.bfloat16)
w = torch.rand(D, device=dev).to(torch.bfloat16)
rstd = torch.rand(T, device=dev) + 0.5
dx = torch.empty_like(x)
dw = torch.empty_like(w)
ref = None
for nblk in [int(v) for v in os.environ.get("NBLK", "512,1024,2048,4096").split(",")]:
    ws = torch.empty(nblk * D, device=dev, dtype=torch.float32)
    fn = lambda: _lib.call("th_rmsnorm_bwd", dy.data_ptr(), x.data_ptr(), w.data_ptr(), rstd.data_ptr(),  # noqa: E731
                           dx.data_ptr(), dw.data_ptr(), ws.data_ptr(), nblk, T, D, 0, dres.data_ptr(),
                           _lib.stream_ptr(dev))
    fn()
    torch.cuda.synchronize()
    if ref is None:
        ref = (dx.clone(), dw.float().clone())
    else:
        assert torch.equal(dx, ref[0])
        assert ((dw.float() - ref[1]).abs().max() / ref[1].abs().max()).item() < 1e-2
    ts = []
    for _ in range(7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 5)
    ms = statistics.median(ts)
    print(json.dumps({"nblk": nblk, "ms": round(ms, 4), "TBps": round(4 * T * D * 2 / ms / 1e9, 2)}), flush=True)
