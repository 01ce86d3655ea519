"""RMSNorm forward (plain and with the fused residual add) at the Llama-3-8B shape (T 32768, D 4096): the
in-tree library against builds with more rows per workgroup (profiles/r05_step/rmsnorm_fwd_rows.patch applied, then scripts/build_variant_lib.sh NAME
-DTH_RMS_FWD_ROWS=N rmsnorm), loaded side by side and timed in interleaved rounds; outputs must be
bit-identical.  AB_VARIANTS="name=path,...".  Prints one JSON line per (library, kernel)."""
import ctypes as C
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tensorhive_fixed_amd.ops import _lib  # noqa: E402


def open_lib(path):
    lib = C.CDLL(path)
    for name, argtypes in _lib._SIGS.items():
        fn = getattr(lib, name, None)
        if fn is not None:
            fn.argtypes = argtypes
            fn.restype = C.c_int
    return lib


libs = {"rows1": _lib.load()}
for spec in filter(None, os.environ.get("AB_VARIANTS", "").split(",")):
    name, path = spec.split("=", 1)
    libs[name] = open_lib(path)
T, D = 32768, 4096
dev = torch.device("cuda")
st = _lib.stream_ptr(dev)
x = torch.randn(T, D, device=dev).to(torch.bfloat16)
a = torch.randn(T, D, device=dev).to(torch.bfloat16)
w = torch.rand(D, device=dev).to(torch.bfloat16)
outs = {n: (torch.empty_like(x), torch.empty_like(x), torch.empty(T, device=dev)) for n in libs}


def call(n, kind):
    lib, (xs, y, rstd) = libs[n], outs[n]
    if kind == "add":
        rc = lib.th_rmsnorm_add_fwd(x.data_ptr(), a.data_ptr(), w.data_ptr(), xs.data_ptr(), y.data_ptr(),
                                    rstd.data_ptr(), T, D, 1e-5, st)
    else:
        rc = lib.th_rmsnorm_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), rstd.data_ptr(), T, D, 1e-5, st)
    assert rc == 0, rc


for kind, nbytes in (("add", 4 * T * D * 2), ("plain", 2 * T * D * 2)):
    for n in libs:
        call(n, kind)
    torch.cuda.synchronize()
    for n in libs:
        for i in ((0, 1, 2) if kind == "add" else (1, 2)):
            assert torch.equal(outs[n][i], outs["rows1"][i]), (n, kind, i)
    ts = {n: [] for n in libs}
    for _ in range(9):
        for n in libs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                call(n, kind)
            e1.record()
            torch.cuda.synchronize()
            ts[n].append(e0.elapsed_time(e1) / 10)
    for n in libs:
        ms = statistics.median(ts[n])
        print(json.dumps({"lib": n, "kernel": kind, "us": round(ms * 1000, 1),
                          "TBps": round(nbytes / ms / 1e9, 2)}), flush=True)
