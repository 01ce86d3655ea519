"""SwiGLU kernels at the Llama-3-8B MLP shape (T 32768, F 14336): forward and the backward that also
writes the transposed gradient, in TB/s of the bytes they move; with AB_BASE_LIB set the in-tree
library and the base library alternate in one process."""
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


libs = {"new": _lib.load()}
if os.environ.get("AB_BASE_LIB"):
    libs["base"] = open_lib(os.environ["AB_BASE_LIB"])
T, F = 32768, 14336
dev = torch.device("cuda")
gu = torch.randn(T, 2 * F, device=dev, dtype=torch.bfloat16)
a = torch.empty(T, F, device=dev, dtype=torch.bfloat16)
da = torch.randn(T, F, device=dev, dtype=torch.bfloat16)
dgu = torch.empty_like(gu)
dguT = torch.empty(2 * F, T, device=dev, dtype=torch.bfloat16)
st = lambda: _lib.stream_ptr(dev)  # noqa: E731
ops = {
    "fwd": (lambda: _lib.call("th_swiglu_fwd", gu.data_ptr(), a.data_ptr(), T, F, st()), 3 * T * F * 2),
    "bwd_t": (lambda: _lib.call("th_swiglu_bwd_t", da.data_ptr(), gu.data_ptr(), dgu.data_ptr(), dguT.data_ptr(),
                                T, F, st()), 7 * T * F * 2),
}
# correctness of the transposed output against the row-major one (new library)
ops["bwd_t"][0]()
torch.cuda.synchronize()
assert torch.equal(dguT, dgu.t()), "dguT != dgu^T"
times = {(k, o): [] for k in libs for o in ops}
for rnd in range(8):
    for k in (list(libs) if rnd % 2 else list(libs)[::-1]):
        _lib._lib = libs[k]
        for o, (fn, _) in ops.items():
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                fn()
            e1.record()
            torch.cuda.synchronize()
            times[(k, o)].append(e0.elapsed_time(e1) / 5)
for o, (_, nbytes) in ops.items():
    row = {"op": o}
    for k in libs:
        ms = statistics.median(times[(k, o)])
        row[k + "_ms"] = round(ms, 4)
        row[k + "_TBps"] = round(nbytes / ms / 1e9, 2)
    print(json.dumps(row), flush=True)
