"""AdamW flat-step bandwidth: th_adamw_step over one 128M-parameter bucket (the trainer's 256 MB
bucket) and over 1.07B parameters, in TB/s of the 28 B/param it moves, plus a bf16 device copy as the
streaming reference. With AB_BASE_LIB set, the in-tree library and the base library alternate in
one process (interleaved rounds)."""
import ctypes as C
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tensorhive_fixed_amd.ops import _lib  # noqa: E402
from tensorhive_fixed_amd.ops.adamw import adamw_flat_  # noqa: E402


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
dev = torch.device("cuda")
norm = torch.ones(1, device=dev)


def timed(fn, reps=5):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for n in (128 << 20, 1 << 30):
    p = torch.randn(n, device=dev).to(torch.bfloat16)
    master, m, v = p.float(), torch.zeros(n, device=dev), torch.rand(n, device=dev)
    g = torch.randn(n, device=dev).to(torch.bfloat16)
    step = lambda: adamw_flat_(p, master, m, v, g, lr=1e-4, beta1=0.9, beta2=0.95, eps=1e-8,  # noqa: E731
                               weight_decay=0.1, step=3, norm_sq=norm, clip=1.0)
    times = {k: [] for k in libs}
    for rnd in range(8):
        for k in (list(libs) if rnd % 2 else list(libs)[::-1]):
            _lib._lib = libs[k]
            times[k].append(timed(step))
    row = {"params": n}
    for k in libs:
        ms = statistics.median(times[k])
        row[k + "_ms"] = round(ms, 4)
        row[k + "_TBps"] = round(28 * n / ms / 1e9, 2)
    src = torch.empty(2 * n, device=dev, dtype=torch.bfloat16)
    dst = torch.empty_like(src)
    ms = timed(lambda: dst.copy_(src))
    row["copy_TBps"] = round(2 * src.numel() * 2 / ms / 1e9, 2)
    print(json.dumps(row), flush=True)
    del p, master, m, v, g, src, dst
