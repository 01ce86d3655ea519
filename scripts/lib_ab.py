"""In-process A/B of two builds of the kernel library (the in-tree libthk.so vs AB_BASE_LIB): the
flash forward and backward at B8 S4096 32/8 heads d128 causal, both libraries loaded side by side
and swapped between interleaved timing rounds (no process-to-process clock drift)."""
import ctypes as C
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tensorhive_fixed_amd.ops import _lib  # noqa: E402
from tensorhive_fixed_amd.ops.attention import flash_bwd, flash_fwd  # noqa: E402


def open_lib(path):
    lib = C.CDLL(path)
    for name, argtypes in _lib._SIGS.items():
        fn = getattr(lib, name, None)
        if fn is not None:
            fn.argtypes = argtypes
            fn.restype = C.c_int
    return lib


libs = {"new": _lib.load(), "base": open_lib(os.environ["AB_BASE_LIB"])}
# AB_VARIANTS="name=path,...": more builds timed in the same rotation (each reported against base)
for spec in filter(None, os.environ.get("AB_VARIANTS", "").split(",")):
    name, path = spec.split("=", 1)
    libs[name] = open_lib(path)
B, S, Hq, Hkv, D = int(os.environ.get("FA_B", "8")), 4096, 32, 8, 128
qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
o, lse = flash_fwd(qkv, B, S, Hq, Hkv, D)
do = torch.randn_like(o)
ops = {"fwd": lambda: flash_fwd(qkv, B, S, Hq, Hkv, D), "bwd": lambda: flash_bwd(do, qkv, o, lse, B, S, Hq, Hkv, D)}
times = {(k, op): [] for k in libs for op in ops}
for rnd in range(int(os.environ.get("AB_ROUNDS", "16"))):
    names = list(libs)
    for k in (names if rnd % 2 else names[::-1]):
        _lib._lib = libs[k]
        for op, fn in ops.items():
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                fn()
            e1.record()
            torch.cuda.synchronize()
            times[(k, op)].append(e0.elapsed_time(e1) / 3)
for op in ops:
    row = {"op": op}
    for k in libs:
        row[k + "_ms_median"] = round(statistics.median(times[(k, op)]), 4)
        row[k + "_ms_min"] = round(min(times[(k, op)]), 4)
    for k in libs:
        if k != "base":
            row[k + "_vs_base"] = round(row["base_ms_median"] / row[k + "_ms_median"], 4)
    print(json.dumps(row), flush=True)
