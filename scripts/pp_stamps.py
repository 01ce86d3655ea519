"""Segment anatomy of the ping-pong flash forward (diagnostic library built with -DTH_PP_STAMP=1):
s_memtime at each segment boundary of workgroup 0 (the heaviest q block), per wave and step."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from tensorhive_fixed_amd.ops import _lib  # noqa: E402
from tensorhive_fixed_amd.ops.attention import flash_fwd  # noqa: E402


def main():
    lib = _lib.load()
    B, S, Hq, Hkv, D = 8, 4096, 32, 8, 128
    qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        flash_fwd(qkv, B, S, Hq, Hkv, D, variant=64)
    torch.cuda.synchronize()
    buf = np.zeros(8 * 72 * 5, dtype=np.uint64)
    raw = ctypes.CDLL(str(_lib._LIB_PATH))
    rc = raw.th_pp_stamps(ctypes.c_void_p(buf.ctypes.data))
    assert rc == 0, rc
    st = buf.reshape(8, 72, 5).astype(np.int64)
    t0 = st[:, 0, 0].min()
    names = ["mfma", "wait+bar1", "softmax", "dma+pref+wait+bar2"]
    for w in range(8):
        steps = [i for i in range(1, 60) if st[w, i, 0] and st[w, i, 4]]
        seg = np.array([[st[w, i, k + 1] - st[w, i, k] for k in range(4)] for i in steps])
        per_step = np.array([st[w, i + 1, 0] - st[w, i, 0] for i in steps if st[w, i + 1, 0]])
        print(json.dumps({"wave": w, "steps": len(steps),
                          **{n: int(np.median(seg[:, k])) for k, n in enumerate(names)},
                          "step_cycles_median": int(np.median(per_step)) if len(per_step) else None,
                          "first_start": int(st[w, 0, 0] - t0)}), flush=True)
    # phase alignment: A wave 0's MFMA segment vs B wave 4's softmax in the same phase
    for i in (10, 30, 50):
        print(json.dumps({"step": i, "A0": [int(x - t0) for x in st[0, i]], "B4": [int(x - t0) for x in st[4, i]]}))


if __name__ == "__main__":
    main()
