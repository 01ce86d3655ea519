"""Round-5 one-wave-per-SIMD flash forward (fa_fwd_w1_kernel, variant bit 5 = 32 + 15): fp32 check of O and
LSE against a PyTorch reference (causal and not, GQA), then timing against the default forward at the
training shape (B 8, S 4096, 32 / 8 heads, d 128, causal)."""
import json
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorhive_fixed_amd.ops import _lib  # noqa: E402
from tensorhive_fixed_amd.ops.attention import flash_fwd  # noqa: E402

W1 = 32 + 15


def ref(qkv, B, S, Hq, Hkv, D, causal):
    q, k, v = qkv.float().split([Hq * D, Hkv * D, Hkv * D], dim=1)
    q = q.view(B, S, Hq, D).transpose(1, 2)
    k = k.view(B, S, Hkv, D).transpose(1, 2).repeat_interleave(Hq // Hkv, dim=1)
    v = v.view(B, S, Hkv, D).transpose(1, 2).repeat_interleave(Hq // Hkv, dim=1)
    s = q @ k.transpose(-1, -2) / math.sqrt(D)
    if causal:
        s = s.masked_fill(torch.triu(torch.ones(S, S, dtype=torch.bool, device=qkv.device), 1), float("-inf"))
    lse = torch.logsumexp(s, -1)
    o = (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(B * S, Hq * D)
    return o, lse


def timed(fn, iters=10):
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts)


def main():
    _lib.load()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    for (B, S, Hq, Hkv, causal, scale) in ((1, 256, 4, 1, True, 1.0), (2, 512, 8, 2, True, 1.0), (1, 768, 4, 4, False, 1.0),
                                           (1, 1024, 8, 2, True, 4.0), (2, 1024, 8, 8, False, 3.0)):
        D = 128
        qkv = (torch.randn(B * S, (Hq + 2 * Hkv) * D, device=dev, generator=g) * scale).to(torch.bfloat16)
        o_r, lse_r = ref(qkv, B, S, Hq, Hkv, D, causal)
        res = {}
        for name, v in (("default", None), ("w1", W1)):
            o, lse = flash_fwd(qkv, B, S, Hq, Hkv, D, causal=causal, variant=v)
            res[name] = {"o_rel": ((o.float() - o_r).norm() / o_r.norm()).item(),
                         "lse_max_abs": (lse - lse_r).abs().max().item()}
        print(json.dumps({"check": [B, S, Hq, Hkv, causal, scale], **res}), flush=True)
        assert res["w1"]["o_rel"] < 1e-2 and res["w1"]["lse_max_abs"] < 1e-2, res
    B, S, Hq, Hkv, D = 8, 4096, 32, 8, 128
    qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16)
    o0, l0 = flash_fwd(qkv, B, S, Hq, Hkv, D)
    o1, l1 = flash_fwd(qkv, B, S, Hq, Hkv, D, variant=W1)
    diff = ((o1.float() - o0.float()).norm() / o0.float().norm()).item()
    t = {"default": [], "w1": []}
    for _ in range(3):
        t["default"].append(timed(lambda: flash_fwd(qkv, B, S, Hq, Hkv, D)))
        t["w1"].append(timed(lambda: flash_fwd(qkv, B, S, Hq, Hkv, D, variant=W1)))
    fl = 4.0 * B * Hq * S * S * D / 2
    print(json.dumps({"shape": [B, S, Hq, Hkv, D], "rel_diff_w1_vs_default": diff,
                      "lse_max_abs_diff": (l1 - l0).abs().max().item(),
                      **{k + "_ms": round(min(v), 4) for k, v in t.items()},
                      **{k + "_tflops": round(fl / min(v) / 1e9) for k, v in t.items()}}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
