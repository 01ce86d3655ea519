#!/usr/bin/env python3
"""Attribute the small device kernels of a training step to their Python call sites.

Runs a few steps of the Llama payload (8B layer shapes, fewer layers by default) under
``torch.profiler`` and prints (a) device time per aten op + input shapes, (b) the Python stack of
every elementwise add / copy / fill launched inside the timed step -- the kernels rocprofv3 only
reports by name (``CUDAFunctor_add``, ``FillFunctor``, ``copyBuffer``).

    python scripts/profile_ops.py --layers 2 --micro-batch 8
"""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from tensorhive_fixed_amd.models.llama3 import LlamaConfig  # noqa: E402
from tensorhive_fixed_amd.ops import _lib  # noqa: E402
from tensorhive_fixed_amd.parallel.dist import init_distributed  # noqa: E402
from tensorhive_fixed_amd.workloads.llama3_ddp import Trainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--micro-batch", type=int, default=8)
    ap.add_argument("--seq-len", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=2)
    args = ap.parse_args()
    _lib.load(build_if_missing=True)
    info = init_distributed()
    cfg = LlamaConfig.named("llama3-8b")
    cfg.n_layers = args.layers
    tr = Trainer(cfg, info, args.micro_batch, args.seq_len)
    tr.step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True,
                 with_stack=True) as prof:
        for _ in range(args.steps):
            tr.step()
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_input_shape=True).table(sort_by="self_device_time_total", row_limit=40,
                                                            max_name_column_width=60, max_shapes_column_width=60))
    stacks = collections.Counter()
    for ev in prof.events():
        if ev.name in ("aten::add", "aten::add_", "aten::copy_", "aten::fill_", "aten::zero_", "aten::zeros",
                       "aten::mul", "aten::clone", "aten::contiguous", "aten::to", "aten::_to_copy") \
                and ev.device_time_total > 0:
            st = [f for f in (ev.stack or []) if "tensorhive_fixed_amd" in f or "bench" in f][:4]
            stacks[(ev.name, str(ev.input_shapes)[:80], " <- ".join(st))] += ev.device_time_total
    print("\n== device time of elementwise ops by call site (us, over all profiled steps)")
    for (name, shapes, st), us in stacks.most_common(30):
        print(f"{us:10.0f}  {name:14s} {shapes}\n            {st}")


if __name__ == "__main__":
    main()
