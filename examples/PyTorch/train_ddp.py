"""Minimal data-parallel PyTorch-ROCm training script for the TensorHive task-execution examples.

It accepts both launch styles the job templates generate (core/launcher.py):

* ``torchrun`` template -- rank / world size / rendezvous come from the environment torchrun sets;
* ``torch`` template    -- one process per GPU with explicit flags:
  ``--init-method=tcp://<master>:<port> --backend=nccl --rank=<r> --world-size=<n>``
  (``backend nccl`` is RCCL on ROCm; ``gloo`` runs on CPUs).

The GPU is whatever ``HIP_VISIBLE_DEVICES`` (set by TensorHive from the reservation or the
allocator) leaves visible.  The model is a small MLP on synthetic data; every rank prints one
``[example] rank=.. step=.. loss=..`` line per step and a final ``[example] done`` line.
"""
import argparse
import os
import time

import torch
import torch.distributed as dist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--init-method", default=None, help="tcp://host:port (torch template)")
    ap.add_argument("--backend", default=None, help="nccl (= RCCL) or gloo")
    ap.add_argument("--rank", type=int, default=None)
    ap.add_argument("--world-size", type=int, default=None)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--width", type=int, default=1024)
    a = ap.parse_args()

    cuda = torch.cuda.is_available()
    backend = a.backend or ("nccl" if cuda else "gloo")
    if backend == "nccl" and not cuda:
        backend = "gloo"
    if a.init_method:  # torch template: explicit rendezvous
        dist.init_process_group(backend, init_method=a.init_method, rank=a.rank, world_size=a.world_size)
    else:  # torchrun template: env:// rendezvous
        dist.init_process_group(backend)
    rank, world = dist.get_rank(), dist.get_world_size()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count())) if cuda else torch.device("cpu")
    if cuda:
        torch.cuda.set_device(dev)
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(a.width, a.width), torch.nn.GELU(),
                                torch.nn.Linear(a.width, 10)).to(dev)
    ddp = torch.nn.parallel.DistributedDataParallel(model, device_ids=[dev.index] if cuda else None)
    opt = torch.optim.AdamW(ddp.parameters(), lr=1e-3)
    g = torch.Generator(device="cpu").manual_seed(1000 + rank)
    t0 = time.time()
    for step in range(1, a.steps + 1):
        x = torch.randn(a.batch, a.width, generator=g).to(dev)
        y = torch.randint(0, 10, (a.batch,), generator=g).to(dev)
        loss = torch.nn.functional.cross_entropy(ddp(x), y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        print(f"[example] rank={rank} world={world} step={step} loss={loss.item():.4f}", flush=True)
    # replicas must agree after DDP's all-reduced updates
    flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    ref = flat.clone()
    dist.broadcast(ref, 0)
    same = bool(torch.equal(flat, ref))
    print(f"[example] done rank={rank} world={world} backend={backend} replicas_identical={same} "
          f"seconds={time.time() - t0:.2f}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
