"""NUMA-correct CPU binding of one-process-per-GPU ranks (round-2 verdict item 2).

The reference pinned each worker's environment by hand (``examples/PyTorch/README.md:28-54``).
Here every rank binds ITSELF, before it touches the GPU: local rank -> the HIP device it will use
(``HIP_VISIBLE_DEVICES`` / ``ROCR_VISIBLE_DEVICES`` applied to the KFD topology order, which is
HIP's enumeration order) -> that GPU's PCI BDF -> ``/sys/bus/pci/devices/<bdf>/numa_node`` ->
``/sys/devices/system/node/node<N>/cpulist`` -> ``os.sched_setaffinity``.  Nothing here calls
HIP, so it is safe to run before ``torch.cuda`` initialises (host threads created afterwards --
the data loader, torch's intra-op pool, RCCL's proxy thread -- inherit the mask).

Modes (``TH_CPU_BIND``): ``numa`` (default: every CPU of the GPU's NUMA node), ``exclusive``
(the node's CPUs split evenly between the local ranks whose GPUs sit on that node), ``none``.
"""
from __future__ import annotations

import os
from pathlib import Path

KFD_NODES = Path("/sys/class/kfd/kfd/topology/nodes")
PCI = Path("/sys/bus/pci/devices")
NODES = Path("/sys/devices/system/node")


def parse_cpulist(text: str) -> list[int]:
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11]."""
    out: list[int] = []
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def format_cpulist(cpus: list[int]) -> str:
    cpus = sorted(set(cpus))
    runs, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        runs.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(runs)


def _props(path: Path) -> dict[str, int]:
    out = {}
    try:
        for line in path.read_text().splitlines():
            k, _, v = line.partition(" ")
            if v.strip().lstrip("-").isdigit():
                out[k] = int(v)
    except OSError:
        pass
    return out


DRI = Path("/dev/dri")


def kfd_gpu_bdfs(root: Path = KFD_NODES, dri: Path | None = None) -> list[str]:
    """PCI BDFs of the GPUs this process can open, in KFD topology order (= HIP's physical
    enumeration order).  The sysfs topology lists every GPU of the machine; ROCr enumerates only
    those whose render node the process may open (a container or cgroup may expose a subset),
    so a node whose ``/dev/dri/renderD<minor>`` is missing or inaccessible is skipped."""
    dri = dri or DRI
    nodes = []
    if not root.exists():
        return []
    for d in root.iterdir():
        if not d.name.isdigit():
            continue
        p = _props(d / "properties")
        if p.get("simd_count", 0) <= 0:  # CPU node
            continue
        minor = p.get("drm_render_minor")
        if minor is not None and dri.exists() and not os.access(dri / f"renderD{minor}", os.R_OK | os.W_OK):
            continue
        loc, dom = p.get("location_id", 0), p.get("domain", 0)
        nodes.append((int(d.name), f"{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7:x}"))
    return [b for _n, b in sorted(nodes)]


def visible_physical(n_physical: int, env: dict | None = None) -> list[int]:
    """Physical GPU indices the process sees, in order (ROCR_VISIBLE_DEVICES applies first, then
    HIP_VISIBLE_DEVICES indexes into what ROCr left).  UUID entries are not resolved here."""
    env = os.environ if env is None else env
    order = list(range(n_physical))
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is None or v.strip() == "":
            continue
        try:
            idx = [int(x) for x in v.split(",") if x.strip() != ""]
        except ValueError:
            continue
        order = [order[i] for i in idx if 0 <= i < len(order)]
    return order


def numa_of_bdf(bdf: str, pci: Path = PCI) -> int | None:
    try:
        n = int((pci / bdf / "numa_node").read_text().strip())
    except (OSError, ValueError):
        return None
    return n if n >= 0 else None


def cpus_of_numa(node: int, nodes: Path = NODES) -> list[int]:
    try:
        return parse_cpulist((nodes / f"node{node}" / "cpulist").read_text())
    except OSError:
        return []


def plan(local_rank: int, local_world: int, mode: str = "numa", env: dict | None = None,
         kfd: Path | None = None, pci: Path | None = None, nodes: Path | None = None,
         dri: Path | None = None) -> dict:
    """What :func:`bind` would do for ``local_rank`` (pure; the sysfs/dev roots are parameters)."""
    kfd, pci, nodes = kfd or KFD_NODES, pci or PCI, nodes or NODES
    bdfs = kfd_gpu_bdfs(kfd, dri)
    vis = visible_physical(len(bdfs), env)
    out = {"mode": mode, "bdf": None, "numa_node": None, "cpus": None, "applied": False}
    if not vis:
        out["reason"] = "no GPU topology"
        return out
    phys = vis[local_rank % len(vis)]
    bdf = bdfs[phys]
    node = numa_of_bdf(bdf, pci)
    out.update(bdf=bdf, numa_node=node)
    if node is None:
        out["reason"] = "no NUMA node for the GPU"
        return out
    cpus = cpus_of_numa(node, nodes)
    if mode == "exclusive" and cpus:
        # the local ranks whose GPUs share this NUMA node split its CPUs in rank order
        peers = [r for r in range(local_world) if numa_of_bdf(bdfs[vis[r % len(vis)]], pci) == node]
        k, share = peers.index(local_rank), len(cpus) // max(1, len(peers))
        if share > 0:
            cpus = cpus[k * share:(k + 1) * share]
    out["cpus"] = format_cpulist(cpus) if cpus else None
    return out


def bind(local_rank: int, local_world: int, mode: str | None = None) -> dict:
    """Bind this process to the CPUs of its GPU's NUMA node; returns the plan plus ``applied``."""
    mode = (mode or os.environ.get("TH_CPU_BIND", "numa")).lower()
    if mode == "none":
        return {"mode": "none", "applied": False}
    p = plan(local_rank, local_world, mode)
    if p.get("cpus") and hasattr(os, "sched_setaffinity"):
        want = set(parse_cpulist(p["cpus"]))
        allowed = os.sched_getaffinity(0)
        use = want & allowed  # a cgroup/cpuset may already restrict us
        if use:
            os.sched_setaffinity(0, use)
            p["applied"] = True
            p["cpus"] = format_cpulist(sorted(use))
        else:
            p["reason"] = "NUMA CPUs outside the allowed cpuset"
    return p


def current_affinity() -> str | None:
    return format_cpulist(sorted(os.sched_getaffinity(0))) if hasattr(os, "sched_getaffinity") else None
