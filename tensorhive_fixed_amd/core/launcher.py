"""Launch templates + topology-aware device placement (reference UI
templates ``TaskCreate.vue:201-215,338-460,617-831``).

The reference filled ``CUDA_VISIBLE_DEVICES=<first char>`` and gloo/TF arguments in the browser.
Here the server owns the launch recipe:

* ``torchrun`` -- PyTorch-ROCm, one process per GPU, backend ``nccl`` (= RCCL over xGMI), with
  ``HIP_VISIBLE_DEVICES`` derived from the user's reservation (UUID -> HIP index through the
  telemetry snapshot, never enumeration-order guessing), RCCL/HIP env presets and rank order
  grouped by NUMA node; defaults to the Llama-3 DDP payload.
* ``pytorch_tcp`` -- the reference's explicit ``--init-method/--backend/--rank/--world-size``
  template (kept for user programs that parse those flags; backend defaults to ``nccl``).
* ``tf2`` -- TF_CONFIG (persisted as an env segment -- the reference only previewed it).
* ``tf1`` -- ClusterSpec ``--ps_hosts/--worker_hosts/--job_name/--task_index``.
"""
from __future__ import annotations

import json

# the payload's own presets (parallel/dist.py::rccl_env_defaults, which it applies itself when unset), written
# into the template so a user's torchrun job sees them too; kept equal by tests/test_comm_emu.py
RCCL_ENV = {
    "HSA_ENABLE_IPC_MODE_LEGACY": "0",
    "TORCH_NCCL_ASYNC_ERROR_HANDLING": "1",
    "NCCL_DEBUG": "WARN",
    "TORCH_NCCL_HIGH_PRIORITY": "1",
    "TENSILE_STREAMK_DATA_PARALLEL": "1",
}

TEMPLATES = {
    "torchrun": {
        "description": "PyTorch-ROCm DDP via torchrun (RCCL over xGMI), one process per reserved GPU",
        "command": "torchrun",
        "envs": [{"name": "HIP_VISIBLE_DEVICES", "value": "<from reservation>"}] +
                [{"name": k, "value": v} for k, v in RCCL_ENV.items()],
        "params": [{"name": "--nnodes=", "value": "1"}, {"name": "--nproc_per_node=", "value": "<#GPUs>"},
                   {"name": "--rdzv_backend=", "value": "c10d"},
                   {"name": "--rdzv_endpoint=", "value": "<host>:29500"},
                   {"name": "--max-restarts=", "value": "0"},
                   {"name": "-m", "value": "tensorhive_fixed_amd.workloads.llama3_ddp"}],
    },
    "pytorch_tcp": {
        "description": "explicit rank/world-size flags (reference 'torch' template), backend nccl=RCCL",
        "command": "python train.py",
        "envs": [{"name": "HIP_VISIBLE_DEVICES", "value": "<gpu>"}],
        "params": [{"name": "--init-method=", "value": "tcp://<host>:29500"}, {"name": "--backend=", "value": "nccl"},
                   {"name": "--rank=", "value": "<auto 0..N-1>"}, {"name": "--world-size=", "value": "<auto N>"}],
    },
    "tf2": {"description": "TensorFlow 2 multi-worker via TF_CONFIG (persisted)", "command": "python train.py",
            "envs": [{"name": "TF_CONFIG", "value": "<generated>"}], "params": []},
    "tf1": {"description": "TensorFlow 1 ClusterSpec", "command": "python train.py", "envs": [],
            "params": [{"name": "--ps_hosts=", "value": "<host:port,...>"},
                       {"name": "--worker_hosts=", "value": "<host:port,...>"},
                       {"name": "--job_name=", "value": "worker|ps"}, {"name": "--task_index=", "value": "<auto>"}]},
}


# ----------------------------------------------------------------------- device placement
def devices_for_uuids(snapshot_data: dict, host: str, uuids: list[str]) -> list[int]:
    """Reserved GPU UUIDs -> HIP device indices on ``host`` (via the telemetry snapshot)."""
    gpus = (snapshot_data.get(host) or {}).get("GPU") or {}
    out = []
    for u in uuids:
        g = gpus.get(u)
        if g is None:
            raise KeyError(f"GPU {u} not found on {host}")
        out.append(int(g["index"]))
    return out


def order_for_rings(indices: list[int], topology: dict | None) -> list[int]:
    """Rank order: group devices by NUMA node (CPU affinity, host staging) and, inside a group,
    keep xGMI neighbours adjacent.  MI355X nodes are fully xGMI-connected (every pair one hop),
    so the ring order only matters across NUMA domains."""
    if not topology:
        return sorted(indices)
    info = {g["index"]: g for g in topology.get("gpus", [])}
    return sorted(indices, key=lambda i: (info.get(i, {}).get("numa_node", 0), i))


def rccl_env(cfg=None) -> dict[str, str]:
    """The environment a torchrun task starts with: the fixed RCCL/HIP presets, the rank CPU
    binding mode (applied by every rank itself, ``parallel/affinity.py``) and the RCCL channel /
    algorithm knobs of ``[launcher]`` that are set."""
    env = dict(RCCL_ENV)
    if cfg is None:
        try:
            from ..config import get_config

            cfg = get_config().launcher
        except Exception:  # noqa: BLE001 -- no config installed (library use)
            cfg = None
    env["TH_CPU_BIND"] = getattr(cfg, "cpu_bind", "numa") or "numa"
    for key, var in (("rccl_min_nchannels", "NCCL_MIN_NCHANNELS"), ("rccl_max_nchannels", "NCCL_MAX_NCHANNELS"),
                     ("rccl_algo", "NCCL_ALGO"), ("rccl_proto", "NCCL_PROTO")):
        v = str(getattr(cfg, key, "") or "").strip()
        if v:
            env[var] = v
    return env


def hip_visible_devices(indices: list[int]) -> str:
    return ",".join(str(i) for i in indices)


# --------------------------------------------------------------------------- builders
def torchrun_task(host: str, gpu_indices: list[int] | int, master_host: str, master_port: int = 29500,
                  nnodes: int = 1, module: str = "tensorhive_fixed_amd.workloads.llama3_ddp",
                  script_args: list[tuple[str, str]] | None = None) -> dict:
    """A TaskForm body for one node of a torchrun job.  ``gpu_indices`` is a pinned device list
    or a count; a count becomes ``HIP_VISIBLE_DEVICES=auto:N`` and the allocator picks the
    devices (NUMA-packed, reservation-aware) when the job starts (``core/allocation.py``)."""
    if isinstance(gpu_indices, int):
        devices, n = f"auto:{gpu_indices}", gpu_indices
    else:
        devices, n = hip_visible_devices(gpu_indices), len(gpu_indices)
    envs = [{"name": "HIP_VISIBLE_DEVICES", "value": devices}]
    envs += [{"name": k, "value": v} for k, v in rccl_env().items()]
    params = [{"name": "--nnodes=", "value": str(nnodes)},
              {"name": "--nproc_per_node=", "value": str(n)},
              {"name": "--rdzv_backend=", "value": "c10d"},
              {"name": "--rdzv_endpoint=", "value": f"{master_host}:{master_port}"},
              {"name": "-m", "value": module}]
    params += [{"name": k, "value": v} for k, v in (script_args or [])]
    return {"hostname": host, "command": "torchrun", "cmdsegments": {"envs": envs, "params": params}}


def pytorch_tcp_tasks(placements: list[tuple[str, int]], master: str, port: int = 29500,
                      command: str = "python train.py", backend: str = "nccl") -> list[dict]:
    """One task per (host, gpu) with explicit rank/world-size (reference 'torch' template)."""
    world = len(placements)
    out = []
    for rank, (host, gpu) in enumerate(placements):
        out.append({"hostname": host, "command": command, "cmdsegments": {
            "envs": [{"name": "HIP_VISIBLE_DEVICES", "value": str(gpu)}],
            "params": [{"name": "--init-method=", "value": f"tcp://{master}:{port}"},
                       {"name": "--backend=", "value": backend}, {"name": "--rank=", "value": str(rank)},
                       {"name": "--world-size=", "value": str(world)}]}})
    return out


def tf_config(cluster: dict[str, list[str]], task_type: str, index: int) -> str:
    return json.dumps({"cluster": cluster, "task": {"type": task_type, "index": index}}, separators=(",", ":"))


def tf2_tasks(roles: list[tuple[str, str, int]], base_port: int = 2222, command: str = "python train.py") -> list[dict]:
    """roles: [(host, task_type, gpu)] -> tasks with a persisted TF_CONFIG; ports auto-increment
    per host from ``base_port`` (the reference's "smart TF_CONFIG")."""
    next_port: dict[str, int] = {}
    addrs: list[tuple[str, str]] = []
    for host, ttype, _gpu in roles:
        p = next_port.get(host, base_port)
        next_port[host] = p + 1
        addrs.append((ttype, f"{host}:{p}"))
    cluster: dict[str, list[str]] = {}
    for ttype, addr in addrs:
        cluster.setdefault(ttype, []).append(addr)
    counters: dict[str, int] = {}
    out = []
    for host, ttype, gpu in roles:
        idx = counters.get(ttype, 0)
        counters[ttype] = idx + 1
        out.append({"hostname": host, "command": command, "cmdsegments": {
            "envs": [{"name": "HIP_VISIBLE_DEVICES", "value": str(gpu)},
                     {"name": "TF_CONFIG", "value": tf_config(cluster, ttype, idx)}], "params": []}})
    return out


def tf1_tasks(ps: list[str], workers: list[tuple[str, int]], base_port: int = 2222,
              command: str = "python train.py") -> list[dict]:
    ps_hosts = ",".join(f"{h}:{base_port + i}" for i, h in enumerate(ps))
    worker_hosts = ",".join(f"{h}:{base_port + len(ps) + i}" for i, (h, _g) in enumerate(workers))
    out = []
    for i, h in enumerate(ps):
        out.append({"hostname": h, "command": command, "cmdsegments": {"envs": [{"name": "HIP_VISIBLE_DEVICES", "value": ""}],
                    "params": [{"name": "--ps_hosts=", "value": ps_hosts}, {"name": "--worker_hosts=", "value": worker_hosts},
                               {"name": "--job_name=", "value": "ps"}, {"name": "--task_index=", "value": str(i)}]}})
    for i, (h, g) in enumerate(workers):
        out.append({"hostname": h, "command": command, "cmdsegments": {"envs": [{"name": "HIP_VISIBLE_DEVICES", "value": str(g)}],
                    "params": [{"name": "--ps_hosts=", "value": ps_hosts}, {"name": "--worker_hosts=", "value": worker_hosts},
                               {"name": "--job_name=", "value": "worker"}, {"name": "--task_index=", "value": str(i)}]}})
    return out


def attach_to_reservation(task_form: dict, snapshot_data: dict, reserved_uuids: list[str],
                          topology: dict | None = None) -> dict:
    """Rewrite a task's device segment to the reservation's GPUs (UI 'attach job to
    reservation', reference ``FullCalendarInfo.vue:510-548``) -- HIP indices, never CUDA."""
    idx = order_for_rings(devices_for_uuids(snapshot_data, task_form["hostname"], reserved_uuids), topology)
    segs = task_form.setdefault("cmdsegments", {"envs": [], "params": []})
    envs = [e for e in segs.get("envs", []) if e["name"] not in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")]
    segs["envs"] = [{"name": "HIP_VISIBLE_DEVICES", "value": hip_visible_devices(idx)}] + envs
    for p in segs.get("params", []):
        if p["name"] == "--nproc_per_node=":
            p["value"] = str(len(idx))
    return task_form
