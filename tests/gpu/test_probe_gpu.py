"""Per-GPU device probe (round-2 verdict item 1), on a real MI355X.

The ``th-probe`` agent runs the gfx950 probe kernel on EVERY GPU of the node; the daemon's
monitor (this process, with the agent and th-counters as its children) is never listed as a
tenant, so it neither raises a protection violation on a reserved GPU nor makes a GPU look busy
to the allocator; ``mfma_contention`` is reported for every index libthsmi lists and rises under a
tenant GEMM on the LAST device (device 0 on a one-GPU box)."""
import datetime
import json
import os
import subprocess
import sys
import time

import pytest

pytestmark = pytest.mark.gpu

GEMM_LOAD = """
import time, torch
a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
b = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
print("ready", flush=True)
t0 = time.time()
while time.time() - t0 < 8:
    for _ in range(4):
        a @ b
    torch.cuda.synchronize()
"""


def _n_devices() -> int:
    import torch

    return torch.cuda.device_count()


def test_th_probe_agent_covers_every_device_at_low_duty():
    from tensorhive_fixed_amd.native.build import build_all, path_of

    build_all(strict=False)
    r = subprocess.run([str(path_of("th-probe")), "--count", "3", "--period-ms", "100", "--wg", "8"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    docs = [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]
    assert len(docs) == 3
    n = _n_devices()
    for doc in docs:
        assert sorted(g["hip"] for g in doc["gpus"]) == list(range(n))
        for g in doc["gpus"]:
            assert g["bdf"].count(":") == 2 and len(g["wg"]) == 8
            assert all(w[1] > 0 and w[3] > 0 for w in g["wg"])
            assert len({w[0] for w in g["wg"]}) >= 2  # spread over several XCDs
            kernel_us = max(w[1] + w[2] for w in g["wg"])
            assert kernel_us < 1000.0, kernel_us  # < 0.1 % of a 1 s period


def test_probe_busy_rises_under_a_tenant_gemm_on_the_last_device():
    from tensorhive_fixed_amd.core.telemetry import AmdSmiBackend

    dev = _n_devices() - 1
    b = AmdSmiBackend(probe=True, probe_period=0.1)
    try:
        assert b.probe is not None and b.probe.wait_first(60), b.probe and b.probe.error

        def busy():
            gpus = b.sample("localhost")["GPU"]
            g = next(g for g in gpus.values() if g["index"] == dev)
            return g["metrics"]["mfma_contention"]["value"], g["metrics"]["probe_baseline"]["value"]

        idle = []
        for _ in range(12):
            idle.append(busy()[0])
            time.sleep(0.12)
        env = {**os.environ, "HIP_VISIBLE_DEVICES": str(dev)}
        p = subprocess.Popen([sys.executable, "-c", GEMM_LOAD], stdout=subprocess.PIPE, text=True, env=env)
        try:
            assert p.stdout.readline().strip() == "ready"
            time.sleep(1.0)
            loaded = []
            for _ in range(10):
                loaded.append(busy()[0])
                time.sleep(0.12)
        finally:
            p.wait(timeout=120)
        idle_med = sorted(idle)[len(idle) // 2]
        busy_med = sorted(loaded)[len(loaded) // 2]
        print(f"device {dev}: probe mfma_contention idle median {idle_med:.1f} %, under GEMM {busy_med:.1f} %")
        assert idle_med < 25.0, idle
        assert busy_med >= idle_med + 30.0, (idle, loaded)
        assert b.probe.baselines, "baselines were learned"
    finally:
        b.close()


def test_monitor_is_never_its_own_tenant(cfg, tables, new_user):
    """Probe on: the daemon and its helpers are absent from every process list, mfma_contention is
    reported for every GPU, a reserved GPU 0 raises no violation, an auto:1 job may get GPU 0."""
    from tensorhive_fixed_amd.core import allocation
    from tensorhive_fixed_amd.core.daemon import Daemon
    from tensorhive_fixed_amd.core.services import MonitoringService, ProtectionService
    from tensorhive_fixed_amd.core.telemetry import AmdSmiBackend
    from tensorhive_fixed_amd.models.orm import Reservation, Resource, Restriction
    from tests.test_allocation import _job, _user

    import torch

    torch.ones(1, device="cuda")  # this process (the "daemon") now holds a GPU context too
    smi = AmdSmiBackend(probe=True, probe_period=0.2)
    host = next(iter(cfg.ssh.available_nodes))
    d = Daemon(cfg, backends={h: smi for h in cfg.ssh.available_nodes}, init_key=False, test_ssh=False)
    try:
        assert smi.probe.wait_first(60), smi.probe.error
        mon = MonitoringService(0.2, {host: smi})
        mon.inject(d)
        time.sleep(0.5)
        mon.do_run()
        snap = d.infrastructure.snapshot().data[host]
        own = {os.getpid(), smi.probe.pid}
        gpus = snap["GPU"]
        listed = sorted(g["index"] for g in gpus.values())
        assert listed == list(range(_n_devices()))
        for g in gpus.values():
            assert not {p["pid"] for p in g["processes"]} & own, g["processes"]
            assert g["metrics"]["mfma_contention"]["value"] is not None, g["metrics"]
            assert g["metrics"]["probe_duty"]["value"] < 0.1
        uuid0 = next(u for u, g in gpus.items() if g["index"] == 0)
        Resource(id=uuid0, name="MI355X", hostname=host).save()
        now = datetime.datetime.utcnow()
        Reservation(user_id=new_user.id, title="mine", description="", resource_id=uuid0,
                    start=now - datetime.timedelta(minutes=5), end=now + datetime.timedelta(hours=1)).save()
        seen = []

        class Recorder:
            def trigger_action(self, data):
                seen.append(data)

        prot = ProtectionService(0.2, [Recorder()], level=2)  # strict: any process is a violation
        prot.inject(d)
        prot.do_run()
        assert not seen, seen
        # the allocator sees GPU 0 as free (reserved by new_user: an auto:1 job of theirs gets it)
        g = Restriction(name="all", starts_at=now - datetime.timedelta(days=1), is_global=True)
        g.save()
        g.apply_to_user(new_user)
        j = _job(new_user, "auto:1", host=host)
        plan = allocation.plan_job(j, d.infrastructure.snapshot().data, held=set())
        assert [idx for idx, _u in plan[j.tasks[0].id]] == [0], plan
    finally:
        d.shutdown()
        smi.close()
