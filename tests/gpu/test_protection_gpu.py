"""BASELINE config 1 on real hardware: amdsmi telemetry + reservation calendar; the violation
enforcer finds a foreign process on the reserved MI355X and runs the configured handlers."""
import datetime
import getpass
import os
import subprocess
import sys
import time

import pytest

pytestmark = pytest.mark.gpu

CHILD = r"""
import sys, time, torch
x = torch.ones(64 << 20, device="cuda"); torch.cuda.synchronize()
print("ready", flush=True)
time.sleep(float(sys.argv[1]))
"""


def test_foreign_pid_on_reserved_gpu_is_a_violation(cfg, tables, new_user):
    from tensorhive_fixed_amd.core.daemon import Daemon
    from tensorhive_fixed_amd.core.services import MonitoringService, ProtectionService
    from tensorhive_fixed_amd.core.telemetry import AmdSmiBackend
    from tensorhive_fixed_amd.models.orm import Reservation, Resource

    smi = AmdSmiBackend()
    d = Daemon(cfg, backends={h: smi for h in cfg.ssh.available_nodes}, init_key=False, test_ssh=False)
    host = next(iter(cfg.ssh.available_nodes))
    mon = MonitoringService(0.2, {host: smi})
    mon.inject(d)
    mon.do_run()
    gpus = d.infrastructure.snapshot().data[host]["GPU"]
    uuid = next(u for u, g in gpus.items() if g["index"] == 0)
    Resource(id=uuid, name="MI355X", hostname=host).save()
    now = datetime.datetime.utcnow()
    Reservation(user_id=new_user.id, title="mine", description="", resource_id=uuid,
                start=now - datetime.timedelta(minutes=5), end=now + datetime.timedelta(hours=1)).save()

    seen = []

    class Recorder:
        def trigger_action(self, data):
            seen.append(data)

    prot = ProtectionService(0.2, [Recorder()], level=1)
    prot.inject(d)
    p = subprocess.Popen([sys.executable, "-c", CHILD, "30"], stdout=subprocess.PIPE, text=True,
                         env={**os.environ, "HIP_VISIBLE_DEVICES": "0"})
    try:
        assert p.stdout.readline().strip() == "ready"
        for _ in range(40):
            mon.do_run()
            prot.do_run()
            if any(p.pid in pids for v in seen for pids in v["VIOLATION_PIDS"].values()):
                break
            time.sleep(0.25)
        hits = [v for v in seen if any(p.pid in pids for pids in v["VIOLATION_PIDS"].values())]
        assert hits, f"no violation for pid {p.pid}: {seen[-1:]}"
        v = hits[-1]
        assert v["INTRUDER_USERNAME"] == getpass.getuser()
        assert v["RESERVATIONS"][0]["OWNER_USERNAME"] == "administrantee"
        assert v["RESERVATIONS"][0]["GPU_UUID"] == uuid
    finally:
        p.kill()
        p.wait()
        d.shutdown()
