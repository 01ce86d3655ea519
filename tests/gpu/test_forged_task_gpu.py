"""Round-4 bypass closed on real hardware: a GPU stream started OUTSIDE th-run with a forged
``TENSORHIVE_TASK_ID`` (the reservation owner's task) is a violation; the same stream started by
th-run as that task is not (``core/attribution.py`` against libthsmi's sid / parent chain)."""
import datetime
import getpass
import json
import os
import subprocess
import sys
import time

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def test_forged_task_id_outside_th_run_is_flagged(cfg, tables, new_user, new_job_with_task, tmp_path):
    from tensorhive_fixed_amd.core.attribution import REGISTRY
    from tensorhive_fixed_amd.core.daemon import Daemon
    from tensorhive_fixed_amd.core.services import MonitoringService, ProtectionService
    from tensorhive_fixed_amd.core.telemetry import AmdSmiBackend
    from tensorhive_fixed_amd.models.orm import Reservation, Resource
    from tensorhive_fixed_amd.native.build import build_all, path_of

    build_all(strict=False)
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
    tid = str(new_job_with_task.tasks[0].id)  # a task of the reservation owner

    seen = []

    class Recorder:
        def trigger_action(self, data):
            seen.append(data)

    prot = ProtectionService(0.2, [Recorder()], level=1)
    prot.inject(d)
    stream = [sys.executable, os.path.join(ROOT, "scripts", "hbm_stream.py"), "40", "add"]
    env = {**os.environ, "HIP_VISIBLE_DEVICES": "0", "TENSORHIVE_TASK_ID": tid}
    state = tmp_path / "th-run"
    r = subprocess.run([str(path_of("th-run")), "spawn", "--name", f"tensorhive_task_{tid}", "--log",
                        str(tmp_path / "task.log"), "--state-dir", str(state), "--env", "HIP_VISIBLE_DEVICES=0",
                        "--env", f"TENSORHIVE_TASK_ID={tid}", "--", *stream], capture_output=True, text=True,
                       timeout=30)
    assert r.returncode == 0, r.stderr
    genuine = int(r.stdout.strip().splitlines()[-1])
    sess = json.loads(subprocess.run([str(path_of("th-run")), "status", "--name", f"tensorhive_task_{tid}",
                                      "--state-dir", str(state)], capture_output=True, text=True).stdout)
    REGISTRY.record(host, sess)  # what task_nursery.spawn records from the same round trip
    forged = subprocess.Popen(stream, stdout=subprocess.PIPE, text=True, env=env, start_new_session=True)
    try:
        assert json.loads(forged.stdout.readline()).get("ready")
        hits, procs = [], {}
        for _ in range(60):
            mon.do_run()
            prot.do_run()
            procs = {p["pid"]: p for p in d.infrastructure.node_gpu_processes(host).get(uuid, [])}
            hits = [v for v in seen if any(forged.pid in pids for pids in v["VIOLATION_PIDS"].values())]
            if hits and genuine in procs:
                break
            time.sleep(0.25)
        assert hits, f"forged pid {forged.pid} not flagged: {seen[-1:]} {procs}"
        assert hits[-1]["INTRUDER_USERNAME"] == getpass.getuser()
        assert procs[forged.pid]["task_id"] is None and procs[forged.pid]["claimed_task_id"] == tid
        # the genuine th-run task: same user, same command, same task id -- attested, no violation
        assert genuine in procs, f"th-run task {genuine} not seen on GPU 0: {procs}"
        assert procs[genuine]["task_id"] == tid
        assert not any(genuine in pids for v in seen for pids in v["VIOLATION_PIDS"].values())
    finally:
        forged.kill()
        forged.wait()
        subprocess.run([str(path_of("th-run")), "kill", "--name", f"tensorhive_task_{tid}", "--state-dir",
                        str(state)], capture_output=True, timeout=30)
        d.shutdown()
