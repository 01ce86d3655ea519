"""Benchmark harnesses for the daemon-side metrics of BASELINE.md.

* :func:`poll_latency` -- p50/p99 latency of ``GET /nodes/metrics`` (the dashboard's poll) on a
  simulated cluster of ``nodes`` x ``gpus`` MI355X (stub telemetry, real router, real auth, real
  snapshot path).  The reference re-read a shared dict under no lock and ran ``nvidia-smi`` per
  node per poll interval (``core/monitors/GPUMonitor.py``); here a poll reads one RCU snapshot.
* :func:`launch_latency` -- time from ``PUT /jobs/{id}/enqueue`` to the task's process running on
  a local node through ``th-run`` (event-driven scheduler wake; the reference polled every 30 s,
  ``core/services/JobSchedulingService.py:44``).
* :func:`train_throughput` -- runs ``bench.py`` (the flagship Llama-3-8B DDP step) and returns its
  JSON line.
"""
from __future__ import annotations

import contextlib
import getpass
import json
import os
import statistics
import subprocess
import sys
import tempfile
import time
from datetime import timedelta
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _pct(xs: list[float], q: float) -> float:
    xs = sorted(xs)
    if not xs:
        return float("nan")
    i = min(len(xs) - 1, max(0, int(round(q * (len(xs) - 1)))))
    return xs[i]


@contextlib.contextmanager
def sandbox(hosts: dict[str, str], backend: str = "stub", stub_gpus: int = 8, job_interval: float = 30.0):
    """Temporary config dir + file SQLite DB + installed global config.

    ``hosts`` maps hostname -> transport (``local``/``fake``/``ssh``).  Restores the previous
    config and ``TENSORHIVE_CONFIG_DIR`` on exit."""
    from . import config as C
    from . import database as D

    old_dir = os.environ.get("TENSORHIVE_CONFIG_DIR")
    old_state = os.environ.get("TH_RUN_STATE_DIR")
    old_cfg = C._current
    with tempfile.TemporaryDirectory(prefix="th-bench-") as td:
        d = Path(td)
        user = getpass.getuser()
        (d / "hosts_config.ini").write_text(
            "".join(f"[{h}]\nuser = {user}\ntransport = {t}\n\n" for h, t in hosts.items()))
        (d / "main_config.ini").write_text(f"""
[ssh]
hosts_config_file = {d / 'hosts_config.ini'}
test_on_startup = off
key_file = {d / 'ssh_key'}
[database]
path = {d / 'db.sqlite'}
[monitoring_service]
update_interval = 1
[protection_service]
enabled = off
level = 0
[usage_logging_service]
enabled = off
[job_scheduling_service]
enabled = on
update_interval = {job_interval}
[amd_monitor]
backend = {backend}
stub_gpus = {stub_gpus}
probe_enabled = off
[launcher]
log_dir = {d / 'logs'}
""")
        C.init_config_files(d)
        C.ensure_secret_key(d / "main_config.ini")
        os.environ["TENSORHIVE_CONFIG_DIR"] = str(d)
        os.environ["TH_RUN_STATE_DIR"] = str(d / "th-run")
        cfg = C.load_config(d)
        C.set_config(cfg)
        D.configure(f"sqlite:///{d / 'db.sqlite'}")
        D.create_all()
        try:
            yield cfg, d
        finally:
            D.db_session.remove()
            for k, v in (("TENSORHIVE_CONFIG_DIR", old_dir), ("TH_RUN_STATE_DIR", old_state)):
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            C.set_config(old_cfg)


def _admin(name: str = "bench"):
    from .models.orm import Role, User

    u = User(username=name, password="benchmark password", email=f"{name}@example.org",
             roles=[Role(name="user"), Role(name="admin")])
    u.save()
    return u


def _headers(u) -> dict:
    from .api import auth

    return {"Authorization": "Bearer " + auth.create_access_token(u.id, u.role_names, fresh=True)}


def _lat_stats(lat: list[float], requests: int) -> dict:
    return {"p50_ms": round(_pct(lat, 0.5), 3), "p99_ms": round(_pct(lat, 0.99), 3),
            "mean_ms": round(statistics.fmean(lat), 3), "requests": requests}


def poll_latency(requests: int = 1000, nodes: int = 8, gpus: int = 8, warmup: int = 20) -> dict:
    """p50/p99 of the dashboard poll on ``nodes`` x ``gpus`` simulated GPUs, three ways:

    * ``admin_inprocess`` -- Flask test client, admin (no permission filter);
    * ``user_inprocess`` -- Flask test client, an ordinary user whose restrictions cover half of
      every node's GPUs (per-resource restrictions, so every poll runs the user lookup and
      ``filter_infrastructure_by_user_restrictions``, reference ``controllers/nodes.py:13-50``);
    * ``user_socket`` -- the same user over HTTP/1.1 keep-alive to the threaded WSGI server the
      daemon runs (``api/app.py``), i.e. what a browser pays minus the network."""
    import http.client
    import threading

    from werkzeug.serving import make_server

    from .api.app import create_app
    from .core.daemon import Daemon
    from .core.telemetry import StubBackend
    from .models.orm import Resource, Restriction, Role, User
    from .utils import dates

    hosts = {f"mi355x-{i:02d}": "fake" for i in range(nodes)}
    with sandbox(hosts, stub_gpus=gpus) as (cfg, _d):
        stub = StubBackend(gpus_per_host=gpus)
        daemon = Daemon(cfg, backends={h: stub for h in hosts}, init_key=False, test_ssh=False)
        for h in hosts:
            daemon.infrastructure.publish(h, stub.sample(h))
        app = create_app(daemon)
        client = app.test_client()
        admin = _admin()
        user = User(username="alice", password="benchmark password", email="alice@example.org",
                    roles=[Role(name="user")])
        user.save()
        r = Restriction(name="half", starts_at=dates.utcnow() - timedelta(days=1), is_global=False)
        r.save()
        r.apply_to_user(user)
        for h in hosts:
            for i in range(0, gpus, 2):
                res = Resource(id=stub.gpu_uuid(h, i), name="MI355X", hostname=h)
                res.save()
                r.apply_to_resource(res)
        client.get("/api/nodes/metrics", headers=_headers(admin))  # registers every GPU resource once
        out = {}
        paths = ("/api/nodes/metrics", "/api/nodes/mi355x-00/gpu/metrics?metric_type=utilization")
        for label, who in (("admin_inprocess", admin), ("user_inprocess", user)):
            hdr = _headers(who)
            for path in paths:
                lat = []
                for i in range(warmup + requests):
                    t0 = time.perf_counter()
                    resp = client.get(path, headers=hdr)
                    dt = (time.perf_counter() - t0) * 1e3
                    assert resp.status_code == 200, resp.data[:200]
                    if i >= warmup:
                        lat.append(dt)
                out.setdefault(label, {})[path] = _lat_stats(lat, requests)
        # the user's view really is filtered: half of each node's GPUs
        seen = client.get("/api/nodes/metrics", headers=_headers(user)).get_json()
        visible = sum(len(v.get("GPU") or {}) for v in seen.values())
        from .app.server import quiet_access_log

        quiet_access_log()  # as the daemon's own server (app/server.py serve_wsgi)
        srv = make_server("127.0.0.1", 0, app, threaded=True)
        th = threading.Thread(target=srv.serve_forever, daemon=True)
        th.start()
        try:
            conn = http.client.HTTPConnection("127.0.0.1", srv.server_port, timeout=10)
            hdr = _headers(user)
            for path in paths:
                lat = []
                for i in range(warmup + requests):
                    t0 = time.perf_counter()
                    conn.request("GET", path, headers=hdr)
                    resp = conn.getresponse()
                    body = resp.read()
                    dt = (time.perf_counter() - t0) * 1e3
                    assert resp.status == 200, body[:200]
                    if i >= warmup:
                        lat.append(dt)
                out.setdefault("user_socket", {})[path] = _lat_stats(lat, requests)
            conn.close()
        finally:
            srv.shutdown()
            daemon.shutdown()
        return {"metric": "dashboard_poll_latency", "nodes": nodes, "gpus_per_node": gpus,
                "user_visible_gpus": visible, "results": out}


def launch_latency(trials: int = 5, command: str = "echo started; sleep 2") -> dict:
    """Enqueue -> task process running (scheduler launch log) and -> first line in the task's log
    (BASELINE.md §2 definition), through the real scheduler thread and th-run."""
    from .controllers import task as task_ctl
    from .core.daemon import Daemon
    from .core.services import JobSchedulingService
    from .core.telemetry import StubBackend
    from .models.orm import (CommandSegment, Job, JobStatus, Restriction, SegmentType,
                             Task, TaskStatus)
    from .native.build import build_all
    from .utils import dates

    me = getpass.getuser()
    if me == "root":
        # tasks run as the job owner's UNIX account; "root" is not a valid TensorHive username
        return {"metric": "queued_job_launch_latency", "skipped": "run as an ordinary user"}
    build_all(strict=False)
    with sandbox({"localhost": "local"}, job_interval=3600.0) as (cfg, _d):
        stub = StubBackend(gpus_per_host=8)
        daemon = Daemon(cfg, backends={"localhost": stub}, init_key=False, test_ssh=False)
        daemon.infrastructure.publish("localhost", stub.sample("localhost"))
        sched = JobSchedulingService(3600.0, 5, 10)
        daemon.add_service(sched)
        u = _admin(me)
        r = Restriction(name="all", starts_at=dates.utcnow(), is_global=True)
        r.save()
        r.apply_to_user(u)
        seg = CommandSegment(name="HIP_VISIBLE_DEVICES", _segment_type=SegmentType.env_variable)
        seg.save()
        sched.start()
        lat, first_line = [], []
        try:
            for i in range(trials):
                job = Job(name=f"bench-{i}", description="", user_id=u.id)
                job.save()
                t = Task(command=command, hostname="localhost")
                t.save()
                job.add_task(t)
                t.add_cmd_segment(seg, str(i % 8))
                job.enqueue()
                t0 = time.time()
                daemon.wake("enqueue")
                deadline = time.time() + 30
                while time.time() < deadline:
                    if any(jid == job.id for jid, _ in sched.launch_log):
                        break
                    time.sleep(0.002)
                else:
                    raise TimeoutError(f"job {job.id} was not launched within 30 s")
                ts = dict(sched.launch_log)[job.id]
                lat.append((ts - t0) * 1e3)
                from .core import task_nursery
                from .database import db_session

                tid = job.tasks[0].id
                while time.time() < deadline:
                    try:
                        lines, _ = task_nursery.fetch_log("localhost", u.username, tid)
                    except FileNotFoundError:
                        lines = []
                    if lines:
                        first_line.append((time.time() - t0) * 1e3)
                        break
                    time.sleep(0.002)

                db_session.expire_all()
                t = Task.get(t.id)
                assert t.status is TaskStatus.running and t.pid, t.as_dict()
                task_nursery.terminate(t.pid, "localhost", u.username, gracefully=False)
                task_ctl.synchronize(t.id)
                job = Job.get(job.id)
                job.dequeue() if job.status is JobStatus.pending else None
        finally:
            daemon.shutdown()
        return {"metric": "queued_job_launch_latency", "trials": trials,
                "p50_ms": round(_pct(lat, 0.5), 2), "max_ms": round(max(lat), 2),
                "first_log_line_p50_ms": round(_pct(first_line, 0.5), 2) if first_line else None,
                "reference_ms": 30000.0 / 2, "note": "reference polls every 30 s -> 15 s mean wait"}


def scheduled_training(gpus: int = 1, steps: int = 10, warmup: int = 2, micro_batch: int = 8,
                       model: str = "llama3-8b", timeout_s: float = 900.0, auto: bool = True) -> dict:
    """BASELINE config 3/4: the Llama-3 DDP payload launched BY THE JOB QUEUE -- torchrun template,
    real amdsmi telemetry for the free-GPU check -- and its tokens/s read back from the task log
    (``[th-train]`` lines).  ``auto``: the task asks for ``HIP_VISIBLE_DEVICES=auto:N`` and the
    allocator picks the devices at launch (gang placement, ``core/allocation.py``); otherwise the
    first N HIP indices are pinned."""
    import re

    from .core import task_nursery
    from .core.daemon import Daemon
    from .core.launcher import torchrun_task
    from .core.services import JobSchedulingService
    from .core.telemetry import AmdSmiBackend
    from .controllers import task as task_ctl
    from .models.orm import Job, Restriction
    from .native.build import build_all
    from .utils import dates

    me = getpass.getuser()
    if me == "root":
        return {"metric": "scheduled_training", "skipped": "run as an ordinary user"}
    build_all(strict=False)
    with sandbox({"localhost": "local"}, job_interval=3600.0) as (cfg, _d):
        smi = AmdSmiBackend()
        daemon = Daemon(cfg, backends={"localhost": smi}, init_key=False, test_ssh=False)
        daemon.infrastructure.publish("localhost", smi.sample("localhost"))
        sched = JobSchedulingService(3600.0, 5, 10)
        daemon.add_service(sched)
        u = _admin(me)
        r = Restriction(name="all", starts_at=dates.utcnow(), is_global=True)
        r.save()
        r.apply_to_user(u)
        form = torchrun_task("localhost", gpus if auto else list(range(gpus)), "127.0.0.1", 29533,
                             script_args=[("--steps", str(steps)), ("--warmup", str(warmup)),
                                          ("--micro-batch", str(micro_batch)), ("--model", model)])
        job = Job(name="llama3-ddp", description="scheduled training", user_id=u.id)
        job.save()
        content, status = task_ctl.business_create(form, job.id)
        assert status == 201, content
        tid = content["task"]["id"]
        job = Job.get(job.id)
        job.enqueue()
        sched.start()
        t0 = time.time()
        daemon.wake("enqueue")
        rates, done, lines = [], False, []
        try:
            while time.time() - t0 < timeout_s and not done:
                time.sleep(1.0)
                try:
                    lines, _ = task_nursery.fetch_log("localhost", me, tid)
                except FileNotFoundError:
                    continue
                rates = [float(m.group(1)) for l in lines for m in [re.search(r"tokens/s=([0-9.]+)", l)] if m]
                done = any('"event": "done"' in l for l in lines)
        finally:
            daemon.shutdown()
        steady = rates[1:] or rates
        launched = task_ctl.Task.get(tid).as_dict()
        return {"metric": "scheduled_llama3_ddp_tokens_per_sec", "gpus": gpus, "micro_batch": micro_batch,
                "placement": "auto" if auto else "pinned", "allocated_gpus": launched.get("allocatedGpus"),
                "full_command": launched.get("fullCommand"),
                "steps_logged": len(rates), "tokens_per_sec": round(statistics.fmean(steady), 1) if steady else None,
                "completed": done, "wall_s": round(time.time() - t0, 1), "log_tail": lines[-3:]}


def multitenant(jobs_per_user: int = 8, seed: int = 0, duration_s: tuple[float, float] = (0.4, 1.2),
                arrival_s: float = 0.15, pinned: bool = False) -> dict:
    """BASELINE config 4 on a simulated 8-GPU MI355X node (scaled time): three users with
    overlapping reservations submit two-GPU jobs to the queue; the real scheduler and monitoring
    threads place and start them.  Reports queue wait (enqueue -> running) p50/p99, node GPU
    utilisation over the run and while jobs were waiting, and the violation path (a foreign
    process on a reserved GPU is detected and walled on the intruder's terminal).

    ``pinned=True`` is the reference's model: every job names its device pair up front
    (each user has a favourite pair), so a job waits for THAT pair even when others are free.
    The default lets the allocator pick any free, permitted pair (``HIP_VISIBLE_DEVICES=auto:2``)."""
    import random

    from .core.daemon import Daemon
    from .core.services import JobSchedulingService, MonitoringService, ProtectionService
    from .core.telemetry import StubBackend
    from .core.violation_handlers import MessageSendingBehaviour, ProtectionHandler
    from .models.orm import (CommandSegment, Job, JobStatus, Reservation, Resource, Restriction, Role,
                             SegmentType, Task, User)
    from .utils import dates

    rng = random.Random(seed)
    host = "mi355x-00"
    with sandbox({host: "simulated"}, job_interval=3600.0) as (cfg, _d):
        stub = StubBackend(gpus_per_host=8)
        daemon = Daemon(cfg, backends={host: stub}, init_key=False, test_ssh=False)
        node = daemon.transports.get(host)
        daemon.infrastructure.publish(host, stub.sample(host))
        uuids = [stub.gpu_uuid(host, i) for i in range(8)]
        for u in uuids:
            Resource(id=u, name="MI355X", hostname=host).save()
        names = ("alice", "bob", "carol")
        users = {}
        g = Restriction(name="everyone", starts_at=dates.utcnow() - timedelta(days=1), is_global=True)
        g.save()
        for n in names:
            users[n] = User(username=n, password="benchmark password", email=f"{n}@example.org",
                            roles=[Role(name="user")])
            users[n].save()
            g.apply_to_user(users[n])
        now = dates.utcnow()
        for n, gpus, start in (("alice", (0, 1), now - timedelta(minutes=5)), ("bob", (2, 3), now - timedelta(minutes=5)),
                               ("carol", (4,), now + timedelta(minutes=10))):
            for i in gpus:
                Reservation(user_id=users[n].id, title=f"{n}-{i}", description="", resource_id=uuids[i],
                            start=start, end=start + timedelta(hours=2)).save()
        favourite = {"alice": "0,1", "bob": "2,3", "carol": "6,7"}
        seg = CommandSegment(name="HIP_VISIBLE_DEVICES", segment_type=SegmentType.env_variable)
        seg.save()
        plan = []  # (arrival offset, user, duration)
        t = 0.0
        for k in range(jobs_per_user * len(names)):
            t += rng.expovariate(1.0 / arrival_s)
            plan.append((t, names[k % len(names)], rng.uniform(*duration_s)))
        mon = MonitoringService(0.02, {host: stub})
        sched = JobSchedulingService(0.25, 5, 30)
        daemon.add_service(mon)
        daemon.add_service(sched)
        mon.start()
        sched.start()
        enq: dict[int, float] = {}
        dur: dict[int, float] = {}
        started: dict[int, float] = {}
        busy_samples, waiting_samples = [], []
        violations = {}
        from .database import db_session

        t0 = time.time()
        try:
            pending = list(plan)
            deadline = t0 + 120
            while time.time() < deadline:
                now_s = time.time() - t0
                while pending and pending[0][0] <= now_s:
                    _at, n, d = pending.pop(0)
                    j = Job(name=f"{n}-{len(enq)}", description="", user_id=users[n].id)
                    j.save()
                    tk = Task(command="python train.py", hostname=host)
                    tk.save()
                    tk.add_cmd_segment(seg, favourite[n] if pinned else "auto:2")
                    j.add_task(tk)
                    j.enqueue()
                    enq[j.id], dur[j.id] = time.time(), d
                    daemon.wake("enqueue")
                for jid, ts in list(sched.launch_log):
                    started.setdefault(jid, ts)
                db_session.expire_all()
                for jid, ts in started.items():  # finish jobs whose time is up
                    if dur.get(jid) is not None and time.time() - ts >= dur[jid]:
                        for tk in Job.get(jid).tasks:
                            if tk.pid:
                                node.exit_task(tk.pid)
                        dur[jid] = None
                        daemon.wake("exit")
                sample = stub.sample(host)["GPU"]
                busy_samples.append(sum(1 for x in sample.values() if x["processes"]))
                waiting_samples.append(any(j not in started for j in enq))
                if not violations and now_s > 1.0:  # a foreign process on bob's reserved GPU 2
                    stub.add_process(host, 2, 66666, "mallory")
                    node.ttys = [("mallory", "pts/7")]
                    mon.do_run()
                    prot = ProtectionService(1.0, [ProtectionHandler(MessageSendingBehaviour(daemon.transports))], 1)
                    prot.inject(daemon)
                    prot.do_run()
                    violations = {k: [r["OWNER_USERNAME"] for r in v["RESERVATIONS"]]
                                  for k, v in prot.last_violations.items()}
                    node._drop_gpu_process(66666)
                if not pending and len(started) == len(enq) and all(v is None for v in dur.values()):
                    break
                time.sleep(0.01)
            makespan = time.time() - t0
        finally:
            daemon.shutdown()
        waits = [(started[j] - enq[j]) * 1e3 for j in enq if j in started]
        util = statistics.fmean(busy_samples) / 8 if busy_samples else 0.0
        contended = [b for b, w in zip(busy_samples, waiting_samples) if w]
        return {"metric": "multitenant_queue", "policy": "pinned (reference)" if pinned else "auto:2 gang placement",
                "jobs": len(enq), "completed": sum(1 for v in dur.values() if v is None),
                "queue_wait_p50_ms": round(_pct(waits, 0.5), 1), "queue_wait_p99_ms": round(_pct(waits, 0.99), 1),
                "node_gpu_util": round(util, 3),
                "gpu_util_while_jobs_wait": round(statistics.fmean(contended) / 8, 3) if contended else None,
                "makespan_s": round(makespan, 2), "violations": violations,
                "walled_ttys": [t for t, _ in node.tty_messages],
                "note": "simulated node (th-run protocol in-process), scaled time: job durations "
                        f"{duration_s[0]}-{duration_s[1]} s, mean inter-arrival {arrival_s} s"}


_NODE_JOB = r"""
import sys, time, torch
secs = float(sys.argv[1])
x = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
print("started", torch.cuda.device_count(), repr(time.time()), flush=True)
t0, n = time.time(), 0
while time.time() - t0 < secs:
    y = x @ x
    n += 1
    if n % 32 == 0:
        torch.cuda.synchronize()
torch.cuda.synchronize()
print("done", n, repr(time.time()), flush=True)
"""

_NODE_INTRUDER = r"""
import sys, time, torch
x = torch.ones(64 << 20, device="cuda"); torch.cuda.synchronize()
print("ready", flush=True)
time.sleep(float(sys.argv[1]))
"""


def multitenant_node(jobs_per_user: int = 2, seed: int = 0, duration_s: tuple[float, float] = (6.0, 10.0),
                     arrival_s: float = 2.0, gpus_per_job: int | None = None, timeout_s: float = 600.0,
                     tick_s: float = 30.0) -> dict:
    """BASELINE config 4 on the REAL node, in real time: three users submit GPU jobs to the queue
    (``HIP_VISIBLE_DEVICES=auto:k``); the daemon's own monitoring (amdsmi + KFD, 0.25 s), job
    scheduling (gang placement over the node's actual free GPUs) and ``th-run`` launch them as
    real processes that run bf16 GEMMs on the device until their time is up.  Queue wait is
    enqueue -> ``th-run`` launch; node utilisation is the share of GPU-samples that hold a job's
    process (from the telemetry snapshots, not from the harness's own bookkeeping).  Afterwards a
    foreign process on a GPU that "bob" has reserved is detected by the protection service.

    ``gpus_per_job`` defaults to 2 on a node with >= 2 GPUs (the BASELINE config) and 1 on a
    one-GPU box.  ``tick_s`` is the scheduler's periodic tick, the shipped 30 s by default: a job
    that waits for a busy device is started by the event wake-ups (enqueue, and the monitoring
    service's "a device lost its last process"), so ``handoff_*`` -- a job's exit to the next
    waiting job's launch -- measures those, not the tick.  The simulated, scaled-time variant is
    :func:`multitenant`."""
    import random

    from .core import task_nursery
    from .core.daemon import Daemon
    from .core.services import JobSchedulingService, MonitoringService, ProtectionService
    from .core.telemetry import AmdSmiBackend
    from .database import db_session
    from .models.orm import CommandSegment, Job, Reservation, Resource, Restriction, Role, SegmentType, Task, User
    from .native.build import build_all
    from .utils import dates

    me = getpass.getuser()
    if me == "root":
        return {"metric": "multitenant_node", "skipped": "run as an ordinary user"}
    build_all(strict=False)
    rng = random.Random(seed)
    host = "localhost"
    with sandbox({host: "local"}, job_interval=3600.0) as (cfg, d):
        smi = AmdSmiBackend()
        daemon = Daemon(cfg, backends={host: smi}, init_key=False, test_ssh=False)
        mon = MonitoringService(0.25, {host: smi})
        mon.inject(daemon)
        mon.do_run()
        gpus = daemon.infrastructure.snapshot().data[host]["GPU"]
        n_gpus = len(gpus)
        k = gpus_per_job or (2 if n_gpus >= 2 else 1)
        by_index = {g["index"]: u for u, g in gpus.items()}
        for u in gpus:
            Resource(id=u, name="MI355X", hostname=host).save()
        names = ("alice", "bob", "carol")
        users = {}
        g = Restriction(name="everyone", starts_at=dates.utcnow() - timedelta(days=1), is_global=True)
        g.save()
        for n in names:
            users[n] = User(username=n, password="benchmark password", email=f"{n}@example.org",
                            roles=[Role(name="user")])
            users[n].save()
            g.apply_to_user(users[n])
        script = d / "job.py"
        script.write_text(_NODE_JOB)
        seg = CommandSegment(name="HIP_VISIBLE_DEVICES", segment_type=SegmentType.env_variable)
        seg.save()
        plan, t = [], 0.0
        for j in range(jobs_per_user * len(names)):
            t += rng.expovariate(1.0 / arrival_s)
            plan.append((t, names[j % len(names)], rng.uniform(*duration_s)))
        sched = JobSchedulingService(tick_s, 5, 30)
        daemon.add_service(mon)
        daemon.add_service(sched)
        mon.start()
        sched.start()
        enq: dict[int, float] = {}
        task_of: dict[int, int] = {}
        busy, waiting = [], []
        t0 = time.time()
        try:
            pending = list(plan)
            last_snap = None
            while time.time() - t0 < timeout_s:
                now_s = time.time() - t0
                while pending and pending[0][0] <= now_s:
                    _at, n, dur = pending.pop(0)
                    job = Job(name=f"{n}-{len(enq)}", description="", user_id=users[n].id)
                    job.save()
                    tk = Task(command=f"{sys.executable} {script} {dur:.1f}", hostname=host)
                    tk.save()
                    tk.add_cmd_segment(seg, f"auto:{k}")
                    job.add_task(tk)
                    job.enqueue()
                    enq[job.id] = time.time()
                    task_of[job.id] = tk.id
                    daemon.wake("enqueue")
                snap = daemon.infrastructure.snapshot()
                if snap is not last_snap:  # one utilisation sample per telemetry update
                    last_snap = snap
                    gs = snap.data[host]["GPU"].values()
                    busy.append(sum(1 for x in gs if x.get("processes")))
                    launched = {jid for jid, _ts in sched.launch_log}
                    waiting.append(any(jid not in launched for jid in enq))
                db_session.expire_all()
                if not pending and enq and all(Job.get(j).status.name not in ("pending", "running")
                                               for j in enq):
                    break
                time.sleep(0.05)
            makespan = time.time() - t0
            starts = dict(sched.launch_log)
        except BaseException:
            daemon.shutdown()  # the monitoring thread too; the normal path shuts down after the violation check
            raise
        finally:
            sched.stop()
        waits = [(starts[j] - enq[j]) * 1e3 for j in enq if j in starts]
        # the jobs' own clocks (task logs): launch -> device ready, and the scheduler's hand-off
        # (a job's exit -> the next waiting job's launch) on a contended node
        marks: dict[int, dict] = {}
        for j, tid in task_of.items():
            try:
                lines, _ = task_nursery.fetch_log(host, me, tid)
            except FileNotFoundError:
                continue
            for ln in lines:
                parts = ln.split()
                if len(parts) >= 3 and parts[0] in ("started", "done"):
                    marks.setdefault(j, {})[parts[0]] = float(parts[-1])
        startup = [(m["started"] - starts[j]) * 1e3 for j, m in marks.items() if "started" in m and j in starts]
        ends = sorted(m["done"] for m in marks.values() if "done" in m)
        handoff = []
        for j in sorted(starts, key=starts.get):
            prev = [e for e in ends if e <= starts[j]]
            if prev and enq[j] < prev[-1] and starts[j] - prev[-1] < 60:  # waited for a device a job freed
                handoff.append((starts[j] - prev[-1]) * 1e3)
        # the daemon's part of it: th-run's exit time (its task-exit event, core/events.py) -> the
        # next waiting job's launch; the rest of `handoff` is the job's own teardown after "done"
        exits = sorted(ev.get("ended_ms", ts * 1e3) / 1e3 for ts, _h, ev in daemon.task_events)
        handoff_exit = []
        for j in sorted(starts, key=starts.get):
            prev = [e for e in exits if e <= starts[j]]
            if prev and enq[j] < prev[-1] and starts[j] - prev[-1] < 60:
                handoff_exit.append((starts[j] - prev[-1]) * 1e3)
        statuses = {}
        for j in enq:
            st = Job.get(j).status.name
            statuses[st] = statuses.get(st, 0) + 1
        # violation path on the real device: bob reserves GPU 0, an unscheduled process uses it
        now = dates.utcnow()
        Reservation(user_id=users["bob"].id, title="bob-0", description="", resource_id=by_index[0],
                    start=now - timedelta(minutes=1), end=now + timedelta(hours=1)).save()
        seen = []

        class _Recorder:
            def trigger_action(self, data):
                seen.append(data)

        prot = ProtectionService(0.25, [_Recorder()], level=1)
        prot.inject(daemon)
        p = subprocess.Popen([sys.executable, "-c", _NODE_INTRUDER, "30"], stdout=subprocess.PIPE, text=True,
                             env={**os.environ, "HIP_VISIBLE_DEVICES": "0"})
        detect_ms = None
        try:
            if p.stdout.readline().strip() == "ready":
                t1 = time.time()
                while time.time() - t1 < 15 and detect_ms is None:
                    mon.do_run()
                    prot.do_run()
                    if any(p.pid in pids for v in seen for pids in v["VIOLATION_PIDS"].values()):
                        detect_ms = round((time.time() - t1) * 1e3, 1)
                    time.sleep(0.1)
        finally:
            p.kill()
            p.wait()
            daemon.shutdown()
        hit = next((v for v in seen if any(p.pid in pids for pids in v["VIOLATION_PIDS"].values())), None)
        return {"metric": "multitenant_node", "real_time": True, "gpus_on_node": n_gpus, "gpus_per_job": k,
                "jobs": len(enq), "job_status": statuses, "launched": len(waits),
                "queue_wait_p50_ms": round(_pct(waits, 0.5), 1), "queue_wait_p99_ms": round(_pct(waits, 0.99), 1),
                "node_gpu_util": round(statistics.fmean(busy) / n_gpus, 3) if busy else None,
                "gpu_util_while_jobs_wait": (round(statistics.fmean([b for b, w in zip(busy, waiting) if w]) / n_gpus, 3)
                                             if any(waiting) else None),
                "telemetry_samples": len(busy), "makespan_s": round(makespan, 1),
                "job_startup_p50_ms": round(_pct(startup, 0.5), 1) if startup else None,
                "handoff_p50_ms": round(_pct(handoff, 0.5), 1) if handoff else None,
                "handoff_max_ms": round(max(handoff), 1) if handoff else None,
                "handoff_from_exit_p50_ms": round(_pct(handoff_exit, 0.5), 1) if handoff_exit else None,
                "handoff_from_exit_max_ms": round(max(handoff_exit), 1) if handoff_exit else None,
                "task_exit_events": len(daemon.task_events),
                "violation": None if hit is None else {
                    "intruder": hit["INTRUDER_USERNAME"], "reserved_by": [r["OWNER_USERNAME"] for r in hit["RESERVATIONS"]],
                    "detect_ms": detect_ms},
                "note": f"real node, real time: {jobs_per_user * 3} jobs of {duration_s[0]}-{duration_s[1]} s bf16 GEMM "
                        f"loops, mean inter-arrival {arrival_s} s, each asking HIP_VISIBLE_DEVICES=auto:{k}; "
                        f"scheduler tick {tick_s:g} s (starts come from event wake-ups)"}


def monitoring_overhead(window_s: float = 20.0, train_rounds: int = 2, steps: int = 8, warmup: int = 3) -> dict:
    """What the monitoring costs, on the real node (BASELINE: "monitoring overhead"; the reference ran
    ``nvidia-smi`` plus one SSH round trip per GPU process every 2-5 s, ``core/monitors/GPUMonitor.py``).

    * ``daemon``: a MonitoringService at the shipped 0.25 s cadence over this node's amdsmi backend
      with the per-GPU ``th-probe`` agent on (the shipped defaults): per-sample wall time, and the CPU
      time of this process and of the probe agent over ``window_s``, as a share of one core.
    * ``tenant``: ``bench.py`` tokens/s of a training step started (a) with nothing else running,
      (b) while that monitoring runs, and (c) with the in-task HBM counter tool (``libthhbm`` through
      ``ROCP_TOOL_LIBRARIES``, what ``th-run`` injects into every task), alternating ``train_rounds``
      times in one box."""
    import psutil

    from .core import hbm
    from .core.daemon import Daemon
    from .core.services import MonitoringService
    from .core.telemetry import AmdSmiBackend

    def bench_once(env_extra: dict | None = None) -> float:
        env = {**os.environ, **(env_extra or {})}
        r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--steps", str(steps), "--warmup", str(warmup),
                            "--daemon-bench", "0"], capture_output=True, text=True, env=env, cwd=ROOT)
        for line in reversed(r.stdout.splitlines()):
            if line.startswith("{"):
                return float(json.loads(line)["value"])
        raise RuntimeError(f"bench.py failed ({r.returncode}): {r.stderr[-1500:]}")

    out: dict = {"metric": "monitoring_overhead"}
    with sandbox({"localhost": "local"}, job_interval=3600.0) as (cfg, _d):

        @contextlib.contextmanager
        def monitoring():
            """The shipped monitoring of this node: amdsmi sampler at 0.25 s + the th-probe agent."""
            smi = AmdSmiBackend(probe=True, probe_period=1.0)
            daemon = Daemon(cfg, backends={"localhost": smi}, init_key=False, test_ssh=False)
            mon = MonitoringService(0.25, {"localhost": smi})
            mon.inject(daemon)
            daemon.add_service(mon)
            try:
                mon.do_run()
                mon.start()
                yield daemon, mon
            finally:
                daemon.shutdown()
                smi.close()

        me = psutil.Process()
        with monitoring() as (daemon, mon):
            time.sleep(2.0)  # the probe agent's first idle references
            agent = me.children(recursive=True)
            c0, a0, t0, k0 = me.cpu_times(), sum(sum(c.cpu_times()[:2]) for c in agent), time.time(), mon.ticks
            time.sleep(window_s)
            c1, a1, wall = me.cpu_times(), sum(sum(c.cpu_times()[:2]) for c in agent), time.time() - t0
            snap = daemon.infrastructure.snapshot().data["localhost"]["GPU"] or {}
            out["daemon"] = {"cadence_s": 0.25, "gpus": len(snap), "samples": mon.ticks - k0, "window_s": round(wall, 1),
                             "sample_ms": mon.stats.summary(), "helper_processes": len(agent),
                             "daemon_cpu_pct_of_one_core": round(100 * ((c1.user + c1.system) - (c0.user + c0.system)) / wall, 2),
                             "probe_agent_cpu_pct_of_one_core": round(100 * (a1 - a0) / wall, 2),
                             "probe_duty_pct": [((g.get("metrics") or {}).get("probe_duty") or {}).get("value")
                                                for g in snap.values()],
                             "mfma_contention_pct": [((g.get("metrics") or {}).get("mfma_contention") or {}).get("value")
                                               for g in snap.values()]}
        # tenant impact: alternate (a) nothing else, (b) the monitoring running, (c) the in-task HBM tool
        rates = {"alone": [], "with_monitoring": [], "with_task_hbm_tool": []}
        for _ in range(train_rounds):
            rates["alone"].append(bench_once())
            with monitoring():
                rates["with_monitoring"].append(bench_once())
            rates["with_task_hbm_tool"].append(bench_once(hbm.task_env()))
        alone = statistics.fmean(rates["alone"])
        out["tenant"] = {"tokens_per_sec": rates, "bench": f"bench.py --steps {steps} --warmup {warmup}",
                         "monitoring_cost_pct": round(100 * (1 - statistics.fmean(rates["with_monitoring"]) / alone), 2),
                         "task_hbm_tool_cost_pct": round(100 * (1 - statistics.fmean(rates["with_task_hbm_tool"]) / alone), 2),
                         "task_hbm_tool": hbm.tool_path()}
    return out


def train_throughput(gpus: int = 1, steps: int = 10, warmup: int = 3, bucket_mb: float | None = None,
                     extra: list[str] | None = None) -> dict:
    """Run bench.py (torchrun for gpus>1) and return its JSON line."""
    args = ["--gpus", str(gpus), "--steps", str(steps), "--warmup", str(warmup)]
    if bucket_mb is not None:
        args += ["--bucket-mb", f"{bucket_mb:g}"]
    args += list(extra or [])
    if gpus > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
               "--master-addr", "127.0.0.1", "--master-port", "29511", str(ROOT / "bench.py")] + args
    else:
        cmd = [sys.executable, str(ROOT / "bench.py")] + args
    r = subprocess.run(cmd, capture_output=True, text=True)
    for line in reversed(r.stdout.splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    raise RuntimeError(f"bench.py failed ({r.returncode}): {r.stderr[-2000:]}")


def scaling(gpu_counts: list[int] | None = None, steps: int = 10, warmup: int = 3,
            run=None, available: int | None = None, bucket_mbs: list[float] | None = None) -> dict:
    """Weak-scaling curve of the training payload on one node (N08 c): ``bench.py`` at each GPU
    count (torchrun, one rank per GPU, RCCL), the per-N whole-job tokens/s and the efficiency
    ``tokens_per_sec(N) / (N * tokens_per_sec(1))``.  Counts above the node's GPUs are skipped.

    ``bucket_mbs`` sweeps the gradient bucket size: every multi-GPU count runs once per size (the
    1-GPU point has no collectives and runs once); each point records its size, the best size per
    count is reported in ``best_bucket_mb``.  Each point also keeps the run's rank census
    (``dist``: world size, distinct GPUs, NUMA binding) so the curve is self-verifying."""
    if bucket_mbs:
        sweep = [float(b) for b in bucket_mbs]
        base_run = run or (lambda n, b: train_throughput(n, steps, warmup, bucket_mb=b))
        out = None
        single: dict = {}  # the 1-GPU point has no collectives: measured once, reused by every size

        def run_one(n, b):
            if n == 1:
                if "doc" not in single:
                    single["doc"] = base_run(1, b)
                return single["doc"]
            return base_run(n, b)

        for b in sweep:
            part = scaling(gpu_counts, steps, warmup, run=lambda n, b=b: run_one(n, b), available=available)
            for p in part["points"]:
                p["bucket_mb"] = b
            if out is None:
                out = part
            else:  # the 1-GPU baseline is measured once; later sweeps add only multi-GPU points
                base = out["points"][0]["tokens_per_sec"]
                for p in part["points"]:
                    if p["n_gpus"] > 1:
                        p["efficiency"] = round(p["tokens_per_sec"] / (p["n_gpus"] * base), 4)
                        out["points"].append(p)
        best: dict = {}
        for p in out["points"]:
            if p["n_gpus"] > 1 and (p["n_gpus"] not in best or p["tokens_per_sec"] > best[p["n_gpus"]][1]):
                best[p["n_gpus"]] = (p["bucket_mb"], p["tokens_per_sec"])
        out["best_bucket_mb"] = {str(n): b for n, (b, _v) in sorted(best.items())}
        out["bucket_sweep_mb"] = sweep
        return out
    if available is None:
        import torch

        available = torch.cuda.device_count()
    counts = [n for n in (gpu_counts or [1, 2, 4, 8]) if 1 <= n <= max(available, 1)]
    if 1 not in counts:
        counts = [1] + counts
    run = run or (lambda n: train_throughput(n, steps, warmup))
    points = []
    base = None
    for n in counts:
        doc = run(n)
        v = float(doc["value"])
        if n == 1:
            base = v
        census = doc.get("dist") or {}
        points.append({"n_gpus": n, "tokens_per_sec": v, "ms_per_step": doc.get("ms_per_step"),
                       "tokens_per_sec_per_gpu": round(v / n, 1),
                       "efficiency": round(v / (n * base), 4) if base else None,
                       "zero": (doc.get("config") or {}).get("zero"),
                       "world_size": census.get("world_size"), "distinct_devices": census.get("distinct_devices")})
    return {"metric": "llama3_8b_bf16_ddp_train_tokens_per_sec", "scaling": "weak", "points": points,
            "skipped": [n for n in (gpu_counts or [1, 2, 4, 8]) if n not in counts]}
