"""``tensorhive`` command line (reference ``cli.py:98-268``).

    tensorhive [-v] [-l LEVEL] [-d LOGDIR] [-c CONFIG_DIR]     run the daemon (API + dashboard + services)
    tensorhive init                                             hostname, DB, first account
    tensorhive test                                             SSH connectivity to every host
    tensorhive key                                              print the authorized_keys line
    tensorhive create user [-m]                                 account prompt (repeat with -m)
    tensorhive doctor                                           ROCm / amdsmi / RCCL / xGMI checks (new)
    tensorhive bench poll|launch|train|scheduled|multitenant    N08 benchmark harnesses (new)
    tensorhive profile --task ID                                rocprofv3 wrapper line for a task (new)

Fixes vs. the reference: ``init`` is a function the main command can call (the reference invoked
a click command object, ``cli.py:127-128``); the default log dir is ``~/.config/TensorHive/logs``
instead of ``/home/tensorhive/.logs``; config files are created explicitly, not on import.
"""
from __future__ import annotations

import io
import json
import logging
import os
import signal
import sys
import threading
import time
from pathlib import Path

import click

from . import __version__

LEVELS = {"debug": logging.DEBUG, "info": logging.INFO, "warning": logging.WARNING, "error": logging.ERROR,
          "critical": logging.CRITICAL}
FMT = "%(asctime)s [%(levelname)s] %(threadName)s %(name)s: %(message)s"


class JsonLineFormatter(logging.Formatter):
    def format(self, r: logging.LogRecord) -> str:
        return json.dumps({"ts": r.created, "level": r.levelname, "thread": r.threadName, "logger": r.name,
                           "msg": r.getMessage()})


def setup_logging(log_dir: str | None = None, level: int = logging.INFO, json_lines: bool = False) -> None:
    root = logging.getLogger()
    root.setLevel(level)
    for h in list(root.handlers):
        root.removeHandler(h)
    fmt = JsonLineFormatter() if json_lines else logging.Formatter(FMT)
    sh = logging.StreamHandler()
    sh.setFormatter(fmt)
    root.addHandler(sh)
    if log_dir:
        d = Path(log_dir).expanduser()
        d.mkdir(parents=True, exist_ok=True)
        fh = logging.FileHandler(d / time.strftime("%Y-%m-%d_%H-%M-%S.log"))
        fh.setFormatter(fmt)
        root.addHandler(fh)
    for noisy in ("werkzeug", "urllib3", "sqlalchemy.engine"):
        logging.getLogger(noisy).setLevel(logging.WARNING)


def _use_config(config_dir: str | None) -> None:
    from .config import init_config_files, load_config, set_config

    if config_dir:
        os.environ["TENSORHIVE_CONFIG_DIR"] = str(Path(config_dir).expanduser())
    init_config_files()
    set_config(load_config())


def do_init() -> None:
    """3-step wizard: public hostname -> DB -> first account (reference ``cli.py:169-214``)."""
    import configparser

    from .config import config_dir, ensure_secret_key, get_config, load_config, set_config
    from .core.account_creator import AccountCreator
    from .database import configure, ensure_db_with_current_schema

    click.echo("[1/3] API/web URL")
    host = click.prompt("Public hostname of this machine (leave 0.0.0.0 if private)", default="0.0.0.0")
    path = config_dir() / "main_config.ini"
    cp = configparser.ConfigParser(strict=False)
    cp.read(path)
    if not cp.has_section("api"):
        cp.add_section("api")
    cp.set("api", "url_hostname", host)
    with open(path, "w") as f:
        cp.write(f)
    os.chmod(path, 0o600)
    if ensure_secret_key(path):  # an install upgraded from the reference still has its public key
        click.echo("wrote a new random [auth] secret_key")
    set_config(load_config())
    click.echo("[2/3] database")
    configure()
    ensure_db_with_current_schema()
    click.echo("[3/3] first account")
    AccountCreator().run_prompt()
    click.echo(f"Config files: {config_dir()}  (database: {get_config().db_path})")


@click.group(invoke_without_command=True)
@click.option("-v", "--version", is_flag=True, help="print version and exit")
@click.option("-l", "--log-level", type=click.Choice(list(LEVELS)), default="info")
@click.option("-d", "--log-dir", default="~/.config/TensorHive/logs")
@click.option("-c", "--config", "config_dir", default=None, help="config directory (default ~/.config/TensorHive)")
@click.option("--json-logs", is_flag=True)
@click.pass_context
def main(ctx, version, log_level, log_dir, config_dir, json_logs):
    import faulthandler

    try:  # tracebacks of every thread on SIGSEGV/SIGABRT (daemon threads, native libs)
        faulthandler.enable(file=sys.__stderr__)
    except (AttributeError, ValueError, OSError, io.UnsupportedOperation):
        pass  # no real stderr (embedded / test runner)
    if version:
        click.echo(__version__)
        return
    setup_logging(log_dir if ctx.invoked_subcommand is None else None, LEVELS[log_level], json_logs)
    _use_config(config_dir)
    if ctx.invoked_subcommand is not None:
        return
    run_daemon()


def refuse_insecure_secret(cfg) -> None:
    """Exit when the JWT signing key is empty, public or shorter than 32 characters (anyone reaching
    :1111 could mint -- or brute-force the key of -- an admin token and run jobs as any user);
    ``TENSORHIVE_ALLOW_INSECURE_SECRET=1`` overrides (tests)."""
    from .config import ALLOW_INSECURE_ENV, MIN_SECRET_LEN, insecure_secret_allowed, secret_is_insecure

    if not secret_is_insecure(cfg.auth.secret_key):
        return
    if insecure_secret_allowed():
        logging.getLogger(__name__).warning("[auth] secret_key is insecure; allowed by %s", ALLOW_INSECURE_ENV)
        return
    raise click.ClickException(
        f"[auth] secret_key in {cfg.directory / 'main_config.ini'} is empty, the public default "
        f"'jwt-some-secret' or shorter than {MIN_SECRET_LEN} characters; run `tensorhive init` "
        "(writes a random key) or set a long random one yourself")


def run_daemon(block: bool = True):
    from .api.app import create_app
    from .app.server import AppServer, serve_wsgi
    from .config import get_config
    from .core.daemon import Daemon
    from .database import check_if_db_exists, configure, ensure_db_with_current_schema

    cfg = get_config()
    refuse_insecure_secret(cfg)
    if not check_if_db_exists():
        do_init()
    configure()
    ensure_db_with_current_schema()
    daemon = Daemon(cfg)
    daemon.configure_services_from_config()
    daemon.init()
    api = serve_wsgi(create_app(daemon), cfg.api_server.host, cfg.api_server.port, "api-server")
    web = AppServer(cfg).start()
    logging.getLogger(__name__).info("tensorhive %s: API on %s:%s, dashboard on %s:%s", __version__,
                                     cfg.api_server.host, cfg.api_server.port, cfg.app_server.host, cfg.app_server.port)
    if not block:
        return daemon, api, web
    stop = threading.Event()
    signal.signal(signal.SIGINT, lambda *_: stop.set())
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    stop.wait()
    api.shutdown()
    web.shutdown()
    daemon.shutdown()
    return None


@main.command()
def init():
    """Hostname, database and first account."""
    do_init()


@main.command()
def test():
    """Test SSH connectivity to every configured host."""
    from .config import get_config
    from .core.transport import TransportManager

    cfg = get_config()
    tm = TransportManager.from_config(cfg.ssh.available_nodes, cfg.ssh.key_file, cfg.ssh.proxy, cfg.ssh.timeout)
    results = tm.test_all(cfg.ssh.timeout)
    for h, ok in results.items():
        click.echo(f"{'OK ' if ok else 'FAIL'} {h}")
    sys.exit(0 if all(results.values()) else 1)


@main.command()
def key():
    """Print the line to append to ~/.ssh/authorized_keys on every node."""
    from .config import get_config
    from .core import ssh

    cfg = get_config()
    click.echo(ssh.authorized_keys_entry(cfg.ssh.key_file, cfg.app_server.host))
    click.echo(f"# append it to ~/.ssh/authorized_keys of the accounts listed in {cfg.ssh.hosts_config_file}",
               err=True)


@main.group()
def create():
    """Create objects (accounts)."""


@create.command("user")
@click.option("-m", "--multiple", is_flag=True, help="keep prompting for more accounts")
def create_user(multiple):
    from .core.account_creator import AccountCreator
    from .database import configure, ensure_db_with_current_schema

    configure()
    ensure_db_with_current_schema()
    while True:
        AccountCreator().run_prompt()
        if not multiple or not click.confirm("Create another account?", default=False):
            break


@main.command()
def doctor():
    """Check ROCm, amdsmi, HIP kernels, RCCL and the node's xGMI topology."""
    from .doctor import run_checks

    ok = True
    for name, passed, detail in run_checks():
        ok &= passed or name.startswith("optional")
        click.echo(f"[{'OK' if passed else '--'}] {name}: {detail}")
    sys.exit(0 if ok else 1)


@main.command()
@click.argument("what", type=click.Choice(["poll", "launch", "train", "scheduled", "multitenant", "scaling",
                                           "overhead"]))
@click.option("--requests", default=1000)
@click.option("--gpus", default=1)
@click.option("--pinned", is_flag=True, help="multitenant: reference-style pinned device pairs")
@click.option("--real", is_flag=True, help="multitenant: this node's GPUs, real processes, real time")
@click.option("--bucket-mb", "bucket_mb", multiple=True, type=float,
              help="scaling: gradient bucket sizes to sweep (repeat the option); train: the bucket size")
def bench(what, requests, gpus, pinned, real, bucket_mb):
    """Benchmarks of BASELINE.md: poll latency, queued-job launch latency, multi-tenant queue
    wait / GPU utilisation, training tokens/s, and its 1/2/4/8-GPU weak-scaling curve."""
    from . import benchmarks

    if what == "overhead":  # monitoring cost on this node: daemon CPU, probe duty, tenant tokens/s
        click.echo(json.dumps(benchmarks.monitoring_overhead()))
    elif what == "multitenant" and real:
        click.echo(json.dumps(benchmarks.multitenant_node()))
    elif what == "multitenant":
        click.echo(json.dumps(benchmarks.multitenant(pinned=pinned)))
    elif what == "poll":
        click.echo(json.dumps(benchmarks.poll_latency(requests)))
    elif what == "launch":
        click.echo(json.dumps(benchmarks.launch_latency()))
    elif what == "scheduled":
        click.echo(json.dumps(benchmarks.scheduled_training(gpus)))
    elif what == "scaling":  # 1, 2, 4, 8 GPUs (those the node has), weak-scaling efficiency
        click.echo(json.dumps(benchmarks.scaling([1, 2, 4, 8], bucket_mbs=list(bucket_mb) or None)))
    else:
        click.echo(json.dumps(benchmarks.train_throughput(gpus, bucket_mb=bucket_mb[0] if bucket_mb else None)))


def rocprof_prefix(task_id: int, pmc: str = "") -> str:
    """rocprofv3 in front of a task's program.  Counters (``--pmc``) get their own run without
    tracing; the output lands next to the task logs."""
    if pmc:
        return ("rocprofv3 --pmc %s --output-format csv -d ~/TensorHiveLogs/pmc_task_%d"
                % (pmc.replace(",", " "), task_id))
    return "rocprofv3 --kernel-trace --stats --output-format csv -d ~/TensorHiveLogs/prof_task_%d" % task_id


@main.command()
@click.option("--task", "task_id", required=True, type=int)
@click.option("--pmc", default="", help="comma separated counters (separate run, never with tracing)")
@click.option("--create", is_flag=True, help="add the profiled copy as a new task of the same job")
def profile(task_id, pmc, create):
    """Profile a task under rocprofv3 (kernel trace + stats, or --pmc counters).

    Prints the profiled command line.  The task's environment segments stay in front of
    rocprofv3 and the program itself follows ``--``, because rocprofv3 must start the program
    directly.  ``--create`` stores it as a new task of the same job, ready to run or enqueue."""
    from .database import configure
    from .models.orm import Task

    configure()
    t = Task.get(task_id)
    prof = rocprof_prefix(task_id, pmc)
    envs = " ".join(f"{n}={v}" for n, v in t.envs())
    body = t.full_command[len(envs):].strip() if envs and t.full_command.startswith(envs) else t.full_command
    click.echo(f"{envs} {prof} -- {body}".strip())
    if create:
        from .controllers.task import _apply_segments

        nt = Task(command=f"{prof} -- {t.command}", hostname=t.hostname)
        nt.save()
        _apply_segments(nt, {"envs": [{"name": n, "value": v} for n, v in t.envs()],
                             "params": [{"name": n, "value": v} for n, v in t.params()]})
        nt.save()
        if t.job is not None:
            t.job.add_task(nt)
        click.echo(f"created task {nt.id}")


if __name__ == "__main__":
    main()
