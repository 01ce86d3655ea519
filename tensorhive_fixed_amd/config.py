"""Configuration: INI files in ``~/.config/TensorHive`` (compatible section/key names), typed.

Reference behaviour (``tensorhive/config.py``): templates are copied into the config dir on
*import* (``config.py:31-87``) and values become class constants with fallbacks
(``config.py:113-298``).  Here:

* copying the templates is an explicit :func:`init_config_files` call (the CLI does it), never
  an import side effect;
* :class:`Config` is an immutable-ish object built by :func:`load_config`; the process-wide
  instance is returned by :func:`get_config` and can be replaced (tests, ``--config DIR``);
* both spellings of the reference's quirks are honoured with a warning: ``[auth] secrect_key``
  vs ``secret_key`` (``config.py:289``) and ``[task_scheduling_service]`` vs
  ``[job_scheduling_service]`` (``main_config.ini:68`` vs ``config.py:255``);
* ``TENSORHIVE_<SECTION>_<KEY>`` environment variables override any key;
* new sections ``[amd_monitor]`` and ``[launcher]`` configure the MI355X telemetry and launcher.
"""
from __future__ import annotations

import ast
import configparser
import logging
import os
import re
import secrets
import shutil
import threading
from dataclasses import dataclass, field
from datetime import timedelta
from pathlib import Path
from typing import Any

import yaml

log = logging.getLogger(__name__)

PACKAGE_DIR = Path(__file__).resolve().parent
TEMPLATE_DIR = PACKAGE_DIR / "templates"
DEFAULT_CONFIG_DIR = Path(os.environ.get("TENSORHIVE_CONFIG_DIR", "~/.config/TensorHive")).expanduser()


def config_dir() -> Path:
    return Path(os.environ.get("TENSORHIVE_CONFIG_DIR", str(DEFAULT_CONFIG_DIR))).expanduser()


# signing keys that are public knowledge: the reference ships ``jwt-some-secret`` in its template
# and as the fallback (``tensorhive/config.py:289``, ``main_config.ini:75``), so with it anyone who
# reaches the API can mint an admin token
INSECURE_SECRETS = frozenset({"", "jwt-some-secret", "secret", "changeme"})
ALLOW_INSECURE_ENV = "TENSORHIVE_ALLOW_INSECURE_SECRET"
_SECRET_LINE = re.compile(r"^(\s*secret_key\s*=)[ \t]*(.*)$", re.M)


MIN_SECRET_LEN = 32  # characters; new_secret() writes 64 hex digits (256 bits)


def secret_is_public(secret: str | None) -> bool:
    """Empty or a key published with the reference: replaced by a random one on startup."""
    return (secret or "").strip() in INSECURE_SECRETS


def secret_is_insecure(secret: str | None) -> bool:
    """Public, or too short to resist an offline guess of the HS256 key (a one-character key
    would be found from any token in microseconds): the daemon refuses to start with it."""
    return secret_is_public(secret) or len((secret or "").strip()) < MIN_SECRET_LEN


def insecure_secret_allowed() -> bool:
    return os.environ.get(ALLOW_INSECURE_ENV, "") in ("1", "yes", "true")


def new_secret() -> str:
    return secrets.token_hex(32)  # 256 bits


def ensure_secret_key(path: Path | str) -> bool:
    """Give ``main_config.ini`` a random ``[auth] secret_key`` when it has none or the public
    default (keeps the file's other lines and its 0600 mode). Returns True when it wrote one."""
    p = Path(path).expanduser()
    try:
        text = p.read_text()
    except OSError:
        return False
    cp = configparser.ConfigParser(strict=False)
    cp.read_string(text)
    current = None
    for k in ("secret_key", "secrect_key"):
        if cp.has_option("auth", k):
            current = cp.get("auth", k)
            break
    if current is not None and not secret_is_public(current):
        return False  # the operator's own key: kept (refused at startup if it is too short)
    key = new_secret()
    if current is not None and _SECRET_LINE.search(text):
        text = _SECRET_LINE.sub(lambda m: f"{m.group(1)} {key}", text, count=1)
    elif re.search(r"^\[auth\]\s*$", text, re.M):
        text = re.sub(r"^\[auth\]\s*$", f"[auth]\nsecret_key = {key}", text, count=1, flags=re.M)
    else:
        text = text.rstrip("\n") + f"\n\n[auth]\nsecret_key = {key}\n"
    tmp = p.with_name(p.name + ".tmp")
    fd = os.open(tmp, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
    with os.fdopen(fd, "w") as f:
        f.write(text)
    os.replace(tmp, p)
    log.warning("wrote a new random [auth] secret_key to %s (tokens signed with the old key are void)", p)
    return True


def init_config_files(directory: Path | None = None) -> list[Path]:
    """Copy missing INI templates into ``directory`` (mode 0600); never overwrite. Returns the
    list of files created (reference: ``ConfigInitilizer``, ``config.py:31-69``). A freshly
    created ``main_config.ini`` gets a random 256-bit ``[auth] secret_key``."""
    d = Path(directory or config_dir()).expanduser()
    d.mkdir(parents=True, exist_ok=True)
    created = []
    for name in ("main_config.ini", "hosts_config.ini", "mailbot_config.ini"):
        dst = d / name
        if dst.exists():
            continue
        shutil.copy(TEMPLATE_DIR / name, dst)
        os.chmod(dst, 0o600)
        if name == "main_config.ini":
            ensure_secret_key(dst)
        created.append(dst)
        log.info("created %s", dst)
    return created


def load_ini(path: Path | str, title: str = "") -> configparser.ConfigParser:
    """configparser(strict=False); a missing file only logs (``ConfigLoader``, ``config.py:72-83``)."""
    cp = configparser.ConfigParser(strict=False)
    p = Path(path).expanduser()
    if cp.read(str(p)):
        log.debug("read %s config from %s", title, p)
    else:
        log.info("%s config %s not found, using defaults", title or "a", p)
    return cp


class _Reader:
    """Typed getters over a ConfigParser with env-var overrides and section aliases."""

    def __init__(self, cp: configparser.ConfigParser, env_prefix: str = "TENSORHIVE"):
        self.cp = cp
        self.env_prefix = env_prefix

    def _env(self, section: str, key: str) -> str | None:
        name = f"{self.env_prefix}_{section}_{key}".upper().replace(".", "_").replace("/", "_")
        return os.environ.get(name)

    def raw(self, section: str | tuple[str, ...], key: str | tuple[str, ...], fallback: Any = None):
        sections = (section,) if isinstance(section, str) else section
        keys = (key,) if isinstance(key, str) else key
        for s in sections:
            for k in keys:
                v = self._env(s, k)
                if v is not None:
                    return v
        for i, s in enumerate(sections):
            for j, k in enumerate(keys):
                if self.cp.has_option(s, k):
                    if i or j:
                        log.warning("config: using [%s] %s (alias of [%s] %s)", s, k, sections[0], keys[0])
                    return self.cp.get(s, k)
        return fallback

    def str(self, section, key, fallback=None):
        v = self.raw(section, key, None)
        return fallback if v is None else str(v).strip()

    def float(self, section, key, fallback: float) -> float:
        v = self.raw(section, key, None)
        return fallback if v is None or str(v).strip() == "" else float(v)

    def int(self, section, key, fallback: int) -> int:
        v = self.raw(section, key, None)
        return fallback if v is None or str(v).strip() == "" else int(float(v))

    def bool(self, section, key, fallback: bool) -> bool:
        v = self.raw(section, key, None)
        if v is None:
            return fallback
        s = str(v).strip().lower()
        if s in ("1", "yes", "true", "on"):
            return True
        if s in ("0", "no", "false", "off"):
            return False
        raise ValueError(f"not a boolean: [{section}] {key} = {v}")

    def literal(self, section, key, fallback):
        v = self.raw(section, key, None)
        if v is None:
            return fallback
        try:
            return ast.literal_eval(str(v))
        except (ValueError, SyntaxError):
            log.warning("config: cannot parse [%s] %s = %r, using %r", section, key, v, fallback)
            return fallback


@dataclass
class SSHConfig:
    hosts_config_file: str
    test_on_startup: bool
    timeout: float
    number_of_retries: int
    key_file: str
    available_nodes: dict[str, dict]
    proxy: dict | None


@dataclass
class ApiConfig:
    title: str
    url_schema: str
    url_hostname: str
    url_port: str
    url_prefix: str
    responses: dict
    # /metrics/prometheus: a static scrape token (Prometheus ``bearer_token``; empty = none) and
    # whether non-admin JWTs may scrape (their view is filtered to the GPUs they may use)
    prometheus_token: str = ""
    prometheus_allow_users: bool = False

    @property
    def api_path(self) -> str:
        return f"{self.url_schema}://{self.url_hostname}:{self.url_port}/{self.url_prefix}"


@dataclass
class ServerConfig:
    backend: str
    host: str
    port: int
    debug: bool = False
    workers: int = 1
    loglevel: str = "warning"


@dataclass
class MonitoringConfig:
    enabled: bool
    enable_gpu_monitor: bool
    update_interval: float


@dataclass
class ProtectionConfig:
    level: int
    update_interval: float
    notify_on_pty: bool
    notify_via_email: bool
    kill_processes: int


@dataclass
class MailbotConfig:
    interval: float
    max_emails_per_protection_interval: int
    notify_intruder: bool
    notify_admin: bool
    admin_email: str | None
    smtp_login: str | None
    smtp_password: str | None
    smtp_server: str | None
    smtp_port: int
    intruder_subject: str
    intruder_body_template: str
    admin_subject: str
    admin_body_template: str


@dataclass
class UsageLoggingConfig:
    enabled: bool
    update_interval: float
    log_dir: str
    log_cleanup_action: int


@dataclass
class JobSchedulingConfig:
    enabled: bool
    update_interval: float
    stop_termination_attempts_after_mins: float
    schedule_queued_jobs_when_free_mins: int


@dataclass
class AuthConfig:
    secret_key: str
    blacklist_enabled: bool
    blacklist_token_checks: list
    access_token_expires: timedelta
    refresh_token_expires: timedelta
    token_location: list


@dataclass
class AmdMonitorConfig:
    backend: str
    probe_enabled: bool
    probe_period: float
    stub_gpus: int
    counters_enabled: bool = True
    counters_period_ms: int = 1000
    # tasks count their own HBM bytes (libthhbm via ROCP_TOOL_LIBRARIES, core/hbm.py)
    task_hbm_counters: bool = True
    # remote nodes: "agent" (the node agent streams the full telemetry: probe + HBM files) or "th-smi"
    remote_mode: str = "agent"
    remote_agent: str = "python3 -m tensorhive_fixed_amd.agent"


@dataclass
class LauncherConfig:
    supervisor: str
    log_dir: str
    rdzv_backend: str
    master_port: int
    bucket_mb: int
    restart_delay: float = 5.0  # seconds between a failed run and its restart (task maxRestarts)
    # rank CPU binding (parallel/affinity.py): numa | exclusive | none
    cpu_bind: str = "numa"
    # RCCL knobs written into the torchrun template (empty = RCCL's own choice); bench.py records
    # the effective values in its JSON line
    rccl_min_nchannels: str = ""
    rccl_max_nchannels: str = ""
    rccl_algo: str = ""
    rccl_proto: str = ""
    # node-local path of libthhbm.so on REMOTE nodes (empty = remote tasks are not counted); the
    # daemon's own node always uses this install's copy
    hbm_tool: str = ""
    # task exits as events (core/events.py): th-run notifies the daemon (its own node) or the node
    # agent (remote nodes) when a task has ended; "auto" = the agent binds a private socket and reports
    # its path (a fixed path in /tmp could be squatted by another local user)
    task_events: bool = True
    node_events_socket: str = "auto"


@dataclass
class Config:
    directory: Path
    ssh: SSHConfig
    db_path: str
    db_uri: str
    api: ApiConfig
    app_server: ServerConfig
    api_server: ServerConfig
    monitoring: MonitoringConfig
    protection: ProtectionConfig
    mailbot: MailbotConfig
    usage_logging: UsageLoggingConfig
    job_scheduling: JobSchedulingConfig
    auth: AuthConfig
    amd_monitor: AmdMonitorConfig
    launcher: LauncherConfig
    extra: dict = field(default_factory=dict)


def parse_hosts(path: Path | str) -> tuple[dict[str, dict], dict | None]:
    """Hosts INI -> ({host: {user, port, transport}}, proxy | None)
    (``SSH.hosts_config_to_dict`` / ``proxy_config_to_dict``, ``config.py:121-150``)."""
    cp = load_ini(path, "hosts")
    nodes: dict[str, dict] = {}
    for section in cp.sections():
        if section == "proxy_tunneling":
            continue
        transport = cp.get(section, "transport", fallback="ssh").strip()
        nodes[section] = {
            "user": cp.get(section, "user", fallback=os.environ.get("USER", "root")).strip(),
            "port": cp.getint(section, "port", fallback=22),
            "transport": transport,
        }
    proxy = None
    if cp.has_section("proxy_tunneling") and cp.getboolean("proxy_tunneling", "enabled", fallback=False):
        proxy = {
            "proxy_host": cp.get("proxy_tunneling", "proxy_host"),
            "proxy_user": cp.get("proxy_tunneling", "proxy_user"),
            "proxy_port": cp.getint("proxy_tunneling", "proxy_port", fallback=22),
        }
    return nodes, proxy


def load_responses() -> dict:
    with open(PACKAGE_DIR / "api" / "responses.yml") as f:
        return yaml.safe_load(f)


def load_config(directory: Path | str | None = None) -> Config:
    d = Path(directory or config_dir()).expanduser()
    main = _Reader(load_ini(d / "main_config.ini", "main"))
    mail = _Reader(load_ini(d / "mailbot_config.ini", "mailbot"))
    hosts_file = main.str("ssh", "hosts_config_file", str(d / "hosts_config.ini"))
    if directory is not None and not Path(hosts_file).expanduser().exists():
        hosts_file = str(d / "hosts_config.ini")
    nodes, proxy = parse_hosts(hosts_file)
    db_path = str(Path(main.str("database", "path", str(d / "database.sqlite"))).expanduser())
    db_uri = "sqlite://" if os.environ.get("PYTEST") else f"sqlite:///{db_path}"
    secret = main.str("auth", ("secret_key", "secrect_key"), "")
    tmpl = _Reader(load_ini(TEMPLATE_DIR / "mailbot_config.ini", "mailbot-template"))
    jobs_sections = ("job_scheduling_service", "task_scheduling_service")
    return Config(
        directory=d,
        ssh=SSHConfig(
            hosts_config_file=hosts_file,
            test_on_startup=main.bool("ssh", "test_on_startup", True),
            timeout=main.float("ssh", "timeout", 10.0),
            number_of_retries=main.int("ssh", "number_of_retries", 1),
            key_file=str(Path(main.str("ssh", "key_file", str(d / "ssh_key"))).expanduser()),
            available_nodes=nodes,
            proxy=proxy,
        ),
        db_path=db_path,
        db_uri=db_uri,
        api=ApiConfig(
            title=main.str("api", "title", "TensorHive API"),
            url_schema=main.str("api", "url_schema", "http"),
            url_hostname=main.str("api", "url_hostname", "0.0.0.0"),
            url_port=main.str("api", "url_port", "1111"),
            url_prefix=main.str("api", "url_prefix", "api"),
            responses=load_responses(),
            prometheus_token=main.str("api", "prometheus_token", ""),
            prometheus_allow_users=main.bool("api", "prometheus_allow_users", False),
        ),
        app_server=ServerConfig(
            backend=main.str("web_app.server", "backend", "builtin"),
            host=main.str("web_app.server", "host", "0.0.0.0"),
            port=main.int("web_app.server", "port", 5000),
            workers=main.int("web_app.server", "workers", 4),
            loglevel=main.str("web_app.server", "loglevel", "warning"),
        ),
        api_server=ServerConfig(
            backend=main.str("api.server", "backend", "threaded"),
            host=main.str("api.server", "host", "0.0.0.0"),
            port=main.int("api.server", "port", 1111),
            debug=main.bool("api.server", "debug", False),
        ),
        monitoring=MonitoringConfig(
            enabled=main.bool("monitoring_service", "enabled", True),
            enable_gpu_monitor=main.bool("monitoring_service", "enable_gpu_monitor", True),
            update_interval=main.float("monitoring_service", "update_interval", 2.0),
        ),
        protection=ProtectionConfig(
            level=main.int("protection_service", "level", 1),
            update_interval=main.float("protection_service", "update_interval", 2.0),
            notify_on_pty=main.bool("protection_service", "notify_on_pty", True),
            notify_via_email=main.bool("protection_service", "notify_via_email", False),
            kill_processes=main.int("protection_service", "kill_processes", 0),
        ),
        mailbot=MailbotConfig(
            interval=mail.float("general", "interval", 10.0),
            max_emails_per_protection_interval=mail.int("general", "max_emails_per_protection_interval", 50),
            notify_intruder=mail.bool("general", "notify_intruder", True),
            notify_admin=mail.bool("general", "notify_admin", False),
            admin_email=mail.str("general", "admin_email", None),
            smtp_login=mail.str("smtp", "email", None),
            smtp_password=mail.str("smtp", "password", None),
            smtp_server=mail.str("smtp", "smtp_server", None),
            smtp_port=mail.int("smtp", "smtp_port", 587),
            intruder_subject=mail.str("template/intruder", "subject", tmpl.str("template/intruder", "subject", "")),
            intruder_body_template=mail.str("template/intruder", "html_body",
                                            tmpl.str("template/intruder", "html_body", "{gpus}")),
            admin_subject=mail.str("template/admin", "subject", tmpl.str("template/admin", "subject", "")),
            admin_body_template=mail.str("template/admin", "html_body", tmpl.str("template/admin", "html_body", "{gpus}")),
        ),
        usage_logging=UsageLoggingConfig(
            enabled=main.bool("usage_logging_service", "enabled", True),
            update_interval=main.float("usage_logging_service", "update_interval", 2.0),
            log_dir=str(Path(main.str("usage_logging_service", "log_dir", str(d / "logs"))).expanduser()),
            log_cleanup_action=main.int("usage_logging_service", "log_cleanup_action", 2),
        ),
        job_scheduling=JobSchedulingConfig(
            enabled=main.bool(jobs_sections, "enabled", True),
            update_interval=main.float(jobs_sections, "update_interval", 30.0),
            stop_termination_attempts_after_mins=main.float(jobs_sections, "stop_termination_attempts_after_mins", 5.0),
            schedule_queued_jobs_when_free_mins=main.int(jobs_sections, "schedule_queued_jobs_when_free_mins", 30),
        ),
        auth=AuthConfig(
            secret_key=secret,
            blacklist_enabled=main.bool("auth", "jwt_blacklist_enabled", True),
            blacklist_token_checks=main.literal("auth", "jwt_blacklist_token_checks", ["access", "refresh"]),
            access_token_expires=timedelta(minutes=main.int("auth", "jwt_access_token_expires_minutes", 1)),
            refresh_token_expires=timedelta(days=main.int("auth", "jwt_refresh_token_expires_days", 1)),
            token_location=main.literal("auth", "jwt_token_location", ["headers"]),
        ),
        amd_monitor=AmdMonitorConfig(
            backend=main.str("amd_monitor", "backend", "auto"),
            probe_enabled=main.bool("amd_monitor", "probe_enabled", True),
            probe_period=main.float("amd_monitor", "probe_period", 1.0),
            stub_gpus=main.int("amd_monitor", "stub_gpus", 8),
            counters_enabled=main.bool("amd_monitor", "counters_enabled", True),
            counters_period_ms=main.int("amd_monitor", "counters_period_ms", 1000),
            task_hbm_counters=main.bool("amd_monitor", "task_hbm_counters", True),
            remote_mode=main.str("amd_monitor", "remote_mode", "agent"),
            remote_agent=main.str("amd_monitor", "remote_agent", "python3 -m tensorhive_fixed_amd.agent"),
        ),
        launcher=LauncherConfig(
            supervisor=main.str("launcher", "supervisor", "th-run"),
            log_dir=main.str("launcher", "log_dir", "~/TensorHiveLogs"),
            rdzv_backend=main.str("launcher", "rdzv_backend", "c10d"),
            master_port=main.int("launcher", "master_port", 29500),
            bucket_mb=main.int("launcher", "bucket_mb", 256),
            restart_delay=main.float("launcher", "restart_delay", 5.0),
            cpu_bind=main.str("launcher", "cpu_bind", "numa"),
            rccl_min_nchannels=main.str("launcher", "rccl_min_nchannels", ""),
            rccl_max_nchannels=main.str("launcher", "rccl_max_nchannels", ""),
            rccl_algo=main.str("launcher", "rccl_algo", ""),
            rccl_proto=main.str("launcher", "rccl_proto", ""),
            hbm_tool=main.str("launcher", "hbm_tool", ""),
            task_events=main.bool("launcher", "task_events", True),
            node_events_socket=main.str("launcher", "node_events_socket", "auto"),
        ),
    )


_lock = threading.Lock()
_current: Config | None = None


def get_config() -> Config:
    global _current
    if _current is None:
        with _lock:
            if _current is None:
                _current = load_config()
    return _current


def set_config(cfg: Config | None) -> None:
    """Install a config object (tests / ``tensorhive --config DIR``); None resets to lazy load."""
    global _current
    with _lock:
        _current = cfg
