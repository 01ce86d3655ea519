"""The daemon object (reference ``core/managers/{TensorHiveManager,ServiceManager}.py``).

Explicit dependency injection instead of a metaclass singleton: one :class:`Daemon` owns the
config, infrastructure store, transports, telemetry backends and services; the Flask app gets
it through ``create_app(daemon)``.  Startup mirrors ``TensorHiveManager.__init__``: load/create
the dedicated SSH key, refuse an empty hosts config, optionally test SSH, then build services.
"""
from __future__ import annotations

import logging
import threading
import time

from ..config import Config, get_config
from ..utils.exceptions import ConfigurationException
from .infrastructure import InfrastructureStore
from .services import (JobSchedulingService, MonitoringService, ProtectionService, Service,
                       UsageLoggingService)
from .telemetry import StubBackend, TelemetryBackend, make_backend
from .transport import TransportManager

log = logging.getLogger(__name__)


class Daemon:
    def __init__(self, cfg: Config | None = None, transports: TransportManager | None = None,
                 backends: dict[str, TelemetryBackend] | None = None, init_key: bool = True,
                 test_ssh: bool | None = None):
        self.cfg = cfg or get_config()
        nodes = self.cfg.ssh.available_nodes
        if not nodes:
            raise ConfigurationException(
                f"no hosts configured in {self.cfg.ssh.hosts_config_file}; add at least one [hostname] section")
        self.ssh_key_path = self.cfg.ssh.key_file
        if init_key:
            from . import ssh

            try:
                ssh.init_ssh_key(self.ssh_key_path)
            except Exception as e:  # noqa: BLE001 -- ssh-keygen missing etc.
                log.warning("could not create the dedicated SSH key: %s", e)
        self.transports = transports or TransportManager.from_config(nodes, self.ssh_key_path, self.cfg.ssh.proxy,
                                                                    self.cfg.ssh.timeout)
        if test_ssh if test_ssh is not None else self.cfg.ssh.test_on_startup:
            bad = [h for h, ok in self.transports.test_all(self.cfg.ssh.timeout).items() if not ok]
            if bad:
                log.warning("SSH test failed for: %s", ", ".join(bad))
        from . import task_nursery

        task_nursery.use_transports(self.transports)
        from .attribution import REGISTRY, Attestor

        # every sample is attested as it is published: a process's TENSORHIVE_TASK_ID counts only
        # inside that task's th-run session and uid (core/attribution.py)
        # (session lookups of unseen claims run on the attestor's own worker thread, never on the monitoring
        # pool, the event listener or a node agent's stream reader: ADVICE r05)
        self.attestor = Attestor(REGISTRY, lookup=self.lookup_task_sessions, background=True)
        self.infrastructure = InfrastructureStore(list(nodes), attest=self.attestor.attest_entry)
        if backends is None:
            am = self.cfg.amd_monitor
            shared: dict = {}
            backends = {}
            for h in nodes:
                kind = am.backend
                b = make_backend(kind, h, self.transports, am.stub_gpus, am.probe_enabled, am.probe_period,
                                 stream_ms=int(1000 * self.cfg.monitoring.update_interval),
                                 counters=am.counters_enabled, counters_period_ms=am.counters_period_ms,
                                 task_hbm=am.task_hbm_counters, remote_mode=am.remote_mode,
                                 remote_agent=am.remote_agent,
                                 events_socket=(self.cfg.launcher.node_events_socket
                                                if self.cfg.launcher.task_events else None))
                # one StubBackend / AmdSmiBackend instance is enough for all hosts of that kind
                backends[h] = shared.setdefault(type(b).__name__, b) if isinstance(b, StubBackend) else b
        self.backends = backends
        from .transport import SimulatedNode

        for h, t in self.transports.transports.items():  # simulated nodes report into the stub telemetry
            if isinstance(t, SimulatedNode) and t.telemetry is None and isinstance(backends.get(h), StubBackend):
                t.telemetry = backends[h]
        self.services: list[Service] = []
        self._topology_cache: dict = {}
        self._lock = threading.Lock()
        self.task_events: list[tuple[float, str, dict]] = []  # (unix time, host, event), newest last
        self._event_sampled: dict[str, float] = {}  # host -> time of its last event-triggered sample
        self._event_deferred: dict[str, threading.Timer] = {}  # host -> its pending trailing sample
        self.events = None
        self._start_task_events()

    # ------------------------------------------------------------------ task-exit events
    def _start_task_events(self) -> None:
        """Task exits as events (core/events.py): a listener for the daemon's own node, the node
        agents' event lines for remote nodes, the in-process hook of simulated nodes."""
        from . import task_nursery
        from .telemetry import RemoteBackend
        from .transport import LocalTransport, SimulatedNode

        if not getattr(self.cfg.launcher, "task_events", True):
            return
        local = [h for h, t in self.transports.transports.items() if isinstance(t, LocalTransport)]
        if local:
            from .events import EventListener

            try:
                self.events = EventListener(lambda ev: [self.on_task_event(h, ev) for h in local])
            except OSError as e:
                log.warning("task-exit events unavailable (%s); exits are found by polling", e)
        for h, t in self.transports.transports.items():
            if isinstance(t, SimulatedNode):
                t.on_event = lambda ev, h=h: self.on_task_event(h, ev)
        for h, b in self.backends.items():
            if isinstance(b, RemoteBackend):
                b.on_event = self.on_task_event
        task_nursery.use_event_sockets(self.event_socket_for)

    def event_socket_for(self, host: str) -> str | None:
        """Where a task spawned on ``host`` reports its exit (``th-run --notify``)."""
        from .telemetry import RemoteBackend
        from .transport import LocalTransport

        t = self.transports.transports.get(host)
        if isinstance(t, LocalTransport):
            return self.events.path if self.events is not None else None
        b = self.backends.get(host)
        if isinstance(b, RemoteBackend) and b.node_mode(host) == "agent" and b.stream_ms:
            return b.event_socket(host)  # only a path the node's agent reported having bound
        return None

    # a host is re-sampled for task events at most this often: the node socket takes datagrams from any
    # local user, so a flood must not turn into a flood of telemetry samples (the wake is coalesced anyway)
    EVENT_SAMPLE_MIN_S = 0.02

    def on_task_event(self, host: str, ev: dict) -> None:
        """A task on ``host`` ended: refresh that host's telemetry now (its devices no longer show
        the task's processes) and run the job scheduler, which releases the devices and starts the
        next queued job in the same tick."""
        now = time.time()
        with self._lock:
            self.task_events.append((now, host, dict(ev)))
            del self.task_events[:-256]
            wait = self._event_sampled.get(host, 0.0) + self.EVENT_SAMPLE_MIN_S - now
            if wait <= 0:
                self._event_sampled[host] = now
            elif host in self._event_deferred:
                return  # a trailing sample + wake for this host is already scheduled
            else:
                # inside the window: one trailing sample + wake at its end, so a real exit that follows
                # another event closely is still seen at once
                t = threading.Timer(wait, self._deferred_task_event, args=(host,))
                t.daemon = True
                self._event_deferred[host] = t
                t.start()
                return
        self._sample_and_wake(host)

    def _deferred_task_event(self, host: str) -> None:
        with self._lock:
            self._event_deferred.pop(host, None)
            self._event_sampled[host] = time.time()
        self._sample_and_wake(host)

    def _sample_and_wake(self, host: str) -> None:
        from .services import MonitoringService

        mon = self.service(MonitoringService)
        if mon is not None and host in mon.backends:
            mon.sample_host(host)
        self.wake("task_exit")

    # ------------------------------------------------------------------ services
    def configure_services_from_config(self) -> list[Service]:
        from .violation_handlers import (EmailSendingBehaviour, MessageSendingBehaviour, ProtectionHandler,
                                         SudoProcessKillingBehaviour, UserProcessKillingBehaviour)

        c = self.cfg
        svcs: list[Service] = []
        if c.monitoring.enabled:
            svcs.append(MonitoringService(c.monitoring.update_interval, self.backends if c.monitoring.enable_gpu_monitor
                                          else {h: StubBackend(0) for h in self.backends}))
        if c.protection.level > 0:
            handlers = []
            if c.protection.notify_on_pty:
                handlers.append(ProtectionHandler(MessageSendingBehaviour(self.transports)))
            if c.protection.notify_via_email:
                handlers.append(ProtectionHandler(EmailSendingBehaviour(c.mailbot)))
            if c.protection.kill_processes == 1:
                handlers.append(ProtectionHandler(UserProcessKillingBehaviour(self.transports)))
            elif c.protection.kill_processes == 2:
                handlers.append(ProtectionHandler(SudoProcessKillingBehaviour(self.transports)))
            svcs.append(ProtectionService(c.protection.update_interval, handlers, c.protection.level))
        if c.usage_logging.enabled:
            svcs.append(UsageLoggingService(c.usage_logging.update_interval, c.usage_logging.log_dir,
                                            c.usage_logging.log_cleanup_action))
        if c.job_scheduling.enabled:
            svcs.append(JobSchedulingService(c.job_scheduling.update_interval,
                                             c.job_scheduling.stop_termination_attempts_after_mins,
                                             c.job_scheduling.schedule_queued_jobs_when_free_mins))
        for s in svcs:
            s.inject(self)
        self.services = svcs
        return svcs

    def add_service(self, svc: Service) -> None:
        svc.inject(self)
        self.services.append(svc)

    def service(self, cls):
        for s in self.services:
            if isinstance(s, cls):
                return s
        return None

    def init(self) -> None:
        for s in self.services:
            s.start()

    start = init

    def shutdown(self, timeout: float = 5.0) -> None:
        if self.events is not None:
            self.events.close()
            self.events = None
        with self._lock:
            pending, self._event_deferred = list(self._event_deferred.values()), {}
        for t in pending:
            t.cancel()
        for s in self.services:
            s.stop()
        for s in self.services:
            if s.is_alive():
                s.join(timeout)
        self.attestor.close()
        for b in {id(b): b for b in self.backends.values()}.values():
            try:
                b.close()
            except Exception:  # noqa: BLE001
                pass
        self.transports.close()
        from . import task_nursery

        if task_nursery._transports is self.transports:
            task_nursery.use_transports(None)
        if task_nursery._event_socket_for == self.event_socket_for:
            task_nursery.use_event_sockets(None)

    def lookup_task_sessions(self, host: str, task_id: str) -> None:
        """Refresh the attestation registry for a claimed task it has not seen: list the task
        owner's th-run sessions on ``host`` (which records them).  Claims naming no task of that
        host cost no round trip."""
        from ..database import db_session
        from ..models.orm import Task
        from . import task_nursery

        try:
            t = Task.query.filter(Task.id == int(task_id)).first()
            user = t.job.user.username if t is not None and t.job is not None and t.job.user else None
            if user is None or t.hostname != host:
                return
        except (ValueError, TypeError):
            return
        finally:
            db_session.remove()
        task_nursery.running(host, user)

    def wake(self, reason: str = "") -> None:
        """Event-driven wake-up of the job scheduler (enqueue, reservation change, job stop, and
        ``gpu_freed`` from the monitoring service: a device lost its last process)."""
        s = self.service(JobSchedulingService)
        if s is not None:
            if reason == "gpu_freed":
                s.device_freed()
            else:
                s.wake()

    def scheduling_window(self):
        """How long a GPU must stay free before a queued job may take it
        (``schedule_queued_jobs_when_free_mins``); also the look-ahead of device placement."""
        from datetime import timedelta

        return timedelta(minutes=self.cfg.job_scheduling.schedule_queued_jobs_when_free_mins)

    # ------------------------------------------------------------------ introspection
    def topology(self) -> dict:
        out = {}
        for h, b in self.backends.items():
            if h not in self._topology_cache:
                try:
                    self._topology_cache[h] = b.topology(h)
                except Exception as e:  # noqa: BLE001
                    self._topology_cache[h] = {"error": str(e)}
            out[h] = self._topology_cache[h]
        return out

    def service_stats(self) -> dict:
        return {s.name: {"ticks": s.ticks, "interval_s": s.interval, **s.stats.summary()} for s in self.services}
