"""Reactions to reservation violations (reference ``core/violation_handlers/*.py``).

* :class:`MessageSendingBehaviour` -- ANSI warning on every terminal of the intruder on each
  affected node (``who`` + ``tee /dev/<tty>``, one merged command per node).  Fixed: a node
  where the intruder has no terminal no longer aborts the other nodes (reference ``return`` at
  ``MessageSendingBehaviour.py:69``).
* :class:`EmailSendingBehaviour` -- per-recipient resend timers, intruder and/or admins,
  at most ``max_emails_per_protection_interval`` messages per trigger.
* :class:`UserProcessKillingBehaviour` / :class:`SudoProcessKillingBehaviour` -- ``kill`` as the
  intruder or ``sudo kill`` as the TensorHive account (fixed: the sudo variant no longer runs
  the kill twice, ``SudoProcessKillingBehaviour.py:23,26``).  When the node is the daemon's
  own node and the pid belongs to a th-run task, the whole process group is signalled.
"""
from __future__ import annotations

import datetime
import logging
import queue
import shlex
import smtplib
from textwrap import dedent

from ..utils import dates
from . import ssh
from .mailer import Mailer, Message, MessageBodyTemplater

log = logging.getLogger(__name__)


class ProtectionHandler:
    def __init__(self, behaviour):
        self.behaviour = behaviour

    def trigger_action(self, violation_data: dict) -> None:
        self.behaviour.trigger_action(violation_data)


class MessageSendingBehaviour:
    def __init__(self, transports):
        self.transports = transports

    @staticmethod
    def warning_message(data: dict) -> str:
        return dedent(f"""\
            \\e[41m\\e[97m
            You are using GPU(s) reserved by someone else!
            Please stop your computations on them now.\\e[0m
            \\e[31m\\e[1m
            GPUs: {data['GPUS']}\\e[0m
            Check the TensorHive reservation calendar before starting GPU work.
            -- tensorhive
            \\e[0m""")

    @staticmethod
    def merged_command(ttys: list[dict], msg: str) -> str:
        assert ttys, "List cannot be empty!"
        return ";".join(f"echo -e {shlex.quote(msg)} | tee /dev/{t['TTY']} >/dev/null" for t in ttys)

    def trigger_action(self, violation_data: dict) -> None:
        msg = self.warning_message(violation_data)
        intruder = violation_data["INTRUDER_USERNAME"]
        for host in violation_data.get("HOSTNAMES", []):
            t = self.transports.get(host)
            ttys = [s for s in ssh.node_tty_sessions(t) if s["USER"] == intruder]
            if not ttys:
                continue
            t.run(self.merged_command(ttys, msg))
            for tty in ttys:
                log.warning("violation warning sent to %s on %s:%s", intruder, host, tty["TTY"])


class _Timer:
    def __init__(self):
        self.to_admin = datetime.datetime.min
        self.to_intruder = datetime.datetime.min


class EmailSendingBehaviour:
    def __init__(self, mailbot_cfg, user_lookup=None, smtp_factory=smtplib.SMTP):
        self.cfg = mailbot_cfg
        self.mailer = Mailer(mailbot_cfg.smtp_server, mailbot_cfg.smtp_port, smtp_factory)
        self.interval = datetime.timedelta(minutes=mailbot_cfg.interval)
        self.timers: dict[str, _Timer] = {}
        self.queue: queue.Queue = queue.Queue()
        self._lookup = user_lookup or self._db_email

    @staticmethod
    def _db_email(username: str) -> str | None:
        from ..models.orm import User

        try:
            return User.find_by_username(username).email
        except Exception:  # noqa: BLE001
            return None

    def _smtp_ok(self) -> bool:
        c = self.cfg
        try:
            assert c.smtp_server and c.smtp_port, "Incomplete SMTP server configuration"
            assert c.smtp_login and c.smtp_password, "Incomplete SMTP server credentials"
            if c.notify_admin:
                assert c.admin_email, "Admin contact email not specified despite enabled notifications"
            self.mailer.connect(c.smtp_login, c.smtp_password)
            return True
        except (AssertionError, smtplib.SMTPException, OSError) as e:
            log.error("mailbot disabled for this round: %s", e)
            return False

    def _timer(self, key: str) -> _Timer:
        return self.timers.setdefault(key, _Timer())

    def _due(self, timer: _Timer, admin: bool = False) -> bool:
        last = timer.to_admin if admin else timer.to_intruder
        return last + self.interval <= dates.utcnow()

    def _queue_admin(self, data: dict, timer: _Timer) -> None:
        body = MessageBodyTemplater(self.cfg.admin_body_template).fill_in(data)
        for addr in [a.strip() for a in (self.cfg.admin_email or "").split(",") if a.strip()]:
            self.queue.put(Message(self.cfg.smtp_login, addr, self.cfg.admin_subject, body))
        timer.to_admin = dates.utcnow()

    def _queue_intruder(self, addr: str, data: dict, timer: _Timer) -> None:
        body = MessageBodyTemplater(self.cfg.intruder_body_template).fill_in(data)
        self.queue.put(Message(self.cfg.smtp_login, addr, self.cfg.intruder_subject, body))
        timer.to_intruder = dates.utcnow()

    def trigger_action(self, violation_data: dict) -> None:
        assert {"INTRUDER_USERNAME", "GPUS"} <= set(violation_data), "Missing keys in violation_data"
        if not self._smtp_ok():
            return
        email = self._lookup(violation_data["INTRUDER_USERNAME"])
        violation_data["INTRUDER_EMAIL"] = email
        if not email or email == "<email_missing>":
            timer = self._timer(violation_data["INTRUDER_USERNAME"])
            if self.cfg.notify_admin and self._due(timer, admin=True):
                self._queue_admin(violation_data, timer)
        else:
            timer = self._timer(email)
            if self.cfg.notify_intruder and self._due(timer):
                self._queue_intruder(email, violation_data, timer)
            if self.cfg.notify_admin and self._due(timer, admin=True):
                self._queue_admin(violation_data, timer)
        for _ in range(self.cfg.max_emails_per_protection_interval):
            if self.queue.empty():
                break
            self.mailer.send(self.queue.get())
        self.mailer.disconnect()


class UserProcessKillingBehaviour:
    """``kill <pids>`` over a connection AS the intruder (needs their authorized_keys entry)."""

    def __init__(self, transports):
        self.transports = transports

    def trigger_action(self, violation_data: dict) -> None:
        user = violation_data["INTRUDER_USERNAME"]
        for host, pids in violation_data["VIOLATION_PIDS"].items():
            cmd = "kill " + " ".join(str(int(p)) for p in sorted(pids))
            try:
                r = self.transports.get(host).run(cmd, user=user)
                log.warning("killed %s of %s on %s (rc=%s)", sorted(pids), user, host, r.exit_code)
            except Exception as e:  # noqa: BLE001
                log.error("unable to kill processes of %s on %s: %s", user, host, e)


class SudoProcessKillingBehaviour:
    """``sudo kill <pids>`` as the TensorHive account -- exactly once."""

    def __init__(self, transports):
        self.transports = transports

    def trigger_action(self, violation_data: dict) -> None:
        for host, pids in violation_data["VIOLATION_PIDS"].items():
            cmd = "sudo -n kill " + " ".join(str(int(p)) for p in sorted(pids))
            r = self.transports.get(host).run(cmd)
            if r.ok:
                log.warning("sudo-killed %s on %s", sorted(pids), host)
            else:
                log.error("sudo kill on %s failed: %s", host, r.stderr.strip())
