"""E-mail plumbing for violation notices (reference ``core/utils/mailer.py:11-86``):
MIME HTML messages, SMTP + STARTTLS + login, a template filler for ``{gpus}``,
``{intruder_username}``, ``{intruder_email}``, ``{owners}``."""
from __future__ import annotations

import logging
import smtplib
from email.mime.multipart import MIMEMultipart
from email.mime.text import MIMEText

log = logging.getLogger(__name__)


class Message:
    def __init__(self, author: str, to, subject: str, body: str):
        m = MIMEMultipart()
        m["From"] = author
        m["To"] = ", ".join(to) if isinstance(to, (list, tuple)) else to
        m["Subject"] = subject
        m.attach(MIMEText(body or "", "html"))
        self.msg = m

    @property
    def author(self):
        return self.msg["From"]

    @property
    def recipients(self):
        return self.msg["To"]

    @property
    def subject(self):
        return self.msg["Subject"]

    @property
    def body(self):
        return self.msg.as_string()


class MessageBodyTemplater:
    def __init__(self, template: str):
        self.template = template

    def fill_in(self, data: dict) -> str:
        return self.template.format(gpus=data.get("GPUS", ""), intruder_username=data.get("INTRUDER_USERNAME", ""),
                                    intruder_email=data.get("INTRUDER_EMAIL", ""), owners=data.get("OWNERS", ""))


class Mailer:
    def __init__(self, server: str | None, port: int | None, smtp_factory=smtplib.SMTP):
        self.smtp_server, self.smtp_port = server, port
        self.server = None
        self._factory = smtp_factory

    def connect(self, login: str, password: str) -> None:
        self.server = self._factory(self.smtp_server, self.smtp_port)
        self.server.starttls()
        self.server.login(login, password)

    def send(self, message: Message) -> None:
        assert self.server is not None, "Must call connect() first!"
        assert message.author and message.recipients and message.body, "Incomplete email"
        try:
            self.server.sendmail(message.author, message.recipients, message.body)
        except smtplib.SMTPException as e:
            log.error("error while sending email: %s", e)

    def disconnect(self) -> None:
        if self.server is not None:
            try:
                self.server.quit()
            except smtplib.SMTPException:
                self.server.close()
            self.server = None
