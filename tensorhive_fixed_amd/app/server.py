"""Dashboard web server (reference ``app/web/AppServer.py:12-89``).

Serves the dependency-free dashboard in ``app/static`` from the daemon process on
``[web_app.server] port`` (default 5000) -- gunicorn is not needed -- and writes
``static/config.json`` = ``{apiPath, version}`` which the SPA reads at startup (a version change
makes the SPA drop its localStorage, as in the reference).
"""
from __future__ import annotations

import json
import logging
import os
import threading
from pathlib import Path

from flask import Flask, send_from_directory
from werkzeug.serving import make_server

from .. import __version__

log = logging.getLogger(__name__)
STATIC = Path(__file__).resolve().parent / "static"


class _ServerThread(threading.Thread):
    def __init__(self, app, host: str, port: int, name: str):
        super().__init__(name=name, daemon=True)
        self.srv = make_server(host, port, app, threaded=True)
        self.port = self.srv.server_port

    def run(self):
        self.srv.serve_forever()

    def shutdown(self):
        self.srv.shutdown()


def quiet_access_log() -> None:
    """werkzeug logs every request at INFO: four lines a second per open dashboard at the 0.25 s
    poll, and ~0.1 ms of each poll.  Kept only with TENSORHIVE_ACCESS_LOG=1."""
    if os.environ.get("TENSORHIVE_ACCESS_LOG", "0") != "1":
        logging.getLogger("werkzeug").setLevel(logging.WARNING)


def serve_wsgi(app, host: str, port: int, name: str = "wsgi") -> _ServerThread:
    quiet_access_log()
    t = _ServerThread(app, host, port, name)
    t.start()
    return t


def create_web_app(api_path: str) -> Flask:
    app = Flask(__name__, static_folder=None)
    cfg_json = json.dumps({"apiPath": api_path, "version": __version__})

    @app.route("/static/config.json")
    def config_json():
        return app.response_class(cfg_json, mimetype="application/json")

    @app.route("/", defaults={"path": ""})
    @app.route("/<path:path>")
    def spa(path):
        p = STATIC / path
        if path and p.is_file():
            return send_from_directory(STATIC, path)
        return send_from_directory(STATIC, "index.html")

    return app


class AppServer:
    def __init__(self, cfg):
        self.cfg = cfg
        self.thread: _ServerThread | None = None

    def start(self) -> "AppServer":
        a = self.cfg.api
        api_path = f"{a.url_schema}://{a.url_hostname}:{a.url_port}/{a.url_prefix}"
        self.thread = serve_wsgi(create_web_app(api_path), self.cfg.app_server.host, self.cfg.app_server.port,
                                 "web-app")
        return self

    def shutdown(self) -> None:
        if self.thread is not None:
            self.thread.shutdown()
