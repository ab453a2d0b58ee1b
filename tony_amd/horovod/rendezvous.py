"""HTTP key-value rendezvous server (the role of Horovod's RendezvousServer, TR/horovod_driver.py:32-42).

Speaks the Gloo HTTP-store protocol Horovod workers use: ``PUT /<scope>/<key>``
stores the body, ``GET /<scope>/<key>`` returns it (404 until present),
``DELETE /<scope>/<key>`` removes it.  tony_amd.parallel.hvd uses the same
store to publish the rank-0 TCPStore address for torch.distributed, so a job
started by the Horovod runtime needs nothing but the HOROVOD_GLOO_RENDEZVOUS_*
variables.  The slot plan is also published under ``/rendezvous/plan``.
"""
from __future__ import annotations

import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Dict, Optional


class _Handler(BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"

    def log_message(self, fmt, *args):  # quiet
        pass

    def _reply(self, code: int, body: bytes = b""):
        self.send_response(code)
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        if body:
            self.wfile.write(body)

    def do_GET(self):  # noqa: N802
        with self.server.kv_lock:
            v = self.server.kv.get(self.path)
        if v is None:
            self._reply(404)
        else:
            self._reply(200, v)

    def do_PUT(self):  # noqa: N802
        n = int(self.headers.get("Content-Length", "0"))
        body = self.rfile.read(n) if n else b""
        with self.server.kv_lock:
            self.server.kv[self.path] = body
        self._reply(200)

    do_POST = do_PUT

    def do_DELETE(self):  # noqa: N802
        with self.server.kv_lock:
            self.server.kv.pop(self.path, None)
        self._reply(200)


class RendezvousServer:
    def __init__(self, host: str = "0.0.0.0", port: int = 0):
        self.httpd = ThreadingHTTPServer((host, port), _Handler)
        self.httpd.kv: Dict[str, bytes] = {}
        self.httpd.kv_lock = threading.Lock()
        self.httpd.daemon_threads = True
        self._thread: Optional[threading.Thread] = None

    @property
    def port(self) -> int:
        return self.httpd.server_address[1]

    def start(self) -> int:
        self._thread = threading.Thread(target=self.httpd.serve_forever, name="tony-hvd-rendezvous", daemon=True)
        self._thread.start()
        return self.port

    def init(self, plan_json: str) -> None:
        with self.httpd.kv_lock:
            self.httpd.kv["/rendezvous/plan"] = plan_json.encode()

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()


def kv_get(addr: str, port: int, key: str, timeout_s: float = 60.0, poll_s: float = 0.05) -> bytes:
    """Blocking GET of ``/<key>`` from a rendezvous server."""
    import time
    import urllib.error
    import urllib.request

    deadline = time.monotonic() + timeout_s
    url = f"http://{addr}:{port}/{key.lstrip('/')}"
    while True:
        try:
            with urllib.request.urlopen(url, timeout=5) as r:
                return r.read()
        except urllib.error.HTTPError as e:
            if e.code != 404:
                raise
        except urllib.error.URLError:
            pass
        if time.monotonic() > deadline:
            raise TimeoutError(f"rendezvous key {key} not published within {timeout_s}s")
        time.sleep(poll_s)


def kv_put(addr: str, port: int, key: str, value: bytes) -> None:
    import urllib.request

    req = urllib.request.Request(f"http://{addr}:{port}/{key.lstrip('/')}", data=value, method="PUT")
    with urllib.request.urlopen(req, timeout=10):
        pass
