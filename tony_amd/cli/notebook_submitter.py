"""NotebookSubmitter: a single-node job (e.g. Jupyter) plus a local port forward
(tony-cli NotebookSubmitter.java:46-146).

The job (no ``tony.X.instances`` -> the coordinator's single-node mode, the
command runs beside the coordinator) gets a 24 h application timeout.  The
coordinator reserves ``TB_PORT`` for the notebook process and reports a ``notebook`` TaskInfo whose url is ``host:port``; this submitter
watches task-info updates for it and starts a :class:`ProxyServer` on a free
local port, printing the ``ssh -L`` hint TonY prints.  Killing this process
kills the job.
"""
from __future__ import annotations

import logging
import signal
import sys
import threading
from typing import Optional, Set
from urllib.parse import urlparse

from .. import constants as C
from ..client.tony_client import TonyClient
from ..conf import keys as K
from ..proxy import ProxyServer
from .cluster_submitter import TonySubmitter

LOG = logging.getLogger("tony.cli.notebook")
NOTEBOOK_TIMEOUT_MS = 24 * 60 * 60 * 1000


class NotebookUpdateListener:
    """Keeps the latest task-info set (NotebookSubmitter.java:49-60)."""

    def __init__(self):
        self.task_infos: Optional[Set] = None

    def on_application_id_received(self, app_id: str) -> None:
        pass

    def on_task_infos_updated(self, infos) -> None:
        self.task_infos = set(infos)


def notebook_address(url: str):
    """``host:port`` or ``http://host:port/...`` -> (host, port)."""
    u = urlparse(url if "://" in url else f"tcp://{url}")
    if not u.hostname or not u.port:
        raise ValueError(f"bad notebook url {url!r}")
    return u.hostname, u.port


class NotebookSubmitter(TonySubmitter):
    def __init__(self, client: Optional[TonyClient] = None):
        self.listener = NotebookUpdateListener()
        self.client = client or TonyClient()
        self.client.add_listener(self.listener)
        self.proxy: Optional[ProxyServer] = None
        self.exit_code = -1

    def _start_proxy(self, url: str) -> None:
        host, port = notebook_address(url)
        self.proxy = ProxyServer(host, port, 0)
        local = self.proxy.start_background()
        LOG.info("If you are running NotebookSubmitter on your local box, open [localhost:%d] in your browser. "
                 "Otherwise (e.g. on a gateway) run [ssh -L 18888:localhost:%d <this host>] on your laptop and "
                 "open [localhost:18888]; pick another number if 18888 is taken.", local, local)

    def submit(self, args) -> int:
        args = list(args) + ["--conf", f"{K.APPLICATION_TIMEOUT}={NOTEBOOK_TIMEOUT_MS}"]
        if not self.client.init(args):
            return -1

        def _run():
            self.exit_code = self.client.start()

        t = threading.Thread(target=_run, name="tony-notebook-client", daemon=True)

        def _kill(signum, _frame):
            LOG.info("signal %d: killing the notebook application", signum)
            self.client.force_kill_application()
            sys.exit(-1)

        old = {}
        if threading.current_thread() is threading.main_thread():
            old = {s: signal.signal(s, _kill) for s in (signal.SIGINT, signal.SIGTERM)}
        try:
            t.start()
            while t.is_alive():
                if self.proxy is None and self.listener.task_infos:
                    for ti in self.listener.task_infos:
                        if ti.name == C.NOTEBOOK_JOB_NAME and ti.url:
                            self._start_proxy(ti.url)
                            break
                t.join(0.2)
        finally:
            for s, h in old.items():
                signal.signal(s, h)
            if self.proxy is not None:
                self.proxy.stop()
        return self.exit_code


def main(argv=None) -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    return NotebookSubmitter().submit(sys.argv[1:] if argv is None else argv)


if __name__ == "__main__":
    sys.exit(main() & 0xFF)
