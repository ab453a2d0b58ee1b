"""ClusterSubmitter: the production entry point (tony-cli ClusterSubmitter.java:41-94).

``python -m com.linkedin.tony.cli.ClusterSubmitter <TonyClient options>`` (or
``bin/tony``) submits to the node's coordinator, installs a SIGINT/SIGTERM hook
that kills the whole gang, and exits 0 on success / 255 (-1) on failure.
"""
from __future__ import annotations

import logging
import signal
import sys

from ..client.tony_client import TonyClient

LOG = logging.getLogger("tony.cli")


class TonySubmitter:
    def submit(self, args) -> int:  # tony-cli TonySubmitter.java:7-9
        raise NotImplementedError


class ClusterSubmitter(TonySubmitter):
    def __init__(self, client: TonyClient = None):
        self.client = client or TonyClient()

    def submit(self, args) -> int:
        if not self.client.init(args):
            return -1

        def _kill(signum, _frame):
            LOG.info("signal %d: killing the application", signum)
            self.client.force_kill_application()
            sys.exit(-1)

        old_int = signal.signal(signal.SIGINT, _kill)
        old_term = signal.signal(signal.SIGTERM, _kill)
        try:
            return self.client.start()
        finally:
            signal.signal(signal.SIGINT, old_int)
            signal.signal(signal.SIGTERM, old_term)


def main(argv=None) -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    rc = ClusterSubmitter().submit(sys.argv[1:] if argv is None else argv)
    return rc


if __name__ == "__main__":
    sys.exit(main() & 0xFF)
