"""``python -m tony_amd.portal [--conf tony-site.xml] [--port N]`` == startTonyPortal.sh.

Settings come from tony-default.xml overlaid with ``--conf`` files (or
``$TONY_CONF_DIR/tony-site.xml``): history location / intermediate / finished,
mover and purger intervals, retention, finished-dir timezone, cache size.
"""
from __future__ import annotations

import argparse
import logging
import os
import sys

from ..conf import Configuration
from ..conf import keys as K
from ..events.history import HistoryLayout
from .history import HistoryFileMover, HistoryFilePurger
from .server import CacheWrapper, PortalServer


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="tony-portal")
    ap.add_argument("--conf", action="append", default=[], help="tony-site.xml style overlay (repeatable)")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=19886)
    ap.add_argument("--no-mover", action="store_true")
    ap.add_argument("--no-purger", action="store_true")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    c = Configuration()
    site = os.path.join(os.environ.get("TONY_CONF_DIR", ""), "tony-site.xml")
    if not a.conf and os.environ.get("TONY_CONF_DIR") and os.path.exists(site):
        a.conf.append(site)
    for f in a.conf:
        c.add_resource(f)
    lay = HistoryLayout.from_conf(c)
    for d in (lay.intermediate, lay.finished):
        os.makedirs(d, exist_ok=True)
    cache = CacheWrapper(lay.intermediate, lay.finished, c.get_int(K.PORTAL_CACHE_MAX_ENTRIES, 1000))
    if not a.no_mover:
        HistoryFileMover(lay.intermediate, lay.finished, lay.timezone, on_job_dir=cache.update_caches).start(
            c.get_int(K.HISTORY_MOVER_INTERVAL_MS, 300000))
    if not a.no_purger:
        HistoryFilePurger(lay.intermediate, lay.finished, c.get_int(K.HISTORY_RETENTION_SECONDS, 2592000),
                          lay.timezone).start(c.get_int(K.HISTORY_PURGER_INTERVAL_MS, 21600000))
    srv = PortalServer(cache, a.host, a.port)
    logging.getLogger("tony.portal").info("portal on http://%s:%d (history %s)", a.host, srv.port, lay.location)
    try:
        srv.serve_forever()
    except KeyboardInterrupt:
        pass
    return 0


if __name__ == "__main__":
    sys.exit(main())
