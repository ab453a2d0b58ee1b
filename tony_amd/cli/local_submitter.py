"""LocalSubmitter: run a job in "local mode" (tony-cli LocalSubmitter.java:33-71).

TonY starts an in-process MiniYARN cluster; on one node the coordinator already
is the cluster, so local mode = the same submit path with CPU-only tasks and a
fake GPU inventory (``tony.amd.fake-gpus``, default 8) and a private staging dir
-- the plumbing configuration of BASELINE.json ("tony-mini local mode on CPU").
"""
from __future__ import annotations

import logging
import sys
import tempfile

from ..client.tony_client import TonyClient
from ..conf import keys as K
from .cluster_submitter import ClusterSubmitter


def main(argv=None) -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    args = list(sys.argv[1:] if argv is None else argv)
    client = TonyClient()
    c = client.get_tony_conf()
    if c.get_int(K.AMD_FAKE_GPUS, -1) < 0:
        c.set(K.AMD_FAKE_GPUS, "8", "LocalSubmitter")
    if not c.get_trimmed(K.AMD_STAGING_DIR):
        c.set(K.AMD_STAGING_DIR, tempfile.mkdtemp(prefix="tony-local-"), "LocalSubmitter")
    c.set(K.AMD_VISIBLE_DEVICES_MODE, "none", "LocalSubmitter")
    return ClusterSubmitter(client).submit(args)


if __name__ == "__main__":
    sys.exit(main() & 0xFF)
