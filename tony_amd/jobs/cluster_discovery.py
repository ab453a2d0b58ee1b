"""Generic cluster discovery from TF_CONFIG (the pattern of EX/ray-on-tony/discovery.py:27-37, where a
``head`` jobtype and ``worker`` jobtypes use the tensorflow runtime only as a cluster-spec carrier).

Prints this task's role and the addresses of every jobtype; ``--write FILE`` stores them as JSON so
a framework that bootstraps itself (Ray, Dask, a custom server) can read its peers.

  tony --src_dir tony_amd/jobs --conf tony.head.instances=1 --conf tony.worker.instances=2 \
       --conf tony.head.command="python cluster_discovery.py" --conf tony.worker.command="python cluster_discovery.py"
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from tony_amd.parallel.tf_config import TFConfig  # noqa: E402


def discover() -> dict:
    tc = TFConfig.from_env()
    return {"role": tc.task_type, "index": tc.task_index, "cluster": tc.cluster,
            "head": (tc.cluster.get("head") or tc.cluster.get("chief") or tc.cluster.get("worker") or [None])[0]}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--write", default=None)
    a = ap.parse_args(argv)
    info = discover()
    print(json.dumps(info, sort_keys=True), flush=True)
    if a.write:
        with open(a.write, "w") as f:
            json.dump(info, f)
    return 0 if info["head"] else 1


if __name__ == "__main__":
    sys.exit(main())
