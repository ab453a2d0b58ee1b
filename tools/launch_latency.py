#!/usr/bin/env python3
"""Job-launch latency (BASELINE.json's second metric): ClusterSubmitter-style submit -> every task
of the gang RUNNING its user command, through the real path (TonyClient -> coordinator process ->
task agents -> gang barrier -> runtime env -> user process).

Reference structure (BASELINE.md "Structural latency constants"): the YARN AM heartbeats the RM every
1 s (ApplicationMaster.java:468), executors poll for the gang every 3 s (TaskExecutor.java:294-296)
and the client polls app status every 1 s (TonyClient.java:1035), so a TonY gang needs several
seconds after its containers are allocated.  Here registration is pushed over gRPC and the gang
release is event driven.

Usage: python tools/launch_latency.py [--workers 8] [--ps 1] [--reps 5] [--gpus]
  --gpus: pin each worker to a real GPU from the amd-smi inventory (GPU box); default: fake
          8-GPU inventory with no device env (runs anywhere).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--ps", type=int, default=1)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--gpus", action="store_true")
    args = ap.parse_args()

    from tony_amd.client.tony_client import TonyClient
    from tony_amd.conf import Configuration
    from tony_amd.conf import keys as K

    scripts = os.path.join(ROOT, "tests", "fixtures", "scripts")
    lat = []
    for _ in range(args.reps):
        with tempfile.TemporaryDirectory() as tmp:
            c = Configuration()
            c.set(K.SECURITY_ENABLED, "false")
            c.set(K.AMD_STAGING_DIR, os.path.join(tmp, "staging"))
            if not args.gpus:
                c.set(K.AMD_FAKE_GPUS, "8")
                c.set(K.AMD_VISIBLE_DEVICES_MODE, "none")
            c.set("tony.amd.stop-grace-sec", "3")
            c.set(K.AMD_CLIENT_POLL_MS, "10")  # the client observes RUNNING at this resolution (default 200 ms)
            c.set(K.AM_WAIT_CLIENT_STOP_TIMEOUT, "5")
            client = TonyClient(c)
            ok = client.init(["--src_dir", scripts, "--python_binary_path", sys.executable,
                              "--executes", "sleep_arg.py 1.0",
                              "--conf", f"tony.worker.instances={args.workers}",
                              "--conf", f"tony.worker.gpus={1 if args.gpus else 0}",
                              "--conf", f"tony.ps.instances={args.ps}"])
            if not ok or client.start() != 0:
                print("launch_latency: job failed", file=sys.stderr)
                return 1
            lat.append(client.launch_latency_s())
    rec = {"metric": "job-launch latency (submit -> all tasks RUNNING)", "unit": "s",
           "tasks": args.workers + args.ps, "gpus_pinned": args.gpus, "reps": args.reps,
           "median": round(statistics.median(lat), 3), "min": round(min(lat), 3), "max": round(max(lat), 3),
           "all": [round(v, 3) for v in lat]}
    print(json.dumps(rec))
    return 0


if __name__ == "__main__":
    sys.exit(main())
