"""User-supplied Horovod driver for debug mode: publishes a fake 2-slot plan on port 9999."""
import json
import os
import signal
import sys
import time

workers = os.environ["CLUSTER_WORKER_LIST"]
out = os.environ["DRIVER_OUTPUT_PATH"]
host = workers.split(":")[0]
plan = [{"hostname": host, "rank": 0, "localRank": 0, "crossRank": 0, "size": 2, "localSize": 2, "crossSize": 1},
        {"hostname": host, "rank": 1, "localRank": 1, "crossRank": 1, "size": 2, "localSize": 2, "crossSize": 1}]
with open(os.path.join(out, "9999____HOROVOD_RENDEZVOUS_SERVER____"), "w") as f:
    json.dump(plan, f)
signal.signal(signal.SIGTERM, lambda *_: sys.exit(0))
while True:
    time.sleep(0.5)
