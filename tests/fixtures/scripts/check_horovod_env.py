import os
import sys
keys = ["HOROVOD_CONTROLLER", "HOROVOD_CPU_OPERATIONS", "HOROVOD_GLOO_TIMEOUT_SECONDS", "HOROVOD_GLOO_RENDEZVOUS_PORT",
        "HOROVOD_GLOO_RENDEZVOUS_ADDR", "HOROVOD_CROSS_RANK", "HOROVOD_CROSS_SIZE", "HOROVOD_LOCAL_RANK",
        "HOROVOD_LOCAL_SIZE", "HOROVOD_SIZE", "HOROVOD_RANK", "HOROVOD_HOSTNAME", "JOB_NAME"]
missing = [k for k in keys if not os.environ.get(k)]
print({k: os.environ.get(k) for k in keys})
sys.exit(1 if missing else 0)
