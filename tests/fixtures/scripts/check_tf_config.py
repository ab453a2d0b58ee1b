import json
import os
import sys
cfg = json.loads(os.environ["TF_CONFIG"])
spec = json.loads(os.environ["CLUSTER_SPEC"])
assert cfg["task"]["type"] == os.environ["JOB_NAME"]
assert cfg["task"]["index"] == int(os.environ["TASK_INDEX"])
assert "tensorboard" not in cfg["cluster"]
for job, hosts in spec.items():
    assert all(":" in h and not h.endswith(":0") for h in hosts), spec
print("TF_CONFIG", cfg)
sys.exit(0)
