import os
import sys
ids = os.environ.get("TONY_GPU_IDS", "")
print("TONY_GPU_IDS", ids, "NUMA", os.environ.get("TONY_NUMA_NODE"), "HIP", os.environ.get("HIP_VISIBLE_DEVICES"))
want = int(os.environ.get("EXPECT_GPUS", "1"))
sys.exit(0 if len([g for g in ids.split(",") if g]) == want else 1)
