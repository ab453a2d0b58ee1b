"""Writes this task's GPU pinning env to $RECORD_DIR/<job>_<index>.txt (ps / worker placement tests)."""
import os

d = os.environ["RECORD_DIR"]
keys = ("TONY_GPU_IDS", "TONY_HIP_ORDINALS", "TONY_VISIBLE_MODE", "HIP_VISIBLE_DEVICES", "TONY_PS_SHARED_GPU",
        "TONY_PS_GPUS")
with open(os.path.join(d, f"{os.environ['JOB_NAME']}_{os.environ['TASK_INDEX']}.txt"), "w") as f:
    for k in keys:
        f.write(f"{k}={os.environ.get(k, '')}\n")
