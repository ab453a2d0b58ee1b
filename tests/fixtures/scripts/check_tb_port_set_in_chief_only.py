import os
import sys
tb = os.environ.get("TB_PORT")
job = os.environ["JOB_NAME"]
print("TB_PORT", tb, "JOB_NAME", job)
sys.exit(1 if tb and job != "chief" else 0)
