import os
import sys
for k in ("RANK", "WORLD", "INIT_METHOD", "MASTER_ADDR", "MASTER_PORT", "WORLD_SIZE", "LOCAL_RANK"):
    if os.environ.get(k) is None:
        print("missing", k)
        sys.exit(1)
sys.exit(0)
