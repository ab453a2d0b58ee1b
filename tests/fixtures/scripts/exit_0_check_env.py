import os
import sys
ok = os.environ.get("ENV_CHECK") == "ENV_CHECK"
print("ENV_CHECK ok" if ok else "ENV_CHECK missing")
sys.exit(0 if ok else 1)
