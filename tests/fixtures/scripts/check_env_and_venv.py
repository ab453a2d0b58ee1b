import os
import sys
if not os.path.isfile("venv/123.xml"):
    print("venv/123.xml missing")
    sys.exit(255)
sys.exit(0 if os.environ.get("ENV_CHECK") == "ENV_CHECK" else 1)
