import sys
import time
time.sleep(float(sys.argv[1]) if len(sys.argv) > 1 else 3.0)
