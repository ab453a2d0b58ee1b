"""Touch N MiB of memory (argv[1]) and hold it for argv[2] seconds (memory-limit enforcement test)."""
import sys
import time

mb = int(sys.argv[1]) if len(sys.argv) > 1 else 512
buf = bytearray(mb << 20)
for i in range(0, len(buf), 4096):
    buf[i] = 1
time.sleep(float(sys.argv[2]) if len(sys.argv) > 2 else 30)
