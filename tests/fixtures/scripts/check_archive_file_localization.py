import os
import sys
print(sorted(os.listdir(".")))
for p in ("./common.zip", "./test20.zip", "./test2.zip/123.xml"):
    if not os.path.isfile(p):
        print("missing", p)
        sys.exit(255)
sys.exit(0)
