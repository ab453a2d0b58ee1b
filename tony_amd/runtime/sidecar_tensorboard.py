"""Sidecar TensorBoard task (TR/sidecar_tensorboard.py, T/TonyClient.java:571-600).

Runs ``tensorboard --logdir $TB_LOG_DIR --port $TB_PORT``.  With SIDECAR_TB_TEST
set it only sleeps (TonY's test mode).  TensorBoard is not part of this image:
when it cannot be imported, a minimal static HTTP server lists the log dir on
TB_PORT so the advertised URL still answers.
"""
from __future__ import annotations

import functools
import http.server
import os
import shutil
import subprocess
import sys
import time

from .. import constants as C


def main() -> int:
    log_dir = os.environ.get(C.SIDECAR_TB_LOG_DIR, ".")
    port = int(os.environ.get(C.TB_PORT, "6006"))
    if os.environ.get(C.SIDECAR_TB_TEST):
        time.sleep(float(os.environ.get("SIDECAR_TB_TEST_SLEEP_S", "30")))
        return 0
    tb = shutil.which("tensorboard")
    if tb:
        return subprocess.call([tb, "--logdir", log_dir, "--port", str(port), "--bind_all"])
    os.makedirs(log_dir, exist_ok=True)
    handler = functools.partial(http.server.SimpleHTTPRequestHandler, directory=log_dir)
    with http.server.ThreadingHTTPServer(("0.0.0.0", port), handler) as httpd:
        print(f"serving {log_dir} on :{port} (tensorboard not installed)", flush=True)
        httpd.serve_forever()
    return 0


if __name__ == "__main__":
    sys.exit(main())
