"""Horovod driver: start the rendezvous server, plan slots, publish them via a port file.

Process contract of TR/horovod_driver.py (and its Java wrapper
T/horovod/HorovodDriver.java): ``python -m tony_amd.horovod.driver -w h1:2,h2:1``
starts the rendezvous server, computes the static slot plan and writes it as
JSON to ``<dir>/<port>____HOROVOD_RENDEZVOUS_SERVER____``; the task agent polls
for that file (5 x 2 s), reports ``DriverCallbackInfo`` to the coordinator and
then waits on the driver until the job ends.  ``-t -p PORT`` is TonY's test mode
(fake 2-slot plan, no server), ``-f`` fails fast in test mode.

``HorovodDriver`` is the agent-side wrapper (spawn, poll, parse, wait); debug
mode runs a user supplied driver command with CLUSTER_WORKER_LIST and
DRIVER_OUTPUT_PATH in its environment instead.
"""
from __future__ import annotations

import argparse
import glob
import json
import logging
import os
import signal
import subprocess
import sys
import tempfile
import time
from typing import Dict, Optional

from .. import constants as C
from . import DriverCallbackInfo, fake_host_plan, host_assignments, parse_hosts, slots_json

LOG = logging.getLogger(__name__)
PORT_FILE_SUFFIX = C.HOROVOD_PORT_FILE_SUFFIX


def port_file_path(directory: str, port) -> str:
    return os.path.join(directory, f"{port}{PORT_FILE_SUFFIX}")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="tony_amd Horovod driver")
    ap.add_argument("-w", "--worker_list", required=True)
    ap.add_argument("-a", "--num_proc", default="1")
    ap.add_argument("-e", dest="elastic", action="store_true")
    ap.add_argument("-t", dest="test_mode", action="store_true")
    ap.add_argument("-p", "--fake_port", default=None)
    ap.add_argument("-f", dest="fast_fail", action="store_true")
    ap.add_argument("-o", "--output_dir", default=os.path.dirname(os.path.abspath(__file__)))
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s horovod-driver: %(message)s")
    if a.elastic:
        LOG.error("elastic Horovod is not supported (TonY's elastic path is a stub as well)")
        return 1
    if a.test_mode:
        if a.fast_fail:
            LOG.error("fast-fail test mode")
            return 1
        port = a.fake_port or "9999"
        plan = fake_host_plan(a.worker_list)
        server = None
    else:
        from .rendezvous import RendezvousServer

        plan = host_assignments(parse_hosts(a.worker_list), 1)
        server = RendezvousServer()
        port = server.start()
        server.init(slots_json(plan))
        LOG.info("Rendezvous server started, port: %s", port)
    path = port_file_path(a.output_dir, port)
    with open(path + ".tmp", "w") as f:
        f.write(slots_json(plan))
    os.replace(path + ".tmp", path)
    LOG.info("Host alloc plan written to %s", path)
    stop = {"flag": False}

    def _term(*_):
        stop["flag"] = True

    signal.signal(signal.SIGTERM, _term)
    signal.signal(signal.SIGINT, _term)
    try:
        while not stop["flag"]:
            time.sleep(0.5)
    finally:
        try:
            os.unlink(path)
        except OSError:
            pass
        if server is not None:
            server.stop()
    return 0


class HorovodDriver:
    """Agent-side handle on a running driver process."""

    POLL_TRIES = 5
    POLL_INTERVAL_S = 2.0

    def __init__(self, proc: subprocess.Popen, port: str, host: str, slot_infos, output_dir: str):
        self.proc = proc
        self.port = port
        self.host = host
        self.slot_infos = slot_infos
        self.output_dir = output_dir

    @classmethod
    def create(cls, worker_list: str, env: Dict[str, str], host: str, test_mode=False, fast_fail=False,
               debug_command: Optional[str] = None, python: Optional[str] = None) -> "HorovodDriver":
        out_dir = tempfile.mkdtemp(prefix="tony-hvd-driver-")
        penv = dict(os.environ)
        penv.update(env)
        if debug_command:
            penv[C.HOROVOD_CLUSTER_WORKER_LIST] = worker_list
            penv[C.HOROVOD_DRIVER_OUTPUT_PATH] = out_dir
            proc = subprocess.Popen(["bash", "-c", debug_command], env=penv, start_new_session=True)
        else:
            cmd = [python or sys.executable, "-m", "tony_amd.horovod.driver", "-w", worker_list, "-o", out_dir]
            if test_mode or fast_fail:
                cmd += ["-t", "-p", "9999"]
            if fast_fail:
                cmd.append("-f")
            proc = subprocess.Popen(cmd, env=penv, start_new_session=True)
        pattern = os.path.join(out_dir, f"*{PORT_FILE_SUFFIX}")
        for _ in range(cls.POLL_TRIES * 20):
            files = glob.glob(pattern)
            if files:
                fn = files[0]
                port = os.path.basename(fn)[: -len(PORT_FILE_SUFFIX)]
                with open(fn) as f:
                    slots = json.load(f)
                return cls(proc, port, host, slots, out_dir)
            if proc.poll() is not None:
                raise RuntimeError(f"Horovod driver exited with {proc.returncode} before publishing its port")
            time.sleep(cls.POLL_INTERVAL_S / 20)
        proc.kill()
        raise TimeoutError("Horovod driver did not publish a port file in time")

    def callback_info(self) -> str:
        return DriverCallbackInfo(str(self.port), self.host, self.slot_infos).to_json()

    def wait_for(self, timeout_s: Optional[float] = None) -> int:
        try:
            return self.proc.wait(timeout=timeout_s)
        except subprocess.TimeoutExpired:
            return -1

    def close(self) -> None:
        if self.proc.poll() is None:
            try:
                os.killpg(self.proc.pid, signal.SIGTERM)
            except OSError:
                pass


if __name__ == "__main__":
    sys.exit(main())
