"""Task agent: one per task, the TaskExecutor of TonY (T/TaskExecutor.java:35-452, call stack SURVEY.md §3.3).

Flow: read the env contract (JOB_NAME, TASK_INDEX, TASK_NUM, IS_CHIEF,
DISTRIBUTED_MODE, AM_HOST/AM_PORT, SESSION_ID ...) and tony-final.xml ->
localize resources into the working dir (the NodeManager's job in YARN) and
unpack the src zip / venv -> pin CPUs to the GPU's NUMA node -> connect to the
coordinator, start heartbeats and the metrics monitor -> reserve the task's
port (its ``host:port`` identity) and, if needed, the TensorBoard port ->
register and poll until the gang barrier returns the cluster spec -> release
the ports (unless TF_GRPC_REUSE_PORT / TB_SERVER_REUSE_PORT) -> run the
runtime adapter (env contract + user command) -> report the exit code -> exit
with it.  Test hooks: TEST_TASK_EXECUTOR_NUM_HB_MISS, TEST_TASK_EXECUTOR_SKEW.
"""
from __future__ import annotations

import logging
import os
import shlex
import shutil
import signal
import sys
import threading
import time
from typing import Dict, List, Optional

from .. import constants as C
from .. import native
from ..conf import Configuration
from ..conf import keys as K
from ..rpc.client import RpcClient
from ..runtime.base import get_runtime
from ..utils import core as U
from ..utils.resources import localize_all
from .monitor import TaskMonitor

LOG = logging.getLogger("tony.executor")
MAX_NUM_FAILED_HB_ATTEMPTS = 5
USER_PGID_FILE = "user.pgid"
_SHELL_META = set("|&;<>()$`\\\"'*?[]#~=%{}\n")


class TaskExecutor:
    def __init__(self, env: Optional[Dict[str, str]] = None):
        env = dict(os.environ if env is None else env)
        self.env = env
        self.job_name = env[C.JOB_NAME]
        self.task_index = int(env[C.TASK_INDEX])
        self.num_tasks = int(env[C.TASK_NUM])
        self.task_id = f"{self.job_name}:{self.task_index}"
        self.is_chief = env.get(C.IS_CHIEF, "false").lower() == "true"
        self.distributed_mode = env.get(C.DISTRIBUTED_MODE_NAME, C.DistributedMode.GANG).upper()
        self.app_id = env.get(C.APPID, "")
        self.session_id = env.get(C.SESSION_ID, "0")
        self.am_host = env[C.AM_HOST]
        self.am_port = int(env[C.AM_PORT])
        self.host = U.current_host()
        self.conf = Configuration(load_defaults=False)
        self.conf.add_resource(env.get(C.TONY_CONF_PATH, C.TONY_FINAL_XML), C.TONY_FINAL_XML)
        self.timeout_ms = self.conf.get_int(K.timeout_key(self.job_name),
                                            self.conf.get_int(K.WORKER_TIMEOUT, 0))
        self.hb_interval_ms = self.conf.get_int(K.TASK_HEARTBEAT_INTERVAL_MS, 1000)
        self.poll_s = self.conf.get_int(K.AMD_REGISTRATION_POLL_MS, 100) / 1000.0
        self.shell_env: Dict[str, str] = U.parse_key_value(self.conf.get_strings(K.EXECUTION_ENV))
        self.task_command = self.conf.get(K.execute_command_key(self.job_name), self.conf.get(K.CONTAINERS_COMMAND))
        if not self.task_command:
            raise ValueError("Task command is empty. Please set tony.[jobtype].command or pass --executes")
        self.framework = self.conf.get(K.FRAMEWORK_NAME, "tensorflow")
        self.gpu_ids: List[int] = [int(g) for g in env.get(C.TONY_GPU_IDS, "").split(",") if g.strip()]
        self.cluster_spec: Optional[str] = None
        token = None
        tok_file = env.get(C.TONY_TOKEN_FILE)
        if tok_file and os.path.exists(tok_file):
            with open(tok_file) as f:
                token = f.read().strip()
        self.client = RpcClient.get_instance(self.am_host, self.am_port, token)
        self.rpc_port: Optional[native.PortReservation] = None
        self.tb_port: Optional[native.PortReservation] = None
        self.user_proc: Optional[U.ShellProcess] = None
        self._hb_stop = threading.Event()
        self.monitor: Optional[TaskMonitor] = None
        self.adapter = get_runtime(self.framework).task_adapter(self)

    # -- setup ---------------------------------------------------------------------------
    def localize(self, cwd: str = ".") -> None:
        specs = self.conf.get_strings(K.CONTAINERS_RESOURCES) + self.conf.get_strings(K.resources_key(self.job_name))
        localize_all(specs, cwd)
        staging = self.env.get(C.TONY_JOB_DIR)
        if staging:
            U.link_job_archives(staging, self.app_id, cwd)
        U.extract_resources(self.app_id, cwd)

    def pin_cpus(self) -> None:
        cpus = self.env.get("TONY_CPUS")
        if not cpus:
            return
        try:
            os.sched_setaffinity(0, {int(c) for c in cpus.split(",")})
        except (OSError, ValueError):
            LOG.warning("could not bind to CPUs %s", cpus)

    def _reuse(self, var: str) -> bool:
        return self.shell_env.get(var, os.environ.get(var, "false")).lower() == "true"

    def setup_ports(self) -> None:
        self.rpc_port = native.PortReservation(0, reuse_port=self._reuse("TF_GRPC_REUSE_PORT"))
        if self.adapter.need_reserve_tb_port():
            self.tb_port = native.PortReservation(0, reuse_port=self._reuse("TB_SERVER_REUSE_PORT"))
            url = f"{self.host}:{self.tb_port.port}"
            U.poll_till_non_null(lambda: self.client.register_tensorboard_url(url), 1, 60)
            self.shell_env[C.TB_PORT] = str(self.tb_port.port)

    # -- heartbeats ------------------------------------------------------------------------
    def _heartbeat_loop(self) -> None:
        try:
            to_miss = max(0, int(os.environ.get(C.TEST_TASK_EXECUTOR_NUM_HB_MISS, "0")))
        except ValueError:
            to_miss = 0
        miss_counter = 0
        failures = 0
        while not self._hb_stop.wait(self.hb_interval_ms / 1000.0):
            if miss_counter > 0:
                miss_counter -= 1  # skipping for testing
                continue
            try:
                self.client.task_executor_heartbeat(self.task_id)
                failures = 0
                miss_counter = to_miss
            except Exception:  # noqa: BLE001
                failures += 1
                if failures > MAX_NUM_FAILED_HB_ATTEMPTS:
                    LOG.error("[%s] too many failed heartbeats, stopping heartbeats", self.task_id)
                    return

    def register_and_get_cluster_spec(self) -> Optional[str]:
        threading.Thread(target=self._heartbeat_loop, name="tony-heartbeat", daemon=True).start()
        spec = f"{self.host}:{self.rpc_port.port}"
        return U.poll_till_non_null(lambda: self.client.register_worker_spec(self.task_id, spec), self.poll_s, 0)

    def callback_info_to_am(self, task_id: str, info: str) -> None:
        self.client.register_callback_info(task_id, info)

    # -- user process --------------------------------------------------------------------------
    def _command(self) -> str:
        cmd = self.task_command
        if self.conf.get_bool(K.AMD_PROFILE, False) and \
                self.job_name in self.conf.get_strings(K.AMD_PROFILE_JOBTYPES, ["worker", "chief"]):
            out = os.path.join(self.env.get(C.TONY_JOB_DIR, "."), "profiles", f"{self.job_name}_{self.task_index}")
            os.makedirs(out, exist_ok=True)
            if set(cmd) & _SHELL_META:
                LOG.warning("not profiling a shell pipeline: %s", cmd)
            else:
                # the profiled program itself must follow "--" (no bash -c hop)
                cmd = f"rocprofv3 --kernel-trace --stats -d {shlex.quote(out)} -- {cmd}"
        return cmd

    def run_user_command(self) -> int:
        env = dict(os.environ)
        env.update(self.shell_env)
        from ..utils.docker import wrap_if_enabled

        cmd = wrap_if_enabled(self._command(), env, os.getcwd())
        self.user_proc = U.ShellProcess(cmd, env=env, die_with_parent=True)
        try:  # the coordinator kills this group too when it stops the task
            with open(USER_PGID_FILE, "w") as f:
                f.write(str(self.user_proc.pid))
        except OSError:
            pass
        timeout = self.timeout_ms / 1000.0 if self.timeout_ms > 0 else None
        rc = self.user_proc.wait(timeout)
        return rc if rc >= 0 else 128 - rc

    def _skew_and_hang_if_testing(self) -> None:
        instr = os.environ.get(C.TEST_TASK_EXECUTOR_SKEW)
        if not instr:
            return
        parts = instr.split("#")
        try:
            if len(parts) == 3 and parts[0] == self.job_name and int(parts[1]) == self.task_index:
                time.sleep(int(parts[2]) / 1000.0)
        except ValueError:
            LOG.error("bad skew instruction %s", instr)

    def release_port(self, port: Optional[native.PortReservation]) -> None:
        if port is not None:
            port.release()

    def _on_fault(self, message: str) -> None:
        """A GPU fault (new uncorrectable ECC errors) or a memory-limit breach: stop the user process
        (its exit is then reported with the fault's exit status and diagnostic)."""
        if "GPU fault" in message and not self.conf.get_bool(K.AMD_GPU_FAULT_STOPS_TASK, True):
            return
        LOG.error("[%s] stopping the task: %s", self.task_id, message)
        if self.user_proc is not None:
            self.user_proc.kill(signal.SIGKILL)

    # -- main ------------------------------------------------------------------------------------
    def run(self) -> int:
        self.localize(".")
        self.pin_cpus()
        self.setup_ports()
        mem_limit = 0
        if self.conf.get_bool(K.AMD_MEMORY_ENFORCED, True):
            mem_limit = U.parse_memory_string(self.conf.get(K.resource_key(self.job_name, C.MEMORY),
                                                            K.DEFAULT_MEMORY)) * 2 ** 20
        self.monitor = TaskMonitor(lambda: self.user_proc.pid if self.user_proc else os.getpid(), self.gpu_ids,
                                   self.conf.get_int(K.TASK_METRICS_UPDATE_INTERVAL_MS, 5000),
                                   lambda m: self.client.update_metrics(self.job_name, self.task_index, m),
                                   self.conf.get_bool(K.TASK_GPU_METRICS_ENABLED, True),
                                   on_fault=self._on_fault, memory_limit_bytes=mem_limit)
        self.monitor.start()
        self.cluster_spec = self.register_and_get_cluster_spec()
        LOG.info("[%s] got cluster spec: %s", self.task_id, self.cluster_spec)
        if not self._reuse("TF_GRPC_REUSE_PORT"):
            self.release_port(self.rpc_port)
        if not self._reuse("TB_SERVER_REUSE_PORT"):
            self.release_port(self.tb_port)
        try:
            exit_code = self.adapter.run()
            if self.monitor.fault is not None and exit_code != 0:
                exit_code = self.monitor.fault_code  # stopped by the agent: report why, not the signal
            self._skew_and_hang_if_testing()
            U.poll_till_non_null(lambda: self.client.register_execution_result(
                exit_code, self.job_name, str(self.task_index), self.session_id), 1, 60)
        finally:
            self.release_port(self.rpc_port)
            self.release_port(self.tb_port)
            self._hb_stop.set()
            if self.monitor is not None:
                self.monitor.stop()
        return exit_code


def main() -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s",
                        stream=sys.stderr)
    ex = TaskExecutor()

    def _term(signum, _frame):
        if ex.user_proc is not None:
            ex.user_proc.kill(signal.SIGTERM)
        sys.exit(128 + signum)

    signal.signal(signal.SIGTERM, _term)
    rc = ex.run()
    LOG.info("[%s] user process exited with %d", ex.task_id, rc)
    return rc


if __name__ == "__main__":
    sys.exit(main())
