"""TonyClient: submit a job to the node's coordinator and follow it to completion.

Behavioural parity with T/TonyClient.java:114-1416 (call stack SURVEY.md §3.1):

* options (TonyClient.java:425-436 + Utils.getCommonOptions): -executes,
  -task_params, -shell_env k=v (repeatable), -container_env k=v, -conf k=v,
  -conf_file, -src_dir, -sidecar_tensorboard_log_dir, -hdfs_classpath,
  -python_binary_path, -python_venv, -help; ``-x v``, ``--x v`` and ``--x=v`` all parse;
* configuration layering: tony-default.xml -> (--conf_file | ./tony.xml) ->
  --conf overrides (multi-value keys append) -> $TONY_CONF_DIR/tony-site.xml,
  with Hadoop precedence (programmatic values beat every file, ``final`` wins);
* validation: per-job max instances, tony.task.max-total-instances,
  tony.task.max-total-<resource> (GPUs bounded by the node's GPU count);
* staging (HDFS in TonY, a per-job dir here): src dir zip, venv, resources,
  tony-final.xml; the coordinator is started as a child process (the RM launching
  the AM) and watched over RPC; task tables are logged when they change,
  listeners are notified, the app is killed on ``tony.application.timeout`` and
  the coordinator is told to finish.  Exit code 0 on success, -1 otherwise.
"""
from __future__ import annotations

import json
import logging
import os
import shutil
import signal
import subprocess
import sys
import threading
import time
from typing import Dict, List, Optional, Set

from .. import constants as C
from ..cluster.session import TaskInfo, TaskStatus
from ..conf import Configuration
from ..conf import keys as K
from ..gpu.inventory import discover
from ..rpc.client import RpcClient
from ..utils import core as U
from ..utils.resources import LocalizableResource

LOG = logging.getLogger("tony.client")

OPTIONS_WITH_VALUE = ("executes", "task_params", "shell_env", "container_env", "conf", "conf_file", "src_dir",
                      "sidecar_tensorboard_log_dir", "hdfs_classpath", "python_binary_path", "python_venv")
REPEATABLE = ("shell_env", "container_env", "conf")
FLAGS = ("help",)


class ClientOptionError(ValueError):
    pass


def parse_args(args: List[str]) -> Dict[str, object]:
    """Commons-CLI GnuParser-alike: ``-x v``, ``--x v``, ``--x=v``; stops at the first non-option."""
    out: Dict[str, object] = {k: [] for k in REPEATABLE}
    i = 0
    while i < len(args):
        a = args[i]
        if not a.startswith("-") or a in ("-", "--"):
            out.setdefault("_rest", []).extend(args[i + (1 if a == "--" else 0):])
            break
        name = a.lstrip("-")
        val = None
        if "=" in name:
            name, val = name.split("=", 1)
        if name in FLAGS:
            out[name] = True
            i += 1
            continue
        if name not in OPTIONS_WITH_VALUE:
            raise ClientOptionError(f"Unrecognized option: {a}")
        if val is None:
            if i + 1 >= len(args):
                raise ClientOptionError(f"Missing argument for option: {name}")
            val = args[i + 1]
            i += 2
        else:
            i += 1
        if name in REPEATABLE:
            out[name].append(val)
        else:
            out[name] = val
    return out


def usage() -> str:
    lines = ["usage: TonyClient"]
    for o in OPTIONS_WITH_VALUE + FLAGS:
        lines.append(f"  -{o}{' <arg>' if o in OPTIONS_WITH_VALUE else ''}")
    return "\n".join(lines)


def build_task_command(python_venv: Optional[str], python_binary: Optional[str], executes: Optional[str],
                       task_params: Optional[str]) -> Optional[str]:
    if executes is None:
        return None
    cmd = executes
    if python_binary is not None:
        interp = python_binary if python_binary.startswith("/") or python_venv is None else \
            f"{C.PYTHON_VENV_DIR}/{python_binary}"
        cmd = f"{interp} {executes}"
    if task_params is not None:
        cmd += f" {task_params}"
    return cmd


def merge_tasks(tasks: List[TaskInfo]) -> str:
    """"ps [0, 1] worker [0] " grouping of consecutive same-name tasks (TonyClient.mergeTasks)."""
    out = []
    group: List[str] = []
    for i, t in enumerate(tasks):
        group.append(t.index)
        if i == len(tasks) - 1 or t.name != tasks[i + 1].name:
            out.append(f"{t.name} [{', '.join(group)}] ")
            group = []
    return "".join(out)


STATUS_SORTED_BY_ATTENTION = (TaskStatus.FAILED, TaskStatus.SUCCEEDED, TaskStatus.FINISHED, TaskStatus.RUNNING,
                              TaskStatus.NEW, TaskStatus.READY)


def _task_order(t: TaskInfo):
    return (t.name, int(t.index) if str(t.index).isdigit() else 0)


class TonyClient:
    def __init__(self, conf: Optional[Configuration] = None):
        self.tony_conf = conf if conf is not None else Configuration()
        self.listeners = []
        self.callback_handler = None
        self.app_id: Optional[str] = None
        self.job_dir: Optional[str] = None
        self.task_infos: Set[TaskInfo] = set()
        self._task_snapshot = None
        self.coordinator_proc: Optional[subprocess.Popen] = None
        self.rpc: Optional[RpcClient] = None
        self.src_dir: Optional[str] = None
        self.python_venv: Optional[str] = None
        self.final_status: Optional[str] = None
        self.diagnostics: str = ""
        self.launch_ms = None
        self.all_running_ms = None
        self.finished = threading.Event()

    # -- listeners (T/client/CallbackHandler.java, TaskUpdateListener.java) --------------
    def add_listener(self, listener) -> None:
        self.listeners.append(listener)

    def remove_listener(self, listener) -> None:
        self.listeners.remove(listener)

    def get_tony_conf(self) -> Configuration:
        return self.tony_conf

    # -- init -----------------------------------------------------------------------------
    def init(self, args: List[str]) -> bool:
        try:
            opts = parse_args(list(args))
        except ClientOptionError as e:
            LOG.error("%s\n%s", e, usage())
            return False
        if opts.get("help"):
            print(usage())
            return False
        self.init_tony_conf(self.tony_conf, opts)
        if not self.validate_tony_conf(self.tony_conf):
            return False
        c = self.tony_conf
        self.src_dir = opts.get("src_dir")
        self.python_venv = opts.get("python_venv")
        python_binary = opts.get("python_binary_path")
        cmd = build_task_command(self.python_venv, python_binary, opts.get("executes"), opts.get("task_params"))
        if cmd is not None:
            c.set(K.CONTAINERS_COMMAND, cmd, "--executes")
        if python_binary:
            c.set(K.PYTHON_EXEC_PATH, build_task_command(self.python_venv, python_binary, "", None).strip()
                  if self.python_venv and not python_binary.startswith("/") else python_binary)
        for e in opts["shell_env"]:
            U.append_conf_resources(K.EXECUTION_ENV, e, c)
        for e in opts["container_env"]:
            U.append_conf_resources(K.CONTAINER_LAUNCH_ENV, e, c)
        hdfs_cp = opts.get("hdfs_classpath")
        if hdfs_cp:
            for p in hdfs_cp.split(","):
                U.append_conf_resources(K.CONTAINERS_RESOURCES, p, c)
        tb_dir = opts.get("sidecar_tensorboard_log_dir") or c.get_trimmed(K.TENSORBOARD_LOG_DIR)
        if tb_dir:
            self.set_sidecar_tb_resources(tb_dir)
        return True

    def init_tony_conf(self, conf: Configuration, opts) -> None:
        conf_file = opts.get("conf_file")
        if conf_file:
            conf.add_resource(conf_file, os.path.basename(conf_file))
        elif os.path.exists(C.TONY_XML):
            conf.add_resource(C.TONY_XML, C.TONY_XML)
        for k, v in U.parse_key_value(opts.get("conf", [])).items():
            if k in K.MULTI_VALUE_CONF and conf.get(k) is not None:
                U.append_conf_resources(k, v, conf)
            else:
                conf.set(k, v, "--conf")
        site = os.path.join(os.environ.get(C.TONY_CONF_DIR, C.DEFAULT_TONY_CONF_DIR), C.TONY_SITE_CONF)
        if os.path.exists(site):
            conf.add_resource(site, C.TONY_SITE_CONF)
        from .. import version

        version.inject(conf)

    def validate_tony_conf(self, conf: Configuration) -> bool:
        U.size_gpu_task_memory(conf)
        try:
            requests = U.parse_container_requests(conf)
        except (ValueError, RuntimeError) as e:
            LOG.error("%s", e)
            return False
        total = 0
        for job, req in requests.items():
            mx = conf.get_int(K.max_instances_key(job), -1)
            if 0 <= mx < req.num_instances:
                LOG.error("Job type %s requests %d instances, limit is %d", job, req.num_instances, mx)
                return False
            total += req.num_instances
        mx_total = conf.get_int(K.MAX_TOTAL_INSTANCES, -1)
        if 0 <= mx_total < total:
            LOG.error("Job requests %d instances, tony.task.max-total-instances is %d", total, mx_total)
            return False
        for key in conf.keys():
            m = K.MAX_TOTAL_RESOURCES_REGEX.match(key)
            if not m or m.group(1) == "instances":
                continue
            res = m.group(1)
            # TonyClient.enforceResourceLimits (TonyClient.java:824-857): memory in MB ("2g" = 2048)
            limit = U.parse_memory_string(conf.get(key)) if res == C.MEMORY else conf.get_int(key, -1)
            want = 0
            for j, r in requests.items():
                v = conf.get(K.resource_key(j, res))
                if v is not None:
                    want += (U.parse_memory_string(v) if res == C.MEMORY else int(v)) * r.num_instances
            if 0 <= limit < want:
                LOG.error("Job requests %d %s, %s is %d", want, res, key, limit)
                return False
        gpus_wanted = max([r.gpus for r in requests.values()] + [0])
        if gpus_wanted > 0:
            node = len(discover(conf.get_int(K.AMD_FAKE_GPUS, -1)))
            if gpus_wanted > node:
                LOG.error("A task asks for %d GPUs but this node has %d", gpus_wanted, node)
                return False
            total_gpus = sum(r.gpus * r.num_instances for r in requests.values())
            if total_gpus > node:
                LOG.warning("tasks ask for %d GPUs in total, node has %d: DAG stages / finishing tasks must "
                            "free GPUs for the rest to start", total_gpus, node)
        return True

    def set_sidecar_tb_resources(self, tb_log_dir: str) -> None:
        c = self.tony_conf
        role = C.SIDECAR_TB_ROLE_NAME
        c.set(K.instances_key(role), "1")
        c.set(K.resource_key(role, C.VCORES), "2")
        c.set(K.resource_key(role, C.MEMORY), "2g")
        c.set(K.resource_key(role, C.GPUS), "0")
        c.set(K.TENSORBOARD_LOG_DIR, tb_log_dir)
        side = c.get_strings(K.SIDECAR_JOBTYPES, [role])
        if role not in side:
            side.append(role)
        c.set_strings(K.SIDECAR_JOBTYPES, side)
        c.set(K.execute_command_key(role), f"{sys.executable} -m tony_amd.runtime.sidecar_tensorboard")
        U.append_conf_resources(K.EXECUTION_ENV, f"{C.SIDECAR_TB_LOG_DIR}={tb_log_dir}", c)

    # -- staging ----------------------------------------------------------------------------
    def _staging_root(self) -> str:
        root = self.tony_conf.get_trimmed(K.AMD_STAGING_DIR) or os.path.join(os.path.expanduser("~"), C.TONY_FOLDER)
        os.makedirs(root, exist_ok=True)
        return root

    def _new_app_id(self, root: str) -> str:
        ts = int(time.time() * 1000)
        seq_file = os.path.join(root, ".seq")
        import fcntl

        with open(seq_file, "a+") as f:
            fcntl.flock(f, fcntl.LOCK_EX)
            f.seek(0)
            try:
                seq = int(f.read().strip() or "0") + 1
            except ValueError:
                seq = 1
            f.seek(0)
            f.truncate()
            f.write(str(seq))
        return f"application_{ts}_{seq:04d}"

    def process_final_tony_conf(self) -> str:
        c = self.tony_conf
        if self.src_dir:
            zip_path = os.path.join(self.job_dir, U.tony_src_zip_name(self.app_id))
            U.zip_folder(self.src_dir, zip_path)
            jobs = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "jobs")
            if os.path.realpath(self.src_dir) == os.path.realpath(jobs):
                c.set(K.AMD_SRC_IS_TONY_JOBS, "true")
        if self.python_venv:
            shutil.copy2(self.python_venv, os.path.join(self.job_dir, C.PYTHON_VENV_ZIP))
        self.process_tony_conf_resources(c)
        final = os.path.join(self.job_dir, C.TONY_FINAL_XML)
        c.write_xml(final)
        shutil.copy2(final, os.path.join(self.job_dir, U.client_resource_name(self.app_id, C.TONY_FINAL_XML)))
        return final

    def process_tony_conf_resources(self, c: Configuration) -> None:
        """Stage local resources into the job dir; directories are zipped as ``#archive``."""
        res_dir = os.path.join(self.job_dir, "resources")
        keys = [k for k in c.keys() if K.RESOURCES_REGEX.match(k)] + [K.CONTAINERS_RESOURCES]
        for key in sorted(set(keys)):
            entries = c.get_strings(key)
            if not entries:
                continue
            staged = []
            for spec in entries:
                r = LocalizableResource.parse(spec)
                os.makedirs(res_dir, exist_ok=True)
                if r.is_directory:
                    zip_path = os.path.join(res_dir, os.path.basename(r.source.rstrip("/")) + ".zip")
                    U.zip_folder(r.source, zip_path)
                    staged.append(zip_path + C.ARCHIVE_SUFFIX)
                    continue
                dst = os.path.join(res_dir, os.path.basename(r.source))
                if not os.path.exists(dst):
                    try:
                        os.link(r.source, dst)
                    except OSError:
                        shutil.copy2(r.source, dst)
                s = dst
                if r.localized_name != os.path.basename(r.source):
                    s += C.RESOURCE_DIVIDER + r.localized_name
                if r.is_archive:
                    s += C.ARCHIVE_SUFFIX
                staged.append(s)
            c.set_strings(key, staged)

    # -- run ------------------------------------------------------------------------------------
    def start(self) -> int:
        try:
            ok = self.run()
        except KeyboardInterrupt:
            self.force_kill_application()
            ok = False
        except Exception:  # noqa: BLE001
            LOG.exception("Failed to run TonyClient")
            self.force_kill_application()
            ok = False
        return 0 if ok else -1

    def run(self) -> bool:
        root = self._staging_root()
        self.app_id = self._new_app_id(root)
        self.job_dir = os.path.join(root, self.app_id)
        os.makedirs(os.path.join(self.job_dir, "logs"), exist_ok=True)
        if self.callback_handler is not None:
            self.callback_handler.on_application_id_received(self.app_id)
        final = self.process_final_tony_conf()
        self.launch_ms = time.time()
        self.submit_application(final)
        return self.monitor_application()

    def submit_application(self, final_conf: str) -> None:
        env = dict(os.environ)
        pkg_root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["PYTHONPATH"] = pkg_root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        # the coordinator runs with the container env too (TonY: the AM container's launch context)
        env.update(U.parse_key_value(self.tony_conf.get_strings(K.CONTAINER_LAUNCH_ENV)))
        logs = os.path.join(self.job_dir, "logs")
        out = open(os.path.join(logs, C.AM_STDOUT_FILENAME), "ab")
        err = open(os.path.join(logs, C.AM_STDERR_FILENAME), "ab")
        cmd = [sys.executable, "-m", "tony_amd.cluster.coordinator", "--conf", final_conf, "--job-dir", self.job_dir,
               "--app-id", self.app_id, "--started", str(int(self.launch_ms * 1000))]
        self.coordinator_proc = subprocess.Popen(cmd, env=env, stdout=out, stderr=err, stdin=subprocess.DEVNULL,
                                                 start_new_session=True)
        out.close()
        err.close()
        LOG.info("Submitted application %s (coordinator pid %d, job dir %s)", self.app_id, self.coordinator_proc.pid,
                 self.job_dir)

    def _connect(self) -> bool:
        if self.rpc is not None:
            return True
        ep = os.path.join(self.job_dir, "coordinator.json")
        if not os.path.exists(ep):
            return False
        with open(ep) as f:
            info = json.load(f)
        token = None
        tok = os.path.join(self.job_dir, "token")
        if os.path.exists(tok):
            with open(tok) as f:
                token = f.read().strip()
        self.rpc = RpcClient(info["host"], info["port"], token, retries=2, retry_sleep_s=0.2)
        LOG.info("Coordinator RPC at %s:%s, logs in %s/logs", info["host"], info["port"], self.job_dir)
        return True

    def update_task_info_and_return(self) -> bool:
        if self.rpc is None:
            return False
        try:
            infos = self.rpc.get_task_infos(retries=0)
        except Exception:  # noqa: BLE001
            return False
        snap = sorted((t.name, t.index, int(t.status)) for t in infos)
        changed = snap != self._task_snapshot
        if changed:
            self._task_snapshot = snap
            self.task_infos = set(infos)
            for lst in self.listeners:
                try:
                    lst.on_task_infos_updated(set(infos))
                except Exception:  # noqa: BLE001
                    LOG.exception("listener failed")
            if infos and self.all_running_ms is None and all(
                    t.status in (TaskStatus.RUNNING, TaskStatus.SUCCEEDED) for t in infos):
                self.all_running_ms = time.time()
        return changed

    def log_simplified_task_info(self) -> None:
        tasks = sorted(self.task_infos, key=_task_order)
        for st in STATUS_SORTED_BY_ATTENTION:
            sel = [t for t in tasks if t.status == st]
            if sel:
                LOG.info("%s: %s", st.name, merge_tasks(sel))

    def log_task_info(self) -> None:
        for t in sorted(self.task_infos, key=TaskInfo.sort_key):
            LOG.info("%s, %s, %s, %s", t.status.name, t.name, t.index, t.url)

    def monitor_application(self) -> bool:
        c = self.tony_conf
        poll_s = c.get_int(K.AMD_CLIENT_POLL_MS, 200) / 1000.0
        timeout_ms = c.get_int(K.APPLICATION_TIMEOUT, 0)
        deadline = time.monotonic() + timeout_ms / 1000.0 if timeout_ms > 0 else float("inf")
        status = None
        while True:
            time.sleep(poll_s)
            self._connect()
            if self.update_task_info_and_return():
                self.log_simplified_task_info()
            if self.rpc is not None:
                try:
                    status = self.rpc.get_application_status(retries=0)
                except Exception:  # noqa: BLE001
                    pass
            if status is not None and status["state"] == "FINISHED":
                self.final_status = status["finalStatus"]
                self.diagnostics = status["diagnostics"]
                self.update_task_info_and_return()
                self.log_task_info()
                LOG.info("Application %s finished: %s %s", self.app_id, self.final_status,
                         f"({self.diagnostics})" if self.diagnostics else "")
                self.signal_coordinator_to_finish()
                self._wait_coordinator(30)
                self.finished.set()
                return self.final_status == "SUCCEEDED"
            rc = self.coordinator_proc.poll()
            if rc is not None:
                self.final_status = "KILLED" if rc < 0 else "FAILED"
                self.diagnostics = f"coordinator exited with {rc} before finishing"
                LOG.error("Application %s: %s", self.app_id, self.diagnostics)
                self._kill_leftover_tasks()
                self.finished.set()
                return False
            if time.monotonic() > deadline:
                LOG.error("Application %s timed out after %d ms, killing it", self.app_id, timeout_ms)
                self.force_kill_application()
                self.final_status = "KILLED"
                self.finished.set()
                return False

    def signal_coordinator_to_finish(self) -> None:
        if self.rpc is not None:
            try:
                self.rpc.finish_application(retries=1)
            except Exception:  # noqa: BLE001
                pass

    def _wait_coordinator(self, timeout_s: float) -> None:
        try:
            self.coordinator_proc.wait(timeout=timeout_s)
        except subprocess.TimeoutExpired:
            self.coordinator_proc.kill()
        if self.rpc is not None:
            self.rpc.close()
            self.rpc = None

    def _kill_leftover_tasks(self) -> None:
        for t in self.task_infos:
            if t.pid:
                try:
                    os.killpg(t.pid, signal.SIGKILL)
                except OSError:
                    pass

    def force_kill_application(self) -> None:
        p = self.coordinator_proc
        if p is None or p.poll() is not None:
            return
        LOG.info("Killing application %s", self.app_id)
        try:
            os.killpg(p.pid, signal.SIGTERM)
            p.wait(timeout=20)
        except (OSError, subprocess.TimeoutExpired):
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except OSError:
                pass
        self._kill_leftover_tasks()

    def launch_latency_s(self) -> Optional[float]:
        """Submit -> every task RUNNING (the BASELINE job-launch latency metric)."""
        if self.launch_ms is None or self.all_running_ms is None:
            return None
        return self.all_running_ms - self.launch_ms


def main(argv=None) -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    client = TonyClient()
    if not client.init(sys.argv[1:] if argv is None else argv):
        return -1
    return client.start()


if __name__ == "__main__":
    sys.exit(main() & 0xFF)
