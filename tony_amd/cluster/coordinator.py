"""The coordinator: a single-node gang scheduler standing in for TonY's ApplicationMaster.

Lifecycle parity with T/ApplicationMaster.java:95-1347 (call stack in SURVEY.md §3.2):

init      read tony-final.xml, timeouts, retry count, single-node detection,
          distributed mode, runtime adapter (``validate_and_update_config`` may
          inject job types, e.g. Horovod's ``driver``)
prepare   RPC server (ApplicationRpc + metrics) on loopback, per-job token,
          GPU inventory + allocator, heartbeat monitor, history writer
sessions  for each attempt (``tony.am.retry-count`` + 1): APPLICATION_INITED,
          preprocess / single-node job, TonySession, DAG scheduler; "container
          allocation" = GPU/NUMA slot reservation + posix_spawn of a task agent in
          its own session; monitor loop until training finishes, the client says
          stop, the app times out, a heartbeat expires, an untracked task fails,
          registration times out or a task dies before registering
stop      stop remaining tasks (SIGTERM, grace, SIGKILL -> FINISHED), wait for
          the client's finish signal, APPLICATION_FINISHED, rename the jhist,
          move the job's history to finished/yyyy/MM/dd

Fault-injection hooks of the reference are honoured: TEST_AM_CRASH,
TEST_AM_THROW_EXCEPTION_CRASH, TEST_WORKER_TERMINATION,
TEST_TASK_COMPLETION_NOTIFICATION_DELAYED.
"""
from __future__ import annotations

import argparse
import getpass
import json
import logging
import os
import re
import secrets
import shutil
import signal
import socket
import sys
import threading
import time
from typing import Dict, List, Optional

from .. import constants as C
from .. import native
from ..conf import Configuration
from ..conf import keys as K
from ..events import schema as EV
from ..events.handler import EventHandler
from ..events.history import HistoryLayout, JobMetadata, year_month_day_dir
from ..portal.history import write_owner
from ..gpu.inventory import GpuAllocator, discover, hip_ordinals
from ..rpc import protocol as P
from ..rpc.server import RpcServer
from ..runtime.base import get_runtime
from ..utils import core as U
from .liveliness import HeartbeatMonitor
from .scheduler import TaskScheduler
from .session import KILLED_BY_AM, FinalStatus, TaskStatus, TonySession, TonyTask

LOG = logging.getLogger("tony.coordinator")

ENDPOINT_FILE = "coordinator.json"


def _default_history_root(conf, staging_root: str) -> str:
    loc = conf.get(K.HISTORY_LOCATION, "")
    if not loc or loc.startswith("/path/to/"):
        return os.path.join(staging_root, "history")
    return loc


_TONY_JOBS_DIR = os.path.realpath(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "jobs"))


def _is_tony_amd_program(cmd: str) -> bool:
    """One of tony_amd's own training programs, named exactly: ``-m tony_amd.jobs.<name>``, or a script
    path that resolves into the installed tony_amd/jobs directory.  A user script that merely shares a
    file name (``python inception_ps.py``) or lives under a path containing "tony_amd" does not count."""
    import shlex

    try:
        toks = shlex.split(cmd)
    except ValueError:
        toks = cmd.split()
    for i, t in enumerate(toks):
        if t == "-m" and i + 1 < len(toks) and toks[i + 1].startswith("tony_amd.jobs."):
            return True
        if t.endswith(".py") and os.path.isabs(t) and os.path.dirname(os.path.realpath(t)) == _TONY_JOBS_DIR:
            return True
    return False


def _runs_tony_amd_job(conf) -> bool:
    """Whether the job's task command is one of tony_amd's own training programs (tony_amd/jobs), which
    bring up the tony_amd data planes themselves: an exact entry point, or a relative script shipped from
    tony_amd/jobs itself (the client marks a --src_dir that is that directory)."""
    cmds = [conf.get(K.CONTAINERS_COMMAND) or ""] + [v for k, v in conf.get_val_by_regex(r"^tony\.[a-z]+\.command$").items()]
    if any(_is_tony_amd_program(c) for c in cmds):
        return True
    if conf.get_bool(K.AMD_SRC_IS_TONY_JOBS, False):
        names = {f for f in os.listdir(_TONY_JOBS_DIR) if f.endswith(".py")} if os.path.isdir(_TONY_JOBS_DIR) else set()
        return any(os.path.basename(t) in names for c in cmds for t in c.split() if t.endswith(".py"))
    return False


def resolve_visible_mode(conf) -> str:
    """``tony.amd.visible-devices-mode`` for a job: ``none`` / ``hip`` / ``rocr`` as configured, and for
    ``auto`` (the default) ``none`` only when the job runs a tony_amd data plane that maps a peer GPU's
    memory -- ``tony.amd.collective=hip`` (the xGMI collective kernels), or a TensorFlow job with ps tasks
    that runs tony_amd's PS program (a task command from tony_amd/jobs) or sets ``tony.amd.ps-plane=xgmi``
    itself (parallel/ps_plane.py; the key's xgmi default alone does not count: an ordinary user TF PS job
    keeps its isolation) -- and ``hip`` (per-task HIP_VISIBLE_DEVICES) for everything else, so an
    arbitrary user program that picks ``cuda:0`` or ``cuda:LOCAL_RANK`` cannot land on another task's GPU."""
    mode = (conf.get(K.AMD_VISIBLE_DEVICES_MODE, "auto") or "auto").lower()
    if mode != "auto":
        return mode
    if conf.get(K.AMD_COLLECTIVE, "rccl").lower() in ("hip", "xgmi"):
        return "none"
    framework = conf.get(K.FRAMEWORK_NAME, "tensorflow").lower()
    plane = conf.get(K.AMD_PS_PLANE, "xgmi").lower()
    explicit = (conf.get_source(K.AMD_PS_PLANE) or "tony-default.xml") != "tony-default.xml"
    if framework == "tensorflow" and conf.get_int("tony.ps.instances", 0) > 0 and plane == "xgmi" \
            and (explicit or _runs_tony_amd_job(conf)):
        return "none"
    # an MXNet job whose kvstore servers move GPU payloads on the peer-mapped plane (parallel/kvstore.py)
    if framework == "mxnet" and conf.get_int("tony.server.instances", 0) > 0 \
            and conf.get_int("tony.worker.gpus", 0) > 0 and conf.get(K.AMD_KV_PLANE, "auto").lower() != "gloo":
        return "none"
    return "hip"


def gpu_pinning_env(mode: str, gpus, hip_ordinal, devices) -> dict:
    """Environment that pins a task to its GPUs (SURVEY §7.4 hard part 6: isolation vs P2P).

    ``none``: every GPU stays visible, so RCCL keeps its xGMI P2P transport and the tony_amd data
    planes can map peer memory (hipIpcOpenMemHandle needs the peer device in the process); the task's
    GPUs are named by their HIP ordinals in TONY_HIP_ORDINALS and parallel/bootstrap.py selects the
    first one (``torch.cuda.set_device``).  ``hip`` / ``rocr``: HIP_VISIBLE_DEVICES /
    ROCR_VISIBLE_DEVICES hide every other GPU (hard isolation; a data plane that needs a peer's memory
    cannot run).  ``resolve_visible_mode`` picks between them for ``auto``.  Either way TONY_GPU_BDFS
    lets the task verify it got the GPU it was allocated (gpu/inventory.verify_visible_device)."""
    mode = (mode or "hip").lower()
    if mode not in ("none", "hip", "rocr"):
        raise ValueError(f"tony.amd.visible-devices-mode must be auto, none, hip or rocr, not {mode!r}")
    ordinals = ",".join(str(hip_ordinal.get(g, g)) for g in gpus)
    devs = {d.index: d for d in devices}
    env = {"TONY_GPU_BDFS": ",".join(devs[g].bdf for g in gpus if g in devs), "TONY_VISIBLE_MODE": mode,
           "TONY_HIP_ORDINALS": ordinals}
    if mode == "hip":
        env[C.HIP_VISIBLE_DEVICES] = ordinals
    elif mode == "rocr":
        env[C.ROCR_VISIBLE_DEVICES] = ordinals
    return env


class Coordinator:
    def __init__(self, conf_path: str, job_dir: str, app_id: str, started_ms: Optional[int] = None):
        self.conf_path = conf_path
        self.job_dir = job_dir
        self.app_id = app_id
        self.started_ms = started_ms or int(time.time() * 1000)
        self.user = getpass.getuser()
        self.host = U.current_host()
        self.conf: Optional[Configuration] = None
        self.session: Optional[TonySession] = None
        self.scheduler: Optional[TaskScheduler] = None
        self.adapter = None
        self.rpc: Optional[RpcServer] = None
        self.hb: Optional[HeartbeatMonitor] = None
        self.allocator: Optional[GpuAllocator] = None
        self.events = EventHandler()
        self.metrics: Dict[str, Dict[str, float]] = {}
        self.metrics_lock = threading.Lock()
        self.children: Dict[int, TonyTask] = {}
        self.children_lock = threading.Lock()
        self.pending_requests: List = []
        self.session_id = 0
        self.num_am_retries = 0
        self.client_signal_to_stop = threading.Event()
        self.task_has_missed_hb = False
        self.untracked_task_failed = False
        self.preprocess_exit_code = 0
        self.preprocess_finished = False
        self.single_node = False
        self.proxy_url: Optional[str] = None
        self.tb_url: Optional[str] = None
        self.state = "ACCEPTED"
        self.final_status = FinalStatus.UNDEFINED
        self.diagnostics = ""
        self.container_env: Dict[str, str] = {}
        self.token: Optional[str] = None
        self.history_dir: Optional[str] = None
        self.wake = threading.Event()
        self.launch_lock = threading.RLock()

    # ------------------------------------------------------------------ init --
    def init(self) -> bool:
        self.conf = Configuration(load_defaults=False)
        self.conf.add_resource(self.conf_path, C.TONY_FINAL_XML)
        c = self.conf
        self.app_timeout_ms = c.get_int(K.APPLICATION_TIMEOUT, 0)
        self.retry_count = c.get_int(K.AM_RETRY_COUNT, 0)
        self.registration_timeout_ms = c.get_int(K.CONTAINER_ALLOCATION_TIMEOUT, -1)
        self.hb_interval_ms = c.get_int(K.TASK_HEARTBEAT_INTERVAL_MS, 1000)
        self.max_missed_hb = c.get_int(K.TASK_MAX_MISSED_HEARTBEATS, 25)
        self.monitor_interval_s = c.get_int(K.AMD_MONITOR_INTERVAL_MS, 200) / 1000.0
        self.wait_client_stop_s = c.get_int(K.AM_WAIT_CLIENT_STOP_TIMEOUT, 15)
        self.distributed_mode = c.get(K.APPLICATION_DISTRIBUTED_MODE, C.DistributedMode.GANG).upper()
        self.framework = c.get(K.FRAMEWORK_NAME, "tensorflow")
        self.runtime = get_runtime(self.framework)
        self.adapter = self.runtime.am_adapter()
        if not self.adapter.validate_and_update_config(c):
            self.diagnostics = "runtime rejected the job configuration"
            LOG.error(self.diagnostics)
            return False
        self.single_node = U.get_num_total_tasks(c) == 0
        self.enable_preprocess = c.get_bool(K.ENABLE_PREPROCESSING_JOB, False)
        self.container_env = U.parse_key_value(c.get_strings(K.CONTAINER_LAUNCH_ENV))
        self.container_env[C.APPID] = self.app_id
        return True

    # --------------------------------------------------------------- prepare --
    def _handlers(self):
        return {
            "getTaskInfos": self._rpc_get_task_infos,
            "getClusterSpec": lambda r: P.GetClusterSpecResponseProto(
                cluster_spec=self.session.cluster_spec_json() if self.session else "{}"),
            "registerWorkerSpec": self._rpc_register_worker_spec,
            "registerTensorBoardUrl": self._rpc_register_tb_url,
            "registerExecutionResult": self._rpc_register_execution_result,
            "finishApplication": self._rpc_finish_application,
            "taskExecutorHeartbeat": self._rpc_heartbeat,
            "registerCallbackInfo": self._rpc_register_callback_info,
            "updateMetrics": self._rpc_update_metrics,
            "getApplicationStatus": self._rpc_get_status,
            "reset": self._rpc_reset,
        }

    def prepare(self) -> bool:
        c = self.conf
        if c.get_bool(K.SECURITY_ENABLED, True):
            self.token = secrets.token_hex(16)
            tok_path = os.path.join(self.job_dir, "token")
            fd = os.open(tok_path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
            with os.fdopen(fd, "w") as f:
                f.write(self.token)
        self.rpc = RpcServer(self._handlers(), host=self.host, port=0, token=self.token).start()
        self.container_env[C.AM_HOST] = self.host
        self.container_env[C.AM_PORT] = str(self.rpc.port)
        self.container_env[C.METRICS_RPC_PORT] = str(self.rpc.port)
        fake = c.get_int(K.AMD_FAKE_GPUS, -1)
        devices = discover(fake)
        self.allocator = GpuAllocator(devices)
        self.ps_share_gpu = U.ps_shares_worker_gpu(c)
        # amd-smi index -> HIP ordinal by PCI BDF (raises on a GPU HIP does not show: no silent mis-pinning)
        self.hip_ordinal = hip_ordinals(devices)
        LOG.info("GPU inventory: %d device(s)%s", len(devices), " (fake)" if devices and devices[0].fake else "")
        self.hb = HeartbeatMonitor(self.hb_interval_ms, self.max_missed_hb, self._on_task_deemed_dead)
        self.hb.start()
        staging_root = os.path.dirname(self.job_dir)
        hist_root = _default_history_root(c, staging_root)
        layout = HistoryLayout.from_conf(c)
        inter = layout.intermediate if not layout.intermediate.startswith("/path/to/") else \
            os.path.join(hist_root, C.TONY_HISTORY_INTERMEDIATE)
        self.history_finished_root = layout.finished if not layout.finished.startswith("/path/to/") else \
            os.path.join(hist_root, C.TONY_HISTORY_FINISHED)
        self.history_tz = layout.timezone
        self.history_dir = os.path.join(inter, self.app_id)
        try:
            os.makedirs(self.history_dir, exist_ok=True)
            shutil.copy2(self.conf_path, os.path.join(self.history_dir, C.TONY_FINAL_XML))
            write_owner(self.history_dir, self.job_dir)
        except OSError:
            LOG.exception("cannot set up history dir %s", self.history_dir)
            self.history_dir = None
        self._write_endpoint()
        return True

    def _write_endpoint(self) -> None:
        ep = {"host": self.host, "port": self.rpc.port, "pid": os.getpid(), "appId": self.app_id,
              "historyDir": self.history_dir}
        path = os.path.join(self.job_dir, ENDPOINT_FILE)
        with open(path + ".tmp", "w") as f:
            json.dump(ep, f)
        os.replace(path + ".tmp", path)

    # ------------------------------------------------------------------- run --
    def run(self) -> bool:
        if not self.init():
            self.state, self.final_status = "FINISHED", FinalStatus.FAILED
            return False
        if not self.prepare():
            return False
        md = JobMetadata(self.app_id, self.started_ms, user=self.user)
        if not self.events.set_up(self.history_dir, md):
            return False
        self.events.start()
        self.state = "RUNNING"
        succeeded = False
        while True:
            if os.environ.get(C.TEST_AM_CRASH) == "true":
                LOG.fatal("Error running coordinator (TEST_AM_CRASH)")
                self._finish(False, md, "TEST_AM_CRASH")
                return False
            if os.environ.get(C.TEST_AM_THROW_EXCEPTION_CRASH) == "true":
                self._finish(False, md, "TEST_AM_THROW_EXCEPTION_CRASH")
                raise IOError("AM crashed.")
            self.events.emit(EV.application_inited(self.app_id, U.get_num_total_tasks(self.conf), self.host,
                                                   f"coordinator_{self.app_id}"))
            try:
                self.start()
            except Exception:  # noqa: BLE001
                LOG.exception("Exception when starting the session")
                self._finish(False, md, "session start failed")
                return False
            succeeded = self.monitor()
            if succeeded or self.retry_count == 0 or self.single_node:
                break
            LOG.info("Session %d failed (%s); retrying, %d retries left", self.session_id,
                     self.session.final_message, self.retry_count)
            self.reset()
            self.retry_count -= 1
            self.num_am_retries += 1
            self.container_env[C.NUM_AM_RETRIES] = str(self.num_am_retries)
        self._finish(succeeded, md, self.session.final_message if self.session else None)
        return succeeded

    def _finish(self, succeeded: bool, md: JobMetadata, message: Optional[str]) -> None:
        self.stop()
        self.final_status = FinalStatus.SUCCEEDED if succeeded else FinalStatus.FAILED
        self.diagnostics = message or ""
        self.state = "FINISHED"
        self._wait_for_client_signal()
        s = self.session
        self.events.emit(EV.application_finished(self.app_id, s.num_completed_tasks() if s else 0,
                                                 s.num_failed_tasks() if s else 0))
        md.completed = int(time.time() * 1000)
        md.status = C.SUCCEEDED if succeeded else C.FAILED
        self.events.stop(self.history_dir, md)
        self._move_history(md)
        if self.rpc is not None:
            self.rpc.stop(0.2)
        if self.hb is not None:
            self.hb.stop()
        self.adapter.destroy()

    def _move_history(self, md: JobMetadata) -> None:
        if not self.history_dir or not os.path.isdir(self.history_dir):
            return
        dst_root = year_month_day_dir(self.history_finished_root, md.completed, self.history_tz)
        try:
            os.makedirs(dst_root, exist_ok=True)
            dst = os.path.join(dst_root, self.app_id)
            if os.path.exists(dst):
                shutil.rmtree(dst)
            shutil.move(self.history_dir, dst)
            self.history_dir = dst
            self._write_endpoint()
        except OSError:
            LOG.exception("failed to move history to %s", dst_root)

    def _wait_for_client_signal(self) -> None:
        if self.conf.get_bool("tony.amd.coordinator.standalone", False):
            return
        self.client_signal_to_stop.wait(self.wait_client_stop_s)

    # ----------------------------------------------------------------- start --
    def start(self) -> None:
        self.preprocess_exit_code = 0
        self.preprocess_finished = False
        if self.enable_preprocess or self.single_node:
            self._do_preprocessing_job()
            if self.single_node:
                self.session = TonySession(self.conf, self.session_id, container_requests={})
                self.session.set_final_status(FinalStatus.SUCCEEDED if self.preprocess_exit_code == 0
                                              else FinalStatus.FAILED,
                                              f"single node job exited with {self.preprocess_exit_code}")
                return
        self.session = TonySession(self.conf, self.session_id)
        self.adapter.set_session(self.session)
        self.scheduler = TaskScheduler(self.session, self._request_containers)
        self.scheduler.schedule_tasks()

    def _do_preprocessing_job(self) -> None:
        """Run the job command inside the coordinator (single-node / preprocess mode)."""
        c = self.conf
        cmd = c.get(K.AM_COMMAND) or c.get(K.CONTAINERS_COMMAND)
        if not cmd:
            self.preprocess_exit_code = 0 if not self.single_node else 1
            self.preprocess_finished = True
            return
        env = dict(self.container_env)
        env.update(U.parse_key_value(c.get_strings(K.EXECUTION_ENV)))
        env[C.PREPROCESSING_JOB] = "true"
        workdir = os.path.join(self.job_dir, "coordinator")
        os.makedirs(workdir, exist_ok=True)
        from ..utils.resources import localize_all

        localize_all(c.get_strings(K.CONTAINERS_RESOURCES), workdir)
        U.link_job_archives(self.job_dir, self.app_id, workdir)
        U.extract_resources(self.app_id, workdir)
        env["HOME"] = workdir
        tb = None
        if self.single_node:
            tb = native.PortReservation(0)
            env[C.TB_PORT] = str(tb.port)
            self.proxy_url = f"{self.host}:{tb.port}"
            self.tb_url = f"http://{self.proxy_url}"
            tb.release()
        out_path = os.path.join(self.job_dir, "logs", C.AM_STDOUT_FILENAME)
        os.makedirs(os.path.dirname(out_path), exist_ok=True)
        with open(out_path, "ab") as out, open(os.path.join(self.job_dir, "logs", C.AM_STDERR_FILENAME), "ab") as err:
            p = U.ShellProcess(cmd, env=env, cwd=workdir, stdout=out, stderr=err)
            timeout_ms = c.get_int(K.WORKER_TIMEOUT, 0)
            rc = p.wait(timeout_ms / 1000.0 if timeout_ms > 0 else None)
        self.preprocess_exit_code = rc if rc >= 0 else 128 - rc
        self.preprocess_finished = True
        try:
            with open(out_path, errors="replace") as f:
                for line in f:
                    if "Model parameters: " in line:
                        self.container_env[C.TASK_PARAM_KEY] = line.split("Model parameters: ", 1)[1].strip()
        except OSError:
            pass
        LOG.info("preprocessing job exited with %d", self.preprocess_exit_code)

    # --------------------------------------------------------- task launching --
    def _request_containers(self, req) -> None:
        with self.launch_lock:
            for _ in range(req.num_instances):
                self.pending_requests.append(req)
        self._launch_pending()

    def _launch_pending(self) -> None:
        # called from the monitor loop and from reaper threads (DAG stage unblocked)
        with self.launch_lock:
            still = []
            for req in self.pending_requests:
                if req.gpus > self.allocator.total:
                    self.session.set_final_status(
                        FinalStatus.FAILED, f"job type {req.job_name} asks {req.gpus} GPUs per task, the node has "
                                            f"{self.allocator.total}")
                    self.session.training_finished = True
                    continue
                if req.gpus > 0 and self.allocator.free_count() < req.gpus:
                    still.append(req)  # wait for GPUs to be released
                    continue
                shared = req.gpus == 0 and req.job_name == C.PS_JOB_NAME and self.ps_share_gpu
                if shared and not self._gpu_workers():
                    still.append(req)  # placed beside a worker: wait for the workers' GPUs
                    continue
                task = self.session.init_task(req.job_name)
                if task is None:
                    continue
                owner = f"{task.id}@{task.session_id}"
                if shared:
                    workers = self._gpu_workers()
                    slot = self.allocator.share(owner, workers[int(task.task_index) % len(workers)].gpus[0], req.vcores)
                    task.gpu_shared = True
                else:
                    slot = self.allocator.allocate(owner, req.gpus, req.vcores) if req.gpus > 0 else None
                self._launch(task, req, slot)
            self.pending_requests = still

    def _gpu_workers(self):
        """The chief / worker tasks of this session that hold GPUs, by (job, index)."""
        out = []
        for job in (C.CHIEF_JOB_NAME, C.WORKER_JOB_NAME):
            for t in self.session.job_tasks.get(job, []):
                if t is not None and getattr(t, "gpus", None):
                    out.append(t)
        return out

    def _task_container_id(self, task: TonyTask) -> str:
        return f"container_{self.app_id}_{task.session_id:02d}_{task.job_name}_{task.task_index}"

    def _launch(self, task: TonyTask, req, slot) -> None:
        c = self.conf
        task.info.status = TaskStatus.READY
        cid = self._task_container_id(task)
        log_dir = os.path.join(self.job_dir, "logs", cid)
        work_dir = os.path.join(self.job_dir, "containers", cid)
        os.makedirs(log_dir, exist_ok=True)
        os.makedirs(work_dir, exist_ok=True)
        env = dict(os.environ)
        env.pop("MALLOC_ARENA_MAX", None)
        env.update(self.container_env)
        env.update({
            C.JOB_NAME: task.job_name,
            C.JOB_ID: self.app_id,
            C.TASK_INDEX: task.task_index,
            C.TASK_NUM: str(self.session.total_tracked_tasks()),
            C.DISTRIBUTED_MODE_NAME: self.distributed_mode,
            C.IS_CHIEF: "true" if self.session.is_chief(task.job_name, task.task_index) else "false",
            C.SESSION_ID: str(self.session_id),
            C.ATTEMPT_NUMBER: str(self.session_id),
            C.NUM_AM_RETRIES: str(self.num_am_retries),
            C.TONY_CONF_PATH: self.conf_path,
            C.TONY_JOB_DIR: self.job_dir,
            "TONY_CONTAINER_ID": cid,
        })
        if self.token:
            env[C.TONY_TOKEN_FILE] = os.path.join(self.job_dir, "token")
        # data-plane collectives of the tony_amd jobs: RCCL or the xGMI peer-memory kernels
        env["TONY_COLLECTIVE"] = c.get(K.AMD_COLLECTIVE, "rccl").lower()
        env["TONY_PS_PLANE"] = c.get(K.AMD_PS_PLANE, "xgmi").lower()
        env["TONY_KV_PLANE"] = c.get(K.AMD_KV_PLANE, "auto").lower()
        # whether the ps tasks own GPUs (the Inception PS job picks its topology from it on every task)
        env["TONY_PS_GPUS"] = str(c.get_int("tony.ps.gpus", 0))
        # the ps tasks sit on a worker's GPU, shared (utils/core.ps_shares_worker_gpu): every task learns
        # the topology; the ps task also gets that GPU's pinning below
        env["TONY_PS_SHARED_GPU"] = "1" if self.ps_share_gpu else "0"
        if slot is not None and slot.gpus:
            ids = ",".join(str(g) for g in slot.gpus)
            task.gpus = list(slot.gpus)
            task.numa_node = slot.numa_node
            env[C.TONY_GPU_IDS] = ids
            env[C.TONY_NUMA_NODE] = str(slot.numa_node)
            if slot.cpus and c.get_bool(K.AMD_NUMA_BIND, True):
                env["TONY_CPUS"] = ",".join(str(x) for x in slot.cpus)
            env.update(gpu_pinning_env(resolve_visible_mode(c), slot.gpus, self.hip_ordinal,
                                       self.allocator.devices))
            task.info.gpus = ids
        if c.get_bool(K.DOCKER_ENABLED, False):
            image = c.get(K.docker_image_key(task.job_name)) or c.get(K.DOCKER_CONTAINERS_IMAGE, "")
            env["YARN_CONTAINER_RUNTIME_TYPE"] = "docker"
            env["YARN_CONTAINER_RUNTIME_DOCKER_IMAGE"] = image
            mounts = c.get(K.DOCKER_CONTAINERS_MOUNT)
            if mounts:
                env["YARN_CONTAINER_RUNTIME_DOCKER_CONTAINER_MOUNTS"] = mounts
        argv = [sys.executable, "-m", "tony_amd.agent.executor"]
        pkg_root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["PYTHONPATH"] = pkg_root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        stdout = os.path.join(log_dir, "stdout")
        stderr = os.path.join(log_dir, "stderr")
        task.info.stdout_path, task.info.stderr_path = stdout, stderr
        task.info.url = f"file://{log_dir}"
        task.info.host = self.host
        pid = native.spawn(argv, env, cwd=work_dir, stdout=stdout, stderr=stderr, new_session=True)
        task.pid = pid
        task.info.pid = pid
        task.start_time = time.time()
        with self.children_lock:
            self.children[pid] = task
        task.info.status = TaskStatus.RUNNING
        self.events.emit(EV.task_started(task.job_name, int(task.task_index), self.host, cid))
        threading.Thread(target=self._reap, args=(pid, task), name=f"tony-reap-{task.id}", daemon=True).start()
        LOG.info("launched %s pid=%d gpus=%s", task.id, pid, task.info.gpus or "-")

    def _reap(self, pid: int, task: TonyTask) -> None:
        try:
            _, status = os.waitpid(pid, 0)
        except ChildProcessError:
            status = 0
        if os.WIFEXITED(status):
            code = os.WEXITSTATUS(status)
        else:
            code = 128 + os.WTERMSIG(status) if os.WIFSIGNALED(status) else 1
        if getattr(task, "killed_by_am", False):
            code = KILLED_BY_AM
        native.kill_tree(pid, signal.SIGKILL)  # leftovers of the task's process group
        with self.children_lock:
            self.children.pop(pid, None)
        self._process_finished_task(task, code)

    def _process_finished_task(self, task: TonyTask, exit_code: int) -> None:
        if os.environ.get(C.TEST_TASK_COMPLETION_NOTIFICATION_DELAYED):
            time.sleep(1.0)
        self.allocator.release(f"{task.id}@{task.session_id}")
        if self.session is None or task.session_id != self.session.session_id:
            return  # completion of a past session
        LOG.info("task %s finished with exit status %d", task.id, exit_code)
        diag = None if exit_code == 0 else C.EXIT_DIAGNOSTICS.get(exit_code, f"exit status {exit_code}")
        self.session.on_task_completed(task.job_name, task.task_index, exit_code, diag)
        if self.scheduler is not None:
            self.scheduler.register_dependency_completed(task.job_name)
        with self.metrics_lock:
            ms = self.metrics.get(task.id, {})
        self.events.emit(EV.task_finished(task.job_name, int(task.task_index), task.info.status.name,
                                          [{"name": k, "value": v} for k, v in ms.items()],
                                          diag if exit_code != 0 else "NA"))
        if U.is_untracked_job_type(task.job_name, self.conf) and task.is_failed():
            self.untracked_task_failed = True
        self.hb.unregister(task.id)
        self.wake.set()

    # --------------------------------------------------------------- monitor --
    def monitor(self) -> bool:
        expire = float("inf") if self.app_timeout_ms == 0 else time.monotonic() + self.app_timeout_ms / 1000.0
        last_log = 0.0
        while True:
            if time.monotonic() > expire:
                LOG.error("Application times out.")
                self.session.set_final_status(FinalStatus.FAILED, "Application times out.")
                break
            if self.client_signal_to_stop.is_set():
                LOG.info("Client signals coordinator to exit.")
                break
            if self.session.training_finished:
                break
            if self.preprocess_exit_code != 0:
                self.session.set_final_status(FinalStatus.FAILED,
                                              f"Preprocess failed with exit code: {self.preprocess_exit_code}")
                break
            if self.single_node and self.preprocess_finished:
                break
            if self.task_has_missed_hb:
                break
            if self.untracked_task_failed:
                self.session.set_final_status(FinalStatus.FAILED,
                                              "One of the untracked tasks has failed with a non-zero exit code.")
                break
            if self.scheduler is not None and not self.scheduler.dependency_check_passed:
                break
            if self._registration_timed_out() or self._startup_failed():
                break
            if self.pending_requests:
                self._launch_pending()
            total = self.session.total_tracked_tasks()
            if total > 0:
                done = self.session.num_completed_tracked_tasks()
                if done == total:
                    LOG.info("Completed all %d tracked tasks.", total)
                    break
                if time.monotonic() - last_log > 30:
                    LOG.info("Completed %d out of %d tracked tasks.", done, total)
                    last_log = time.monotonic()
            self.wake.wait(self.monitor_interval_s)
            self.wake.clear()
        if not self.single_node:
            self.session.update_session_status()
        ok = self.session.final_status == FinalStatus.SUCCEEDED
        if not ok:
            LOG.info("Tony session failed: %s", self.session.final_message)
        return ok

    def _registration_timed_out(self) -> bool:
        if self.registration_timeout_ms <= 0:
            return False
        now = time.time()
        for t in self.session.unregistered_tasks():
            if now - t.start_time > self.registration_timeout_ms / 1000.0:
                msg = f"Stopping AM for task [{t.job_name}:{t.task_index}] registration timeout"
                LOG.error(msg)
                self.session.set_final_status(FinalStatus.FAILED, msg)
                return True
        return False

    def _startup_failed(self) -> bool:
        for t in self.session.tasks():
            if t.is_failed() and t.id not in self.session.registered:
                msg = f"Stopping AM for task [{t.job_name}:{t.task_index}] starting failed"
                LOG.error(msg)
                self.session.set_final_status(FinalStatus.FAILED, msg)
                return True
        return False

    def _on_task_deemed_dead(self, task_id: str) -> None:
        msg = f"Task with id [{task_id}] has missed [{self.max_missed_hb}] heartbeats. Ending application!"
        LOG.error(msg)
        self.task_has_missed_hb = True
        self.session.set_final_status(FinalStatus.FAILED, msg)
        self.wake.set()

    # ------------------------------------------------------------ stop/reset --
    def _running_tasks(self) -> List[TonyTask]:
        with self.children_lock:
            return list(self.children.values())

    def _user_pgid(self, t: TonyTask) -> int:
        path = os.path.join(self.job_dir, "containers", self._task_container_id(t), "user.pgid")
        try:
            with open(path) as f:
                return int(f.read().strip())
        except (OSError, ValueError):
            return 0

    def stop_running_tasks(self, grace_s: float = 15.0) -> None:
        tasks = self._running_tasks()
        for t in tasks:
            t.killed_by_am = True
            native.kill_tree(t.pid, signal.SIGTERM)  # the agent forwards it to the user process group
        deadline = time.monotonic() + grace_s
        while self._running_tasks() and time.monotonic() < deadline:
            time.sleep(0.05)
        for t in tasks:
            upg = self._user_pgid(t)
            if upg > 1:
                native.kill_tree(upg, signal.SIGKILL)
        for t in self._running_tasks():
            native.kill_tree(t.pid, signal.SIGKILL)
        deadline = time.monotonic() + 5
        while self._running_tasks() and time.monotonic() < deadline:
            time.sleep(0.02)

    def stop(self) -> None:
        self.stop_running_tasks(min(15.0, float(self.conf.get_int("tony.amd.stop-grace-sec", 15))))

    def reset(self) -> None:
        self.stop_running_tasks()
        self.session_id += 1
        self.pending_requests = []
        self.task_has_missed_hb = False
        self.untracked_task_failed = False
        self.hb.reset()
        with self.metrics_lock:
            self.metrics.clear()

    # ------------------------------------------------------------------- RPC --
    def _rpc_get_task_infos(self, req):
        infos = []
        if self.single_node and self.proxy_url is not None:
            infos = [P.TaskInfoProto(name=C.DRIVER_JOB_NAME, index="0", url=f"file://{self.job_dir}/logs",
                                     taskStatus=TaskStatus.RUNNING if self.state == "RUNNING" else
                                     TaskStatus.SUCCEEDED),
                     P.TaskInfoProto(name=C.NOTEBOOK_JOB_NAME, index="0", url=self.proxy_url,
                                     taskStatus=TaskStatus.RUNNING)]
        elif not self.single_node and self.session is not None and self.session.all_tasks_scheduled():
            for ti in self.session.task_infos():
                infos.append(P.TaskInfoProto(name=ti.name, index=ti.index, url=ti.url, taskStatus=int(ti.status),
                                             host=ti.host, pid=ti.pid, gpus=ti.gpus, exitCode=ti.exit_code,
                                             stdoutPath=ti.stdout_path, stderrPath=ti.stderr_path))
        return P.GetTaskInfosResponseProto(task_infos=infos)

    def _rpc_register_worker_spec(self, req):
        task = self.session.get_task(req.worker) if self.session else None
        if task is None:
            return P.RegisterWorkerSpecResponseProto()
        if task.host is None:
            LOG.info("registration from %s with spec %s", req.worker, req.spec)
            task.set_host_port(req.spec)
            task.registered_at = time.time()
            self.session.add_registered(req.worker)
            self.hb.register(req.worker)
            self._kill_chief_worker_if_testing(req.worker)
        if self.adapter.can_start_task(self.distributed_mode, req.worker):
            spec = self.adapter.construct_cluster_spec(req.worker)
            if spec is not None:
                return P.RegisterWorkerSpecResponseProto(spec=spec)
        return P.RegisterWorkerSpecResponseProto()

    def _rpc_register_tb_url(self, req):
        LOG.info("TensorBoard URL registered: %s", req.spec)
        self.tb_url = req.spec
        return P.RegisterTensorBoardUrlResponseProto(spec=req.spec)

    def _rpc_register_execution_result(self, req):
        LOG.info("result registration: exit %d from %s:%s", req.exitCode, req.jobName, req.jobIndex)
        self.hb.unregister(f"{req.jobName}:{req.jobIndex}")
        return P.RegisterExecutionResultResponseProto(message="RECEIVED")

    def _rpc_finish_application(self, req):
        self.client_signal_to_stop.set()
        self.wake.set()
        return P.EmptyProto()

    def _rpc_heartbeat(self, req):
        self.hb.received_ping(req.taskId)
        return P.HeartbeatResponseProto(sessionId=self.session_id)

    def _rpc_register_callback_info(self, req):
        if not self.adapter.receive_task_callback_info(req.taskId, req.callbackInfo):
            LOG.error("errors receiving callback info from %s", req.taskId)
        return P.EmptyProto()

    def _rpc_update_metrics(self, req):
        with self.metrics_lock:
            self.metrics[f"{req.taskType}:{req.taskIndex}"] = {m.name: m.value for m in req.metrics}
        return P.EmptyProto()

    def _rpc_get_status(self, req):
        progress = 0.0
        if self.session is not None and self.session.total_tracked_tasks():
            progress = self.session.num_completed_tracked_tasks() / self.session.total_tracked_tasks()
        return P.ApplicationStatusProto(appId=self.app_id, state=self.state, finalStatus=self.final_status,
                                        diagnostics=self.diagnostics or "", trackingUrl=self.tb_url or "",
                                        progress=progress, sessionId=self.session_id)

    def _rpc_reset(self, req):
        if self.session is not None:
            self.session.reset_registered()
        return P.EmptyProto()

    def _kill_chief_worker_if_testing(self, task_id: str) -> None:
        if os.environ.get(C.TEST_WORKER_TERMINATED) is None or task_id != C.COORDINATOR_ID:
            return
        for t in self._running_tasks():
            if t.job_name == C.WORKER_JOB_NAME:
                LOG.warning("Simulating worker termination for %s", t.id)
                native.kill_tree(t.pid, signal.SIGKILL)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="tony_amd coordinator (ApplicationMaster)")
    ap.add_argument("--conf", required=True, help="tony-final.xml")
    ap.add_argument("--job-dir", required=True)
    ap.add_argument("--app-id", required=True)
    ap.add_argument("--started", type=int, default=None)
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s",
                        stream=sys.stderr)
    coord = Coordinator(a.conf, a.job_dir, a.app_id, a.started)

    def _term(*_):
        coord.client_signal_to_stop.set()
        coord.wake.set()

    signal.signal(signal.SIGTERM, _term)
    try:
        ok = coord.run()
    except Exception:  # noqa: BLE001
        LOG.exception("coordinator crashed")
        return 255
    return 0 if ok else 255


if __name__ == "__main__":
    sys.exit(main())
