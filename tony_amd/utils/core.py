"""General helpers (behavioural parity with T/util/Utils.java:83-788).

Process execution is MI355X-node specific: user commands run under
``bash -c`` in their own process group (so the whole tree can be killed),
``MALLOC_ARENA_MAX`` is dropped as in TonY (Utils.java:316-317), and an
optional timeout kills the group.
"""
from __future__ import annotations

import json
import logging
import os
import re
import signal
import socket
import struct
import subprocess
import tarfile
import time
import zipfile
from dataclasses import dataclass, field
from typing import Callable, Dict, Iterable, List, Optional, TypeVar

from .. import constants as C
from ..conf import keys as K

LOG = logging.getLogger(__name__)
T = TypeVar("T")


# -- polling (Utils.java:96-150) -------------------------------------------------------
def poll(func: Callable[[], bool], interval_s: float, timeout_s: float) -> bool:
    """Call ``func`` every ``interval_s`` until it returns True; ``timeout_s`` 0 = forever."""
    if interval_s < 0 or timeout_s < 0:
        raise ValueError("interval and timeout must be non-negative")
    deadline = time.monotonic() + timeout_s
    try:
        while timeout_s == 0 or time.monotonic() <= deadline:
            if func():
                return True
            time.sleep(interval_s)
    except Exception:  # noqa: BLE001 - mirror TonY: a throwing poll function ends the poll
        LOG.exception("polled function threw")
    return False


def poll_till_non_null(func: Callable[[], Optional[T]], interval_s: float, timeout_s: float) -> Optional[T]:
    if interval_s < 0 or timeout_s < 0:
        raise ValueError("interval and timeout must be non-negative")
    deadline = time.monotonic() + timeout_s
    try:
        while timeout_s == 0 or time.monotonic() <= deadline:
            r = func()
            if r is not None:
                return r
            time.sleep(interval_s)
    except Exception:  # noqa: BLE001
        LOG.exception("pollTillNonNull function threw")
    return None


# -- parsing -----------------------------------------------------------------------------
def parse_memory_string(memory: str) -> int:
    """"2g" -> 2048, "512m" -> 512, "1024" -> 1024 (MB)."""
    m = str(memory).strip().lower()
    if "m" in m:
        return int(m[:m.index("m")])
    if "g" in m:
        return int(m[:m.index("g")]) * 1024
    return int(m)


def parse_key_value(pairs: Optional[Iterable[str]]) -> Dict[str, str]:
    """["A=1", "B", "C=x=y"] -> {"A": "1", "B": "", "C": "x=y"}."""
    out: Dict[str, str] = {}
    for kv in pairs or []:
        kv = kv.strip()
        if "=" not in kv:
            out[kv] = ""
            continue
        k, v = kv.split("=", 1)
        out[k] = v
    return out


def split_address_port(addr: str):
    m = re.fullmatch(r"([\w.\-]+):(\d+)", addr)
    return (m.group(1), m.group(2)) if m else None


def resolve_name_to_ip(host: str) -> str:
    try:
        return socket.gethostbyname(host)
    except OSError:
        return "127.0.0.1" if host in ("localhost", socket.gethostname()) else host


def current_host() -> str:
    """The address tasks advertise in the cluster spec (loopback unless TONY_HOST is set)."""
    return os.environ.get("TONY_HOST", "127.0.0.1")


# -- archives (Utils.java:165-186, 477-495, 750-763) --------------------------------------
def is_archive(path: str) -> bool:
    try:
        with open(path, "rb") as f:
            head = f.read(4)
    except OSError:
        return False
    if len(head) < 4:
        return False
    sig = struct.unpack(">I", head)[0]
    return sig in (0x504B0304, 0x504B0506, 0x504B0708, 0x74657374, 0x75737461) or (sig & 0xFFFF0000) == 0x1F8B0000


def zip_folder(src_dir: str, zip_path: str) -> None:
    with zipfile.ZipFile(zip_path, "w", zipfile.ZIP_DEFLATED) as z:
        for root, _, files in os.walk(src_dir):
            for fn in files:
                full = os.path.join(root, fn)
                z.write(full, os.path.relpath(full, src_dir))


def unzip_archive(src: str, dst: str) -> bool:
    """Extract a zip / tar(.gz) archive; returns False (and logs) on failure like TonY."""
    try:
        os.makedirs(dst, exist_ok=True)
        if zipfile.is_zipfile(src):
            with zipfile.ZipFile(src) as z:
                for info in z.infolist():
                    target = os.path.realpath(os.path.join(dst, info.filename))
                    if not target.startswith(os.path.realpath(dst)):
                        raise ValueError(f"unsafe path in archive: {info.filename}")
                    z.extract(info, dst)
                    mode = (info.external_attr >> 16) & 0o777
                    if mode and not info.is_dir():
                        os.chmod(target, mode)
            return True
        if tarfile.is_tarfile(src):
            with tarfile.open(src) as t:
                t.extractall(dst, filter="data")
            return True
        LOG.error("%s is not an archive", src)
    except Exception:  # noqa: BLE001
        LOG.exception("failed to unpack %s", src)
    return False


def tony_src_zip_name(app_id: str) -> str:
    return f"tony_src_{app_id}.zip"


def client_resource_name(app_id: str, file_name: str) -> str:
    return f"{app_id}-{file_name}"


def link_job_archives(job_dir: str, app_id: str, cwd: str) -> None:
    """Make the job's src zip and venv.zip visible in a task working dir (hard link or copy)."""
    import shutil

    for fn in (tony_src_zip_name(app_id), C.PYTHON_VENV_ZIP):
        src = os.path.join(job_dir, fn)
        dst = os.path.join(cwd, fn)
        if os.path.exists(src) and not os.path.exists(dst):
            try:
                os.link(src, dst)
            except OSError:
                shutil.copy2(src, dst)


def extract_resources(app_id: str, cwd: str = ".") -> None:
    src_zip = os.path.join(cwd, tony_src_zip_name(app_id))
    if os.path.exists(src_zip):
        unzip_archive(src_zip, cwd)
    venv = os.path.join(cwd, C.PYTHON_VENV_ZIP)
    if os.path.isfile(venv):
        unzip_archive(venv, os.path.join(cwd, C.PYTHON_VENV_DIR))


# -- job types (Utils.java:371-475, 655-682) ---------------------------------------------------
def get_all_job_types(conf) -> List[str]:
    types = set()
    for k in conf.keys():
        m = K.INSTANCES_REGEX.match(k)
        if m:
            types.add(m.group(1))
    return sorted(types)


def get_num_total_tasks(conf) -> int:
    return sum(conf.get_int(K.instances_key(t), 0) for t in get_all_job_types(conf))


def get_untracked_job_types(conf) -> List[str]:
    return conf.get_strings(K.UNTRACKED_JOBTYPES, ["ps"])


def get_sidecar_job_types(conf) -> List[str]:
    # TonY passes the key itself as the default here (Utils.java:660, a latent bug);
    # the documented default is "tensorboard".
    return conf.get_strings(K.SIDECAR_JOBTYPES, [C.SIDECAR_TB_ROLE_NAME])


def get_stop_on_failure_job_types(conf) -> List[str]:
    return conf.get_strings(K.STOP_ON_FAILURE_JOBTYPES, [])


def is_sidecar_job_type(job: str, conf) -> bool:
    return job in get_sidecar_job_types(conf)


def is_untracked_job_type(job: str, conf) -> bool:
    return job in get_untracked_job_types(conf)


def is_job_type_monitored(job: str, conf) -> bool:
    return job not in set(get_untracked_job_types(conf)) | set(get_sidecar_job_types(conf))


@dataclass
class JobContainerRequest:
    """Per job type resource request (T/tensorflow/JobContainerRequest.java:10-63) + GPU pinning hints."""

    job_name: str
    num_instances: int
    memory_mb: int
    vcores: int
    gpus: int
    priority: int
    node_label: Optional[str] = None
    depends_on: List[str] = field(default_factory=list)

    @property
    def memory(self) -> int:
        return self.memory_mb


def ensure_staged_tasks_integrity(prepare: List[str], training: List[str], all_types: Iterable[str]) -> None:
    all_types = list(all_types)
    if not prepare and training:
        prepare.extend(t for t in all_types if t not in training)
        LOG.warning("no prepare-stage tasks given, auto-filling with %s", prepare)
    elif prepare and not training:
        training.extend(t for t in all_types if t not in prepare)
        LOG.warning("no training-stage tasks given, auto-filling with %s", training)
    elif not prepare and not training:
        return
    if len(prepare) + len(training) != len(all_types):
        raise ValueError(
            f"cannot parse application stages: {len(prepare)} prepare-stage and {len(training)} training-stage "
            f"job types, but {len(all_types)} job types in total")


def ps_shares_worker_gpu(conf) -> bool:
    """TonY's ``ps`` tasks request no GPU (tony-default.xml has only memory / vcores for them), yet in
    the reference's PS jobs the ps owns the variables and the optimizer.  On one MI355X node a 0-GPU
    ps of a TensorFlow job whose chief / workers have GPUs is placed on a worker's GPU, shared
    (``tony.amd.ps-share-gpu``, default true): it keeps the fp32 variables in that GPU's HBM and
    runs the xGMI PS data plane's apply kernels there (parallel/ps_plane.py), next to the worker."""
    if not conf.get_bool(K.AMD_PS_SHARE_GPU, True):
        return False
    if conf.get(K.FRAMEWORK_NAME, "tensorflow").lower() != "tensorflow":
        return False
    if conf.get_int(K.instances_key(C.PS_JOB_NAME), 0) <= 0 or conf.get_int(K.resource_key(C.PS_JOB_NAME, C.GPUS), 0) > 0:
        return False
    return any(conf.get_int(K.instances_key(j), 0) > 0 and conf.get_int(K.resource_key(j, C.GPUS), 0) > 0
               for j in (C.WORKER_JOB_NAME, C.CHIEF_JOB_NAME))


def size_gpu_task_memory(conf) -> Dict[str, int]:
    """MI355X-sized memory for GPU jobtypes whose ``tony.<job>.memory`` was left at tony-default.xml's
    YARN-era 2g.  A PyTorch-ROCm rank alone exceeds 2 GB of RSS, and the task agent enforces the limit
    (tony.amd.memory-enforced, like YARN's pmem check), so such a job used to be SIGKILLed.  Such a
    jobtype gets ``tony.amd.gpu-task-memory-per-gpu`` (default 32g) x its GPUs, set explicitly in the conf
    (and so in tony-final.xml); an explicit user value is never changed.  Returns {job: MB} changed."""
    changed = {}
    per_gpu = parse_memory_string(conf.get(K.AMD_GPU_TASK_MEMORY, "32g"))
    shared_ps = ps_shares_worker_gpu(conf)
    for job in get_all_job_types(conf):
        key = K.resource_key(job, C.MEMORY)
        gpus = conf.get_int(K.resource_key(job, C.GPUS), 0)
        if job == C.PS_JOB_NAME and shared_ps:
            gpus = 1  # a ps on a shared GPU is a GPU process (HIP runtime + torch) all the same
        src = conf.get_source(key)
        if gpus <= 0 or per_gpu <= 0 or (src is not None and src != "tony-default.xml"):
            continue
        cur = parse_memory_string(conf.get(key, K.DEFAULT_MEMORY))
        want = gpus * per_gpu
        if want > cur:
            conf.set(key, f"{want}m", source=f"{K.AMD_GPU_TASK_MEMORY} x {gpus} GPU(s)")
            changed[job] = want
            LOG.info("tony.%s.memory left at the default %d MB for a %d-GPU task: using %d MB (%s)", job, cur, gpus,
                     want, K.AMD_GPU_TASK_MEMORY)
    return changed


def parse_container_requests(conf, gpus_available: Optional[int] = None) -> Dict[str, JobContainerRequest]:
    """Job types -> requests with unique priorities and prepare->training stage dependencies."""
    job_types = get_all_job_types(conf)
    untracked = set(get_untracked_job_types(conf))
    prepare = conf.get_strings(K.APPLICATION_PREPARE_STAGE)
    training = conf.get_strings(K.APPLICATION_TRAINING_STAGE)
    ensure_staged_tasks_integrity(prepare, training, job_types)
    depend_targets = [t for t in prepare if t not in untracked]
    out: Dict[str, JobContainerRequest] = {}
    priority = 0
    for job in job_types:
        n = conf.get_int(K.instances_key(job), 0)
        mem = parse_memory_string(conf.get(K.resource_key(job, C.MEMORY), K.DEFAULT_MEMORY))
        vcores = conf.get_int(K.resource_key(job, C.VCORES), K.DEFAULT_VCORES)
        gpus = conf.get_int(K.resource_key(job, C.GPUS), K.DEFAULT_GPUS)
        if gpus > 0 and gpus_available is not None and gpus_available <= 0:
            raise RuntimeError(f"User requested {gpus} GPUs for job '{job}' but GPU is not available on the cluster.")
        deps = list(depend_targets) if job in training else []
        if n > 0:
            out[job] = JobContainerRequest(job, n, mem, vcores, gpus, priority, conf.get(K.node_label_key(job)), deps)
            priority += 1
    return out


# -- TF_CONFIG (Utils.java:503-524, TFConfig.java) ------------------------------------------------
def construct_tf_config(cluster_spec_json: str, job_name: str, task_index: int) -> str:
    spec = json.loads(cluster_spec_json)
    spec.pop(C.SIDECAR_TB_ROLE_NAME, None)
    if job_name.lower() != C.EVALUATOR_JOB_NAME:
        for k in [k for k in spec if k.lower() == C.EVALUATOR_JOB_NAME]:
            spec.pop(k)
    return json.dumps({"cluster": spec, "task": {"type": job_name, "index": int(task_index)}})


def parse_cluster_spec_for_pytorch(cluster_spec_json: str) -> Optional[str]:
    spec = json.loads(cluster_spec_json)
    workers = spec.get(C.WORKER_JOB_NAME) or []
    if not workers:
        return None
    return C.COMMUNICATION_BACKEND + workers[0]


def parse_cluster_spec_for_mxnet(cluster_spec_json: str):
    spec = json.loads(cluster_spec_json)
    sched = (spec.get(C.SCHEDULER_JOB_NAME) or [None])[0]
    if sched is None:
        return None
    hp = split_address_port(sched)
    if hp is None:
        return None
    return resolve_name_to_ip(hp[0]), hp[1]


# -- config resources (Utils.java:684-718) -----------------------------------------------------------
def append_conf_resources(key: str, resource: Optional[str], conf) -> None:
    if resource is None:
        return
    cur = conf.get_strings(key)
    cur.append(resource)
    conf.set_strings(key, cur)


# -- process execution (Utils.java:299-328) ------------------------------------------------------------
def _pdeathsig():  # runs in the child between fork and exec
    import ctypes

    try:
        ctypes.CDLL("libc.so.6").prctl(1, signal.SIGKILL)  # PR_SET_PDEATHSIG
    except OSError:
        pass


_PDEATH_HELPER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "native", "tony_pdeath")


class ShellProcess:
    """A ``bash -c`` child in its own session/process group."""

    def __init__(self, command: str, env: Optional[Dict[str, str]] = None, cwd: Optional[str] = None,
                 stdout=None, stderr=None, extra_env_unset=("MALLOC_ARENA_MAX",), die_with_parent: bool = False):
        penv = dict(os.environ)
        for k in extra_env_unset:
            penv.pop(k, None)
        if env:
            penv.update({k: str(v) for k, v in env.items()})
        exe = command.strip().split(" ")[0]
        if exe and os.path.isfile(exe) and not os.access(exe, os.X_OK):
            try:
                os.chmod(exe, os.stat(exe).st_mode | 0o111)
            except OSError:
                LOG.warning("failed to make %s executable", exe)
        self.command = command
        argv, preexec = ["bash", "-c", command], None
        if die_with_parent:
            if os.access(_PDEATH_HELPER, os.X_OK):
                # native helper: no Python (and no gRPC at-fork handlers) between fork and exec
                argv = [_PDEATH_HELPER, str(os.getpid())] + argv
            else:
                preexec = _pdeathsig
        self.proc = subprocess.Popen(argv, env=penv, cwd=cwd, stdout=stdout, stderr=stderr,
                                     start_new_session=True, preexec_fn=preexec)
        self.pid = self.proc.pid

    def wait(self, timeout_s: Optional[float] = None) -> int:
        try:
            return self.proc.wait(timeout=timeout_s)
        except subprocess.TimeoutExpired:
            LOG.warning("command timed out after %ss, killing process group %d", timeout_s, self.pid)
            self.kill()
            return self.proc.wait()

    def poll(self) -> Optional[int]:
        return self.proc.poll()

    def kill(self, sig=signal.SIGKILL, grace_s: float = 0.0) -> None:
        kill_process_group(self.pid, sig, grace_s)


def kill_process_group(pgid: int, sig=signal.SIGKILL, grace_s: float = 0.0) -> None:
    """SIGTERM (optional grace) then ``sig`` to a whole process group."""
    try:
        if grace_s > 0:
            os.killpg(pgid, signal.SIGTERM)
            deadline = time.monotonic() + grace_s
            while time.monotonic() < deadline:
                try:
                    os.killpg(pgid, 0)
                except ProcessLookupError:
                    return
                time.sleep(0.05)
        os.killpg(pgid, sig)
    except (ProcessLookupError, PermissionError):
        pass


def execute_shell(command: str, timeout_ms: int = 0, env: Optional[Dict[str, str]] = None,
                  cwd: Optional[str] = None, stdout=None, stderr=None) -> int:
    """Run ``command`` under bash; returns its exit code (127 for command-not-found, like bash)."""
    LOG.info("Executing command: %s", command)
    p = ShellProcess(command, env=env, cwd=cwd, stdout=stdout, stderr=stderr)
    rc = p.wait(timeout_ms / 1000.0 if timeout_ms and timeout_ms > 0 else None)
    return rc if rc >= 0 else 128 - rc  # signal -> 128+sig like a shell


def links_to_be_displayed_on_page(job_id: Optional[str]) -> Dict[str, str]:
    if job_id is None:
        return {}
    return dict(sorted({"Logs": f"/{C.LOGS_SUFFIX}/{job_id}", "Events": f"/{C.JOBS_SUFFIX}/{job_id}"}.items()))
