"""Session and task state (behavioural parity with T/tensorflow/TonySession.java:46-633).

A *session* is one attempt of the whole gang (``SESSION_ID``; a retry after a
failed session builds a new one).  It owns the task table ``job -> [TonyTask]``,
the registration set behind the gang barrier, the cluster spec, completion
accounting (tracked vs untracked vs sidecar job types) and the final-status
policy:

* a non-zero, non-"killed by coordinator" exit of the chief (``chief:0``, or
  ``worker:0`` when there is no chief), of a stop-on-failure job type, or of any
  task when ``fail-on-worker-failure`` is on, ends training immediately as FAILED;
* otherwise, after all tracked tasks complete, the session FAILS only if
  fail-on-worker-failure is on or EVERY tracked task failed -- some failed
  non-chief workers still make a SUCCEEDED job (TonySession.java:331-344);
* a task stopped by the coordinator ends FINISHED (exit code ``KILLED_BY_AM``).

Unlike TonY every structure here is guarded by one lock: the RPC threads, the
process reaper and the monitor loop all mutate it (TonY's HashSet-from-RPC-
threads race, SURVEY.md §5.2, is not reproduced).
"""
from __future__ import annotations

import json
import threading
import time
from dataclasses import dataclass, field
from enum import IntEnum
from typing import Dict, List, Optional

from .. import constants as C
from ..conf import keys as K
from ..utils import core as U

KILLED_BY_AM = -105   # YARN ContainerExitStatus.KILLED_BY_APPMASTER
SUCCESS = 0


class TaskStatus(IntEnum):
    NEW = 0
    READY = 1
    RUNNING = 2
    FAILED = 3
    SUCCEEDED = 4
    FINISHED = 5


# Sort order "by attention" used by the client task table (T/rpc/TaskInfo.java:15-86)
_ATTENTION = {TaskStatus.FAILED: 0, TaskStatus.SUCCEEDED: 1, TaskStatus.FINISHED: 2, TaskStatus.RUNNING: 3,
              TaskStatus.NEW: 4, TaskStatus.READY: 5}


@dataclass
class TaskInfo:
    name: str
    index: str
    url: str = ""
    status: TaskStatus = TaskStatus.NEW
    host: str = ""
    pid: int = 0
    gpus: str = ""
    exit_code: int = -1
    stdout_path: str = ""
    stderr_path: str = ""

    def sort_key(self):
        return (_ATTENTION.get(self.status, 9), self.name, int(self.index) if self.index.isdigit() else 0)

    def __hash__(self):
        return hash((self.name, self.index))


class FinalStatus:
    UNDEFINED = "UNDEFINED"
    SUCCEEDED = "SUCCEEDED"
    FAILED = "FAILED"
    KILLED = "KILLED"


@dataclass
class TonyTask:
    job_name: str
    task_index: str
    session_id: int
    start_time: float = field(default_factory=time.time)
    host: Optional[str] = None
    port: int = -1
    exit_status: int = -1
    completed: bool = False
    info: Optional[TaskInfo] = None
    pid: int = 0
    gpus: List[int] = field(default_factory=list)
    numa_node: int = -1
    registered_at: float = 0.0

    @property
    def id(self) -> str:
        return f"{self.job_name}:{self.task_index}"

    def host_port(self) -> str:
        return f"{self.host}:{self.port if self.port >= 0 else 0}"

    def set_host_port(self, spec: str) -> None:
        h, p = spec.rsplit(":", 1)
        self.host = h
        self.port = int(p)

    def set_exit_status(self, status: int) -> None:
        if self.exit_status != -1 or self.completed:
            return  # first verdict wins (TonySession.java:506-523)
        self.exit_status = status
        if self.info is not None:
            self.info.exit_code = status
            if status == SUCCESS:
                self.info.status = TaskStatus.SUCCEEDED
            elif status == KILLED_BY_AM:
                self.info.status = TaskStatus.FINISHED
            else:
                self.info.status = TaskStatus.FAILED
        self.completed = True

    def is_failed(self) -> bool:
        return self.info is not None and self.info.status == TaskStatus.FAILED


class TonySession:
    def __init__(self, conf, session_id: int = 0, container_requests=None):
        self.conf = conf
        self.session_id = session_id
        self.lock = threading.RLock()
        self.container_requests = container_requests if container_requests is not None else \
            U.parse_container_requests(conf)
        self.job_tasks: Dict[str, List[Optional[TonyTask]]] = {
            job: [None] * req.num_instances for job, req in self.container_requests.items()}
        self.registered: set = set()
        self.num_expected_tasks = 0
        self.training_finished = False
        self.final_status = FinalStatus.UNDEFINED
        self.final_message: Optional[str] = None
        self.untracked = set(U.get_untracked_job_types(conf))
        self.sidecar = set(U.get_sidecar_job_types(conf))
        self.stop_on_failure = set(U.get_stop_on_failure_job_types(conf))
        self.fail_on_worker_failure = conf.get_bool(K.FAIL_ON_WORKER_FAILURE_ENABLED, False)

    # -- task table ---------------------------------------------------------------------------
    def is_monitored(self, job: str) -> bool:
        return job not in self.untracked and job not in self.sidecar

    def init_task(self, job: str, index: Optional[int] = None) -> Optional[TonyTask]:
        """Create the next unscheduled task of ``job`` (the allocation -> task match)."""
        with self.lock:
            tasks = self.job_tasks.get(job)
            if tasks is None:
                return None
            slots = [index] if index is not None else range(len(tasks))
            for i in slots:
                if tasks[i] is None:
                    t = TonyTask(job, str(i), self.session_id)
                    t.info = TaskInfo(job, str(i))
                    tasks[i] = t
                    return t
        return None

    def get_task(self, task_id: str) -> Optional[TonyTask]:
        try:
            job, idx = task_id.split(":")
            with self.lock:
                return self.job_tasks[job][int(idx)]
        except (KeyError, ValueError, IndexError):
            return None

    def tasks(self) -> List[TonyTask]:
        with self.lock:
            return [t for ts in self.job_tasks.values() for t in ts if t is not None]

    def all_tasks_scheduled(self) -> bool:
        with self.lock:
            return all(t is not None and t.info is not None for ts in self.job_tasks.values() for t in ts)

    def total_tasks(self) -> int:
        return sum(len(v) for v in self.job_tasks.values())

    def total_tracked_tasks(self) -> int:
        return sum(len(v) for k, v in self.job_tasks.items() if self.is_monitored(k))

    def num_completed_tasks(self) -> int:
        return sum(1 for t in self.tasks() if t.completed)

    def num_completed_tracked_tasks(self) -> int:
        return sum(1 for t in self.tasks() if t.completed and self.is_monitored(t.job_name))

    def num_failed_tasks(self) -> int:
        return sum(1 for t in self.tasks() if t.is_failed())

    def add_num_expected(self, n: int) -> None:
        with self.lock:
            self.num_expected_tasks += n

    # -- registration / gang barrier -------------------------------------------------------------
    def add_registered(self, task_id: str) -> None:
        with self.lock:
            self.registered.add(task_id)

    def reset_registered(self) -> None:
        with self.lock:
            self.registered = set()

    def num_registered(self) -> int:
        with self.lock:
            return len(self.registered)

    def unregistered_tasks(self) -> List[TonyTask]:
        return [t for t in self.tasks() if t.host is None]

    def cluster_spec(self) -> Dict[str, List[str]]:
        with self.lock:
            return {job: [t.host_port() for t in ts if t is not None] for job, ts in self.job_tasks.items()}

    def cluster_spec_json(self) -> str:
        return json.dumps(self.cluster_spec())

    # -- completion / verdicts ---------------------------------------------------------------------
    def is_chief(self, job: str, index: str) -> bool:
        return job == C.CHIEF_JOB_NAME or (C.CHIEF_JOB_NAME not in self.job_tasks and job == C.WORKER_JOB_NAME
                                           and str(index) == "0")

    def on_task_completed(self, job: str, index: str, exit_code: int, diagnostic: Optional[str] = None) -> None:
        with self.lock:
            task = self.get_task(f"{job}:{index}")
            if task is None:
                return
            task.set_exit_status(exit_code)
            if exit_code not in (SUCCESS, KILLED_BY_AM):
                if self.is_chief(job, index) or job in self.stop_on_failure or self.fail_on_worker_failure:
                    self.training_finished = True
                    msg = f"Exit status: {exit_code}"
                    if diagnostic:
                        msg += f". Error msg: {diagnostic}"
                    self.set_final_status(FinalStatus.FAILED, msg)

    def set_final_status(self, status: str, message: Optional[str]) -> None:
        with self.lock:
            self.final_status = status
            self.final_message = message

    def update_session_status(self) -> None:
        with self.lock:
            if self.final_status == FinalStatus.FAILED:
                return
            failures = 0
            for job, tasks in self.job_tasks.items():
                if not self.is_monitored(job):
                    continue
                for t in tasks:
                    if t is None:
                        self.set_final_status(FinalStatus.FAILED, "Job is null, this should not happen.")
                        return
                    if not t.completed:
                        self.set_final_status(FinalStatus.FAILED, f"Job {t.id} hasn't finished yet.")
                        return
                    if t.exit_status != 0:
                        failures += 1
            if failures > 0:
                if self.fail_on_worker_failure or failures >= self.total_tracked_tasks():
                    self.set_final_status(FinalStatus.FAILED,
                                          f"At least one job task exited with non-zero status, failedCnt={failures}")
                else:
                    self.set_final_status(FinalStatus.SUCCEEDED,
                                          f"Training completed with some worker jobs failure, failedCnt={failures}")
            else:
                self.set_final_status(FinalStatus.SUCCEEDED, None)

    def task_infos(self) -> List[TaskInfo]:
        return sorted((t.info for t in self.tasks() if t.info is not None), key=TaskInfo.sort_key)
