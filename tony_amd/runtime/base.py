"""Framework runtime SPI (T/Framework.java:31-68, T/FrameworkRuntimeProvider.java:26-68).

A runtime contributes two adapters:

coordinator side (``AMAdapter``, 6 hooks)
    construct_cluster_spec(task_id), destroy(), set_session(session),
    can_start_task(mode, task_id)  -- the gang barrier decision,
    validate_and_update_config(conf), receive_task_callback_info(task_id, info)
task-agent side (``TaskAdapter``)
    need_reserve_tb_port(), run() -> exit code (default: build env + run the
    user command)

Runtimes register under their framework name (``tony.application.framework``,
case-insensitive) in ``REGISTRY``; third-party runtimes can be added through
the ``tony_amd.runtimes`` entry-point group (the analogue of TonY's
ServiceLoader file META-INF/services/com.linkedin.tony.AbstractFrameworkRuntime).
"""
from __future__ import annotations

import logging
import re
import time
from typing import Dict, List, Optional, Type

from .. import constants as C

LOG = logging.getLogger(__name__)

REGISTRATION_STATUS_INTERVAL_S = 15.0


class AMAdapter:
    def __init__(self):
        self.session = None
        self.illegal_conf_key_regexes: List[str] = []
        self._last_status_log = 0.0

    def set_session(self, session) -> None:
        self.session = session

    def destroy(self) -> None:
        pass

    def construct_cluster_spec(self, task_id: str) -> str:
        return self.session.cluster_spec_json()

    def receive_task_callback_info(self, task_id: str, info: str) -> bool:
        return True

    def can_start_task(self, mode: str, task_id: str) -> bool:
        if mode == C.DistributedMode.GANG:
            if self.session.num_registered() == self.session.num_expected_tasks:
                return True
            self._print_pending()
            return False
        if mode == C.DistributedMode.FCFS:
            return True
        LOG.error("unknown distributed mode %s", mode)
        return False

    def validate_and_update_config(self, conf) -> bool:
        illegal = [k for rx in self.illegal_conf_key_regexes for k in conf.keys() if re.match(rx, k)]
        if illegal:
            LOG.error("Not allowed to configure illegal conf in Runtime. Illegal keys: %s", illegal)
            return False
        return True

    def _print_pending(self) -> None:
        now = time.monotonic()
        if now - self._last_status_log < REGISTRATION_STATUS_INTERVAL_S:
            return
        self._last_status_log = now
        pending = self.session.unregistered_tasks()
        LOG.info("Received registrations from %d tasks, awaiting registration from %d tasks.",
                 self.session.num_registered(), self.session.num_expected_tasks - self.session.num_registered())
        for t in pending:
            LOG.info("Awaiting registration from task %s", t.id)


class TaskAdapter:
    def __init__(self, executor):
        self.executor = executor

    def need_reserve_tb_port(self) -> bool:
        ex = self.executor
        sidecar_tb = bool(ex.conf.get_trimmed("tony.application.tensorboard-log-dir"))
        if not sidecar_tb and ex.is_chief:
            return True
        return sidecar_tb and ex.job_name == C.SIDECAR_TB_ROLE_NAME

    def build_task_env(self) -> None:
        raise NotImplementedError

    def run(self) -> int:
        self.build_task_env()
        return self.executor.run_user_command()


class FrameworkRuntime:
    name = ""

    def am_adapter(self) -> AMAdapter:
        return AMAdapter()

    def task_adapter(self, executor) -> TaskAdapter:
        raise NotImplementedError


REGISTRY: Dict[str, Type[FrameworkRuntime]] = {}


def register(cls: Type[FrameworkRuntime]) -> Type[FrameworkRuntime]:
    REGISTRY[cls.name.upper()] = cls
    return cls


def _load_entry_points() -> None:
    try:
        from importlib.metadata import entry_points
    except ImportError:  # pragma: no cover
        return
    try:
        eps = entry_points()
        group = eps.select(group="tony_amd.runtimes") if hasattr(eps, "select") else eps.get("tony_amd.runtimes", [])
    except Exception:  # noqa: BLE001
        return
    for ep in group:
        try:
            register(ep.load())
        except Exception:  # noqa: BLE001
            LOG.exception("failed to load runtime entry point %s", ep)


def get_runtime(framework: str) -> FrameworkRuntime:
    from . import horovod, mxnet, pytorch, standalone, tensorflow  # noqa: F401  (register built-ins)

    key = (framework or "tensorflow").upper()
    if key not in REGISTRY:
        _load_entry_points()
    if key not in REGISTRY:
        raise ValueError(f"Unsupported framework {framework!r}; known: {sorted(REGISTRY)}")
    return REGISTRY[key]()


def base_env(executor) -> Dict[str, str]:
    """JOB_NAME / TASK_INDEX / TASK_NUM / DISTRIBUTED_MODE shared by every ML runtime."""
    return {
        C.JOB_NAME: executor.job_name,
        C.TASK_INDEX: str(executor.task_index),
        C.TASK_NUM: str(executor.num_tasks),
        C.DISTRIBUTED_MODE_NAME: executor.distributed_mode,
    }


def parse_spec(cluster_spec: Optional[str]):
    import json

    return json.loads(cluster_spec) if cluster_spec else {}
