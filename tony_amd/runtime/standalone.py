"""``standalone`` runtime (T/runtime/StandaloneRuntime.java:29-101): exactly one task, no extra env."""
from __future__ import annotations

import logging

from ..utils.core import get_num_total_tasks
from .base import AMAdapter, FrameworkRuntime, TaskAdapter, register

LOG = logging.getLogger(__name__)


class StandaloneAM(AMAdapter):
    def validate_and_update_config(self, conf) -> bool:
        n = get_num_total_tasks(conf)
        if n != 1:
            LOG.error("Standalone runtime requires exactly 1 task, got %d", n)
            return False
        return super().validate_and_update_config(conf)

    def can_start_task(self, mode, task_id) -> bool:
        return True


class StandaloneTask(TaskAdapter):
    def need_reserve_tb_port(self) -> bool:
        return False

    def build_task_env(self) -> None:
        pass


@register
class StandaloneRuntime(FrameworkRuntime):
    name = "standalone"

    def am_adapter(self):
        return StandaloneAM()

    def task_adapter(self, executor):
        return StandaloneTask(executor)
