"""``tensorflow`` runtime (T/runtime/TFRuntime.java:26-61, T/TFConfig.java).

Env: JOB_NAME, TASK_INDEX, TASK_NUM, DISTRIBUTED_MODE; in GANG mode also
CLUSTER_SPEC (raw ``{job: [host:port]}``) and TF_CONFIG
(``{"cluster": ..., "task": {"type", "index"}}`` without the tensorboard sidecar,
and without the evaluator unless this task is the evaluator).  TensorFlow is
not part of the MI355X stack: TF_CONFIG is consumed by tony_amd's own
parameter-server / all-reduce programs (tony_amd.parallel.tf_config).
"""
from __future__ import annotations

from .. import constants as C
from ..utils.core import construct_tf_config
from .base import FrameworkRuntime, TaskAdapter, base_env, register


class TFTask(TaskAdapter):
    def build_task_env(self) -> None:
        ex = self.executor
        env = ex.shell_env
        env.update(base_env(ex))
        if ex.distributed_mode == C.DistributedMode.GANG and ex.cluster_spec:
            env[C.CLUSTER_SPEC] = ex.cluster_spec
            env[C.TF_CONFIG] = construct_tf_config(ex.cluster_spec, ex.job_name, int(ex.task_index))


@register
class TFRuntime(FrameworkRuntime):
    name = "tensorflow"

    def task_adapter(self, executor) -> TaskAdapter:
        return TFTask(executor)
