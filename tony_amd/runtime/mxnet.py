"""``mxnet`` runtime (T/runtime/MXNetRuntime.java:26-68, T/util/Utils.java:610-637).

Env: DMLC_ROLE = job name (so job types must be named scheduler/server/worker),
DMLC_PS_ROOT_URI / DMLC_PS_ROOT_PORT = the scheduler task's address (resolved
to an IP), DMLC_LOCAL = 0, DMLC_NUM_SERVER = tony.server.instances,
DMLC_NUM_WORKER = tony.worker.instances.  MXNet itself is not in this stack:
tony_amd.parallel.kvstore implements the ``dist_sync`` / ``dist_async`` kvstore
semantics these variables describe.
"""
from __future__ import annotations

from .. import constants as C
from ..conf import keys as K
from ..utils.core import parse_cluster_spec_for_mxnet
from .base import FrameworkRuntime, TaskAdapter, base_env, register


class MXNetTask(TaskAdapter):
    def build_task_env(self) -> None:
        ex = self.executor
        env = ex.shell_env
        env.update(base_env(ex))
        if not ex.cluster_spec:
            return
        addr = parse_cluster_spec_for_mxnet(ex.cluster_spec)
        if addr is None:
            raise RuntimeError("MXNet job needs a 'scheduler' job type in the cluster spec")
        env[C.DMLC_ROLE] = ex.job_name
        env[C.DMLC_PS_ROOT_URI] = addr[0]
        env[C.DMLC_PS_ROOT_PORT] = str(addr[1])
        env[C.DMLC_LOCAL] = "0"
        env[C.DMLC_NUM_SERVER] = str(ex.conf.get_int(K.instances_key(C.SERVER_JOB_NAME), 0))
        env[C.DMLC_NUM_WORKER] = str(ex.conf.get_int(K.instances_key(C.WORKER_JOB_NAME), 0))


@register
class MXNetRuntime(FrameworkRuntime):
    name = "mxnet"

    def task_adapter(self, executor) -> TaskAdapter:
        return MXNetTask(executor)
