"""``pytorch`` runtime (T/runtime/PyTorchRuntime.java:26-58, T/util/Utils.java:598-608).

TonY's contract: INIT_METHOD = tcp://<worker:0 host:port>, RANK = task index,
WORLD = TASK_NUM (total tracked tasks).  tony_amd adds the torch.distributed
standard variables so ``init_process_group("nccl")`` -- RCCL over xGMI on
MI355X -- works without arguments: MASTER_ADDR / MASTER_PORT (worker:0's
reserved port, released by its agent just before the user process starts so
rank 0 can host the c10d TCPStore there), WORLD_SIZE, LOCAL_RANK,
LOCAL_WORLD_SIZE.  GPU pinning variables (HIP_VISIBLE_DEVICES, TONY_CPUS) come from the coordinator's
slot assignment (cluster/coordinator.py, gpu/inventory.py).
"""
from __future__ import annotations

from .. import constants as C
from ..utils.core import parse_cluster_spec_for_pytorch
from .base import FrameworkRuntime, TaskAdapter, base_env, parse_spec, register


class PyTorchTask(TaskAdapter):
    def build_task_env(self) -> None:
        ex = self.executor
        env = ex.shell_env
        env.update(base_env(ex))
        if not ex.cluster_spec:
            return
        init = parse_cluster_spec_for_pytorch(ex.cluster_spec)
        if init is None:
            raise RuntimeError("Failed to parse the worker:0 address from the cluster spec")
        env[C.INIT_METHOD] = init
        env[C.RANK] = str(ex.task_index)
        env[C.WORLD] = str(ex.num_tasks)
        host, port = init[len(C.COMMUNICATION_BACKEND):].rsplit(":", 1)
        spec = parse_spec(ex.cluster_spec)
        workers = spec.get(C.WORKER_JOB_NAME, [])
        env[C.MASTER_ADDR] = host
        env[C.MASTER_PORT] = port
        env[C.WORLD_SIZE] = str(ex.num_tasks)
        # single node: the local rank is the rank among this node's workers
        local = [i for i, hp in enumerate(workers) if hp.rsplit(":", 1)[0] == ex.host]
        env[C.LOCAL_RANK] = str(local.index(int(ex.task_index)) if int(ex.task_index) in local else ex.task_index)
        env[C.LOCAL_WORLD_SIZE] = str(len(local) or ex.num_tasks)


@register
class PyTorchRuntime(FrameworkRuntime):
    name = "pytorch"

    def task_adapter(self, executor) -> TaskAdapter:
        return PyTorchTask(executor)
