"""``horovod`` runtime (T/runtime/HorovodRuntime.java:54-356).

Coordinator side: forbids user ``tony.driver.*`` keys (except in driver debug
mode, which requires ``tony.driver.command``), injects one untracked ``driver``
task; GANG only; the driver may start once every task registered, workers only
after the driver reported its rendezvous endpoint and slot plan.
Agent side: the driver task runs ``HorovodDriver`` and posts its callback info;
a worker picks its slot by its position among same-host task indices and gets
HOROVOD_{CONTROLLER,CPU_OPERATIONS,GLOO_TIMEOUT_SECONDS,GLOO_RENDEZVOUS_ADDR,
GLOO_RENDEZVOUS_PORT,RANK,SIZE,LOCAL_RANK,LOCAL_SIZE,CROSS_RANK,CROSS_SIZE,HOSTNAME}.
"""
from __future__ import annotations

import logging
from typing import List

from .. import constants as C
from ..conf import keys as K
from ..horovod import DriverCallbackInfo, HorovodClusterSpec, SlotInfo
from .base import AMAdapter, FrameworkRuntime, TaskAdapter, base_env, register

LOG = logging.getLogger(__name__)
DRIVER = C.DRIVER_JOB_NAME
DEBUG_DRIVER_CONF_KEY = "tony.driver.command"


class HorovodAM(AMAdapter):
    def __init__(self):
        super().__init__()
        self.driver_ready = False
        self.slot_infos: List[dict] = []
        self.rendezvous_port = ""
        self.rendezvous_host = ""
        self.debug_mode = False

    def _is_driver(self, task_id: str) -> bool:
        t = self.session.get_task(task_id)
        return t is not None and t.job_name == DRIVER

    def build_worker_list(self, task_host: str, same_host: List[int]) -> str:
        counts = {}
        for t in self.session.tasks():
            if t.job_name == DRIVER:
                continue
            counts[t.host] = counts.get(t.host, 0) + 1
            if t.host == task_host:
                same_host.append(int(t.task_index))
        return ",".join(f"{h}:{n}" for h, n in counts.items())

    def construct_cluster_spec(self, task_id: str) -> str:
        task = self.session.get_task(task_id)
        same: List[int] = []
        workers = self.build_worker_list(task.host, same)
        same.sort()
        if self._is_driver(task_id):
            return workers
        if not self.driver_ready:
            LOG.error("Horovod driver is not ready; no cluster spec for %s", task_id)
            return None
        return HorovodClusterSpec(self.slot_infos, self.rendezvous_port, self.rendezvous_host, same).to_json()

    def receive_task_callback_info(self, task_id: str, info: str) -> bool:
        if not self._is_driver(task_id):
            LOG.error("callback info from a non-driver task %s", task_id)
            return False
        cb = DriverCallbackInfo.from_json(info)
        self.slot_infos = cb.slotInfos
        self.rendezvous_port = cb.port
        self.rendezvous_host = cb.host
        self.driver_ready = True
        return True

    def can_start_task(self, mode: str, task_id: str) -> bool:
        if mode != C.DistributedMode.GANG:
            self.session.set_final_status("FAILED", f"Horovod don't support {mode} distributed mode.")
            self.session.training_finished = True
            return False
        if self.session.num_registered() != self.session.num_expected_tasks:
            self._print_pending()
            return False
        return self._is_driver(task_id) or self.driver_ready

    def validate_and_update_config(self, conf) -> bool:
        self.debug_mode = conf.get_bool(K.HOROVOD_DRIVER_DEBUG_MODE, False)
        if self.debug_mode:
            if not conf.get_trimmed(DEBUG_DRIVER_CONF_KEY):
                LOG.error("Should set tony.driver.command conf when in horovod driver debug mode.")
                return False
        else:
            self.illegal_conf_key_regexes = [r"tony\.driver\.([a-z]+)"]
            if not super().validate_and_update_config(conf):
                return False
        conf.set(K.instances_key(DRIVER), "1")
        conf.set(K.resource_key(DRIVER, C.VCORES), "1")
        conf.set(K.UNTRACKED_JOBTYPES, DRIVER)
        return True


class HorovodTask(TaskAdapter):
    def need_reserve_tb_port(self) -> bool:
        return self.executor.job_name != DRIVER and super().need_reserve_tb_port()

    def build_task_env(self) -> None:
        ex = self.executor
        env = ex.shell_env
        env.update(base_env(ex))
        env[C.CLUSTER_SPEC] = ex.cluster_spec or ""
        if ex.job_name == DRIVER:
            return
        spec = HorovodClusterSpec.from_json(ex.cluster_spec)
        mine = sorted((SlotInfo.from_dict(s) for s in spec.slotInfos if s["hostname"] == ex.host),
                      key=lambda s: s.localRank)
        seq = spec.sameHostTaskIndexList.index(int(ex.task_index))
        slot = mine[seq]
        env.update({
            "HOROVOD_CONTROLLER": "gloo",
            "HOROVOD_CPU_OPERATIONS": "gloo",
            "HOROVOD_GLOO_TIMEOUT_SECONDS": "2000",
            "HOROVOD_GLOO_RENDEZVOUS_PORT": str(spec.port),
            "HOROVOD_GLOO_RENDEZVOUS_ADDR": spec.amHost,
            "HOROVOD_CROSS_RANK": str(slot.crossRank),
            "HOROVOD_CROSS_SIZE": str(slot.crossSize),
            "HOROVOD_LOCAL_RANK": str(slot.localRank),
            "HOROVOD_LOCAL_SIZE": str(slot.localSize),
            "HOROVOD_SIZE": str(slot.size),
            "HOROVOD_RANK": str(slot.rank),
            "HOROVOD_HOSTNAME": slot.hostname,
        })

    def run(self) -> int:
        ex = self.executor
        self.build_task_env()
        if ex.job_name != DRIVER:
            return ex.run_user_command()
        from ..horovod.driver import HorovodDriver

        conf = ex.conf
        debug_cmd = conf.get_trimmed(DEBUG_DRIVER_CONF_KEY) if conf.get_bool(K.HOROVOD_DRIVER_DEBUG_MODE) else None
        driver = HorovodDriver.create(ex.cluster_spec, ex.shell_env, ex.host,
                                      test_mode=conf.get_bool(K.HOROVOD_TEST_MODE, False),
                                      fast_fail=conf.get_bool(K.HOROVOD_TEST_FAST_FAIL, False),
                                      debug_command=debug_cmd)
        ex.callback_info_to_am(f"{ex.job_name}:{ex.task_index}", driver.callback_info())
        LOG.info("Horovod driver has started; it ends when the job finishes.")
        rc = driver.wait_for()
        driver.close()
        return rc


@register
class HorovodRuntime(FrameworkRuntime):
    name = "horovod"

    def am_adapter(self):
        return HorovodAM()

    def task_adapter(self, executor):
        return HorovodTask(executor)
