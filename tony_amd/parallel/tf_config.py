"""TF_CONFIG reader: the cluster-spec contract of TonY's tensorflow runtime as a process group.

TonY hands every task ``TF_CONFIG={"cluster": {job: ["host:port", ...]}, "task":
{"type": job, "index": i}}`` (T/runtime/TFRuntime.java:45-59, T/util/Utils.java:503-524:
``tensorboard`` is dropped and ``evaluator`` only appears in the evaluator's own
view).  TF would start gRPC servers on those ports; here the same document
defines one torch.distributed group:

* ranks are assigned in the order chief, master, worker, ps (index order
  inside a job) -- every task computes the same table from the same JSON;
* rank 0's advertised ``host:port`` (the port TonY's agent reserved for it and
  released before exec) hosts the TCPStore, so no extra port is needed;
* the evaluator is not part of the training group (``rank = -1``);
* ``ps`` ranks are where a dedicated :class:`ParameterServer` keeps variables.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field, replace
from typing import Dict, List, Tuple

RANK_ORDER = ("chief", "master", "worker", "ps")


@dataclass
class TFConfig:
    cluster: Dict[str, List[str]]
    task_type: str
    task_index: int
    roles: Tuple[str, ...] = field(default=RANK_ORDER)

    def without_ps(self) -> "TFConfig":
        """Rank table of the training tasks only (colocated PS: ``ps`` tasks just ``server.join()``)."""
        return replace(self, roles=tuple(r for r in self.roles if r != "ps"))

    @classmethod
    def from_json(cls, s: str) -> "TFConfig":
        d = json.loads(s)
        task = d.get("task", {})
        return cls({k: list(v) for k, v in d.get("cluster", {}).items()}, task.get("type", "worker"),
                   int(task.get("index", 0)))

    @classmethod
    def from_env(cls) -> "TFConfig":
        s = os.environ.get("TF_CONFIG")
        if s:
            return cls.from_json(s)
        # low-level TonY contract: CLUSTER_SPEC + JOB_NAME + TASK_INDEX (mnist_distributed.py:200-210)
        spec = os.environ.get("CLUSTER_SPEC")
        if spec:
            return cls(json.loads(spec), os.environ.get("JOB_NAME", "worker"), int(os.environ.get("TASK_INDEX", "0")))
        return cls({"worker": ["localhost:0"]}, "worker", 0)

    # -- rank table --------------------------------------------------------------------------
    @property
    def members(self) -> List[Tuple[str, int, str]]:
        out = []
        for job in self.roles:
            for i, addr in enumerate(self.cluster.get(job, [])):
                out.append((job, i, addr))
        return out

    @property
    def world(self) -> int:
        return len(self.members)

    @property
    def rank(self) -> int:
        for r, (job, i, _) in enumerate(self.members):
            if job == self.task_type and i == self.task_index:
                return r
        return -1

    def ranks_of(self, job: str) -> List[int]:
        return [r for r, (j, _, _) in enumerate(self.members) if j == job]

    @property
    def ps_ranks(self) -> List[int]:
        return self.ranks_of("ps")

    @property
    def worker_ranks(self) -> List[int]:
        return [r for r, (j, _, _) in enumerate(self.members) if j in ("chief", "master", "worker")]

    @property
    def num_workers(self) -> int:
        return len(self.worker_ranks)

    @property
    def is_chief(self) -> bool:
        """TF semantics: the chief task, or worker 0 when there is no chief."""
        if "chief" in self.cluster or "master" in self.cluster:
            return self.task_type in ("chief", "master") and self.task_index == 0
        return self.task_type == "worker" and self.task_index == 0

    @property
    def is_evaluator(self) -> bool:
        return self.task_type == "evaluator"

    @property
    def master_address(self) -> Tuple[str, int]:
        host, port = self.members[0][2].rsplit(":", 1)
        return host, int(port)

    @property
    def local_rank(self) -> int:
        """Index among the training tasks on this host (for device choice when GPUs are not masked)."""
        me = self.rank
        if me < 0:
            return 0
        my_host = self.members[me][2].rsplit(":", 1)[0]
        return sum(1 for r, (_, _, a) in enumerate(self.members) if r < me and a.rsplit(":", 1)[0] == my_host)

    def global_batch(self, per_worker: int) -> int:
        """mnist_keras_distributed.py:56-62: global batch = per-worker batch x number of workers."""
        return per_worker * self.num_workers
