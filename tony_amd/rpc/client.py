"""Coordinator RPC client (T/rpc/impl/ApplicationRpcClient.java:41-143).

One client per (host, port) (TonY keeps a singleton), calls retried on
UNAVAILABLE / DEADLINE_EXCEEDED up to ``retries`` times with a fixed sleep (TonY:
RetryProxy, 10 retries x 2 s).  Method names mirror ``ApplicationRpc``.
"""
from __future__ import annotations

import logging
import threading
import time
from typing import Dict, List, Optional, Tuple

import grpc

from ..cluster.session import TaskInfo, TaskStatus
from . import protocol as P
from .server import TOKEN_KEY

LOG = logging.getLogger(__name__)
_RETRYABLE = (grpc.StatusCode.UNAVAILABLE, grpc.StatusCode.DEADLINE_EXCEEDED)


class RpcClient:
    _instances: Dict[Tuple[str, int], "RpcClient"] = {}
    _ilock = threading.Lock()

    def __init__(self, host: str, port: int, token: Optional[str] = None, retries: int = 10,
                 retry_sleep_s: float = 2.0, timeout_s: float = 30.0):
        self.host, self.port = host, int(port)
        self.token = token
        self.retries = retries
        self.retry_sleep_s = retry_sleep_s
        self.timeout_s = timeout_s
        self._channel = grpc.insecure_channel(f"{host}:{self.port}")
        self._stubs = {}
        for name, (req, resp) in P.METHODS.items():
            self._stubs[name] = self._channel.unary_unary(
                P.method_path(name), request_serializer=P.MESSAGES[req].SerializeToString,
                response_deserializer=P.MESSAGES[resp].FromString)

    @classmethod
    def get_instance(cls, host: str, port: int, token: Optional[str] = None, **kw) -> "RpcClient":
        with cls._ilock:
            key = (host, int(port))
            if key not in cls._instances:
                cls._instances[key] = cls(host, port, token, **kw)
            return cls._instances[key]

    @classmethod
    def reset_instances(cls) -> None:
        with cls._ilock:
            for c in cls._instances.values():
                c.close()
            cls._instances.clear()

    def close(self) -> None:
        self._channel.close()

    def _call(self, method: str, request, retries: Optional[int] = None):
        md = ((TOKEN_KEY, self.token),) if self.token else None
        attempts = (self.retries if retries is None else retries) + 1
        last = None
        for i in range(attempts):
            try:
                return self._stubs[method](request, timeout=self.timeout_s, metadata=md)
            except grpc.RpcError as e:
                last = e
                if e.code() not in _RETRYABLE or i == attempts - 1:
                    raise
                time.sleep(self.retry_sleep_s)
        raise last  # pragma: no cover

    # -- ApplicationRpc -----------------------------------------------------------------
    def get_task_infos(self, retries=None) -> List[TaskInfo]:
        r = self._call("getTaskInfos", P.GetTaskInfosRequestProto(), retries)
        return [TaskInfo(t.name, t.index, t.url, TaskStatus(t.taskStatus), t.host, t.pid, t.gpus, t.exitCode,
                         t.stdoutPath, t.stderrPath) for t in r.task_infos]

    def get_cluster_spec(self) -> str:
        return self._call("getClusterSpec", P.GetClusterSpecRequestProto()).cluster_spec

    def register_worker_spec(self, worker: str, spec: str) -> Optional[str]:
        r = self._call("registerWorkerSpec", P.RegisterWorkerSpecRequestProto(worker=worker, spec=spec))
        return r.spec if r.HasField("spec") else None

    def register_tensorboard_url(self, url: str) -> str:
        return self._call("registerTensorBoardUrl", P.RegisterTensorBoardUrlRequestProto(spec=url)).spec

    def register_execution_result(self, exit_code: int, job: str, index: str, session_id: str) -> str:
        return self._call("registerExecutionResult", P.RegisterExecutionResultRequestProto(
            exitCode=int(exit_code), jobName=job, jobIndex=str(index), sessionId=str(session_id))).message

    def finish_application(self, retries=None) -> None:
        self._call("finishApplication", P.EmptyProto(), retries)

    def task_executor_heartbeat(self, task_id: str, retries=0) -> int:
        return self._call("taskExecutorHeartbeat", P.HeartbeatRequestProto(taskId=task_id), retries).sessionId

    def register_callback_info(self, task_id: str, info: str) -> None:
        self._call("registerCallbackInfo", P.RegisterCallbackInfoRequestProto(taskId=task_id, callbackInfo=info))

    # -- metrics / status / local-only --------------------------------------------------
    def update_metrics(self, task_type: str, index: int, metrics: Dict[str, float], retries=0) -> None:
        self._call("updateMetrics", P.UpdateMetricsRequestProto(
            taskType=task_type, taskIndex=int(index),
            metrics=[P.MetricProto(name=k, value=float(v)) for k, v in metrics.items()]), retries)

    def get_application_status(self, retries=None) -> Dict:
        r = self._call("getApplicationStatus", P.EmptyProto(), retries)
        return {"appId": r.appId, "state": r.state, "finalStatus": r.finalStatus, "diagnostics": r.diagnostics,
                "trackingUrl": r.trackingUrl, "progress": r.progress, "sessionId": r.sessionId}

    def reset(self) -> None:
        self._call("reset", P.EmptyProto())
