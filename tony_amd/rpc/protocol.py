"""The coordinator RPC protocol, as protobuf messages built at import time.

Message and field names follow TonY's ``TensorFlowClusterService``
(tony-core/src/main/proto/tensorflow_cluster_service_protos.proto:11-20 and
yarn_tensorflow_cluster_protos.proto:8-79) so the wire contract reads the same:
``getTaskInfos, getClusterSpec, registerWorkerSpec, registerTensorBoardUrl,
registerExecutionResult, finishApplication, taskExecutorHeartbeat,
registerCallbackInfo``.  The metrics channel (TonY's separate Hadoop Writable
``MetricsRpc.updateMetrics``, T/rpc/MetricsRpc.java:11-15) is one more method
of the same service here, plus ``reset`` and ``getApplicationStatus`` used by
the local client.

No ``protoc`` exists in this image, so the FileDescriptorProto is assembled
programmatically and concrete message classes come from the message factory;
the encoding is ordinary protobuf (proto2 syntax, every field optional).
TaskInfo carries MI355X additions (host, pid, GPU ids, log paths) as new field
numbers so a TonY-era reader still parses it.
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

PACKAGE = "tony"
SERVICE = "TensorFlowClusterService"
FULL_SERVICE = f"{PACKAGE}.{SERVICE}"

F = descriptor_pb2.FieldDescriptorProto
_T = {"string": F.TYPE_STRING, "int32": F.TYPE_INT32, "int64": F.TYPE_INT64, "double": F.TYPE_DOUBLE,
      "bool": F.TYPE_BOOL}

TASK_STATUS = ("NEW", "READY", "RUNNING", "FAILED", "SUCCEEDED", "FINISHED")

# message name -> [(field, type, number, repeated)]; nested types are prefixed
_MESSAGES = {
    "EmptyProto": [],
    "GetTaskInfosRequestProto": [],
    "TaskInfoProto": [("name", "string", 1, False), ("index", "string", 2, False), ("url", "string", 3, False),
                      ("taskStatus", "enum:TaskStatus", 4, False),
                      # MI355X additions
                      ("host", "string", 10, False), ("pid", "int64", 11, False), ("gpus", "string", 12, False),
                      ("exitCode", "int32", 13, False), ("stdoutPath", "string", 14, False),
                      ("stderrPath", "string", 15, False)],
    "GetTaskInfosResponseProto": [("task_infos", "msg:TaskInfoProto", 1, True)],
    "GetClusterSpecRequestProto": [],
    "GetClusterSpecResponseProto": [("cluster_spec", "string", 1, False)],
    "RegisterWorkerSpecRequestProto": [("worker", "string", 1, False), ("spec", "string", 2, False)],
    "RegisterWorkerSpecResponseProto": [("spec", "string", 1, False)],
    "RegisterTensorBoardUrlRequestProto": [("spec", "string", 1, False)],
    "RegisterTensorBoardUrlResponseProto": [("spec", "string", 1, False)],
    "RegisterExecutionResultRequestProto": [("exitCode", "int32", 1, False), ("jobName", "string", 2, False),
                                            ("jobIndex", "string", 3, False), ("sessionId", "string", 4, False)],
    "RegisterExecutionResultResponseProto": [("message", "string", 1, False)],
    "HeartbeatRequestProto": [("taskId", "string", 1, False)],
    "HeartbeatResponseProto": [("sessionId", "int32", 1, False)],
    "RegisterCallbackInfoRequestProto": [("taskId", "string", 1, False), ("callbackInfo", "string", 2, False)],
    "MetricProto": [("name", "string", 1, False), ("value", "double", 2, False)],
    "UpdateMetricsRequestProto": [("taskType", "string", 1, False), ("taskIndex", "int32", 2, False),
                                  ("metrics", "msg:MetricProto", 3, True)],
    "ApplicationStatusProto": [("appId", "string", 1, False), ("state", "string", 2, False),
                               ("finalStatus", "string", 3, False), ("diagnostics", "string", 4, False),
                               ("trackingUrl", "string", 5, False), ("progress", "double", 6, False),
                               ("sessionId", "int32", 7, False)],
}

# method -> (request, response)
METHODS = {
    "getTaskInfos": ("GetTaskInfosRequestProto", "GetTaskInfosResponseProto"),
    "getClusterSpec": ("GetClusterSpecRequestProto", "GetClusterSpecResponseProto"),
    "registerWorkerSpec": ("RegisterWorkerSpecRequestProto", "RegisterWorkerSpecResponseProto"),
    "registerTensorBoardUrl": ("RegisterTensorBoardUrlRequestProto", "RegisterTensorBoardUrlResponseProto"),
    "registerExecutionResult": ("RegisterExecutionResultRequestProto", "RegisterExecutionResultResponseProto"),
    "finishApplication": ("EmptyProto", "EmptyProto"),
    "taskExecutorHeartbeat": ("HeartbeatRequestProto", "HeartbeatResponseProto"),
    "registerCallbackInfo": ("RegisterCallbackInfoRequestProto", "EmptyProto"),
    "updateMetrics": ("UpdateMetricsRequestProto", "EmptyProto"),
    "getApplicationStatus": ("EmptyProto", "ApplicationStatusProto"),
    "reset": ("EmptyProto", "EmptyProto"),
}


def _build():
    fdp = descriptor_pb2.FileDescriptorProto()
    fdp.name = "tony_amd/tensorflow_cluster.proto"
    fdp.package = PACKAGE
    fdp.syntax = "proto2"
    enum = fdp.enum_type.add()
    enum.name = "TaskStatus"
    for i, s in enumerate(TASK_STATUS):
        v = enum.value.add()
        v.name = s
        v.number = i
    for mname, fields in _MESSAGES.items():
        m = fdp.message_type.add()
        m.name = mname
        for fname, ftype, num, repeated in fields:
            f = m.field.add()
            f.name = fname
            f.number = num
            f.label = F.LABEL_REPEATED if repeated else F.LABEL_OPTIONAL
            if ftype.startswith("msg:"):
                f.type = F.TYPE_MESSAGE
                f.type_name = f".{PACKAGE}.{ftype[4:]}"
            elif ftype.startswith("enum:"):
                f.type = F.TYPE_ENUM
                f.type_name = f".{PACKAGE}.{ftype[5:]}"
            else:
                f.type = _T[ftype]
    svc = fdp.service.add()
    svc.name = SERVICE
    for meth, (req, resp) in METHODS.items():
        md = svc.method.add()
        md.name = meth
        md.input_type = f".{PACKAGE}.{req}"
        md.output_type = f".{PACKAGE}.{resp}"
    pool = descriptor_pool.DescriptorPool()
    fd = pool.Add(fdp)
    classes = {}
    for mname in _MESSAGES:
        classes[mname] = message_factory.GetMessageClass(pool.FindMessageTypeByName(f"{PACKAGE}.{mname}"))
    return fd, classes


FILE_DESCRIPTOR, MESSAGES = _build()
globals().update(MESSAGES)


def method_path(method: str) -> str:
    return f"/{FULL_SERVICE}/{method}"
