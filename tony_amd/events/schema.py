"""TonY's history event schema (tony-core/src/main/avro/*.avsc), as one Avro schema.

Records: Event{type: EventType, event: union[ApplicationInited, ApplicationFinished,
TaskStarted, TaskFinished], timestamp: long}; Metric{name, value}.
"""
from __future__ import annotations

import time

from .avro import Schema

NS = "com.linkedin.tony.events"

METRIC = {"type": "record", "name": "Metric", "namespace": NS,
          "fields": [{"name": "name", "type": "string"}, {"name": "value", "type": "double"}]}
EVENT_TYPE = {"type": "enum", "name": "EventType", "namespace": NS,
              "symbols": ["APPLICATION_INITED", "APPLICATION_FINISHED", "TASK_STARTED", "TASK_FINISHED"]}
APPLICATION_INITED = {"type": "record", "name": "ApplicationInited", "namespace": NS, "fields": [
    {"name": "applicationId", "type": "string"}, {"name": "numTasks", "type": "int"},
    {"name": "host", "type": "string"},
    {"name": "containerID", "type": ["null", "string"], "default": None}]}
APPLICATION_FINISHED = {"type": "record", "name": "ApplicationFinished", "namespace": NS, "fields": [
    {"name": "applicationId", "type": "string"}, {"name": "finishedTasks", "type": "int"},
    {"name": "failedTasks", "type": "int"}, {"name": "metrics", "type": {"type": "array", "items": METRIC}}]}
TASK_STARTED = {"type": "record", "name": "TaskStarted", "namespace": NS, "fields": [
    {"name": "taskType", "type": "string"}, {"name": "taskIndex", "type": "int"},
    {"name": "host", "type": "string"},
    {"name": "containerID", "type": ["null", "string"], "default": None}]}
TASK_FINISHED = {"type": "record", "name": "TaskFinished", "namespace": NS, "fields": [
    {"name": "taskType", "type": "string"}, {"name": "taskIndex", "type": "int"},
    {"name": "status", "type": "string"},
    {"name": "metrics", "type": {"type": "array", "items": f"{NS}.Metric"}},
    {"name": "containerDiagnostic", "type": ["null", "string"], "default": None}]}
EVENT = {"type": "record", "name": "Event", "namespace": NS, "fields": [
    {"name": "type", "type": EVENT_TYPE},
    {"name": "event", "type": [APPLICATION_INITED, APPLICATION_FINISHED, TASK_STARTED, TASK_FINISHED]},
    {"name": "timestamp", "type": "long"}]}


def event_schema() -> Schema:
    return Schema(EVENT)


_BRANCH = {
    "APPLICATION_INITED": "ApplicationInited",
    "APPLICATION_FINISHED": "ApplicationFinished",
    "TASK_STARTED": "TaskStarted",
    "TASK_FINISHED": "TaskFinished",
}


def make_event(event_type: str, payload: dict, timestamp_ms: int = None) -> dict:
    return {"type": event_type, "event": {_BRANCH[event_type]: payload},
            "timestamp": int(time.time() * 1000) if timestamp_ms is None else int(timestamp_ms)}


def application_inited(app_id, num_tasks, host, container_id=None):
    return make_event("APPLICATION_INITED", {"applicationId": app_id, "numTasks": int(num_tasks), "host": host,
                                             "containerID": container_id})


def application_finished(app_id, finished, failed, metrics=()):
    return make_event("APPLICATION_FINISHED", {"applicationId": app_id, "finishedTasks": int(finished),
                                               "failedTasks": int(failed), "metrics": list(metrics)})


def task_started(task_type, index, host, container_id=None):
    return make_event("TASK_STARTED", {"taskType": task_type, "taskIndex": int(index), "host": host,
                                       "containerID": container_id})


def task_finished(task_type, index, status, metrics=(), diagnostic=None):
    return make_event("TASK_FINISHED", {"taskType": task_type, "taskIndex": int(index), "status": status,
                                        "metrics": [{"name": m["name"], "value": float(m["value"])} for m in metrics],
                                        "containerDiagnostic": diagnostic})
