"""The ``tony.*`` configuration schema (parity with T/TonyConfigurationKeys.java:13-337).

Key strings are the external contract and are identical to TonY's; defaults
live in ``tony-default.xml`` next to this file (a parity test checks that every
key with a default here appears there and vice versa).  MI355X-specific keys
are under ``tony.amd.*``.
"""
from __future__ import annotations

import re

PREFIX = "tony."

# -- version info (injected at submit, VersionInfo.java:133-141) --------------
VERSION_INFO_PREFIX = PREFIX + "version-info."
VERSION_INFO_KEYS = ("version", "revision", "branch", "user", "date", "url", "checksum")

OTHER_NAMENODES_TO_ACCESS = PREFIX + "other.namenodes"

# -- history / portal -----------------------------------------------------------
HISTORY_LOCATION = PREFIX + "history.location"
HISTORY_INTERMEDIATE = PREFIX + "history.intermediate"
HISTORY_FINISHED = PREFIX + "history.finished"
HISTORY_MOVER_INTERVAL_MS = PREFIX + "history.mover-interval-ms"
HISTORY_FINISHED_DIR_TIMEZONE = PREFIX + "history.finished-dir-timezone"
HISTORY_RETENTION_SECONDS = PREFIX + "history.retention-sec"
HISTORY_PURGER_INTERVAL_MS = PREFIX + "history.purger-interval-ms"
PORTAL_CACHE_MAX_ENTRIES = PREFIX + "portal.cache.max-entries"
KEYTAB_USER = PREFIX + "keytab.user"
KEYTAB_LOCATION = PREFIX + "keytab.location"
HTTPS_PORT = PREFIX + "https.port"
HTTPS_KEYSTORE_PATH = PREFIX + "https.keystore.path"
HTTPS_KEYSTORE_TYPE = PREFIX + "https.keystore.type"
HTTPS_KEYSTORE_PASSWORD = PREFIX + "https.keystore.password"
HTTPS_KEYSTORE_ALGORITHM = PREFIX + "https.keystore.algorithm"
HTTP_PORT = PREFIX + "http.port"
SECRET_KEY = PREFIX + "secret.key"
PORTAL_URL = PREFIX + "portal.url"

YARN_QUEUE_NAME = PREFIX + "yarn.queue"

# -- application --------------------------------------------------------------
APP = PREFIX + "application."
APPLICATION_NAME = APP + "name"
APPLICATION_TYPE = APP + "type"
FRAMEWORK_NAME = APP + "framework"
APPLICATION_NODE_LABEL = APP + "node-label"
ENABLE_PREPROCESSING_JOB = APP + "enable-preprocess"
APPLICATION_TIMEOUT = APP + "timeout"
RM_CLIENT_CONNECT_RETRY_MULTIPLIER = APP + "num-client-rm-connect-retries"
APPLICATION_TAGS = APP + "tags"
APPLICATION_PREPARE_STAGE = APP + "prepare-stage"
APPLICATION_TRAINING_STAGE = APP + "training-stage"
APPLICATION_DISTRIBUTED_MODE = APP + "distributed-mode"
APPLICATION_HADOOP_LOCATION = APP + "hadoop.location"
APPLICATION_HADOOP_CLASSPATH = APP + "hadoop.classpath"
UNTRACKED_JOBTYPES = APP + "untracked.jobtypes"
SIDECAR_JOBTYPES = APP + "sidecar.jobtypes"
STOP_ON_FAILURE_JOBTYPES = APP + "stop-on-failure-jobtypes"
FAIL_ON_WORKER_FAILURE_ENABLED = APP + "fail-on-worker-failure-enabled"
SECURITY_ENABLED = APP + "security.enabled"
HDFS_CONF_LOCATION = APP + "hdfs-conf-path"
YARN_CONF_LOCATION = APP + "yarn-conf-path"
MAPRED_CONF_LOCATION = APP + "mapred-conf-path"
TENSORBOARD_LOG_DIR = APP + "tensorboard-log-dir"

# -- tasks -----------------------------------------------------------------------
TASK = PREFIX + "task."
MAX_TOTAL_INSTANCES = TASK + "max-total-instances"
TASK_AM_JVM_OPTS = TASK + "am.jvm.opts"
TASK_EXECUTOR_JVM_OPTS = TASK + "executor.jvm.opts"
TASK_HEARTBEAT_INTERVAL_MS = TASK + "heartbeat-interval-ms"
TASK_MAX_MISSED_HEARTBEATS = TASK + "max-missed-heartbeats"
TASK_METRICS_UPDATE_INTERVAL_MS = TASK + "metrics-interval-ms"
TASK_GPU_METRICS_ENABLED = TASK + "gpu-metrics.enabled"

# -- AM (coordinator) --------------------------------------------------------------
AM_RETRY_COUNT = PREFIX + "am.retry-count"
AM_MEMORY = PREFIX + "am.memory"
AM_VCORES = PREFIX + "am.vcores"
AM_GPUS = PREFIX + "am.gpus"
AM_WAIT_CLIENT_STOP_TIMEOUT = PREFIX + "am.wait-client-signal-stop-timeout-sec"
AM_COMMAND = PREFIX + "am.command"

INSTANCES_REGEX = re.compile(r"^tony\.([a-z]+)\.instances$")
MAX_TOTAL_RESOURCES_REGEX = re.compile(r"^tony\.task\.max-total-([a-z]+)$")
RESOURCES_REGEX = re.compile(r"^tony\.([a-z]+)\.resources$")
DEFAULT_MEMORY = "2g"
DEFAULT_VCORES = 1
DEFAULT_GPUS = 0

CONTAINER_ALLOCATION_TIMEOUT = PREFIX + "container.allocation.timeout"
WORKER_TIMEOUT = PREFIX + "worker.timeout"

DOCKER_ENABLED = PREFIX + "docker.enabled"
CONTAINER_LAUNCH_ENV = PREFIX + "containers.envs"
EXECUTION_ENV = PREFIX + "execution.envs"
GPU_PATH_TO_EXEC = PREFIX + "gpu-exec-path"
PYTHON_EXEC_PATH = PREFIX + "python-exec-path"
CONTAINERS_RESOURCES = PREFIX + "containers.resources"
CONTAINERS_COMMAND = PREFIX + "containers.command"
DOCKER_CONTAINERS_IMAGE = PREFIX + "docker.containers.image"
DOCKER_CONTAINERS_MOUNT = PREFIX + "docker.containers.mount"

# -- horovod -------------------------------------------------------------------------
HOROVOD_TEST_MODE = PREFIX + "horovod.mode.test"
HOROVOD_TEST_FAST_FAIL = PREFIX + "horovod.mode.test.fast.fail"
HOROVOD_DRIVER_DEBUG_MODE = PREFIX + "horovod.driver.mode.debug"

# -- MI355X-native additions (tony.amd.*) ---------------------------------------------
AMD = PREFIX + "amd."
AMD_VISIBLE_DEVICES_MODE = AMD + "visible-devices-mode"   # auto | hip | rocr | none
AMD_PS_SHARE_GPU = AMD + "ps-share-gpu"                  # 0-GPU ps on a worker's GPU
AMD_PS_PLANE = AMD + "ps-plane"                          # xgmi | rccl (dedicated ps data plane)
AMD_KV_PLANE = AMD + "kv-plane"                          # auto | xgmi | gloo (mxnet kvstore server payloads)
AMD_NUMA_BIND = AMD + "numa-bind"                          # bind task CPUs to its GPU's NUMA node
AMD_COLLECTIVE = AMD + "collective"                        # rccl | hip
AMD_FAKE_GPUS = AMD + "fake-gpus"                          # CI: pretend the node has N GPUs (-1 = detect)
AMD_REGISTRATION_POLL_MS = AMD + "registration-poll-ms"    # executor gang-barrier poll
AMD_MONITOR_INTERVAL_MS = AMD + "monitor-interval-ms"      # coordinator monitor loop
AMD_CLIENT_POLL_MS = AMD + "client-poll-ms"                # client app-status poll
AMD_STAGING_DIR = AMD + "staging-dir"                      # job dirs (YARN app dir equivalent)
AMD_PROFILE = AMD + "profile"                              # wrap tasks in rocprofv3 --kernel-trace --stats
AMD_PROFILE_JOBTYPES = AMD + "profile.jobtypes"
AMD_GPU_TASK_MEMORY = AMD + "gpu-task-memory-per-gpu"    # memory of a GPU task left at the 2g default
AMD_MEMORY_ENFORCED = AMD + "memory-enforced"              # stop tasks whose RSS exceeds tony.<job>.memory
AMD_GPU_FAULT_STOPS_TASK = AMD + "gpu-fault-stops-task"    # new uncorrectable ECC errors stop the task
# set by the client when --src_dir is tony_amd's own job directory (tony_amd/jobs): the task commands then
# run tony_amd's training programs, which bring up its peer-mapping data planes (coordinator auto mode)
AMD_SRC_IS_TONY_JOBS = AMD + "src-is-tony-jobs"

# multi-value keys are appended (not overridden) by --conf (TonyConfigurationKeys.java:307-308)
MULTI_VALUE_CONF = (CONTAINER_LAUNCH_ENV, EXECUTION_ENV, CONTAINERS_RESOURCES)


def instances_key(job: str) -> str:
    return f"{PREFIX}{job}.instances"


def max_instances_key(job: str) -> str:
    return f"{PREFIX}{job}.max-instances"


def resource_key(job: str, resource: str) -> str:
    return f"{PREFIX}{job}.{resource}"


def node_label_key(job: str) -> str:
    return f"{PREFIX}{job}.node-label"


def depends_on_key(job: str) -> str:
    return f"{PREFIX}{job}.depends-on"


def max_total_resource_key(resource: str) -> str:
    return f"{TASK}max-total-{resource}"


def resources_key(job: str) -> str:
    return f"{PREFIX}{job}.resources"


def execute_command_key(job: str) -> str:
    return f"{PREFIX}{job}.command"


def docker_image_key(job: str) -> str:
    return f"{PREFIX}docker.{job}.image"


def timeout_key(job: str) -> str:
    return f"{PREFIX}{job}.timeout"
