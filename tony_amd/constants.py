"""Names that form TonY's external contract (parity with T/Constants.java:13-196).

Environment variable names, file names, job-type names, metric names and the
fault-injection hooks are kept byte-identical so user scripts, tony.xml files
and history tooling written for TonY work unchanged.
"""

# -- environment contract -------------------------------------------------------
TB_PORT = "TB_PORT"
TASK_INDEX = "TASK_INDEX"
TASK_NUM = "TASK_NUM"
IS_CHIEF = "IS_CHIEF"
CLUSTER_SPEC = "CLUSTER_SPEC"
TF_CONFIG = "TF_CONFIG"
COORDINATOR_ID = "worker:0"
COMMUNICATION_BACKEND = "tcp://"
RANK = "RANK"
WORLD = "WORLD"
INIT_METHOD = "INIT_METHOD"
DMLC_ROLE = "DMLC_ROLE"
DMLC_PS_ROOT_URI = "DMLC_PS_ROOT_URI"
DMLC_PS_ROOT_PORT = "DMLC_PS_ROOT_PORT"
DMLC_NUM_SERVER = "DMLC_NUM_SERVER"
DMLC_NUM_WORKER = "DMLC_NUM_WORKER"
DMLC_LOCAL = "DMLC_LOCAL"
PS_VERBOSE = "PS_VERBOSE"
JOB_NAME = "JOB_NAME"
JOB_ID = "JOB_ID"
SESSION_ID = "SESSION_ID"
PREPROCESSING_JOB = "PREPROCESSING_JOB"
TASK_PARAM_KEY = "MODEL_PARAMS"
AM_HOST = "AM_HOST"
AM_PORT = "AM_PORT"
METRICS_RPC_PORT = "METRICS_RPC_PORT"
APPID = "appid"
ATTEMPT_NUMBER = "ATTEMPT_NUMBER"
NUM_AM_RETRIES = "NUM_AM_RETRIES"
DISTRIBUTED_MODE_NAME = "DISTRIBUTED_MODE"
TONY_CONF_DIR = "TONY_CONF_DIR"
DEFAULT_TONY_CONF_DIR = "/export/apps/tony/conf"
SKIP_HADOOP_PATH = "SKIP_HADOOP_PATH"
SIDECAR_TB_LOG_DIR = "TB_LOG_DIR"
SIDECAR_TB_TEST_KEY = "SIDECAR_TB_TEST"
HOROVOD_CLUSTER_WORKER_LIST = "CLUSTER_WORKER_LIST"
HOROVOD_DRIVER_OUTPUT_PATH = "DRIVER_OUTPUT_PATH"

# torch-standard bootstrap + MI355X pinning (new in tony_amd)
MASTER_ADDR = "MASTER_ADDR"
MASTER_PORT = "MASTER_PORT"
WORLD_SIZE = "WORLD_SIZE"
LOCAL_RANK = "LOCAL_RANK"
LOCAL_WORLD_SIZE = "LOCAL_WORLD_SIZE"
HIP_VISIBLE_DEVICES = "HIP_VISIBLE_DEVICES"
ROCR_VISIBLE_DEVICES = "ROCR_VISIBLE_DEVICES"
TONY_GPU_IDS = "TONY_GPU_IDS"
TONY_NUMA_NODE = "TONY_NUMA_NODE"
TONY_TOKEN_FILE = "TONY_TOKEN_FILE"
TONY_JOB_DIR = "TONY_JOB_DIR"
TONY_CONF_PATH = "TONY_CONF_PATH"
TONY_EXECUTION_ENV_FILE = "TONY_EXECUTION_ENV_FILE"

# -- file names -------------------------------------------------------------------
TONY_FOLDER = ".tony"
TONY_DEFAULT_XML = "tony-default.xml"
TONY_XML = "tony.xml"
TONY_SITE_CONF = "tony-site.xml"
TONY_FINAL_XML = "tony-final.xml"
TONY_JAR_NAME = "tony.jar"
PYTHON_VENV_ZIP = "venv.zip"
PYTHON_VENV_DIR = "venv"
AM_STDOUT_FILENAME = "amstdout.log"
AM_STDERR_FILENAME = "amstderr.log"
ARCHIVE_SUFFIX = "#archive"
RESOURCE_DIVIDER = "::"
SIDECAR_TB_SCRIPT_FILE_NAME = "sidecar_tensorboard.py"
HOROVOD_DRIVER_SCRIPT = "horovod_driver.py"
PORT_FILE_SUFFIX = "___PORT___"
HOROVOD_PORT_FILE_SUFFIX = "____HOROVOD_RENDEZVOUS_SERVER____"

# -- history ------------------------------------------------------------------------
JOBS_SUFFIX = "jobs"
CONFIG_SUFFIX = "config"
LOGS_SUFFIX = "logs"
HISTFILE_SUFFIX = "jhist"
INPROGRESS = "inprogress"
SUCCEEDED = "SUCCEEDED"
FAILED = "FAILED"
RUNNING = "RUNNING"
KILLED = "KILLED"
TONY_HISTORY_INTERMEDIATE = "intermediate"
TONY_HISTORY_FINISHED = "finished"
APP_TYPE = "TONY"

# -- job types ----------------------------------------------------------------------
AM_NAME = "am"
CHIEF_JOB_NAME = "chief"
SCHEDULER_JOB_NAME = "scheduler"
SERVER_JOB_NAME = "server"
PS_JOB_NAME = "ps"
WORKER_JOB_NAME = "worker"
EVALUATOR_JOB_NAME = "evaluator"
NOTEBOOK_JOB_NAME = "notebook"
DRIVER_JOB_NAME = "driver"
SIDECAR_TB_ROLE_NAME = "tensorboard"

# -- resources -----------------------------------------------------------------------
MEMORY = "memory"
VCORES = "vcores"
GPUS = "gpus"

# -- metrics (TaskMonitor) -------------------------------------------------------------
MAX_MEMORY_BYTES = "MAX_MEMORY_BYTES"
AVG_MEMORY_BYTES = "AVG_MEMORY_BYTES"
MAX_GPU_UTILIZATION = "MAX_GPU_UTILIZATION"
AVG_GPU_UTILIZATION = "AVG_GPU_UTILIZATION"
MAX_GPU_FB_MEMORY_USAGE = "MAX_GPU_FB_MEMORY_USAGE"
AVG_GPU_FB_MEMORY_USAGE = "AVG_GPU_FB_MEMORY_USAGE"
MAX_GPU_MAIN_MEMORY_USAGE = "MAX_GPU_MAIN_MEMORY_USAGE"
AVG_GPU_MAIN_MEMORY_USAGE = "AVG_GPU_MAIN_MEMORY_USAGE"
# MI355X additions
MAX_GPU_POWER_WATTS = "MAX_GPU_POWER_WATTS"
AVG_GPU_POWER_WATTS = "AVG_GPU_POWER_WATTS"
MAX_GPU_TEMPERATURE = "MAX_GPU_TEMPERATURE"
GPU_ECC_UNCORRECTABLE = "GPU_ECC_UNCORRECTABLE"  # new uncorrectable ECC errors on the task's GPUs
MAX_XGMI_READ_GBPS = "MAX_XGMI_READ_GBPS"
AVG_XGMI_READ_GBPS = "AVG_XGMI_READ_GBPS"
MAX_XGMI_WRITE_GBPS = "MAX_XGMI_WRITE_GBPS"
AVG_XGMI_WRITE_GBPS = "AVG_XGMI_WRITE_GBPS"
MAX_REPEATED_GPU_ERROR_ALLOWED = 10
# exit statuses the agent reports for failures the user process did not cause (coordinator diagnostics)
EXIT_GPU_FAULT = 75          # new uncorrectable ECC errors on a pinned GPU: the task was stopped
EXIT_MEMORY_LIMIT = 76       # the task's process tree exceeded tony.<job>.memory
EXIT_DIAGNOSTICS = {EXIT_GPU_FAULT: "GPU fault: uncorrectable ECC errors on the task's GPU(s); task stopped",
                    EXIT_MEMORY_LIMIT: "task exceeded its memory limit (tony.<job>.memory); task stopped"}

# -- fault injection hooks (test-only env vars read by production code) -----------------
TEST_AM_CRASH = "TEST_AM_CRASH"
TEST_AM_THROW_EXCEPTION_CRASH = "TEST_AM_THROW_EXCEPTION_CRASH"
TEST_WORKER_TERMINATED = "TEST_WORKER_TERMINATION"
TEST_TASK_COMPLETION_NOTIFICATION_DELAYED = "TEST_TASK_COMPLETION_NOTIFICATION_DELAYED"
TEST_TASK_EXECUTOR_NUM_HB_MISS = "TEST_TASK_EXECUTOR_NUM_HB_MISS"
TEST_TASK_EXECUTOR_SKEW = "TEST_TASK_EXECUTOR_SKEW"

DEFAULT_VALUE_OF_CONTAINER_LOG_LINK = "NA"


class DistributedMode:
    GANG = "GANG"
    FCFS = "FCFS"
