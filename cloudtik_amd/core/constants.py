"""Environment-tunable constants of the control plane.

Names and defaults follow the reference's ``core/_private/constants.py:108-278`` so that
existing ``CLOUDTIK_*`` environment settings keep working (update interval 5 s, heartbeat
period 1 s, heartbeat timeout 30 s, metrics port 44217, ...).  MI355X additions are marked.
"""
import os


def env_integer(key, default):
    v = os.environ.get(key)
    if v is None or v == "":
        return default
    try:
        return int(v)
    except ValueError:
        return default


def env_bool(key, default):
    v = os.environ.get(key)
    if v is None or v == "":
        return default
    return v.lower() in ("1", "true", "yes", "on")


# --- state service ---------------------------------------------------------------------
CLOUDTIK_DEFAULT_PORT = env_integer("CLOUDTIK_DEFAULT_PORT", 6789)
CLOUDTIK_ADDRESS_ENV = "CLOUDTIK_ADDRESS"
CLOUDTIK_STATE_PASSWORD = os.environ.get("CLOUDTIK_STATE_PASSWORD", "434C4F554454494B")
CLOUDTIK_START_STATE_WAIT_RETRIES = env_integer("CLOUDTIK_START_REDIS_WAIT_RETRIES", 16)

# --- logging -----------------------------------------------------------------------------
CLOUDTIK_LOGGING_LEVEL_ENV = "CLOUDTIK_LOGGING_LEVEL"
LOGGER_FORMAT = "%(asctime)s\t%(levelname)s %(filename)s:%(lineno)s -- %(message)s"
LOGGER_LEVEL_INFO = "info"
LOGGER_LEVEL_CHOICES = ["debug", "info", "warning", "error", "critical"]
LOGGING_ROTATE_MAX_BYTES = env_integer("CLOUDTIK_LOGGING_ROTATE_MAX_BYTES", 512 * 1024 * 1024)
LOGGING_ROTATE_BACKUP_COUNT = env_integer("CLOUDTIK_LOGGING_ROTATE_BACKUP_COUNT", 5)
LOG_FILE_CHANNEL = "CLOUDTIK_LOG_CHANNEL"
LOG_MONITOR_MAX_OPEN_FILES = env_integer("CLOUDTIK_LOG_MONITOR_MAX_OPEN_FILES", 200)
LOG_MONITOR_NUM_LINES_TO_READ = env_integer("CLOUDTIK_LOG_MONITOR_NUM_LINES_TO_READ", 1000)

# --- templates / config ----------------------------------------------------------------
CLOUDTIK_USER_TEMPLATES = "CLOUDTIK_USER_TEMPLATES"
CLOUDTIK_RESOURCES_ENV = "CLOUDTIK_OVERRIDE_RESOURCES"
CLOUDTIK_CONFIG_SECRET = "CLOUDTIK_CONFIG_SECRET"
CLOUDTIK_DEFAULT_MAX_WORKERS = env_integer("CLOUDTIK_DEFAULT_MAX_WORKERS", 32)

# --- scaler / controller ---------------------------------------------------------------
CLOUDTIK_UPDATE_INTERVAL_S = env_integer("CLOUDTIK_UPDATE_INTERVAL_S", 5)
CLOUDTIK_HEARTBEAT_PERIOD_SECONDS = env_integer("CLOUDTIK_HEARTBEAT_PERIOD_SECONDS", 1)
CLOUDTIK_HEARTBEAT_TIMEOUT_S = env_integer("CLOUDTIK_HEARTBEAT_TIMEOUT_S", 30)
CLOUDTIK_SCALER_STARTUP_BACKOFF_S = env_integer("CLOUDTIK_SCALER_STARTUP_BACKOFF_S", 30)
CLOUDTIK_SCALING_STATE_TIMEOUT_S = env_integer("CLOUDTIK_SCALING_STATE_TIMEOUT_S", 10)
CLOUDTIK_NODE_RESOURCE_STATE_TIMEOUT_S = env_integer("CLOUDTIK_NODE_RESOURCE_STATE_TIMEOUT_S", 10)
CLOUDTIK_MAX_NUM_FAILURES = env_integer("CLOUDTIK_MAX_NUM_FAILURES", 5)
CLOUDTIK_MAX_LAUNCH_BATCH = env_integer("CLOUDTIK_MAX_LAUNCH_BATCH", 5)
CLOUDTIK_MAX_CONCURRENT_LAUNCHES = env_integer("CLOUDTIK_MAX_CONCURRENT_LAUNCHES", 10)
CLOUDTIK_NODE_START_WAIT_S = env_integer("CLOUDTIK_NODE_START_WAIT_S", 900)
CLOUDTIK_NODE_SSH_INTERVAL_S = env_integer("CLOUDTIK_NODE_SSH_INTERVAL_S", 5)
CLOUDTIK_CONSERVE_GPU_NODES = env_integer("CLOUDTIK_CONSERVE_GPU_NODES", 1)
CLOUDTIK_NODE_AVAILABILITY_MAX_STALENESS_S = env_integer("CLOUDTIK_NODE_AVAILABILITY_MAX_STALENESS_S", 30 * 60)
CLOUDTIK_RESOURCE_UTILIZATION_SCORER_KEY = "CLOUDTIK_RESOURCE_UTILIZATION_SCORER"
CLOUDTIK_MAX_RESOURCE_DEMAND_VECTOR_SIZE = 1000
CLOUDTIK_METRIC_PORT = env_integer("CLOUDTIK_METRIC_PORT", 44217)
CLOUDTIK_FATESHARE_WORKERS = env_bool("CLOUDTIK_FATESHARE_WORKERS", False)
CLOUDTIK_MAX_NODES_TRACKED = 1500
MAX_PARALLEL_SHUTDOWN_WORKERS = env_integer("MAX_PARALLEL_SHUTDOWN_WORKERS", 50)
MAX_PARALLEL_EXEC_NODES = env_integer("MAX_PARALLEL_EXEC_NODES", 50)

# --- processes -------------------------------------------------------------------------
PROCESS_TYPE_STATE_SERVER = "cloudtik_state_server"
PROCESS_TYPE_CLUSTER_CONTROLLER = "cloudtik_cluster_controller"
PROCESS_TYPE_NODE_MONITOR = "cloudtik_node_monitor"
PROCESS_TYPE_LOG_MONITOR = "cloudtik_log_monitor"
PROCESS_TYPE_REAPER = "cloudtik_process_reaper"

ERROR_CLUSTER_CONTROLLER_DIED = "cluster_controller_died"
ERROR_NODE_MONITOR_DIED = "node_monitor_died"
ERROR_LOG_MONITOR_DIED = "log_monitor_died"

SESSION_LATEST = "session_latest"
KV_NAMESPACE_SESSION = "session"
KV_NAMESPACE_HEALTHCHECK = "healthcheck"
KV_NAMESPACE_SCALING = "scaling"
KV_NAMESPACE_ERRORS = "errors"

# --- cluster status ----------------------------------------------------------------------
CLOUDTIK_CLUSTER_STATUS_STOPPED = "STOPPED"
CLOUDTIK_CLUSTER_STATUS_UNHEALTHY = "UNHEALTHY"
CLOUDTIK_CLUSTER_STATUS_RUNNING = "RUNNING"
CLOUDTIK_WAIT_FOR_CLUSTER_READY_TIMEOUT_S = env_integer("CLOUDTIK_WAIT_FOR_CLUSTER_READY_TIMEOUT_S", 600)
CLOUDTIK_WAIT_FOR_CLUSTER_READY_INTERVAL_S = env_integer("CLOUDTIK_WAIT_FOR_CLUSTER_READY_INTERVAL_S", 5)
CLOUDTIK_WAIT_FOR_JOB_FINISHED_INTERVAL_S = env_integer("CLOUDTIK_WAIT_FOR_JOB_FINISHED_INTERVAL_S", 5)

# --- runtime environment injected into node commands ---------------------------------------
CLOUDTIK_RUNTIME_ENV_RUNTIMES = "CLOUDTIK_RUNTIMES"
CLOUDTIK_RUNTIME_ENV_WORKSPACE = "CLOUDTIK_WORKSPACE"
CLOUDTIK_RUNTIME_ENV_CLUSTER = "CLOUDTIK_CLUSTER"
CLOUDTIK_RUNTIME_ENV_HEAD_IP = "CLOUDTIK_HEAD_IP"
CLOUDTIK_RUNTIME_ENV_HEAD_HOST = "CLOUDTIK_HEAD_HOST"
CLOUDTIK_RUNTIME_ENV_NODE_ID = "CLOUDTIK_NODE_ID"
CLOUDTIK_RUNTIME_ENV_NODE_IP = "CLOUDTIK_NODE_IP"
CLOUDTIK_RUNTIME_ENV_NODE_HOST = "CLOUDTIK_NODE_HOST"
CLOUDTIK_RUNTIME_ENV_NODE_SEQ_ID = "CLOUDTIK_NODE_SEQ_ID"
CLOUDTIK_RUNTIME_ENV_NODE_TYPE = "CLOUDTIK_NODE_TYPE"
CLOUDTIK_RUNTIME_ENV_PROVIDER_TYPE = "CLOUDTIK_PROVIDER_TYPE"
CLOUDTIK_RUNTIME_ENV_PYTHON_VERSION = "CLOUDTIK_PYTHON_VERSION"
CLOUDTIK_RUNTIME_ENV_SECRETS = "CLOUDTIK_SECRETS"

# --- storage -----------------------------------------------------------------------------
CLOUDTIK_DATA_DISK_MOUNT_POINT = "/mnt/cloudtik"
CLOUDTIK_DATA_DISK_MOUNT_NAME_PREFIX = "data_disk_"
CLOUDTIK_FS_PATH = "/cloudtik/fs"
DEFAULT_PROXY_PORT = 6000

# --- MI355X / ROCm (new) -----------------------------------------------------------------
# GPU resource name used in node resources and scaling demands.  The reference uses "GPU"
# for NVIDIA devices; MI355X devices are reported under the same key so existing
# resource-based scaling configs keep working, with the accelerator type recorded separately.
CLOUDTIK_GPU_RESOURCE = "GPU"
CLOUDTIK_ACCELERATOR_TYPE_PREFIX = "accelerator_type:"
CLOUDTIK_ROCM_VISIBLE_ENVS = ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")
CLOUDTIK_GPU_HEALTH_TEMP_C = env_integer("CLOUDTIK_GPU_HEALTH_TEMP_C", 100)
# a worker whose GPUs stay unhealthy (RAS uncorrectable errors, over-temperature) this long
# is terminated and replaced by the scaler
CLOUDTIK_GPU_UNHEALTHY_TIMEOUT_S = env_integer("CLOUDTIK_GPU_UNHEALTHY_TIMEOUT_S", 60)
