"""Node tags (labels) that carry control-plane state on the nodes themselves.

Same tag keys / values as the reference (``core/tags.py``): providers persist them with
each node, and the cluster operator / scaler read them back (tags-as-state).
"""

CLOUDTIK_TAG_NODE_NAME = "cloudtik-node-name"
CLOUDTIK_TAG_CLUSTER_NAME = "cloudtik-cluster-name"
CLOUDTIK_TAG_WORKSPACE_NAME = "cloudtik-workspace-name"

CLOUDTIK_TAG_NODE_KIND = "cloudtik-node-kind"
NODE_KIND_HEAD = "head"
NODE_KIND_WORKER = "worker"
NODE_KIND_UNMANAGED = "unmanaged"

CLOUDTIK_TAG_USER_NODE_TYPE = "cloudtik-user-node-type"

CLOUDTIK_TAG_NODE_STATUS = "cloudtik-node-status"
STATUS_UNINITIALIZED = "uninitialized"
STATUS_WAITING_FOR_SSH = "waiting-for-ssh"
STATUS_BOOTSTRAPPING_DATA_DISKS = "mounting-disks"
STATUS_SYNCING_FILES = "syncing-files"
STATUS_SETTING_UP = "setting-up"
STATUS_UPDATE_FAILED = "update-failed"
STATUS_UP_TO_DATE = "up-to-date"

CLOUDTIK_TAG_LAUNCH_CONFIG = "cloudtik-launch-config"
CLOUDTIK_TAG_RUNTIME_CONFIG = "cloudtik-runtime-config"
CLOUDTIK_TAG_FILE_MOUNTS_CONTENTS = "cloudtik-file-mounts-contents"

CLOUDTIK_GLOBAL_VARIABLE_KEY_PREFIX = "x-"
CLOUDTIK_GLOBAL_VARIABLE_KEY = CLOUDTIK_GLOBAL_VARIABLE_KEY_PREFIX + "{}"

CLOUDTIK_TAG_NODE_SEQ_ID = "cloudtik-node-seq-id"
CLOUDTIK_TAG_HEAD_NODE_SEQ_ID = 1

CLOUDTIK_TAG_QUORUM_ID = "cloudtik-quorum-id"
CLOUDTIK_TAG_QUORUM_JOIN = "cloudtik-quorum-join"
QUORUM_JOIN_STATUS_INIT = "init"
QUORUM_JOIN_STATUS_SUCCESS = "success"
QUORUM_JOIN_STATUS_FAILED = "failed"

NODE_STATUSES_UPDATING = (STATUS_WAITING_FOR_SSH, STATUS_BOOTSTRAPPING_DATA_DISKS,
                          STATUS_SYNCING_FILES, STATUS_SETTING_UP)
