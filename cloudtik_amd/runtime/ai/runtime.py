"""AI runtime: PyTorch-ROCm + RCCL training stack, MLflow tracking server, cloudtik-run.

Reference: runtime/ai/runtime.py:15 (AIRuntime), runtime/ai/utils.py:49-128 (config
discovery, env, service registration), scripts/install.sh:47-102 (framework install:
CUDA torch / Horovod / OpenMPI / oneAPI), configure.sh:92-123 (MLflow backend store and
artifact root), services.sh (mlflow server on head).

MI355X redesign:
* the framework stack is PyTorch-ROCm + this repository's HIP op library; GPU detection is
  AMD (``/dev/kfd`` + KFD topology / amdsmi) and ``AI_WITH_GPU`` is resolved per node;
* collectives are RCCL over xGMI (torch ``nccl`` backend) -- no Horovod/MPI/oneCCL install;
  the ``horovod`` launcher type is served by the built-in Horovod-compatible
  DistributedOptimizer (cloudtik_amd.parallel.horovod);
* the node environment carries the RCCL / HIP settings a one-process-per-GPU job needs.
"""
from __future__ import annotations

import os
from typing import Any, Dict, List

from cloudtik_amd.core import service_discovery as sd
from cloudtik_amd.runtime.common.runtime_base import RuntimeBase, standard_commands

MLFLOW_PORT = 5001
BUILT_IN_RUNTIME_AI = "ai"


def detect_amd_gpus() -> int:
    from cloudtik_amd.core.resources import detect_amd_gpu_count
    return detect_amd_gpu_count()


class AIRuntime(RuntimeBase):
    name = BUILT_IN_RUNTIME_AI

    def get_runtime_commands(self, cluster_config):
        return standard_commands(self.name)

    def get_defaults_config(self, cluster_config):
        return {"runtime": {"ai": {"with_gpu": "auto", "mlflow": {"port": MLFLOW_PORT},
                                   "rccl": {"min_channels": 32}}}}

    # ---------------------------------------------------------------- config pipeline
    def prepare_config(self, cluster_config):
        ai = cluster_config.setdefault("runtime", {}).setdefault("ai", {}) or {}
        cluster_config["runtime"]["ai"] = ai
        # MLflow backend store discovery: explicit database > discovered mysql/postgres
        if not ai.get("database"):
            types = cluster_config.get("runtime", {}).get("types", [])
            for db in ("mysql", "postgres"):
                if db in types:
                    ai["database"] = {"engine": db, "address": "$CLOUDTIK_HEAD_IP", "discovered": "cluster"}
                    break
        if not ai.get("hdfs_namenode_uri") and "hdfs" in cluster_config.get("runtime", {}).get("types", []):
            ai["hdfs_namenode_uri"] = "hdfs://$CLOUDTIK_HEAD_IP:8020"
        return cluster_config

    def validate_config(self, cluster_config):
        ai = cluster_config.get("runtime", {}).get("ai", {}) or {}
        wg = ai.get("with_gpu", "auto")
        if wg not in (True, False, "auto", "true", "false"):
            raise ValueError("runtime.ai.with_gpu must be true, false or auto")

    # ---------------------------------------------------------------- node env
    def with_environment_variables(self, config, provider, node_id):
        ai = (config or {}).get("runtime", {}).get("ai", {}) or {}
        wg = ai.get("with_gpu", "auto")
        if wg == "auto":
            ngpu = detect_amd_gpus()
            with_gpu = ngpu > 0
        else:
            with_gpu = str(wg).lower() == "true"
        env = {
            "AI_ENABLED": "true",
            "AI_WITH_GPU": "true" if with_gpu else "false",
            "MLFLOW_PORT": str((ai.get("mlflow") or {}).get("port", MLFLOW_PORT)),
            "MLFLOW_HOME": "$RUNTIME_PATH/mlflow",
        }
        if with_gpu:
            rccl = ai.get("rccl") or {}
            env.update({
                # one process per GPU over xGMI: many channels so rings cover all 7 links
                "NCCL_MIN_NCHANNELS": str(rccl.get("min_channels", 32)),
                "HSA_ENABLE_IPC_MODE_LEGACY": "0",
                "TORCH_NCCL_ASYNC_ERROR_HANDLING": "1",
                "MIOPEN_FIND_MODE": str(ai.get("miopen_find_mode", "FAST")),
            })
        db = ai.get("database") or {}
        if db:
            env["AI_DATABASE_ENGINE"] = db.get("engine", "")
            env["AI_DATABASE_HOST"] = db.get("address", "")
        if ai.get("hdfs_namenode_uri"):
            env["HDFS_NAMENODE_URI"] = ai["hdfs_namenode_uri"]
        return env

    # ---------------------------------------------------------------- services
    def get_runtime_services(self, cluster_config):
        cluster = cluster_config.get("cluster_name", "default")
        port = (cluster_config.get("runtime", {}).get("ai", {}).get("mlflow") or {}).get("port", MLFLOW_PORT)
        return {f"{cluster}-mlflow": sd.define_runtime_service(
            "ai", "mlflow", port, sd.SERVICE_DISCOVERY_PROTOCOL_HTTP,
            features=[sd.SERVICE_DISCOVERY_FEATURE_AI])}

    def get_head_service_ports(self):
        return {"mlflow": {"protocol": "http", "port": MLFLOW_PORT}}

    def get_runtime_endpoints(self, cluster_config, cluster_head_ip):
        return {"mlflow": {"name": "MLflow", "url": f"http://{cluster_head_ip}:{MLFLOW_PORT}"}}

    def cluster_booting_completed(self, cluster_config, head_node_id):
        # workspace registration happens through the cluster operator's service publisher
        return None

    def get_processes(self):
        return [["mlflow.server", False, "MLflow", "head"]]

    def get_logs(self):
        return {"mlflow": "$RUNTIME_PATH/mlflow/logs"}

    def get_dependencies(self):
        return ["mysql", "postgres", "mount"]

    def get_runnable_command(self, target, runtime_options):
        if target.endswith(".py"):
            return ["cloudtik-run"] + list(runtime_options or []) + [target]
        return None

    # ---------------------------------------------------------------- node-side steps
    def install_steps(self, head):
        # MI355X nodes are provisioned from a ROCm image: verify the stack, never fetch it
        return [
            "python3 -c 'import torch; assert torch.version.hip' 2>/dev/null || "
            "echo '[ai] PyTorch-ROCm not found: install torch for ROCm before using the AI runtime' >&2",
            "python3 -c 'import mlflow' 2>/dev/null || "
            "echo '[ai] mlflow not installed: the tracking server will not be started' >&2",
        ]

    def configure_steps(self, head):
        return ["mkdir -p $RUNTIME_PATH/mlflow/logs $RUNTIME_PATH/mlflow/artifacts"]

    def start_steps(self, head):
        if not head:
            return []
        return [
            "python3 -c 'import mlflow' 2>/dev/null || exit 0; "
            "STORE=${AI_DATABASE_ENGINE:+${AI_DATABASE_ENGINE}://cloudtik@${AI_DATABASE_HOST}/mlflow}; "
            "STORE=${STORE:-sqlite:///$RUNTIME_PATH/mlflow/mlflow.db}; "
            "nohup mlflow server --host 0.0.0.0 --port ${MLFLOW_PORT:-5001} --backend-store-uri $STORE "
            "--default-artifact-root ${HDFS_NAMENODE_URI:-$RUNTIME_PATH/mlflow/artifacts} "
            "> $RUNTIME_PATH/mlflow/logs/mlflow.log 2>&1 & echo $! > $RUNTIME_PATH/mlflow/mlflow.pid",
        ]

    def stop_steps(self, head):
        # stop exactly the server this node started (pid file), never by name pattern
        return ["P=$RUNTIME_PATH/mlflow/mlflow.pid; [ -f $P ] && kill $(cat $P) 2>/dev/null; rm -f $P; true"] \
            if head else []
