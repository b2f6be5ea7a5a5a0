"""Public Python API (reference core/api.py:22-980): ``Workspace``, ``Cluster`` (drive a
cluster from anywhere) and ``ThisCluster`` (the same operations from ON the head, against
its bootstrap config).

    from cloudtik_amd.core.api import Cluster
    c = Cluster("cluster.yaml")
    c.start()
    c.wait_for_ready(min_workers=2)
    c.submit("train.py", ["--epochs", "3"])
    print(c.get_info())
    c.stop()
"""
from __future__ import annotations

import os
from typing import Any, Callable, Dict, List, Optional, Union

import yaml

from cloudtik_amd.core import cluster_operator as op
from cloudtik_amd.core import tags as T
from cloudtik_amd.core.event_system import CreateClusterEvent, global_event_system

DEFAULT_HEAD_CONFIG = "~/cloudtik_bootstrap_config.yaml"


def _load_dict(cfg: Union[dict, str]) -> Dict[str, Any]:
    if isinstance(cfg, dict):
        return cfg
    from cloudtik_amd.core.config.loader import load_config_file
    return load_config_file(cfg)


class Workspace:
    def __init__(self, workspace_config: Union[dict, str]) -> None:
        from cloudtik_amd.core import workspace as ws
        self._ws = ws
        self.config = ws.prepare_workspace_config(_load_dict(workspace_config))

    def create(self) -> None:
        self._ws.create_workspace(self.config)

    def delete(self, delete_managed_storage: bool = False, delete_managed_database: bool = False) -> None:
        self._ws.delete_workspace(self.config, delete_managed_storage, delete_managed_database)

    def update(self) -> None:
        self._ws.update_workspace(self.config)

    def get_status(self):
        return self._ws.workspace_status(self.config)

    def get_info(self) -> Dict[str, Any]:
        return self._ws.workspace_info(self.config)

    def list_clusters(self) -> Optional[Dict[str, Any]]:
        return self._ws.list_workspace_clusters(self.config)


class _ClusterOps:
    """Operations shared by Cluster and ThisCluster; ``self.config`` is bootstrapped."""
    config: Dict[str, Any]

    def exec(self, cmd: str, node_ip: Optional[str] = None, all_nodes: bool = False, with_output: bool = False,
             run_env: str = "auto", env: Optional[Dict[str, Any]] = None):
        return op.exec_cluster(self.config, cmd, node_ip, all_nodes, with_output, run_env, env=env)

    def run(self, script: str, script_args: Optional[List[str]] = None, node_ip: Optional[str] = None,
            with_output: bool = False):
        return op.submit_and_exec(self.config, script, script_args, node_ip, with_output=with_output)

    def rsync(self, source: str, target: str, down: bool, node_ip: Optional[str] = None, all_workers: bool = False):
        return op.rsync(self.config, source, target, down, node_ip, all_workers)

    def scale(self, num_cpus: Optional[int] = None, num_gpus: Optional[int] = None, workers: Optional[int] = None,
              worker_type: Optional[str] = None, resources: Optional[Dict[str, float]] = None,
              up_only: bool = False) -> Dict[str, Any]:
        return op.scale_cluster(self.config, num_cpus, num_gpus, workers, worker_type, resources, up_only)

    def start_node(self, node_ip: Optional[str] = None, all_nodes: bool = False):
        """Re-run the start commands of a node (restart its CloudTik daemons and runtimes)."""
        from cloudtik_amd.core.cluster_config import merged_commands_for
        return self._run_node_commands("start", node_ip, all_nodes)

    def stop_node(self, node_ip: Optional[str] = None, all_nodes: bool = False):
        return self._run_node_commands("stop", node_ip, all_nodes)

    def _run_node_commands(self, stage: str, node_ip, all_nodes):
        from cloudtik_amd.core.cluster_config import merged_commands_for
        provider = op._provider(self.config)
        nodes = provider.non_terminated_nodes({T.CLOUDTIK_TAG_CLUSTER_NAME: self.config["cluster_name"]}) \
            if all_nodes else [op._node_by_ip(self.config, provider, node_ip)]
        for n in nodes:
            head = provider.node_tags(n).get(T.CLOUDTIK_TAG_NODE_KIND) == T.NODE_KIND_HEAD
            ip = provider.internal_ip(n)
            for cmd in merged_commands_for(self.config, head, stage):
                op.exec_cluster(self.config, cmd, node_ip=ip, env={"CLOUDTIK_NODE_IP": ip})

    def kill_node(self, node_ip: Optional[str] = None, hard: bool = False) -> Optional[str]:
        return op.kill_node(self.config, node_ip, hard)

    def get_head_node_ip(self, public: bool = False) -> str:
        return op.get_head_node_ip(self.config)

    def get_worker_node_ips(self, runtime: Optional[str] = None, node_status: Optional[str] = None) -> List[str]:
        return op.get_worker_node_ips(self.config, runtime, node_status)

    def get_head_node_host(self) -> str:
        return self.get_head_node_ip()

    def get_worker_node_hosts(self, node_status: Optional[str] = None) -> List[str]:
        return self.get_worker_node_ips(node_status=node_status)

    def get_nodes(self) -> List[Dict[str, Any]]:
        return op.get_cluster_nodes_info(self.config)

    def get_info(self) -> Dict[str, Any]:
        return op.get_cluster_info(self.config)

    def wait_for_ready(self, min_workers: Optional[int] = None, timeout: Optional[int] = None) -> int:
        kw = {"timeout": timeout} if timeout else {}
        return op.wait_for_ready(self.config, min_workers, **kw)

    def get_default_cloud_storage(self):
        return op._provider(self.config).get_default_cloud_storage()

    def get_default_cloud_database(self):
        return op._provider(self.config).get_default_cloud_database()

    def health_check(self) -> Dict[str, Any]:
        return op.health_check(self.config)

    def get_runtime_endpoints(self) -> Dict[str, Any]:
        return self.get_info().get("endpoints", {})


class Cluster(_ClusterOps):
    def __init__(self, cluster_config: Union[dict, str], should_bootstrap: bool = True, no_config_cache: bool = True,
                 verbosity: Optional[int] = None, skip_runtime_bootstrap: bool = False) -> None:
        from cloudtik_amd.core.cluster_config import bootstrap_config
        cfg = _load_dict(cluster_config)
        cfg.setdefault("cluster_name", "default")
        self.config = bootstrap_config(cfg, no_config_cache) if should_bootstrap else cfg
        self.verbosity = verbosity

    def start(self, no_restart: bool = False, restart_only: bool = False) -> None:
        op.create_or_update_cluster(self.config, no_restart=no_restart, restart_only=restart_only)

    def stop(self, workers_only: bool = False, keep_min_workers: bool = False, hard: bool = False) -> None:
        op.teardown_cluster(self.config, workers_only, keep_min_workers, hard=hard)

    def submit(self, script_file: str, script_args: Optional[List[str]] = None, job_waiter: Optional[str] = None,
               with_output: bool = False):
        return op.submit_and_exec(self.config, script_file, script_args, job_waiter=job_waiter,
                                  with_output=with_output)

    def register_callback(self, event: CreateClusterEvent, callback: Callable[[Dict[str, Any]], None]) -> None:
        global_event_system.add_callback_handler(event, callback, self.config["cluster_name"])


class ThisCluster(_ClusterOps):
    """On the head node: operations against the head's bootstrap config."""

    def __init__(self, verbosity: Optional[int] = None, config_file: str = DEFAULT_HEAD_CONFIG) -> None:
        path = os.path.expanduser(config_file)
        if not os.path.exists(path):
            raise RuntimeError(f"not running on a cluster head ({path} is missing)")
        with open(path) as f:
            self.config = yaml.safe_load(f)
        self.verbosity = verbosity
