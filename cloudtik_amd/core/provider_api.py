"""Workspace / storage / database / load-balancer provider contracts, scaling policy and
job waiter contracts (reference: core/workspace_provider.py, core/storage_provider.py,
core/database_provider.py, core/load_balancer_provider.py, core/scaling_policy.py,
core/job_waiter.py)."""
from __future__ import annotations

from typing import Any, Dict, List, Optional


class WorkspaceProvider:
    """Shared infrastructure of a set of clusters plus the workspace-wide service registry
    (``publish/subscribe_global_variables``)."""

    def __init__(self, provider_config: Dict[str, Any], workspace_name: str):
        self.provider_config = provider_config
        self.workspace_name = workspace_name

    def create_workspace(self, config: Dict[str, Any]):
        return None

    def delete_workspace(self, config: Dict[str, Any], delete_managed_storage: bool = False,
                         delete_managed_database: bool = False):
        return None

    def update_workspace(self, config: Dict[str, Any], delete_managed_storage: bool = False,
                         delete_managed_database: bool = False):
        return None

    def check_workspace_existence(self, config: Dict[str, Any]):
        from cloudtik_amd.core.workspace import Existence
        return Existence.COMPLETED

    def check_workspace_integrity(self, config: Dict[str, Any]) -> bool:
        return True

    def list_clusters(self, config: Dict[str, Any]) -> Optional[Dict[str, Any]]:
        return None

    def list_storages(self, config):
        return None

    def list_databases(self, config):
        return None

    def publish_global_variables(self, cluster_config: Dict[str, Any], global_variables: Dict[str, Any]):
        raise NotImplementedError

    def subscribe_global_variables(self, cluster_config: Dict[str, Any]) -> Dict[str, Any]:
        raise NotImplementedError

    def get_workspace_info(self, config: Dict[str, Any]):
        return {}

    @staticmethod
    def validate_config(provider_config):
        return None

    @staticmethod
    def bootstrap_workspace_config(config):
        return config


class StorageProvider:
    def __init__(self, provider_config: Dict[str, Any], workspace_name: str, storage_name: str):
        self.provider_config = provider_config
        self.workspace_name = workspace_name
        self.storage_name = storage_name

    def create(self, config):
        raise NotImplementedError

    def delete(self, config):
        raise NotImplementedError

    def get_info(self, config):
        return {}

    @staticmethod
    def validate_config(provider_config):
        return None

    @staticmethod
    def bootstrap_config(config):
        return config


class DatabaseProvider(StorageProvider):
    pass


class LoadBalancerProvider:
    """Load balancers of a workspace (reference core/load_balancer_provider.py).

    A load balancer config is ``{"name", "type": "network"|"application", "scheme":
    "internet-facing"|"internal", "tags", "service_groups": [{"listeners": [{"protocol",
    "port"}], "services": [{"name", "protocol", "port", "route_path", "service_path",
    "default", "targets": [{"address", "port", "node_id", "seq_id"}]}]}]}``; ``list`` maps
    name -> ``{"name", "type", "scheme", "tags", ...provider ids}``.  Implementations:
    core/load_balancer.py (HAProxy on the node, for local / on-premise) and
    providers/cloud/load_balancer.py (AWS ELBv2, GCP, Azure)."""

    def __init__(self, provider_config: Dict[str, Any], workspace_name: str):
        self.provider_config = provider_config
        self.workspace_name = workspace_name

    def support_multi_service_group(self) -> bool:
        return True

    def list(self) -> Dict[str, Dict[str, Any]]:
        raise NotImplementedError

    def get(self, load_balancer_name: str) -> Optional[Dict[str, Any]]:
        return self.list().get(load_balancer_name)

    def create(self, load_balancer_config: Dict[str, Any]):
        raise NotImplementedError

    def update(self, load_balancer: Dict[str, Any], load_balancer_config: Dict[str, Any]):
        raise NotImplementedError

    def delete(self, load_balancer: Dict[str, Any]):
        raise NotImplementedError

    def validate_config(self, provider_config: Dict[str, Any]):
        return None

    @staticmethod
    def bootstrap_config(config: Dict[str, Any], provider_config: Dict[str, Any]) -> Dict[str, Any]:
        return provider_config


class ScalingState:
    """What a scaling policy tells the scaler: autoscaling instructions (resource demands
    / requests), per-node resource states, lost nodes."""

    def __init__(self, autoscaling_instructions=None, node_resource_states=None, lost_nodes=None):
        self.autoscaling_instructions = autoscaling_instructions
        self.node_resource_states = node_resource_states
        self.lost_nodes = lost_nodes


class ScalingPolicy:
    def __init__(self, config: Dict[str, Any], head_ip: str) -> None:
        self.config = config
        self.head_ip = head_ip

    def name(self) -> str:
        raise NotImplementedError

    def reset(self, config):
        self.config = config

    def get_scaling_state(self) -> Optional[ScalingState]:
        return None


class JobWaiter:
    def __init__(self, config: Dict[str, Any] = None) -> None:
        self.config = config

    def wait_for_completion(self, node_id: str, cmd: str, session_name: str = None, timeout: int = None):
        raise NotImplementedError
