"""Runtime plugin contract (reference ``core/runtime.py:13-292``).

A runtime contributes config defaults, config validation/bootstrap hooks, node
environment variables, install/configure/services steps, service definitions for
discovery, scaling policy, job waiter, health checks, logs and processes.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional


class Runtime:
    def __init__(self, runtime_config: Dict[str, Any]) -> None:
        self.runtime_config = runtime_config or {}

    # config pipeline
    def prepare_config(self, cluster_config: Dict[str, Any]) -> Dict[str, Any]:
        return cluster_config

    def validate_config(self, cluster_config: Dict[str, Any]):
        return None

    def bootstrap_config(self, cluster_config: Dict[str, Any]) -> Dict[str, Any]:
        return cluster_config

    def verify_config(self, cluster_config: Dict[str, Any]):
        return None

    def prepare_config_on_head(self, cluster_config: Dict[str, Any]) -> Dict[str, Any]:
        return cluster_config

    def bootstrap_config_on_head(self, cluster_config: Dict[str, Any]) -> Dict[str, Any]:
        return cluster_config

    # node side
    def with_environment_variables(self, config: Dict[str, Any], provider, node_id: str) -> Dict[str, Any]:
        return {}

    def node_configure(self, head: bool):
        return None

    def node_services(self, command: str, head: bool):
        return None

    def get_runtime_shared_memory_ratio(self, runtime_config, config, node_type: str) -> float:
        return 0.0

    def cluster_booting_completed(self, cluster_config: Dict[str, Any], head_node_id: str) -> None:
        return None

    def get_runnable_command(self, target: str, runtime_options: Optional[List[str]]):
        return None

    def get_runtime_commands(self, cluster_config: Dict[str, Any]) -> Dict[str, Any]:
        return {}

    def get_defaults_config(self, cluster_config: Dict[str, Any]) -> Dict[str, Any]:
        return {}

    def get_runtime_endpoints(self, cluster_config: Dict[str, Any], cluster_head_ip: str):
        return {}

    def get_head_service_ports(self) -> Dict[str, Any]:
        return {}

    def get_runtime_services(self, cluster_config: Dict[str, Any]):
        return {}

    def get_node_constraints(self, cluster_config: Dict[str, Any], node_type: Optional[str] = None):
        """None, or (needs minimal nodes before setup, forms a quorum, quorum can grow) for the
        given worker node type (reference core/runtime.py:193)."""
        return None

    def node_constraints_reached(self, cluster_config, node_type, head_info, nodes_info, quorum_id=None):
        return None

    def get_scaling_policy(self, cluster_config: Dict[str, Any], head_ip: str):
        return None

    def get_job_waiter(self, cluster_config: Dict[str, Any]):
        return None

    def get_health_check(self, cluster_config: Dict[str, Any]):
        return None

    def get_logs(self) -> Dict[str, List[str]]:
        return {}

    def get_processes(self) -> List[List]:
        return []

    @staticmethod
    def get_dependencies() -> List[str]:
        return []

    @staticmethod
    def get_required() -> List[str]:
        return []
