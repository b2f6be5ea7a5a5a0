"""NodeProvider: the contract every infrastructure backend implements.

Method set and semantics follow the reference ``core/node_provider.py:52-381`` so that
existing provider configs / external provider classes port over unchanged.  Nodes are
identified by opaque string ids; all control-plane state about a node lives in its tags
(see core.tags).
"""
from __future__ import annotations

import contextlib
import copy
import threading
from typing import Any, Dict, List, Optional


class NodeLaunchException(Exception):
    """A structured launch failure (records category + description for the availability
    tracker, reference node_launcher.py:97)."""

    def __init__(self, category: str, description: str, src_exc_info=None):
        super().__init__(f"{category}: {description}")
        self.category = category
        self.description = description
        self.src_exc_info = src_exc_info


class NodeProvider:
    def __init__(self, provider_config: Dict[str, Any], cluster_name: str) -> None:
        self.provider_config = provider_config
        self.cluster_name = cluster_name
        self._internal_ip_cache: Dict[str, str] = {}
        self._external_ip_cache: Dict[str, str] = {}

    # ------------------------------------------------------------------ queries
    def non_terminated_nodes(self, tag_filters: Dict[str, str]) -> List[str]:
        raise NotImplementedError

    # A provider instance is bound to one cluster: its listing filters on the cluster-name tag.
    # The workspace registry needs the head nodes of EVERY cluster of a workspace (reference
    # providers/_private/aws/workspace_provider.py:57-91 _get_workspace_head_nodes): inside
    # ``workspace_scope()`` the cloud providers drop the cluster filter (thread-local, so a
    # scaler thread sharing the instance keeps its own scope).
    _scope = threading.local()

    @contextlib.contextmanager
    def workspace_scope(self):
        prev = getattr(self._scope, "all_clusters", False)
        self._scope.all_clusters = True
        try:
            yield
        finally:
            self._scope.all_clusters = prev

    def cluster_filter(self) -> Dict[str, str]:
        """The cluster-name tag filter this instance lists with ({} in a workspace scope)."""
        if getattr(self._scope, "all_clusters", False):
            return {}
        from cloudtik_amd.core import tags as T
        return {T.CLOUDTIK_TAG_CLUSTER_NAME: self.cluster_name}

    def workspace_head_nodes(self, workspace_name: str) -> Dict[str, Dict[str, str]]:
        """Running head nodes of every cluster in ``workspace_name``: {key: tags}.  The keys
        are opaque (a head of another cluster may not be addressable through this instance)."""
        from cloudtik_amd.core import tags as T
        with self.workspace_scope():
            ids = self.non_terminated_nodes({T.CLOUDTIK_TAG_WORKSPACE_NAME: workspace_name,
                                             T.CLOUDTIK_TAG_NODE_KIND: T.NODE_KIND_HEAD})
            return {i: self.node_tags(i) for i in ids}

    def is_running(self, node_id: str) -> bool:
        raise NotImplementedError

    def is_terminated(self, node_id: str) -> bool:
        raise NotImplementedError

    def node_tags(self, node_id: str) -> Dict[str, str]:
        raise NotImplementedError

    def external_ip(self, node_id: str) -> Optional[str]:
        raise NotImplementedError

    def internal_ip(self, node_id: str) -> Optional[str]:
        raise NotImplementedError

    def get_node_id(self, ip_address: str, use_internal_ip: bool = False) -> str:
        def find(ip_fn, cache):
            if ip_address in cache:
                return cache[ip_address]
            for nid in self.non_terminated_nodes({}):
                ip = ip_fn(nid)
                cache[ip] = nid
                if ip == ip_address:
                    return nid
            return None
        nid = (find(self.internal_ip, self._internal_ip_cache) if use_internal_ip
               else find(self.external_ip, self._external_ip_cache))
        if nid is None:
            raise ValueError(f"no node with ip {ip_address}")
        return nid

    # ------------------------------------------------------------------ mutations
    def create_node(self, node_config: Dict[str, Any], tags: Dict[str, str], count: int) -> Optional[Dict[str, Any]]:
        raise NotImplementedError

    def create_node_with_resources(self, node_config, tags, count, resources):
        return self.create_node(node_config, tags, count)

    def set_node_tags(self, node_id: str, tags: Dict[str, str]) -> None:
        raise NotImplementedError

    def terminate_node(self, node_id: str) -> Optional[Dict[str, Any]]:
        raise NotImplementedError

    def terminate_nodes(self, node_ids: List[str]) -> Optional[Dict[str, Any]]:
        for nid in node_ids:
            self.terminate_node(nid)
        return None

    # ------------------------------------------------------------------ execution
    def get_command_executor(self, call_context, log_prefix: str, node_id: str, auth_config,
                             cluster_name: str, process_runner, use_internal_ip: bool,
                             docker_config=None):
        from cloudtik_amd.core.executor import create_default_command_executor
        return create_default_command_executor(
            call_context, log_prefix, node_id, self, auth_config, cluster_name, process_runner,
            use_internal_ip, docker_config)

    # ------------------------------------------------------------------ config hooks
    def prepare_config_for_head(self, cluster_config: Dict[str, Any], remote_config: Dict[str, Any]):
        return remote_config

    def prepare_node_config_for_launch_hash(self, node_config: Dict[str, Any]) -> Dict[str, Any]:
        return node_config

    def prepare_config_for_runtime_hash(self, cluster_config: Dict[str, Any]) -> Dict[str, Any]:
        return cluster_config

    def cleanup_cluster(self, cluster_config: Dict[str, Any], deep: bool = False):
        pass

    def get_node_info(self, node_id: str) -> Dict[str, str]:
        tags = self.node_tags(node_id)
        from cloudtik_amd.core import tags as T
        return {
            "node_id": node_id,
            "instance_type": tags.get("instance_type", ""),
            "private_ip": self.internal_ip(node_id),
            "public_ip": self.external_ip(node_id),
            "instance_status": "running" if self.is_running(node_id) else "terminated",
            T.CLOUDTIK_TAG_NODE_KIND: tags.get(T.CLOUDTIK_TAG_NODE_KIND),
            T.CLOUDTIK_TAG_NODE_STATUS: tags.get(T.CLOUDTIK_TAG_NODE_STATUS),
            T.CLOUDTIK_TAG_USER_NODE_TYPE: tags.get(T.CLOUDTIK_TAG_USER_NODE_TYPE),
            T.CLOUDTIK_TAG_NODE_SEQ_ID: tags.get(T.CLOUDTIK_TAG_NODE_SEQ_ID),
        }

    def with_environment_variables(self, node_type_config: Dict[str, Any], node_id: str):
        return {}

    def get_default_cloud_storage(self):
        return None

    def get_default_cloud_database(self):
        return None

    # ------------------------------------------------------------------ static config pipeline
    @staticmethod
    def prepare_config(cluster_config: Dict[str, Any]) -> Dict[str, Any]:
        return cluster_config

    @staticmethod
    def post_prepare(cluster_config: Dict[str, Any]) -> Dict[str, Any]:
        return cluster_config

    @staticmethod
    def validate_config(provider_config: Dict[str, Any]) -> None:
        return None

    @staticmethod
    def bootstrap_config(cluster_config: Dict[str, Any]) -> Dict[str, Any]:
        return cluster_config

    @staticmethod
    def bootstrap_config_for_api(cluster_config: Dict[str, Any]) -> Dict[str, Any]:
        return cluster_config

    @staticmethod
    def verify_config(provider_config: Dict[str, Any]) -> None:
        return None

    @staticmethod
    def fillout_available_node_types_resources(cluster_config: Dict[str, Any]) -> Dict[str, Any]:
        return cluster_config


def copy_config(c):
    return copy.deepcopy(c)
