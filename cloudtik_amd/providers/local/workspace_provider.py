"""Workspace provider for local / on-premise / virtual clusters, and the workspace-wide
service registry every provider type shares.

The registry (global variables) lives WITH THE CLUSTERS, as tags on their head nodes,
reached through the node provider (reference providers/_private/local/workspace_provider.py
:54-80 and aws/workspace_provider.py:57-91): ``publish`` tags this cluster's running head with
``x-<name>``; ``subscribe`` lists the running heads of every cluster of the workspace
(``NodeProvider.workspace_head_nodes``) and collects their ``x-`` tags.  So any machine that
reaches the provider -- a second CLI host, or a head node running discovery -- sees the same
registry, and a cluster's entries disappear with its head.  Long values are stored in
numbered pieces (cloud tag values are limited, e.g. 256 characters on EC2).

The workspace marker (created / resources) stays a small locked JSON file."""
from __future__ import annotations

import os
from typing import Any, Dict

from cloudtik_amd.core import tags as T
from cloudtik_amd.core.provider_api import WorkspaceProvider
from cloudtik_amd.core.state.file_state_store import FileStateStore

STATE_DIR = os.path.expanduser(os.environ.get("CLOUDTIK_LOCAL_STATE_DIR", "~/.cloudtik/local"))
TAG_VALUE_MAX = 240          # below EC2's 256-character tag value limit
_PIECE = "~"


def encode_global_variables(global_variables: Dict[str, Any]) -> Dict[str, str]:
    """{name: value} -> head-node tags: ``x-<name>``, or ``x-<name>~<i>`` pieces + a count."""
    out: Dict[str, str] = {}
    for name, value in global_variables.items():
        v = "" if value is None else str(value)
        key = T.CLOUDTIK_GLOBAL_VARIABLE_KEY.format(name)
        if len(v) <= TAG_VALUE_MAX:
            out[key] = v
            continue
        pieces = [v[i:i + TAG_VALUE_MAX] for i in range(0, len(v), TAG_VALUE_MAX)]
        out[key] = f"{_PIECE}{len(pieces)}"
        for i, piece in enumerate(pieces):
            out[f"{key}{_PIECE}{i}"] = piece
    return out


def decode_global_variables(tags: Dict[str, str]) -> Dict[str, str]:
    """Inverse of encode_global_variables over one head's tags."""
    prefix = T.CLOUDTIK_GLOBAL_VARIABLE_KEY_PREFIX
    out: Dict[str, str] = {}
    for key, value in tags.items():
        if not key.startswith(prefix) or _PIECE in key[len(prefix):]:
            continue
        name = key[len(prefix):]
        if value.startswith(_PIECE) and value[1:].isdigit():
            parts = [tags.get(f"{key}{_PIECE}{i}") for i in range(int(value[1:]))]
            if any(p is None for p in parts):
                continue                          # torn write: skip, the next read sees it whole
            value = "".join(parts)
        out[name] = value
    return out


class LocalWorkspaceProvider(WorkspaceProvider):
    def __init__(self, provider_config, workspace_name):
        super().__init__(provider_config, workspace_name)
        self.store = FileStateStore(os.path.join(STATE_DIR, f"workspace-{workspace_name}.json"))

    def create_workspace(self, config):
        with self.store.transaction() as st:
            st.setdefault("workspace", {"name": self.workspace_name, "created": True})
            st.setdefault("global_variables", {})

    def delete_workspace(self, config, delete_managed_storage=False, delete_managed_database=False):
        with self.store.transaction() as st:
            st.clear()
            st["nodes"] = {}

    def check_workspace_existence(self, config):
        from cloudtik_amd.core.workspace import Existence
        return Existence.COMPLETED if self.store.get().get("workspace") else Existence.NOT_EXIST

    def _node_provider(self, cluster_config: Dict[str, Any]):
        from cloudtik_amd.core.provider_factory import get_node_provider
        pc = dict(cluster_config.get("provider") or self.provider_config)
        return get_node_provider(pc, cluster_config.get("cluster_name") or f"{self.workspace_name}-registry")

    def workspace_heads(self, config: Dict[str, Any]) -> Dict[str, Dict[str, str]]:
        return self._node_provider(config).workspace_head_nodes(self.workspace_name)

    def list_clusters(self, config):
        clusters = {}
        for tags in self.workspace_heads(config).values():
            name = tags.get(T.CLOUDTIK_TAG_CLUSTER_NAME)
            if name:
                clusters[name] = {"head_status": tags.get(T.CLOUDTIK_TAG_NODE_STATUS)}
        return clusters

    def publish_global_variables(self, cluster_config: Dict[str, Any], global_variables: Dict[str, Any]):
        from cloudtik_amd.core.cluster_utils import get_head_node
        provider = self._node_provider(cluster_config)
        head = get_head_node(provider, cluster_config["cluster_name"])
        if head is None:
            raise RuntimeError(f"cluster {cluster_config['cluster_name']}: no running head node to publish "
                               f"global variables on")
        provider.set_node_tags(head, encode_global_variables(global_variables))

    def subscribe_global_variables(self, cluster_config: Dict[str, Any]) -> Dict[str, Any]:
        out: Dict[str, Any] = {}
        heads = self.workspace_heads(cluster_config)
        for key in sorted(heads):
            out.update(decode_global_variables(heads[key]))
        return out

    def unpublish_cluster(self, cluster_name: str):
        """Nothing to remove: the entries are tags of the cluster's head, gone with it."""

    def get_workspace_info(self, config):
        st = self.store.get()
        cfg = dict(config or {}, provider=(config or {}).get("provider") or self.provider_config)
        try:
            clusters = sorted(self.list_clusters(cfg) or {})
            n_vars = len(self.subscribe_global_variables(cfg))
        except Exception:  # noqa: BLE001 - provider unreachable: show the marker only
            clusters, n_vars = [], None
        return {"name": self.workspace_name, "provider": self.provider_config.get("type"),
                "created": bool(st.get("workspace")), "clusters": clusters, "global_variables": n_vars}
