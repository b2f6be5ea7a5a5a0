"""Workspace provider for local / on-premise / virtual clusters: the workspace-wide service
registry (global variables) is stored in a shared locked JSON file (the reference stores
them as head-node tags, providers/_private/local/workspace_provider.py)."""
from __future__ import annotations

import os
from typing import Any, Dict

from cloudtik_amd.core.provider_api import WorkspaceProvider
from cloudtik_amd.core.state.file_state_store import FileStateStore

STATE_DIR = os.path.expanduser(os.environ.get("CLOUDTIK_LOCAL_STATE_DIR", "~/.cloudtik/local"))


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

    def list_clusters(self, config):
        gv = self.store.get().get("global_variables", {})
        clusters = {}
        for k in gv:
            if k.startswith("service."):
                clusters.setdefault(k.split(".")[1], {})
        return clusters

    def publish_global_variables(self, cluster_config: Dict[str, Any], global_variables: Dict[str, Any]):
        with self.store.transaction() as st:
            st.setdefault("global_variables", {}).update(global_variables)

    def subscribe_global_variables(self, cluster_config: Dict[str, Any]) -> Dict[str, Any]:
        return dict(self.store.get().get("global_variables", {}))

    def unpublish_cluster(self, cluster_name: str):
        with self.store.transaction() as st:
            gv = st.setdefault("global_variables", {})
            for k in [k for k in gv if k.startswith(f"service.{cluster_name}.")]:
                gv.pop(k)

    def get_workspace_info(self, config):
        st = self.store.get()
        return {"name": self.workspace_name, "provider": self.provider_config.get("type"),
                "clusters": sorted(self.list_clusters(config) or {}),
                "global_variables": len(st.get("global_variables", {}))}
