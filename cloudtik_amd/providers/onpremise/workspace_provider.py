"""On-premise workspaces live in the cloud simulator that owns the pool (reference
providers/_private/onpremise/workspace_provider.py + workspace_config.py): create / delete /
existence are simulator calls, so every CLI host of the pool sees the same workspaces; the
service registry is the head-node tags of the workspace's clusters, as for every provider
(providers/local/workspace_provider.py), listed through the simulator."""
from __future__ import annotations

from cloudtik_amd.providers.local.workspace_provider import LocalWorkspaceProvider


class OnPremiseWorkspaceProvider(LocalWorkspaceProvider):
    def _client(self, config=None):
        from cloudtik_amd.providers.onpremise.node_provider import SimulatorClient
        from cloudtik_amd.providers.onpremise.simulator import simulator_address
        pc = (config or {}).get("provider") or self.provider_config
        return SimulatorClient(simulator_address(pc.get("cloud_simulator_address")))

    def create_workspace(self, config):
        if self._client(config).call("get_workspace", workspace_name=self.workspace_name) is None:
            self._client(config).call("create_workspace", workspace_name=self.workspace_name)

    def delete_workspace(self, config, delete_managed_storage=False, delete_managed_database=False):
        if self._client(config).call("get_workspace", workspace_name=self.workspace_name) is not None:
            self._client(config).call("delete_workspace", workspace_name=self.workspace_name)

    def check_workspace_existence(self, config):
        from cloudtik_amd.core.workspace import Existence
        got = self._client(config).call("get_workspace", workspace_name=self.workspace_name)
        return Existence.COMPLETED if got is not None else Existence.NOT_EXIST

    def check_workspace_integrity(self, config) -> bool:
        from cloudtik_amd.core.workspace import Existence
        return self.check_workspace_existence(config) == Existence.COMPLETED

    def get_workspace_info(self, config):
        info = super().get_workspace_info(config)
        info["created"] = self.check_workspace_existence(config).name == "COMPLETED"
        return info
