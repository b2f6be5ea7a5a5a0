"""Cloud workspace provider (reference providers/_private/<cloud>/workspace_provider.py: VPC,
subnets, NAT, firewall, IAM and the global-variable registry stored as cloud tags).

Here the workspace-wide service registry (publish / subscribe global variables) works for
every provider type through a shared JSON state file, so service discovery between
clusters of one workspace is provider independent; creating cloud network resources
requires the provider SDK and is not part of this build."""
from __future__ import annotations

from cloudtik_amd.providers.local.workspace_provider import LocalWorkspaceProvider


class CloudWorkspaceProvider(LocalWorkspaceProvider):
    def create_workspace(self, config):
        ptype = self.provider_config.get("type")
        if not self.provider_config.get("use_existing_network", True):
            raise NotImplementedError(f"{ptype}: creating cloud network resources is not supported in this build; "
                                      "set provider.use_existing_network")
        super().create_workspace(config)
