"""Cloud workspace provider (reference providers/_private/<cloud>/workspace_provider.py: VPC,
subnets, NAT, firewall, IAM and the global-variable registry).

``create_workspace`` / ``delete_workspace`` / ``check_workspace_existence`` run the cloud's
step plan (providers/cloud/workspace.py: GCP and Azure over REST, AWS over boto3) unless the
workspace is declared on an existing network (``provider.use_working_vpc`` /
``use_existing_network``) -- then only the registry below is set up.  The workspace-wide
service registry (publish / subscribe global variables) is the same shared JSON state for
every provider type, so service discovery between clusters of one workspace is provider
independent.  Aliyun / Huawei Cloud workspaces are step plans over the clouds' signed APIs
(providers/cloud/signed_workspace.py); a Kubernetes
workspace is its namespace, service accounts and RBAC plus the EKS / GKE / AKS workload
identity of the pods (providers/kubernetes/workspace.py)."""
from __future__ import annotations

from cloudtik_amd.providers.local.workspace_provider import LocalWorkspaceProvider


class CloudWorkspaceProvider(LocalWorkspaceProvider):
    def _plan(self):
        if self.provider_config.get("use_working_vpc") or self.provider_config.get("use_existing_network"):
            return None
        from cloudtik_amd.providers.cloud.workspace import cloud_workspace
        return cloud_workspace(self.provider_config, self.workspace_name)

    def _builder(self, config):
        from cloudtik_amd.providers.cloud.workspace import WorkspaceBuilder
        plan = self._plan()
        if plan is None:
            return None, None
        return plan, WorkspaceBuilder(plan.steps(config.get("provider", config)), log=self._log)

    @staticmethod
    def _log(msg):
        print(f"[workspace] {msg}", flush=True)

    def create_workspace(self, config):
        plan, b = self._builder(config)
        if b is not None:
            b.create()
        super().create_workspace(config)
        if plan is not None:
            with self.store.transaction() as st:
                st.setdefault("workspace", {})["resources"] = plan.info()

    def delete_workspace(self, config, delete_managed_storage=False, delete_managed_database=False):
        _, b = self._builder(config)
        if b is not None:
            b.delete(delete_managed_storage, delete_managed_database)
        super().delete_workspace(config, delete_managed_storage, delete_managed_database)

    def check_workspace_existence(self, config):
        _, b = self._builder(config)
        if b is None:
            return super().check_workspace_existence(config)
        return b.existence()

    def check_workspace_integrity(self, config) -> bool:
        from cloudtik_amd.core.workspace import Existence
        return self.check_workspace_existence(config) == Existence.COMPLETED

    def get_workspace_info(self, config):
        info = super().get_workspace_info(config)
        res = self.store.get().get("workspace", {}).get("resources")
        if res:
            info["resources"] = res
        return info
