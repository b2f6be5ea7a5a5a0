"""Managed storage / database providers (reference core/storage_provider.py,
core/database_provider.py and the per-cloud implementations).

A managed bucket / database belongs to a workspace: these providers run only the managed
steps of the workspace's step plan (providers/cloud/workspace.py) -- GCS bucket / Cloud SQL,
ADLS Gen2 account + container / MySQL flexible server, S3 bucket / RDS -- so ``cloudtik
storage create`` and ``cloudtik workspace create`` with ``managed_cloud_storage`` build the
same resource; Aliyun / Huawei Cloud manage an OSS / OBS bucket the same way
(providers/cloud/signed_workspace.py; reference aliyun/storage_provider.py,
huaweicloud/storage_provider.py).  Neither of those two clouds has a managed database in the
reference: the mysql / postgres runtimes serve their clusters."""
from __future__ import annotations

from cloudtik_amd.core.provider_api import DatabaseProvider, StorageProvider


class _ManagedSteps:
    KIND = ""

    def _steps(self, config):
        from cloudtik_amd.providers.cloud.workspace import WorkspaceBuilder, cloud_workspace
        plan = cloud_workspace(self.provider_config, self.workspace_name)
        if plan is None:
            raise NotImplementedError(f"managed {self.KIND} on {self.provider_config.get('type')}: use the "
                                      f"{'hdfs or minio' if self.KIND == 'storage' else 'mysql or postgres'} runtime")
        flags = {"managed_cloud_storage": self.KIND == "storage", "managed_cloud_database": self.KIND == "database"}
        steps = [s for s in plan.steps(dict(config.get("provider", {}), **flags)) if s.managed == self.KIND]
        if not steps:
            raise NotImplementedError(f"managed {self.KIND} on {self.provider_config.get('type')}: use the "
                                      f"{'hdfs or minio' if self.KIND == 'storage' else 'mysql or postgres'} runtime")
        return plan, WorkspaceBuilder(steps, log=lambda m: print(f"[{self.KIND}] {m}", flush=True))

    def create(self, config):
        return self._steps(config)[1].create()

    def delete(self, config):
        kw = {"delete_managed_storage": self.KIND == "storage", "delete_managed_database": self.KIND == "database"}
        return self._steps(config)[1].delete(**kw)

    def get_info(self, config):
        plan, b = self._steps(config)
        info = plan.info()
        key = "bucket" if self.KIND == "storage" else "database"
        return {"name": self.storage_name, "provider": self.provider_config.get("type"), "managed": True,
                key: info.get(key, info.get("storage_account")), "exists": all(b.status().values())}


class CloudStorageProvider(_ManagedSteps, StorageProvider):
    KIND = "storage"


class CloudDatabaseProvider(_ManagedSteps, DatabaseProvider):
    KIND = "database"
