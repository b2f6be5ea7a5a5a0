"""Managed storage / database providers (reference core/storage_provider.py,
core/database_provider.py and the per-cloud implementations: S3 / GCS / ADLS / OSS / OBS
buckets, RDS / Cloud SQL ...).  The interface is kept; on-premise MI355X deployments use the
hdfs / minio / mysql / postgres runtimes instead, so the managed-cloud variants report the
SDK they would need."""
from __future__ import annotations

from cloudtik_amd.core.provider_api import DatabaseProvider, StorageProvider


class CloudStorageProvider(StorageProvider):
    def create(self, config):
        raise NotImplementedError(f"managed storage on {self.provider_config.get('type')} needs the cloud SDK; "
                                  "use the hdfs or minio runtime for cluster storage")

    def delete(self, config):
        raise NotImplementedError("managed storage is not supported in this build")

    def get_info(self, config):
        return {"name": self.storage_name, "provider": self.provider_config.get("type"), "managed": False}


class CloudDatabaseProvider(DatabaseProvider):
    def create(self, config):
        raise NotImplementedError(f"managed databases on {self.provider_config.get('type')} need the cloud SDK; "
                                  "use the mysql or postgres runtime")

    def delete(self, config):
        raise NotImplementedError("managed databases are not supported in this build")

    def get_info(self, config):
        return {"name": self.storage_name, "provider": self.provider_config.get("type"), "managed": False}
