"""Spark runtime cluster API (reference runtime/spark/api.py:10-60): ``SparkCluster`` /
``ThisSparkCluster`` add YARN application queries (ResourceManager REST API on the head,
reached through an ssh tunnel from outside the cluster), the runtime's default storage and
its service endpoints."""
from __future__ import annotations

import json
from typing import Any, Dict, Optional

from cloudtik_amd.core.api import Cluster, ThisCluster

YARN_WEB_PORT = 8088


def request_rest_applications(config: Dict[str, Any], endpoint: str = "", on_head: bool = False) -> Dict[str, Any]:
    """GET ws/v1/cluster/apps[/<endpoint>] from the YARN ResourceManager."""
    from cloudtik_amd.core.cluster_tunnel_request import _request_rest_to_head
    path = "ws/v1/cluster/apps" + (f"/{endpoint.lstrip('/')}" if endpoint else "")
    return json.loads(_request_rest_to_head(config, path, YARN_WEB_PORT, on_head=on_head) or b"{}")


def get_runtime_default_storage(config: Dict[str, Any]) -> Optional[Dict[str, Any]]:
    """fs.defaultFS of the cluster: HDFS in the cluster, a workspace HDFS/MinIO service, or
    the provider's managed cloud storage."""
    from cloudtik_amd.core.cluster_operator import get_head_node_ip
    from cloudtik_amd.runtime.common import discovery
    head = get_head_node_ip(config, missing_ok=True)
    uri = discovery.discover_service("hdfs", config, head_ip=head, consumer="spark")
    if uri:
        return {"default_storage_uri": uri}
    uri = discovery.discover_service("minio", config, head_ip=head, consumer="spark")
    if uri:
        return {"default_storage_uri": "s3a://", "endpoint": uri}
    storage = (config.get("provider") or {}).get("storage") or {}
    return {"default_storage_uri": storage.get("uri")} if storage.get("uri") else None


class _SparkOps:
    def applications(self, endpoint: str = "") -> Dict[str, Any]:
        return request_rest_applications(self.config, endpoint, on_head=isinstance(self, ThisCluster))

    def get_default_storage(self):
        return get_runtime_default_storage(self.config)

    def get_endpoints(self) -> Dict[str, Any]:
        return self.get_runtime_endpoints()


class SparkCluster(_SparkOps, Cluster):
    pass


class ThisSparkCluster(_SparkOps, ThisCluster):
    pass
