"""Public-cloud node providers (reference providers/_private/{aws,gcp,azure,aliyun,
huaweicloud}/node_provider.py; SURVEY.md §2.9 "keep interface; not needed for the MI355X
node").

The provider interface, config schema, defaults and instance templates are kept so cluster
YAML stays portable.  ``AWSNodeProvider`` is implemented against boto3 (EC2 instances as
nodes, tags as node tags, ``cloudtik-cluster-name`` filters); it needs boto3 and
credentials at run time.  GCP and Azure are implemented over their REST APIs in
rest_providers.py, Aliyun and Huawei Cloud over their signed HTTP APIs in signed_providers.py.
"""
from __future__ import annotations

import importlib
from typing import Any, Dict, List

from cloudtik_amd.core import tags as T
from cloudtik_amd.core.node_provider import NodeLaunchException, NodeProvider


def _require(module: str, provider: str):
    try:
        return importlib.import_module(module)
    except ImportError as e:
        raise RuntimeError(f"the {provider} provider needs the '{module}' package (pip install {module}); "
                           "it is not available in this environment") from e


class AWSNodeProvider(NodeProvider):
    """EC2-backed nodes (reference providers/_private/aws/node_provider.py)."""

    def __init__(self, provider_config, cluster_name):
        super().__init__(provider_config, cluster_name)
        boto3 = _require("boto3", "aws")
        self.ec2 = boto3.resource("ec2", region_name=provider_config.get("region"))
        self.client = self.ec2.meta.client
        self._cache: Dict[str, Any] = {}

    def _filters(self, tag_filters):
        f = [{"Name": "instance-state-name", "Values": ["pending", "running"]},
             {"Name": f"tag:{T.CLOUDTIK_TAG_CLUSTER_NAME}", "Values": [self.cluster_name]}]
        f += [{"Name": f"tag:{k}", "Values": [v]} for k, v in tag_filters.items()]
        return f

    def non_terminated_nodes(self, tag_filters):
        nodes = list(self.ec2.instances.filter(Filters=self._filters(tag_filters)))
        self._cache.update({n.id: n for n in nodes})
        return [n.id for n in nodes]

    def _node(self, node_id):
        n = self._cache.get(node_id)
        if n is None:
            n = self.ec2.Instance(node_id)
            self._cache[node_id] = n
        return n

    def is_running(self, node_id):
        return self._node(node_id).state["Name"] == "running"

    def is_terminated(self, node_id):
        return self._node(node_id).state["Name"] not in ("running", "pending")

    def node_tags(self, node_id):
        return {t["Key"]: t["Value"] for t in (self._node(node_id).tags or [])}

    def external_ip(self, node_id):
        return self._node(node_id).public_ip_address

    def internal_ip(self, node_id):
        return self._node(node_id).private_ip_address

    def create_node(self, node_config, tags, count):
        conf = dict(node_config)
        tags = dict(tags, **{T.CLOUDTIK_TAG_CLUSTER_NAME: self.cluster_name})
        conf.setdefault("TagSpecifications", []).append(
            {"ResourceType": "instance", "Tags": [{"Key": k, "Value": v} for k, v in tags.items()]})
        conf["MinCount"] = conf["MaxCount"] = count
        if "instance_type" in conf:
            conf["InstanceType"] = conf.pop("instance_type")
        try:
            created = self.ec2.create_instances(**conf)
        except Exception as e:  # noqa: BLE001 -- botocore ClientError
            raise NodeLaunchException(getattr(e, "response", {}).get("Error", {}).get("Code", "Unknown"), str(e))
        return {n.id: n for n in created}

    def set_node_tags(self, node_id, tags):
        self.client.create_tags(Resources=[node_id], Tags=[{"Key": k, "Value": v} for k, v in tags.items()])
        self._cache.pop(node_id, None)

    def terminate_node(self, node_id):
        self.client.terminate_instances(InstanceIds=[node_id])

    def terminate_nodes(self, node_ids: List[str]):
        if node_ids:
            self.client.terminate_instances(InstanceIds=list(node_ids))


# GCP and Azure speak the clouds' REST APIs directly (no SDK needed): rest_providers.py
from cloudtik_amd.providers.cloud.rest_providers import AzureNodeProvider, GCPNodeProvider  # noqa: E402,F401


# Aliyun and Huawei Cloud speak the clouds' signed HTTP APIs (no SDK needed): signed_providers.py
from cloudtik_amd.providers.cloud.signed_providers import AliyunNodeProvider, HuaweiCloudNodeProvider  # noqa: E402,F401,E501
