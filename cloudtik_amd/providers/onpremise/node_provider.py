"""On-premise provider: nodes come from the pool owned by a ``cloudtik-simulator`` service
(reference providers/_private/onpremise/node_provider.py:14 + cloud_simulator_scheduler.py:23).

    provider:
        type: onpremise
        cloud_simulator_address: 10.0.0.2:8282
    available_node_types:
        worker.mi355x:
            node_config: {instance_type: mi355x-8gpu}

Commands reach the hosts over SSH (``auth``), or locally when the host is the CLI machine;
node resources are filled from the simulator's instance-type table.
"""
from __future__ import annotations

import json
import urllib.request
from typing import Any, Dict, List

from cloudtik_amd.core.node_provider import NodeLaunchException, NodeProvider


class SimulatorClient:
    def __init__(self, address: str, timeout: float = 30.0):
        if "://" not in address:
            address = "http://" + address
        self.url = address.rstrip("/") + "/api"
        self.timeout = timeout

    def call(self, method: str, **params):
        req = urllib.request.Request(self.url, data=json.dumps({"method": method, "params": params}).encode(),
                                     headers={"Content-Type": "application/json"})
        try:
            with urllib.request.urlopen(req, timeout=self.timeout) as r:
                res = json.loads(r.read())
        except urllib.error.HTTPError as e:
            res = json.loads(e.read() or b"{}")
        if "error" in res:
            raise RuntimeError(res["error"])
        return res.get("result")


class OnPremiseNodeProvider(NodeProvider):
    def __init__(self, provider_config, cluster_name):
        super().__init__(provider_config, cluster_name)
        from cloudtik_amd.providers.onpremise.simulator import simulator_address
        # configured, or discovered from the process file of a simulator on this machine
        self.client = SimulatorClient(simulator_address(provider_config.get("cloud_simulator_address")))

    def non_terminated_nodes(self, tag_filters):
        return self.client.call("non_terminated_nodes", cluster_name=self.cluster_name if self.cluster_filter() else None,
                                tag_filters=tag_filters)

    def is_running(self, node_id):
        return self.client.call("is_running", node_id=node_id)

    def is_terminated(self, node_id):
        return self.client.call("is_terminated", node_id=node_id)

    def node_tags(self, node_id):
        return self.client.call("node_tags", node_id=node_id)

    def internal_ip(self, node_id):
        return self.client.call("internal_ip", node_id=node_id)

    def external_ip(self, node_id):
        return self.client.call("external_ip", node_id=node_id)

    def create_node(self, node_config, tags, count):
        try:
            ids = self.client.call("create_node", cluster_name=self.cluster_name, node_config=node_config,
                                   tags=tags, count=count)
        except RuntimeError as e:
            raise NodeLaunchException("NoAvailableHost", str(e))
        return {i: {"ip": i} for i in ids}

    def set_node_tags(self, node_id, tags):
        self.client.call("set_node_tags", node_id=node_id, tags=tags)

    def terminate_node(self, node_id):
        self.client.call("terminate_node", node_id=node_id)

    def terminate_nodes(self, node_ids: List[str]):
        self.client.call("terminate_nodes", node_ids=list(node_ids))

    def get_node_info(self, node_id) -> Dict[str, Any]:
        info = super().get_node_info(node_id)
        info.update(self.client.call("node_info", node_id=node_id))
        return info

    @staticmethod
    def validate_config(provider_config):
        if not provider_config.get("cloud_simulator_address"):
            raise ValueError("onpremise provider needs provider.cloud_simulator_address")

    @staticmethod
    def fillout_available_node_types_resources(cluster_config):
        addr = cluster_config["provider"].get("cloud_simulator_address")
        if not addr:
            return cluster_config
        try:
            types = SimulatorClient(addr, timeout=5).call("get_instance_types")
        except Exception:  # noqa: BLE001 -- simulator not reachable at config time
            return cluster_config
        for nt in cluster_config.get("available_node_types", {}).values():
            it = (nt.get("node_config") or {}).get("instance_type")
            if it in types and not nt.get("resources"):
                nt["resources"] = dict(types[it])
        return cluster_config
