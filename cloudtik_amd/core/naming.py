"""Cluster node naming (reference core/_private/service_discovery/naming.py:28-172).

Node names are ``<cluster>-<seq_id>`` (seq id 1 = head); with a DNS runtime in the cluster
(consul / coredns / bind / dnsmasq) nodes are also resolvable by short name
``<node>.<cluster>.node`` and fully-qualified name ``<node>.<cluster>.<workspace>.cloudtik``;
otherwise hosts fall back to IP addresses.
"""
from __future__ import annotations

import ipaddress
from typing import Any, Dict, Optional

DNS_RUNTIMES = ("consul", "coredns", "bind", "dnsmasq")


def get_cluster_node_name(cluster_name: str, seq_id) -> str:
    return f"{cluster_name}-{seq_id}"


def get_cluster_node_sqdn(node_name: str, cluster_name: str) -> str:
    return f"{node_name}.{cluster_name}.node"


def get_cluster_node_fqdn(node_name: str, cluster_name: str, workspace_name: str) -> str:
    return f"{node_name}.{cluster_name}.{workspace_name}.cloudtik"


def get_address_type_of_hostname(hostname: str) -> str:
    try:
        ip = ipaddress.ip_address(hostname)
        return "ipv6" if ip.version == 6 else "ipv4"
    except ValueError:
        return "hostname"


def dns_naming_runtime(config: Dict[str, Any]) -> Optional[str]:
    types = (config.get("runtime", {}) or {}).get("types", []) or []
    for t in DNS_RUNTIMES:
        if t in types:
            return t
    return None


def is_cluster_hostname_available(config: Dict[str, Any]) -> bool:
    return dns_naming_runtime(config) is not None


def get_cluster_node_host(config: Dict[str, Any], node_seq_id, node_ip: str) -> str:
    if not is_cluster_hostname_available(config):
        return node_ip
    name = get_cluster_node_name(config["cluster_name"], node_seq_id)
    return get_cluster_node_fqdn(name, config["cluster_name"], config.get("workspace_name", "default"))


def get_cluster_head_host(config: Dict[str, Any], head_ip: str) -> str:
    return get_cluster_node_host(config, 1, head_ip)


def with_node_host_environment_variables(config, node_seq_id, node_ip, env: Dict[str, Any]) -> Dict[str, Any]:
    env["CLOUDTIK_NODE_HOST"] = get_cluster_node_host(config, node_seq_id, node_ip)
    return env


def with_head_host_environment_variables(config, head_ip, env: Dict[str, Any]) -> Dict[str, Any]:
    env["CLOUDTIK_HEAD_HOST"] = get_cluster_head_host(config, head_ip)
    return env
