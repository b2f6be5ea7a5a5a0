"""Local provider: one cluster over a static list of hosts (reference
providers/_private/local/node_provider.py:16, local_scheduler.py:30-171, config.py:207-246).

``provider.nodes`` lists the hosts (``[{ip: 10.0.0.2}, ...]`` or plain IP strings); when it
is empty the cluster is just this host (the CLI host becomes the head).  Node ids are the
host IPs.  A launched node is "running" in the locked file state; terminating it marks it
terminated (the host itself is not powered off).  Instance types are filled out from the
detected CPU / memory / AMD GPU resources of each host (``core.resources``), so a single
8 x MI355X host reports ``{"CPU": .., "GPU": 8, "accelerator_type:MI355X": 8}``.
"""
from __future__ import annotations

import copy
import logging
import os
import threading
from typing import Any, Dict, List, Optional

from cloudtik_amd.core import tags as T
from cloudtik_amd.core.executor import local_ips
from cloudtik_amd.core.node_provider import NodeProvider, NodeLaunchException
from cloudtik_amd.core.state.file_state_store import FileStateStore

logger = logging.getLogger(__name__)

STATE_DIR = os.path.expanduser(os.environ.get("CLOUDTIK_LOCAL_STATE_DIR", "~/.cloudtik/local"))


def _node_ips(provider_config: Dict[str, Any]) -> List[str]:
    out = []
    for n in provider_config.get("nodes", []) or []:
        out.append(n["ip"] if isinstance(n, dict) else str(n))
    if not out:
        out = [_this_host_ip()]
    return out


def _this_host_ip() -> str:
    ips = [ip for ip in local_ips() if ip.count(".") == 3 and not ip.startswith("127.")]
    return ips[0] if ips else "127.0.0.1"


class LocalScheduler:
    """Allocates hosts from the static pool for create_node requests."""

    def __init__(self, provider_config: Dict[str, Any], cluster_name: str):
        self.provider_config = provider_config
        self.cluster_name = cluster_name
        self.lock = threading.RLock()
        path = os.path.join(STATE_DIR, f"{cluster_name}.json")
        self.store = FileStateStore(path)
        self.ips = _node_ips(provider_config)
        with self.store.transaction() as st:
            nodes = st.setdefault("nodes", {})
            for ip in self.ips:
                nodes.setdefault(ip, {"state": "terminated", "tags": {}, "ip": ip})

    def get_non_terminated_nodes(self, tag_filters):
        out = []
        for nid, n in self.store.get_nodes().items():
            if n.get("state") == "terminated":
                continue
            tags = n.get("tags", {})
            if all(tags.get(k) == v for k, v in tag_filters.items()):
                out.append(nid)
        return out

    def is_running(self, node_id):
        n = self.store.get_node(node_id)
        return bool(n) and n.get("state") == "running"

    def is_terminated(self, node_id):
        n = self.store.get_node(node_id)
        return not n or n.get("state") == "terminated"

    def get_node_tags(self, node_id):
        n = self.store.get_node(node_id)
        return dict(n.get("tags", {})) if n else {}

    def set_node_tags(self, node_id, tags):
        self.store.update_node_tags(node_id, tags)

    def create_node(self, node_config, tags, count):
        with self.lock, self.store.transaction() as st:
            nodes = st["nodes"]
            is_head = tags.get(T.CLOUDTIK_TAG_NODE_KIND) == T.NODE_KIND_HEAD
            free = [ip for ip in self.ips if nodes.get(ip, {}).get("state") == "terminated"]
            if is_head:
                # the head must be this host when it is in the pool (commands run locally)
                me = set(local_ips())
                free.sort(key=lambda ip: ip not in me)
            if len(free) < count:
                raise NodeLaunchException("NoAvailableHost",
                                          f"requested {count} node(s), {len(free)} free host(s) in the pool")
            created = {}
            for ip in free[:count]:
                nodes[ip] = {"state": "running", "tags": dict(tags), "ip": ip,
                             "instance_type": node_config.get("instance_type", "default")}
                created[ip] = nodes[ip]
            return created

    def terminate_node(self, node_id):
        with self.store.transaction() as st:
            n = st["nodes"].get(node_id)
            if n:
                n["state"] = "terminated"
                n["tags"] = {}


class LocalNodeProvider(NodeProvider):
    def __init__(self, provider_config, cluster_name):
        super().__init__(provider_config, cluster_name)
        self.scheduler = LocalScheduler(provider_config, cluster_name)

    def workspace_head_nodes(self, workspace_name):
        """Every local cluster keeps its node state in its own file of the state directory
        (the same host serves as head of several clusters, so node ids -- host IPs -- repeat
        across clusters): scan them all; keys are ``<cluster>/<ip>``."""
        out = {}
        try:
            files = sorted(f for f in os.listdir(STATE_DIR) if f.endswith(".json") and not f.startswith("workspace-"))
        except OSError:
            return out
        for f in files:
            try:
                nodes = FileStateStore(os.path.join(STATE_DIR, f)).get_nodes()
            except (OSError, ValueError):
                continue
            for ip, n in nodes.items():
                tags = n.get("tags", {})
                if n.get("state") != "terminated" and tags.get(T.CLOUDTIK_TAG_NODE_KIND) == T.NODE_KIND_HEAD and \
                        tags.get(T.CLOUDTIK_TAG_WORKSPACE_NAME) == workspace_name:
                    out[f"{f[:-5]}/{ip}"] = dict(tags)
        return out

    def non_terminated_nodes(self, tag_filters):
        return self.scheduler.get_non_terminated_nodes(tag_filters)

    def is_running(self, node_id):
        return self.scheduler.is_running(node_id)

    def is_terminated(self, node_id):
        return self.scheduler.is_terminated(node_id)

    def node_tags(self, node_id):
        return self.scheduler.get_node_tags(node_id)

    def external_ip(self, node_id):
        return node_id

    def internal_ip(self, node_id):
        return node_id

    def create_node(self, node_config, tags, count):
        return self.scheduler.create_node(node_config, tags, count)

    def set_node_tags(self, node_id, tags):
        self.scheduler.set_node_tags(node_id, tags)

    def terminate_node(self, node_id):
        self.scheduler.terminate_node(node_id)

    def get_node_info(self, node_id):
        info = super().get_node_info(node_id)
        n = self.scheduler.store.get_node(node_id) or {}
        info["instance_type"] = n.get("instance_type", "default")
        return info

    # ------------------------------------------------------------------ config hooks
    @staticmethod
    def prepare_config(cluster_config):
        return cluster_config

    @staticmethod
    def validate_config(provider_config):
        for n in provider_config.get("nodes", []) or []:
            if isinstance(n, dict) and "ip" not in n:
                raise ValueError("local provider: every entry of provider.nodes needs an 'ip'")

    @staticmethod
    def fillout_available_node_types_resources(cluster_config):
        """Fill ``resources`` of node types without explicit resources from this host's
        detected CPU / memory / AMD GPUs (all local hosts are assumed homogeneous)."""
        from cloudtik_amd.core.resources import detect_resources
        detected = None
        for name, nt in cluster_config.get("available_node_types", {}).items():
            if nt.get("resources"):
                continue
            if detected is None:
                detected = detect_resources()
            nt["resources"] = {k: v for k, v in detected.items() if k != "memory"}
            nt["resources"]["memory"] = int(detected.get("memory", 0) * 0.7)
        return cluster_config

    @staticmethod
    def bootstrap_config(cluster_config):
        cfg = copy.deepcopy(cluster_config)
        ips = _node_ips(cfg["provider"])
        workers = [t for t in cfg.get("available_node_types", {}) if t != cfg["head_node_type"]]
        # cap worker max_workers by the pool size (one node is the head)
        cap = max(0, len(ips) - 1)
        for t in workers:
            nt = cfg["available_node_types"][t]
            nt["max_workers"] = min(nt.get("max_workers", cap), cap)
            nt["min_workers"] = min(nt.get("min_workers", 0), nt["max_workers"])
        cfg["max_workers"] = min(cfg.get("max_workers", cap), cap)
        return cfg
