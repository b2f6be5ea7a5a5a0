"""Virtual provider: a multi-node cluster on ONE host (reference
providers/_private/virtual/node_provider.py + virtual_container_scheduler.py, which create a
docker container per node on the host's bridge network).

Each virtual node gets

* a node id ``<cluster>-<seq>`` and its own loopback address ``127.<a>.<b>.<seq>`` (all of
  127/8 routes to the host on Linux, so per-node services can bind distinct addresses and
  the same ports -- the role the docker bridge IPs play in the reference);
* its own home directory (``$CLOUDTIK_LOCAL_STATE_DIR/virtual/<cluster>/<node>``) that
  commands run in with ``HOME`` pointed at it, so file mounts / logs / pid files of nodes do
  not collide;
* when ``docker.enabled`` with an image is configured, the node's commands run inside a
  per-node ROCm container instead (``DockerCommandExecutor``; /dev/kfd + /dev/dri passed
  through, GPUs split between nodes with ``HIP_VISIBLE_DEVICES``).

With ``provider.use_containers: true`` every node is instead a docker container on the
workspace's bridge network with an exclusive GPU / NUMA-local CPU slice, memory limit and data
disks (providers/virtual/containers.py), addressed by its bridge IP -- the reference's
virtual container scheduler, laid out for MI355X.

On an 8 x MI355X host this lets one box rehearse multi-node layouts, e.g. 4 nodes x 2 GPUs.
"""
from __future__ import annotations

import hashlib
import os
import shlex
from typing import Any, Dict, List, Optional

from cloudtik_amd.core import tags as T
from cloudtik_amd.core.executor import (LocalCommandExecutor, DockerCommandExecutor,
                                        with_environment_variables, run_cmd_with_runner)
from cloudtik_amd.core.node_provider import NodeProvider, NodeLaunchException
from cloudtik_amd.core.state.file_state_store import FileStateStore


def _state_dir() -> str:
    return os.path.expanduser(os.environ.get("CLOUDTIK_LOCAL_STATE_DIR", "~/.cloudtik/local"))


def _cluster_prefix(cluster_name: str) -> str:
    h = int(hashlib.sha1(cluster_name.encode()).hexdigest(), 16)
    return f"127.{1 + h % 250}.{(h >> 8) % 256}"


class VirtualCommandExecutor(LocalCommandExecutor):
    """Runs node commands on this host inside the virtual node's home directory."""

    def __init__(self, call_context, log_prefix, auth_config, cluster_name, process_runner,
                 node_id, provider, home: str, env: Dict[str, str]):
        super().__init__(call_context, log_prefix, auth_config, cluster_name, process_runner,
                         node_id, provider)
        self.home = home
        self.env = env

    def _map(self, path: str) -> str:
        if path.startswith("~/") or path == "~":
            return os.path.join(self.home, path[2:])
        return path

    def run(self, cmd=None, timeout=120, exit_on_fail=False, port_forward=None, with_output=False,
            environment_variables=None, run_env="auto", ssh_options_override_ssh_key="",
            shutdown_after_run=False, cmd_to_print=None, silent=False):
        if not cmd:
            return None
        env = dict(self.env)
        env.update(environment_variables or {})
        full = with_environment_variables(f"cd {shlex.quote(self.home)} && {cmd}", env)
        full = f"export HOME={shlex.quote(self.home)}; " + full
        return run_cmd_with_runner(self.process_runner, ["bash", "-c", full], with_output=with_output,
                                   silent=silent)

    def run_rsync_up(self, source, target, options=None):
        target = self._map(target)
        os.makedirs(os.path.dirname(target.rstrip("/")) or ".", exist_ok=True)
        self._copy(source, target)

    def run_rsync_down(self, source, target, options=None):
        self._copy(self._map(source), target)


class VirtualNodeProvider(NodeProvider):
    def __init__(self, provider_config, cluster_name):
        super().__init__(provider_config, cluster_name)
        self.root = os.path.join(_state_dir(), "virtual", cluster_name)
        os.makedirs(self.root, exist_ok=True)
        self.store = FileStateStore(os.path.join(self.root, "nodes.json"))
        self.prefix = _cluster_prefix(cluster_name)
        self.containers = None
        if provider_config.get("use_containers"):
            from cloudtik_amd.providers.virtual.containers import DockerNodes
            self.containers = DockerNodes(provider_config, cluster_name,
                                          provider_config.get("workspace_name", cluster_name), self.root,
                                          runner=provider_config.get("_docker_runner"),
                                          gpus=provider_config.get("_host_gpus"),
                                          numa_cpus=provider_config.get("_host_numa_cpus"))

    # ------------------------------------------------------------------ queries
    def _nodes(self):
        return self.store.get_nodes()

    def workspace_head_nodes(self, workspace_name):
        """Heads of every virtual cluster on this host (one state directory per cluster)."""
        from cloudtik_amd.core import tags as T
        base = os.path.join(_state_dir(), "virtual")
        out = {}
        try:
            names = sorted(os.listdir(base))
        except OSError:
            return out
        for cname in names:
            path = os.path.join(base, cname, "nodes.json")
            if not os.path.exists(path):
                continue
            for nid, n in FileStateStore(path).get_nodes().items():
                t = n.get("tags", {})
                if n.get("state") == "running" and t.get(T.CLOUDTIK_TAG_NODE_KIND) == T.NODE_KIND_HEAD and \
                        t.get(T.CLOUDTIK_TAG_WORKSPACE_NAME) == workspace_name:
                    out[f"{cname}/{nid}"] = dict(t)
        return out

    def non_terminated_nodes(self, tag_filters):
        out = []
        for nid, n in self._nodes().items():
            if n.get("state") != "running":
                continue
            tags = n.get("tags", {})
            if all(tags.get(k) == v for k, v in tag_filters.items()):
                out.append(nid)
        return sorted(out, key=lambda x: int(x.rsplit("-", 1)[1]))

    def is_running(self, node_id):
        n = self._nodes().get(node_id)
        return bool(n) and n.get("state") == "running"

    def is_terminated(self, node_id):
        return not self.is_running(node_id)

    def node_tags(self, node_id):
        n = self._nodes().get(node_id)
        return dict(n.get("tags", {})) if n else {}

    def internal_ip(self, node_id):
        n = self._nodes().get(node_id)
        return n.get("ip") if n else None

    def external_ip(self, node_id):
        return self.internal_ip(node_id)

    def node_home(self, node_id) -> str:
        return os.path.join(self.root, node_id)

    # ------------------------------------------------------------------ mutations
    def create_node(self, node_config, tags, count):
        max_nodes = int(self.provider_config.get("max_nodes", 64))
        created = {}
        with self.store.transaction() as st:
            nodes = st.setdefault("nodes", {})
            live = [n for n in nodes.values() if n.get("state") == "running"]
            if len(live) + count > max_nodes:
                raise NodeLaunchException("QuotaExceeded",
                                          f"virtual provider limit of {max_nodes} nodes reached")
            seq = st.get("next_seq", 1)
            for _ in range(count):
                if seq > 254:
                    raise NodeLaunchException("AddressExhausted", "no free virtual node address")
                nid = f"{self.cluster_name}-{seq}"
                node = {"state": "running", "ip": f"{self.prefix}.{seq}", "tags": dict(tags),
                        "instance_type": node_config.get("instance_type", "virtual"),
                        "gpu_ids": node_config.get("gpu_ids"), "seq": seq, "node_config": node_config}
                if self.containers is not None:
                    # sizes: the reference's instance_type {CPU, memory, GPU} or resources
                    res = dict(node_config.get("resources") or {})
                    if isinstance(node_config.get("instance_type"), dict):
                        res.update(node_config["instance_type"])
                    alloc_tab = st.setdefault("alloc", {})
                    alloc = self.containers.scheduler.allocate(
                        alloc_tab, int(node_config.get("gpus", res.get("GPU", 0)) or 0),
                        int(node_config.get("cpus", res.get("CPU", 1)) or 1))
                    alloc_tab[nid] = alloc
                    ctags = dict(tags, **{T.CLOUDTIK_TAG_CLUSTER_NAME: self.cluster_name})
                    try:
                        node["ip"] = self.containers.start(nid, node_config, ctags, alloc, seq)
                    except Exception as e:  # noqa: BLE001 - docker failed: release the slice
                        alloc_tab.pop(nid, None)
                        raise NodeLaunchException("ContainerStartFailed", str(e))
                    node.update(container=nid, gpu_ids=None, alloc=alloc)
                nodes[nid] = node
                created[nid] = node
                os.makedirs(self.node_home(nid), exist_ok=True)
                seq += 1
            st["next_seq"] = seq
        return created

    def set_node_tags(self, node_id, tags):
        self.store.update_node_tags(node_id, tags)

    def terminate_node(self, node_id):
        with self.store.transaction() as st:
            n = st.get("nodes", {}).get(node_id)
            if n:
                n["state"] = "terminated"
                if n.get("container") and self.containers is not None:
                    self.containers.stop(n["container"], n.get("node_config"), seq=n.get("seq", 0))
                    st.get("alloc", {}).pop(node_id, None)

    # ------------------------------------------------------------------ execution
    def get_command_executor(self, call_context, log_prefix, node_id, auth_config, cluster_name,
                             process_runner, use_internal_ip, docker_config=None):
        n = self._nodes().get(node_id) or {}
        env = {"CLOUDTIK_VIRTUAL_NODE": node_id}
        if n.get("gpu_ids") is not None:
            env["HIP_VISIBLE_DEVICES"] = ",".join(str(g) for g in n["gpu_ids"])
        host = VirtualCommandExecutor(call_context, log_prefix, auth_config, cluster_name,
                                      process_runner, node_id, self, self.node_home(node_id), env)
        if n.get("container"):
            from cloudtik_amd.providers.virtual.containers import ContainerExecutor
            return ContainerExecutor(host, n["container"], (self.provider_config.get("docker_cmd") or ["docker"])[0])
        if docker_config and docker_config.get("enabled") and docker_config.get("image"):
            dc = dict(docker_config)
            dc.setdefault("container_name", f"cloudtik-{node_id}")
            return DockerCommandExecutor(call_context, host, dc)
        return host

    def get_node_info(self, node_id):
        info = super().get_node_info(node_id)
        info["instance_type"] = (self._nodes().get(node_id) or {}).get("instance_type", "virtual")
        return info

    def cleanup_cluster(self, cluster_config, deep=False):
        if deep:
            with self.store.transaction() as st:
                if self.containers is not None:
                    for nid, n in st.get("nodes", {}).items():
                        if n.get("container") and n.get("state") == "running":
                            self.containers.stop(n["container"], n.get("node_config"), seq=n.get("seq", 0))
                st["nodes"] = {}
                st["alloc"] = {}
                st["next_seq"] = 1

    # ------------------------------------------------------------------ config hooks
    @staticmethod
    def fillout_available_node_types_resources(cluster_config):
        from cloudtik_amd.core.resources import detect_resources
        detected = None
        for nt in cluster_config.get("available_node_types", {}).values():
            if nt.get("resources"):
                continue
            if detected is None:
                detected = detect_resources()
            nt["resources"] = {"CPU": max(1, int(detected.get("CPU", 1)) // 4),
                               "memory": int(detected.get("memory", 0) * 0.1)}
        return cluster_config

    @staticmethod
    def validate_config(provider_config):
        if int(provider_config.get("max_nodes", 64)) > 254:
            raise ValueError("virtual provider supports at most 254 nodes per cluster")
