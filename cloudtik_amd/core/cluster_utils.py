"""Helpers shared by the cluster operator (CLI side) and the cluster scaler (head side):
launch / runtime hashes, node tags, node environment and updater construction
(reference core/_private/cluster/cluster_operator.py:get_or_create_head_node and
cluster_scaler.py:_create_node_updater / spawn_updater).
"""
from __future__ import annotations

import os
import sys
from typing import Any, Dict, Optional

from cloudtik_amd.core import constants as C
from cloudtik_amd.core import tags as T
from cloudtik_amd.core import runtime_factory as rf
from cloudtik_amd.core.cluster_config import (get_runtime_types, hash_launch_conf, hash_runtime_conf,
                                              merged_commands_for)
from cloudtik_amd.core.updater import NodeUpdater, NodeUpdaterThread

BOOTSTRAP_CONFIG_REMOTE = "~/cloudtik_bootstrap_config.yaml"


def launch_hash(config: Dict[str, Any], node_type: str, provider=None) -> str:
    nc = dict(config["available_node_types"][node_type].get("node_config", {}))
    if provider is not None:
        nc = provider.prepare_node_config_for_launch_hash(nc)
    return hash_launch_conf(nc, config.get("auth", {}))


def runtime_hashes(config: Dict[str, Any], provider=None):
    cfg = provider.prepare_config_for_runtime_hash(config) if provider is not None else config
    extra = [cfg.get("merged_commands"), cfg.get("runtime"), cfg.get("docker")]
    mounts = {k: v for k, v in (cfg.get("file_mounts") or {}).items() if k != BOOTSTRAP_CONFIG_REMOTE}
    return hash_runtime_conf(mounts, cfg.get("cluster_synced_files"), extra,
                             generate_file_mounts_contents_hash=True)


def node_tags(config: Dict[str, Any], node_type: str, kind: str, seq_id: Optional[int] = None,
              provider=None) -> Dict[str, str]:
    t = {
        T.CLOUDTIK_TAG_CLUSTER_NAME: config["cluster_name"],
        T.CLOUDTIK_TAG_NODE_KIND: kind,
        T.CLOUDTIK_TAG_USER_NODE_TYPE: node_type,
        T.CLOUDTIK_TAG_NODE_STATUS: T.STATUS_UNINITIALIZED,
        T.CLOUDTIK_TAG_LAUNCH_CONFIG: launch_hash(config, node_type, provider),
        T.CLOUDTIK_TAG_NODE_NAME: f"cloudtik-{config['cluster_name']}-{kind}",
        # the workspace the node belongs to: the workspace registry (global variables as
        # head-node tags) lists the heads of all its clusters by this tag
        T.CLOUDTIK_TAG_WORKSPACE_NAME: config.get("workspace_name") or "default",
    }
    if seq_id is not None:
        t[T.CLOUDTIK_TAG_NODE_SEQ_ID] = str(seq_id)
    return t


def next_seq_id(provider, cluster_name: str) -> int:
    used = set()
    for nid in provider.non_terminated_nodes({T.CLOUDTIK_TAG_CLUSTER_NAME: cluster_name}):
        s = provider.node_tags(nid).get(T.CLOUDTIK_TAG_NODE_SEQ_ID)
        if s and s.isdigit():
            used.add(int(s))
    i = T.CLOUDTIK_TAG_HEAD_NODE_SEQ_ID + 1
    while i in used:
        i += 1
    return i


def node_environment(config: Dict[str, Any], provider, node_id: str, head_ip: Optional[str],
                     is_head: bool) -> Dict[str, Any]:
    env: Dict[str, Any] = {
        C.CLOUDTIK_RUNTIME_ENV_RUNTIMES: ",".join(get_runtime_types(config)),
        C.CLOUDTIK_RUNTIME_ENV_WORKSPACE: config.get("workspace_name", "default"),
    }
    if head_ip:
        env[C.CLOUDTIK_RUNTIME_ENV_HEAD_IP] = head_ip
    for t in get_runtime_types(config):
        rt = rf.get_runtime(t, config.get("runtime", {}).get(t, {}) or {})
        env.update(rt.with_environment_variables(config, provider, node_id) or {})
    nt = config["available_node_types"].get(provider.node_tags(node_id).get(T.CLOUDTIK_TAG_USER_NODE_TYPE, ""), {})
    env.update(provider.with_environment_variables(nt, node_id) or {})
    if config["provider"].get("type") in ("local", "virtual") or os.environ.get("CLOUDTIK_INHERIT_PYTHONPATH"):
        # same-host nodes run the CLI of this checkout even when it is not pip-installed
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["PYTHONPATH"] = root
        env["CLOUDTIK_PYTHON"] = sys.executable
        env["CLOUDTIK_BIN_DIR"] = os.path.join(root, "bin")
    return env


def create_updater(config: Dict[str, Any], provider, node_id: str, is_head: bool, head_ip: Optional[str],
                   restart_only: bool = False, for_recovery: bool = False, threaded: bool = False,
                   file_mounts: Optional[Dict[str, str]] = None, call_context=None,
                   ready_timeout: Optional[float] = None):
    rh, fmh = runtime_hashes(config, provider)
    mounts = dict(config.get("file_mounts") or {})
    mounts.update(file_mounts or {})
    nt = provider.node_tags(node_id).get(T.CLOUDTIK_TAG_USER_NODE_TYPE)
    resources = config["available_node_types"].get(nt, {}).get("resources")
    cls = NodeUpdaterThread if threaded else NodeUpdater
    return cls(
        node_id=node_id, provider_config=config["provider"], provider=provider,
        auth_config=config.get("auth", {}), cluster_name=config["cluster_name"], file_mounts=mounts,
        initialization_commands=merged_commands_for(config, is_head, "initialization"),
        setup_commands=merged_commands_for(config, is_head, "setup"),
        bootstrap_commands=merged_commands_for(config, is_head, "bootstrap"),
        start_commands=merged_commands_for(config, is_head, "start"),
        runtime_hash=rh, file_mounts_contents_hash=fmh, is_head_node=is_head,
        node_resources=resources, cluster_synced_files=config.get("cluster_synced_files"),
        use_internal_ip=not is_head or config["provider"].get("use_internal_ips", False),
        docker_config=config.get("docker"), restart_only=restart_only, for_recovery=for_recovery,
        environment_variables=node_environment(config, provider, node_id, head_ip, is_head),
        call_context=call_context, ready_timeout=ready_timeout,
        shared_memory_ratio=shared_memory_ratio(config, nt))


def shared_memory_ratio(config: Dict[str, Any], node_type: Optional[str]) -> float:
    """/dev/shm share of a container's memory: the largest any enabled runtime asks for
    (Runtime.get_runtime_shared_memory_ratio), or docker.shared_memory_ratio."""
    ratio = float((config.get("docker") or {}).get("shared_memory_ratio", 0.0) or 0.0)
    from cloudtik_amd.core.runtime_factory import get_runtime, get_runtime_types
    rc = config.get("runtime") or {}
    for name in get_runtime_types(config):
        try:
            ratio = max(ratio, float(get_runtime(name, rc).get_runtime_shared_memory_ratio(rc, config, node_type) or 0))
        except Exception:  # noqa: BLE001 - a runtime without the hook
            continue
    return ratio


def get_head_node(provider, cluster_name: str) -> Optional[str]:
    heads = provider.non_terminated_nodes({T.CLOUDTIK_TAG_CLUSTER_NAME: cluster_name,
                                           T.CLOUDTIK_TAG_NODE_KIND: T.NODE_KIND_HEAD})
    return heads[0] if heads else None


def get_worker_nodes(provider, cluster_name: str):
    return provider.non_terminated_nodes({T.CLOUDTIK_TAG_CLUSTER_NAME: cluster_name,
                                          T.CLOUDTIK_TAG_NODE_KIND: T.NODE_KIND_WORKER})
