"""Cluster config bootstrap pipeline (reference ``core/_private/cluster/cluster_config.py:37-150``
+ ``utils.py`` prepare/validate/merge_commands/hashing).

    prepare_config     provider.prepare_config -> fill_with_defaults (from: + provider
                       defaults) -> runtime defaults -> merged node commands (built-in +
                       provider + runtime, per node kind, runtime dependency order) ->
                       docker flags -> min/max workers -> node resources
    post_prepare       provider.post_prepare -> runtime.prepare_config
    validate_config    JSON schema + head/worker node types + provider + runtimes
    bootstrap          provider.bootstrap_config -> runtime.bootstrap_config -> verify
    cache              encrypted JSON keyed by the config hash (~/.cloudtik/configs)
"""
from __future__ import annotations

import copy
import hashlib
import json
import logging
import os
import sys
from typing import Any, Dict, List, Optional

import yaml

from cloudtik_amd.core import constants
from cloudtik_amd.core.config import loader, schema as jschema
from cloudtik_amd.core.config.crypto import decrypt_config, encrypt_config
from cloudtik_amd.core.config.merge import merge_config
from cloudtik_amd.core.provider_factory import get_node_provider_cls
from cloudtik_amd.core import runtime_factory as rf

logger = logging.getLogger(__name__)

SCHEMA_DIR = os.path.join(loader.PKG_ROOT, "schema")
CONFIG_CACHE_DIR = os.path.expanduser(os.environ.get("CLOUDTIK_CONFIG_CACHE", "~/.cloudtik/configs"))
CONFIG_CACHE_VERSION = 1

COMMAND_KEYS = ["initialization_commands", "setup_commands", "bootstrap_commands",
                "start_commands", "stop_commands"]


def load_schema(name: str = "cluster") -> Dict[str, Any]:
    with open(os.path.join(SCHEMA_DIR, f"{name}.json")) as f:
        return json.load(f)


def config_hash(config: Dict[str, Any]) -> str:
    return hashlib.sha1(json.dumps(config, sort_keys=True, default=str).encode()).hexdigest()


# --------------------------------------------------------------------------------- helpers
def get_head_node_type(config) -> str:
    return config["head_node_type"]


def get_available_node_types(config) -> Dict[str, Any]:
    return config.get("available_node_types", {})


def get_worker_node_types(config) -> List[str]:
    head = config.get("head_node_type")
    return [t for t in get_available_node_types(config) if t != head]


def get_runtime_types(config) -> List[str]:
    return rf.get_runtime_types(config)


def is_docker_enabled(config) -> bool:
    return bool(config.get("docker", {}).get("enabled"))


def with_head_node_ip_env(config) -> Dict[str, str]:
    return {}


# --------------------------------------------------------------------------------- commands
def _builtin_commands() -> Dict[str, Any]:
    return loader.load_yaml(os.path.join(loader.PROVIDERS_DIR, "commands.yaml"))


def _provider_commands(provider: Dict[str, Any]) -> Dict[str, Any]:
    from cloudtik_amd.core.provider_factory import get_provider_home
    p = os.path.join(get_provider_home(provider), "commands.yaml")
    return loader.load_yaml(p) if os.path.exists(p) else {}


def head_start_command(config) -> str:
    return ("cloudtik node start --head --node-ip=$CLOUDTIK_NODE_IP "
            f"--port={constants.CLOUDTIK_DEFAULT_PORT} --state")


def head_controller_command(config) -> str:
    if config.get("no_controller_on_head"):
        return "true"
    return "cloudtik node start --head --node-ip=$CLOUDTIK_NODE_IP --controller"


def worker_start_command(config) -> str:
    return ("cloudtik node start --node-ip=$CLOUDTIK_NODE_IP "
            f"--address=$CLOUDTIK_HEAD_IP:{constants.CLOUDTIK_DEFAULT_PORT}")


def merge_commands(config: Dict[str, Any]) -> Dict[str, Any]:
    """Combine built-in, provider, user and runtime commands into
    ``config['merged_commands'][head|worker][initialization|setup|start|stop]``."""
    builtin = _builtin_commands()
    provider_cmds = _provider_commands(config["provider"])
    runtimes = rf.reorder_runtimes_for_dependency(get_runtime_types(config))
    rt_cmds = [rf.get_runtime(t, config.get("runtime", {}).get(t, {})).get_runtime_commands(config) or {}
               for t in runtimes]

    def collect(kind: str, stage: str) -> List[str]:
        out: List[str] = []
        for src in (builtin, provider_cmds, config):
            if stage == "initialization" and is_docker_enabled(config) and src is builtin:
                d = builtin.get("docker", {})
                out += d.get("initialization_commands", []) + d.get(f"{kind}_initialization_commands", [])
            out += list(src.get(f"{stage}_commands", []) or [])
            out += list(src.get(f"{kind}_{stage}_commands", []) or [])
        return out

    merged = {}
    for kind in ("head", "worker"):
        m = {"initialization": collect(kind, "initialization"), "setup": collect(kind, "setup"),
             "bootstrap": collect(kind, "bootstrap"), "start": [], "stop": []}
        if kind == "head":
            m["start"].append(head_start_command(config))
        for c in rt_cmds:
            m["setup"] += list(c.get(f"{kind}_setup_commands", []) or [])
        m["start"] += collect(kind, "start")
        for c in rt_cmds:
            m["start"] += list(c.get(f"{kind}_start_commands", []) or [])
        if kind == "head":
            m["start"].append(head_controller_command(config))
        else:
            m["start"].insert(0, worker_start_command(config))
        for c in reversed(rt_cmds):
            m["stop"] += list(c.get(f"{kind}_stop_commands", []) or [])
        m["stop"] += collect(kind, "stop")
        m["stop"].append("cloudtik node stop")
        merged[kind] = m
    config["merged_commands"] = merged
    return config


def merged_commands_for(config, head: bool, stage: str) -> List[str]:
    return list(config.get("merged_commands", {}).get("head" if head else "worker", {}).get(stage, []))


# --------------------------------------------------------------------------------- pipeline
def fill_runtime_defaults(config: Dict[str, Any]) -> Dict[str, Any]:
    types = rf.add_required_runtimes(get_runtime_types(config))
    config.setdefault("runtime", {})["types"] = types
    for t in types:
        d = rf.get_runtime(t, config["runtime"].get(t, {})).get_defaults_config(config) or {}
        if "runtime" in d:      # a runtime may return a full {"runtime": {...}} fragment
            d = d["runtime"].get(t, {})
        user = config["runtime"].get(t) or {}
        config["runtime"][t] = merge_config(copy.deepcopy(d), user)
    return config


def fill_node_type_min_max_workers(config: Dict[str, Any]) -> Dict[str, Any]:
    head = config.get("head_node_type")
    total_max = config.get("max_workers", constants.CLOUDTIK_DEFAULT_MAX_WORKERS)
    for name, nt in get_available_node_types(config).items():
        if name == head:
            nt.setdefault("min_workers", 0)
            nt["max_workers"] = 0
        else:
            nt.setdefault("min_workers", 0)
            nt.setdefault("max_workers", total_max)
    config["max_workers"] = total_max
    return config


def prepare_config(config: Dict[str, Any]) -> Dict[str, Any]:
    cfg = copy.deepcopy(config)
    cls = get_node_provider_cls(cfg["provider"])
    cfg = cls.prepare_config(cfg)
    cfg = loader.fill_with_defaults(cfg)
    cfg = fill_runtime_defaults(cfg)
    cfg = fill_node_type_min_max_workers(cfg)
    cfg = cls.fillout_available_node_types_resources(cfg)
    return cfg


def post_prepare(config: Dict[str, Any]) -> Dict[str, Any]:
    cls = get_node_provider_cls(config["provider"])
    config = cls.post_prepare(config)
    for t in get_runtime_types(config):
        config = rf.get_runtime(t, config["runtime"].get(t, {})).prepare_config(config) or config
    return merge_commands(config)


def validate_config(config: Dict[str, Any]) -> None:
    jschema.validate(config, load_schema("cluster"))
    if config.get("runtime"):
        jschema.validate(config["runtime"], load_schema("runtime"), path=["runtime"])
    nts = get_available_node_types(config)
    head = config.get("head_node_type")
    if head not in nts:
        raise ValueError(f"head_node_type '{head}' must be one of available_node_types {list(nts)}")
    for name, nt in nts.items():
        if nt.get("min_workers", 0) > nt.get("max_workers", 0) and name != head:
            raise ValueError(f"node type {name}: min_workers > max_workers")
    get_node_provider_cls(config["provider"]).validate_config(config["provider"])
    for t in get_runtime_types(config):
        rf.get_runtime(t, config["runtime"].get(t, {})).validate_config(config)


def _cache_path(h: str) -> str:
    return os.path.join(CONFIG_CACHE_DIR, f"cloudtik-config-{h}")


def bootstrap_config(config: Dict[str, Any], no_config_cache: bool = False,
                     init_config_cache: bool = False) -> Dict[str, Any]:
    """Full pipeline with an encrypted on-disk cache keyed by the input config's hash."""
    h = config_hash(config)
    path = _cache_path(h)
    if not no_config_cache and os.path.exists(path):
        try:
            with open(path) as f:
                cached = json.load(f)
            if cached.get("_version") == CONFIG_CACHE_VERSION:
                return decrypt_config(cached["config"])
        except (OSError, ValueError, KeyError):
            pass
    cfg = prepare_config(config)
    cfg = post_prepare(cfg)
    validate_config(cfg)
    cls = get_node_provider_cls(cfg["provider"])
    cfg = cls.bootstrap_config(cfg)
    for t in get_runtime_types(cfg):
        cfg = rf.get_runtime(t, cfg["runtime"].get(t, {})).bootstrap_config(cfg) or cfg
    cls.verify_config(cfg["provider"])
    for t in get_runtime_types(cfg):
        rf.get_runtime(t, cfg["runtime"].get(t, {})).verify_config(cfg)
    cfg["bootstrapped"] = True
    cfg["config_hash"] = h
    if not no_config_cache or init_config_cache:
        try:
            os.makedirs(CONFIG_CACHE_DIR, exist_ok=True)
            with open(path, "w") as f:
                json.dump({"_version": CONFIG_CACHE_VERSION, "config": encrypt_config(cfg)}, f)
        except OSError:
            logger.warning("could not write config cache %s", path)
    return cfg


def load_cluster_config(config_file: str, override_cluster_name: Optional[str] = None,
                        overrides: Optional[Dict[str, Any]] = None, no_config_cache: bool = False,
                        should_bootstrap: bool = True) -> Dict[str, Any]:
    cfg = loader.load_config_file(config_file, overrides)
    if override_cluster_name:
        cfg["cluster_name"] = override_cluster_name
    if "provider" not in cfg:
        raise ValueError(f"{config_file}: missing 'provider'")
    cfg.setdefault("cluster_name", "default")
    return bootstrap_config(cfg, no_config_cache) if should_bootstrap else cfg


def dump_yaml(config: Dict[str, Any], stream=None):
    return yaml.safe_dump(config, stream or sys.stdout, sort_keys=False)


# --------------------------------------------------------------------------------- hashing
def hash_launch_conf(node_config: Dict[str, Any], auth: Dict[str, Any]) -> str:
    """Launch hash: node_config + auth (with key *contents*): decides head relaunch
    (reference utils.py:1516)."""
    full = dict(auth or {})
    for k in ("ssh_private_key", "ssh_public_key"):
        if k in full:
            try:
                with open(os.path.expanduser(full[k])) as f:
                    full[k] = f.read()
            except OSError:
                pass
    return hashlib.sha1(json.dumps([node_config, full], sort_keys=True).encode()).hexdigest()


def _hash_path_contents(hasher, path: str, allow_missing: bool = False):
    path = os.path.expanduser(path)
    if not os.path.exists(path):
        if allow_missing:
            return
        raise ValueError(f"file mount source {path} does not exist")
    if os.path.isdir(path):
        for root, dirs, files in os.walk(path):
            dirs.sort()
            for fn in sorted(files):
                p = os.path.join(root, fn)
                hasher.update(os.path.relpath(p, path).encode())
                with open(p, "rb") as f:
                    hasher.update(f.read())
    else:
        with open(path, "rb") as f:
            hasher.update(f.read())


def hash_runtime_conf(file_mounts: Dict[str, str], cluster_synced_files: Optional[List[str]],
                      extra_objs: Any, generate_file_mounts_contents_hash: bool = False):
    """(runtime_hash, file_mounts_contents_hash): runtime hash decides whether setup
    re-runs; the contents hash whether file syncing is needed (reference utils.py:1588)."""
    contents = hashlib.sha1()
    for local in sorted((file_mounts or {}).values()):
        _hash_path_contents(contents, local)
    head_contents = contents.hexdigest()
    rh = hashlib.sha1()
    rh.update(json.dumps(file_mounts or {}, sort_keys=True).encode())
    rh.update(json.dumps(extra_objs, sort_keys=True, default=str).encode())
    rh.update(head_contents.encode())
    fm_hash = None
    if generate_file_mounts_contents_hash:
        for p in sorted(cluster_synced_files or []):
            _hash_path_contents(contents, p, allow_missing=True)
        fm_hash = contents.hexdigest()
    return rh.hexdigest(), fm_hash
