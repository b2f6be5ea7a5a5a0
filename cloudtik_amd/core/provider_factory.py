"""Provider registries (reference ``core/_private/provider_factory.py:119``).

``type`` in the provider config selects a NodeProvider / WorkspaceProvider /
StorageProvider / DatabaseProvider class.  ``type: external`` loads ``provider_class``
(and ``workspace_provider_class``) by dotted path.  Providers import lazily so the
control plane does not pull in backends it does not use.
"""
from __future__ import annotations

import importlib
import os
import threading
from typing import Any, Dict

_lock = threading.RLock()
_cache: Dict[Any, Any] = {}


def load_class(path: str):
    mod, _, cls = path.rpartition(".")
    return getattr(importlib.import_module(mod), cls)


def _lazy(module: str, cls: str):
    return lambda: getattr(importlib.import_module(module), cls)


_NODE_PROVIDERS = {
    "local": _lazy("cloudtik_amd.providers.local.node_provider", "LocalNodeProvider"),
    "onpremise": _lazy("cloudtik_amd.providers.onpremise.node_provider", "OnPremiseNodeProvider"),
    "virtual": _lazy("cloudtik_amd.providers.virtual.node_provider", "VirtualNodeProvider"),
    "aws": _lazy("cloudtik_amd.providers.cloud.node_provider", "AWSNodeProvider"),
    "gcp": _lazy("cloudtik_amd.providers.cloud.node_provider", "GCPNodeProvider"),
    "azure": _lazy("cloudtik_amd.providers.cloud.node_provider", "AzureNodeProvider"),
    "aliyun": _lazy("cloudtik_amd.providers.cloud.node_provider", "AliyunNodeProvider"),
    "huaweicloud": _lazy("cloudtik_amd.providers.cloud.node_provider", "HuaweiCloudNodeProvider"),
    "kubernetes": _lazy("cloudtik_amd.providers.kubernetes.node_provider", "KubernetesNodeProvider"),
    "mock": _lazy("cloudtik_amd.providers.mock.node_provider", "MockProvider"),
    "external": None,
}

_WORKSPACE_PROVIDERS = {
    "local": _lazy("cloudtik_amd.providers.local.workspace_provider", "LocalWorkspaceProvider"),
    "onpremise": _lazy("cloudtik_amd.providers.onpremise.workspace_provider", "OnPremiseWorkspaceProvider"),
    "virtual": _lazy("cloudtik_amd.providers.local.workspace_provider", "LocalWorkspaceProvider"),
    "aws": _lazy("cloudtik_amd.providers.cloud.workspace_provider", "CloudWorkspaceProvider"),
    "gcp": _lazy("cloudtik_amd.providers.cloud.workspace_provider", "CloudWorkspaceProvider"),
    "azure": _lazy("cloudtik_amd.providers.cloud.workspace_provider", "CloudWorkspaceProvider"),
    "aliyun": _lazy("cloudtik_amd.providers.cloud.workspace_provider", "CloudWorkspaceProvider"),
    "huaweicloud": _lazy("cloudtik_amd.providers.cloud.workspace_provider", "CloudWorkspaceProvider"),
    "kubernetes": _lazy("cloudtik_amd.providers.cloud.workspace_provider", "CloudWorkspaceProvider"),
    "mock": _lazy("cloudtik_amd.providers.local.workspace_provider", "LocalWorkspaceProvider"),
}

_STORAGE_PROVIDERS = {
    "aws": _lazy("cloudtik_amd.providers.cloud.storage_provider", "CloudStorageProvider"),
    "gcp": _lazy("cloudtik_amd.providers.cloud.storage_provider", "CloudStorageProvider"),
    "azure": _lazy("cloudtik_amd.providers.cloud.storage_provider", "CloudStorageProvider"),
    "aliyun": _lazy("cloudtik_amd.providers.cloud.storage_provider", "CloudStorageProvider"),
    "huaweicloud": _lazy("cloudtik_amd.providers.cloud.storage_provider", "CloudStorageProvider"),
}
_DATABASE_PROVIDERS = {k: _lazy("cloudtik_amd.providers.cloud.storage_provider", "CloudDatabaseProvider")
                       for k in _STORAGE_PROVIDERS}

_PROVIDER_HOMES = {
    "local": "local", "onpremise": "onpremise", "virtual": "virtual", "aws": "aws", "gcp": "gcp",
    "azure": "azure", "aliyun": "aliyun", "huaweicloud": "huaweicloud", "kubernetes": "kubernetes",
    "mock": "local",
}


def register_node_provider(type_name: str, cls_or_factory, home: str = None):
    """Used by tests (the reference registers a "mock" provider the same way,
    tests/unit/test_cloudtik.py:619-620)."""
    _NODE_PROVIDERS[type_name] = cls_or_factory if callable(cls_or_factory) and not isinstance(cls_or_factory, type) \
        else (lambda: cls_or_factory)
    if home:
        _PROVIDER_HOMES[type_name] = home


def get_provider_home(provider_config: Dict[str, Any]) -> str:
    from cloudtik_amd.core.config.loader import PROVIDERS_DIR
    t = provider_config["type"]
    if t == "external":
        home = provider_config.get("provider_home")
        return home or PROVIDERS_DIR
    sub = _PROVIDER_HOMES.get(t)
    if sub is None:
        raise NotImplementedError(f"unsupported provider type {t}")
    if os.path.isabs(sub):
        return sub
    return os.path.join(PROVIDERS_DIR, sub)


def get_node_provider_cls(provider_config: Dict[str, Any]):
    t = provider_config["type"]
    if t == "external":
        return load_class(provider_config["provider_class"])
    f = _NODE_PROVIDERS.get(t)
    if f is None:
        raise NotImplementedError(f"Unsupported node provider: {t}")
    return f()


def get_node_provider(provider_config: Dict[str, Any], cluster_name: str, use_cache: bool = True):
    key = (provider_config.get("type"), repr(sorted(provider_config.items(), key=lambda kv: kv[0])), cluster_name)
    with _lock:
        if use_cache and key in _cache:
            return _cache[key]
        p = get_node_provider_cls(provider_config)(provider_config, cluster_name)
        if use_cache:
            _cache[key] = p
        return p


def get_workspace_provider(provider_config: Dict[str, Any], workspace_name: str):
    t = provider_config["type"]
    if t == "external":
        return load_class(provider_config["workspace_provider_class"])(provider_config, workspace_name)
    return _WORKSPACE_PROVIDERS[t]()(provider_config, workspace_name)


def get_storage_provider(provider_config, workspace_name, storage_name):
    return _STORAGE_PROVIDERS[provider_config["type"]]()(provider_config, workspace_name, storage_name)


def get_database_provider(provider_config, workspace_name, database_name):
    return _DATABASE_PROVIDERS[provider_config["type"]]()(provider_config, workspace_name, database_name)


def clear_cache():
    with _lock:
        _cache.clear()
