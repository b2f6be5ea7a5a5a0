"""Layered config loading: ``from:`` template inheritance + provider system defaults.

Resolution order (reference ``utils.py:465-597``):

1. a config with ``from: <template>`` is merged ON TOP of that template, recursively
   (user template dirs from ``$CLOUDTIK_USER_TEMPLATES`` first, then the built-in
   ``cloudtik_amd/templates``, then the generated provider size / GPU-family templates of
   ``instance_templates.py``);
2. the root of the chain is merged on top of the provider's system defaults
   (``providers/<type>/defaults.yaml``, which itself chains ``from: defaults`` to the global
   ``providers/defaults.yaml``).

Objects other than clusters (workspace / storage / database) use
``<object>-defaults.yaml`` files the same way.
"""
from __future__ import annotations

import copy
import os
from typing import Any, Dict, Optional

import yaml

from cloudtik_amd.core import constants
from .merge import merge_config

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PROVIDERS_DIR = os.path.join(PKG_ROOT, "providers")
TEMPLATES_DIR = os.path.join(PKG_ROOT, "templates")


def load_yaml(path: str) -> Dict[str, Any]:
    with open(os.path.expanduser(path)) as f:
        return yaml.safe_load(f) or {}


def _user_template(name: str) -> Optional[str]:
    dirs = os.environ.get(constants.CLOUDTIK_USER_TEMPLATES, "")
    for d in (x.strip() for x in dirs.split(",") if x.strip()):
        p = os.path.join(os.path.expanduser(d), name)
        if os.path.exists(p):
            return p
    return None


def template_path(name: str, system: bool = False) -> str:
    if not name.endswith(".yaml"):
        name += ".yaml"
    if system:
        return os.path.join(PROVIDERS_DIR, name)
    p = _user_template(name)
    return p or os.path.join(TEMPLATES_DIR, name)


def provider_home(provider: Dict[str, Any]) -> str:
    from cloudtik_amd.core.provider_factory import get_provider_home
    return get_provider_home(provider)


def _defaults_file(provider: Dict[str, Any], object_name: Optional[str]) -> str:
    fname = "defaults.yaml" if object_name is None else f"{object_name}-defaults.yaml"
    return os.path.join(provider_home(provider), fname)


def merge_config_hierarchy(provider: Dict[str, Any], config: Dict[str, Any], system: bool = False,
                           object_name: Optional[str] = None) -> Dict[str, Any]:
    base = config.get("from")
    if base:
        path = template_path(base, system)
        if os.path.exists(path) or system:
            tmpl = load_yaml(path)
        else:
            # provider size / GPU-family templates are generated (core/config/instance_templates.py)
            from .instance_templates import synthesize
            tmpl = synthesize(base)
            if tmpl is None:
                raise FileNotFoundError(f"no template {base!r} ({path} does not exist and it is not a "
                                        f"known <provider>/<size> or <provider>/gpu/<family>/<size> template)")
        tp = tmpl.get("provider", {}).get("type")
        if tp and tp != provider.get("type"):
            raise RuntimeError(f"Template provider type ({tp}) doesn't match ({provider.get('type')})!")
        merged_base = merge_config_hierarchy(provider, tmpl, system, object_name)
        return merge_config(merged_base, config)
    if system:
        return config
    path = _defaults_file(provider, object_name)
    defaults = load_yaml(path) if os.path.exists(path) else {}
    merged = merge_config_hierarchy(provider, defaults, True, object_name)
    return copy.deepcopy(merge_config(merged, config))


def fill_with_defaults(config: Dict[str, Any], object_name: Optional[str] = None) -> Dict[str, Any]:
    merged = merge_config_hierarchy(config["provider"], copy.deepcopy(config), object_name=object_name)
    merged["auth"] = merged.get("auth", {}) or {}
    merged.pop("min_workers", None)
    merged.pop("from", None)
    return merged


def load_config_file(path: str, overrides: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
    cfg = load_yaml(path)
    if overrides:
        cfg = merge_config(cfg, overrides)
    return cfg
