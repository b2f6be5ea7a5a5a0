"""Deep-merge rules of the layered YAML config (reference ``utils.py:2137-2236``).

* mappings merge recursively;
* a one-element list of a ``{"name": ...}`` mapping merges INTO the target's one-element
  list when the names match (used for e.g. node disk lists);
* ``key++: [...]`` appends after and ``++key: [...]`` prepends before the target list;
* anything else replaces.
"""
from __future__ import annotations

import collections.abc
import copy
from typing import Any, Dict


def _only_named_child(v):
    if not isinstance(v, list) or len(v) != 1:
        return None
    c = v[0]
    if not isinstance(c, collections.abc.Mapping) or "name" not in c:
        return None
    return c


def _is_append_key(k, v) -> bool:
    return isinstance(v, list) and isinstance(k, str) and (k.endswith("++") or k.startswith("++"))


def update_nested_dict(target: Dict[str, Any], new: Dict[str, Any],
                       match_list_item_with_name: bool = True,
                       advanced_list_appending: bool = True) -> Dict[str, Any]:
    appends = {}
    for k, v in new.items():
        if isinstance(v, collections.abc.Mapping):
            base = target.get(k)
            target[k] = update_nested_dict(base if isinstance(base, dict) else {}, v,
                                           match_list_item_with_name, advanced_list_appending)
            continue
        if match_list_item_with_name:
            ni, ti = _only_named_child(v), _only_named_child(target.get(k))
            if ni is not None and ti is not None and ni["name"] == ti["name"]:
                target[k][0] = update_nested_dict(ti, ni, match_list_item_with_name,
                                                  advanced_list_appending)
                continue
        if advanced_list_appending and _is_append_key(k, v):
            appends[k] = v
        else:
            target[k] = v
    for k, v in appends.items():
        if k.startswith("++"):
            key = k[2:]
            cur = target.get(key)
            target[key] = v + cur if cur is not None else v
        else:
            key = k[:-2]
            cur = target.get(key)
            target[key] = cur + v if cur is not None else v
    return target


def merge_config(config: Dict[str, Any], updates: Dict[str, Any]) -> Dict[str, Any]:
    return update_nested_dict(config, updates)


def merged_copy(base: Dict[str, Any], updates: Dict[str, Any]) -> Dict[str, Any]:
    return update_nested_dict(copy.deepcopy(base), copy.deepcopy(updates))
