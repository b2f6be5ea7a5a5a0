"""Script alias registry (reference core/_private/script_registry.py:20-52).

Runtime packages export ``_script_aliases_ = {alias: module}``; ``cloudtik submit`` turns a
registered alias into ``python -m <module>`` on the target node.  Only the direct
sub-packages of ``cloudtik_amd.runtime`` are scanned.
"""
from __future__ import annotations

import importlib
import pkgutil
from typing import Dict, Optional

SCRIPT_ALIASES = "_script_aliases_"

_registry: Optional[Dict[str, str]] = None


def _scan() -> Dict[str, str]:
    import cloudtik_amd.runtime as runtime
    reg: Dict[str, str] = {}
    for info in pkgutil.iter_modules(runtime.__path__):
        if not info.ispkg:
            continue
        try:
            mod = importlib.import_module(f"{runtime.__name__}.{info.name}")
        except ImportError:
            continue
        reg.update(getattr(mod, SCRIPT_ALIASES, {}) or {})
    return reg


def register(alias: str, target: str):
    registry()[alias] = target


def registry() -> Dict[str, str]:
    global _registry
    if _registry is None:
        _registry = _scan()
    return _registry


def get_registered_script(alias: str) -> Optional[str]:
    return registry().get(alias)
