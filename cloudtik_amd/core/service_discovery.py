"""Runtime service model: what a runtime exposes and how other runtimes / clusters find it.

Mirrors the reference's ``core/_private/service_discovery/utils.py:173-382`` and
``runtime_services.py``: a service has a name, port, protocol, scope (cluster-local or
workspace-wide), node kind (head/worker/all), feature tags and an optional selector used by
consumers.  Workspace-wide services are published as workspace global variables
(``WorkspaceProvider.publish_global_variables``) and discovered by name/runtime type.
"""
from __future__ import annotations

import json
from typing import Any, Dict, List, Optional

SERVICE_SCOPE_LOCAL = "local"
SERVICE_SCOPE_WORKSPACE = "workspace"

SERVICE_DISCOVERY_PROTOCOL_TCP = "tcp"
SERVICE_DISCOVERY_PROTOCOL_HTTP = "http"

SERVICE_DISCOVERY_NODE_KIND_HEAD = "head"
SERVICE_DISCOVERY_NODE_KIND_WORKER = "worker"
SERVICE_DISCOVERY_NODE_KIND_NODE = "node"

SERVICE_DISCOVERY_FEATURE_DATABASE = "database"
SERVICE_DISCOVERY_FEATURE_STORAGE = "storage"
SERVICE_DISCOVERY_FEATURE_METRICS = "metrics"
SERVICE_DISCOVERY_FEATURE_DNS = "dns"
SERVICE_DISCOVERY_FEATURE_LOAD_BALANCER = "load-balancer"
SERVICE_DISCOVERY_FEATURE_SCHEDULER = "scheduler"
SERVICE_DISCOVERY_FEATURE_ANALYTICS = "analytics"
SERVICE_DISCOVERY_FEATURE_KEY_VALUE = "kv"
SERVICE_DISCOVERY_FEATURE_AI = "ai"


class ServiceRegister(dict):
    """One service definition (name, port, protocol, node_kind, scope, tags, features)."""


def define_runtime_service(service_type: str, name: str, port: int,
                           protocol: str = SERVICE_DISCOVERY_PROTOCOL_TCP,
                           node_kind: str = SERVICE_DISCOVERY_NODE_KIND_HEAD,
                           scope: str = SERVICE_SCOPE_WORKSPACE, features: Optional[List[str]] = None,
                           metrics: bool = False) -> ServiceRegister:
    return ServiceRegister(service_type=service_type, name=name, port=int(port), protocol=protocol,
                           node_kind=node_kind, scope=scope, features=list(features or []),
                           metrics=metrics)


def define_runtime_service_on_head(service_type, name, port, **kw):
    return define_runtime_service(service_type, name, port, node_kind=SERVICE_DISCOVERY_NODE_KIND_HEAD, **kw)


def define_runtime_service_on_worker(service_type, name, port, **kw):
    return define_runtime_service(service_type, name, port, node_kind=SERVICE_DISCOVERY_NODE_KIND_WORKER, **kw)


def define_runtime_service_on_all(service_type, name, port, **kw):
    return define_runtime_service(service_type, name, port, node_kind=SERVICE_DISCOVERY_NODE_KIND_NODE, **kw)


def get_service_selector_for_update(config: Dict[str, Any], key: str) -> Dict[str, Any]:
    sel = config.get(key) or {}
    config[key] = sel
    return sel


def include_runtime_for_selector(selector: Dict[str, Any], runtime: str) -> Dict[str, Any]:
    rts = selector.setdefault("runtimes", [])
    if runtime not in rts:
        rts.append(runtime)
    return selector


LABEL_CLUSTER, LABEL_RUNTIME, LABEL_SERVICE = "cloudtik-cluster", "cloudtik-runtime", "cloudtik-service"


def service_tags(service: Dict[str, Any]) -> set:
    """Implicit tags of a service record: ``cloudtik-c-<cluster>``, ``cloudtik-r-<runtime>``,
    ``cloudtik-f-<feature>`` (the tags Consul registrations carry) plus explicit ``tags``."""
    out = set(service.get("tags") or [])
    if service.get("cluster"):
        out.add(f"cloudtik-c-{service['cluster']}")
    if service.get("service_type"):
        out.add(f"cloudtik-r-{service['service_type']}")
    out.update(f"cloudtik-f-{f}" for f in service.get("features") or [])
    return out


def service_labels(service: Dict[str, Any]) -> Dict[str, str]:
    labels = {LABEL_CLUSTER: service.get("cluster"), LABEL_RUNTIME: service.get("service_type"),
              LABEL_SERVICE: service.get("name")}
    labels.update(service.get("labels") or {})
    return {k: v for k, v in labels.items() if v is not None}


def match_service(service: Dict[str, Any], selector: Optional[Dict[str, Any]]) -> bool:
    """Selector keys (reference service_discovery/utils.py SERVICE_SELECTOR_*): services,
    service_types / runtimes, clusters (+ exclude_* of each), tags (all required), features
    (any), labels (all equal), exclude_labels (none equal)."""
    if not selector:
        return True
    for key, field in (("services", "name"), ("service_types", "service_type"),
                       ("runtimes", "service_type"), ("clusters", "cluster")):
        want = selector.get(key)
        if want and service.get(field) not in want:
            return False
        ex = selector.get(f"exclude_{key}")
        if ex and service.get(field) in ex:
            return False
    feats = selector.get("features")
    if feats and not set(feats) & set(service.get("features", [])):
        return False
    tags = selector.get("tags")
    if tags and not set(tags) <= service_tags(service):
        return False
    labels = service_labels(service)
    for k, v in (selector.get("labels") or {}).items():
        if labels.get(k) != v:
            return False
    for k, v in (selector.get("exclude_labels") or {}).items():
        if labels.get(k) == v:
            return False
    return True


# ------------------------------------------------------------------ global-variable encoding
def service_global_key(cluster_name: str, service_name: str) -> str:
    return f"service.{cluster_name}.{service_name}"


def encode_service_address(service: Dict[str, Any], host: str, hosts: Optional[List[str]] = None) -> str:
    """``host`` is where head-kind services listen; worker/all-kind services list every node."""
    return json.dumps({**service, "host": host, "hosts": list(hosts) if hosts else [host]}, sort_keys=True)


def decode_service_address(value: str) -> Dict[str, Any]:
    try:
        return json.loads(value)
    except (TypeError, ValueError):
        host, _, port = str(value).partition(":")
        return {"host": host, "port": int(port) if port.isdigit() else None}


def discover_services(global_variables: Dict[str, str], selector: Optional[Dict[str, Any]] = None):
    out = []
    for k, v in (global_variables or {}).items():
        if not k.startswith("service."):
            continue
        _, cluster, _name = k.split(".", 2)
        svc = decode_service_address(v)
        svc.setdefault("cluster", cluster)
        if match_service(svc, selector):
            out.append(svc)
    return sorted(out, key=lambda s: (s.get("cluster", ""), s.get("name", "")))
