"""Runtime registry (reference ``core/_private/runtime_factory.py:244``) and dependency
ordering of runtimes for command merging (reference ``utils.py:776``
``reorder_runtimes_for_dependency``)."""
from __future__ import annotations

import importlib
from typing import Any, Dict, List

BUILT_IN_RUNTIME_AI = "ai"
BUILT_IN_RUNTIME_NONE = "none"

_CUSTOM = {
    "ai": ("cloudtik_amd.runtime.ai.runtime", "AIRuntime"),
    # self-configuring Hadoop family: conf files rendered per node, executor sizing, YARN
    # scaling policy / job waiter (cloudtik_amd/runtime/hadoop)
    "hadoop": ("cloudtik_amd.runtime.hadoop.runtimes", "HadoopRuntime"),
    "hdfs": ("cloudtik_amd.runtime.hadoop.runtimes", "HdfsRuntime"),
    "yarn": ("cloudtik_amd.runtime.hadoop.runtimes", "YarnRuntime"),
    "spark": ("cloudtik_amd.runtime.hadoop.runtimes", "SparkRuntime"),
    # service runtimes that render their own configuration (cloudtik_amd/runtime/configured.py)
    **{n: ("cloudtik_amd.runtime.configured", c) for n, c in (
        ("zookeeper", "ZooKeeperRuntime"), ("kafka", "KafkaRuntime"), ("redis", "RedisRuntime"),
        ("mongodb", "MongoDBRuntime"), ("consul", "ConsulRuntime"), ("etcd", "EtcdRuntime"),
        ("coredns", "CoreDNSRuntime"), ("mysql", "MySQLRuntime"), ("postgres", "PostgresRuntime"),
        ("prometheus", "PrometheusRuntime"), ("grafana", "GrafanaRuntime"), ("haproxy", "HAProxyRuntime"),
        ("loadbalancer", "LoadBalancerRuntime"))},
    # part 2: query engines, frameworks, stores, gateways, DNS, poolers, node utilities
    **{n: ("cloudtik_amd.runtime.configured_more", c) for n, c in (
        ("metastore", "MetastoreRuntime"), ("presto", "PrestoRuntime"), ("trino", "TrinoRuntime"),
        ("flink", "FlinkRuntime"), ("ray", "RayRuntime"), ("minio", "MinIORuntime"),
        ("elasticsearch", "ElasticsearchRuntime"), ("nginx", "NginxRuntime"), ("kong", "KongRuntime"),
        ("apisix", "APISIXRuntime"), ("dnsmasq", "DnsmasqRuntime"), ("bind", "BindRuntime"),
        ("pgbouncer", "PgBouncerRuntime"), ("pgpool", "PgpoolRuntime"), ("mount", "MountRuntime"),
        ("sshserver", "SSHServerRuntime"), ("xinetd", "XinetdRuntime"), ("nodex", "NodexRuntime"))},
}


def _catalog_names():
    from cloudtik_amd.runtime.catalog import SPEC_BY_NAME
    return list(SPEC_BY_NAME)


def list_runtimes() -> List[str]:
    return sorted(set(_CUSTOM) | set(_catalog_names()))


_cls_cache: Dict[str, Any] = {}


def get_runtime_cls(name: str):
    if name in _cls_cache:
        return _cls_cache[name]
    if name in _CUSTOM:
        mod, cls = _CUSTOM[name]
        c = getattr(importlib.import_module(mod), cls)
    else:
        from cloudtik_amd.runtime.catalog import SPEC_BY_NAME, make_runtime_class
        if name not in SPEC_BY_NAME:
            raise NotImplementedError(f"Unsupported runtime: {name}")
        c = make_runtime_class(name)
    _cls_cache[name] = c
    return c


def register_runtime(name: str, cls):
    _cls_cache[name] = cls
    _CUSTOM[name] = (cls.__module__, cls.__name__)


def get_runtime(name: str, runtime_config: Dict[str, Any]):
    return get_runtime_cls(name)(runtime_config)


def get_runtime_types(config: Dict[str, Any]) -> List[str]:
    return list((config.get("runtime") or {}).get("types") or [])


def _deps(name: str) -> List[str]:
    cls = get_runtime_cls(name)
    try:
        return list(cls({}).get_dependencies())
    except Exception:  # noqa: BLE001
        return []


def reorder_runtimes_for_dependency(types: List[str]) -> List[str]:
    """Stable topological order: a runtime comes after the runtimes it depends on (only
    those present in ``types``)."""
    present = set(types)
    order, state = [], {}

    def visit(n):
        if state.get(n) == 2:
            return
        if state.get(n) == 1:
            raise ValueError(f"runtime dependency cycle at {n}")
        state[n] = 1
        for d in _deps(n):
            if d in present:
                visit(d)
        state[n] = 2
        order.append(n)

    for t in types:
        visit(t)
    return order


def add_required_runtimes(types: List[str]) -> List[str]:
    """Append runtimes that a selected runtime requires (reference ``get_required``)."""
    out = list(types)
    changed = True
    while changed:
        changed = False
        for t in list(out):
            for r in get_runtime_cls(t)({}).get_required():
                if r not in out:
                    out.insert(out.index(t), r)
                    changed = True
    return out
