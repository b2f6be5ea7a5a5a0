"""Runtime service discovery (reference core/_private/service_discovery/runtime_discovery.py:1-300).

A runtime that depends on another service (Spark on HDFS, Presto on a metastore, Kafka on
ZooKeeper, a metastore on MySQL ...) finds it in one of two places:

* ``*_on_head``       -- the same cluster runs the service runtime: address it through the
  head (or the worker list for worker services) directly from the cluster config;
* ``*_from_workspace`` -- another cluster in the workspace published it as a workspace
  global variable (``service.<cluster>.<name>`` -> JSON service record, see
  ``cluster_operator._publish_services``); a ``<runtime>.<service>_service_selector`` in
  the runtime config narrows the candidates (clusters, features, names).

* ``*_from_consul``    -- a Consul agent on the node knows every registered instance of the
  service (healthy ones only), across clusters, selected by the same selector.

Each helper returns the URI the consumer's config needs (``hdfs://h:8020``,
``thrift://h:9083``, ``h1:2181,h2:2181`` ...) or ``None``.  Discovery of a dependency is on
unless the consumer sets ``<dependency>_service_discovery: false`` (then only the explicit
URI in its config counts).  ``with_database_environment_variables`` turns the database a
runtime uses (explicit ``database`` section, same cluster, Consul or workspace) into the
``CLOUDTIK_DATABASE_*`` variables its scripts read.
"""
from __future__ import annotations

from typing import Any, Callable, Dict, List, Optional

from cloudtik_amd.core import service_discovery as sd

# runtime type -> (service name, port, uri formatter over "host:port" addresses)
_KNOWN: Dict[str, tuple] = {
    "hdfs": ("hdfs-rpc", 8020, lambda a: f"hdfs://{a[0]}"),
    "minio": ("minio", 9000, lambda a: f"http://{a[0]}"),
    "metastore": ("metastore", 9083, lambda a: f"thrift://{a[0]}"),
    "zookeeper": ("zookeeper", 2181, lambda a: ",".join(a)),
    "etcd": ("etcd", 2379, lambda a: ",".join(f"http://{x}" for x in a)),
    "consul": ("consul", 8500, lambda a: a[0]),
    "mysql": ("mysql", 3306, lambda a: a[0]),
    "postgres": ("postgres", 5432, lambda a: a[0]),
}
DATABASE_RUNTIMES = ("mysql", "postgres")


def _runtime_types(config: Dict[str, Any]) -> List[str]:
    return list((config.get("runtime", {}) or {}).get("types", []) or [])


def _selector(config: Dict[str, Any], consumer: Optional[str], runtime_type: str) -> Dict[str, Any]:
    sel: Dict[str, Any] = {}
    if consumer:
        rc = (config.get("runtime", {}) or {}).get(consumer, {}) or {}
        sel = dict(rc.get(f"{runtime_type}_service_selector") or {})
    sel.setdefault("runtimes", [runtime_type])
    # a cluster does not discover its own services through the workspace
    ex = list(sel.get("exclude_clusters") or [])
    if config.get("cluster_name") and config["cluster_name"] not in ex:
        ex.append(config["cluster_name"])
    sel["exclude_clusters"] = ex
    return sel


def discover_runtime_services(global_variables: Dict[str, str], selector: Dict[str, Any]) -> List[Dict[str, Any]]:
    return sd.discover_services(global_variables, selector)


def service_addresses(service: Dict[str, Any]) -> List[str]:
    port = service.get("port")
    return [f"{h}:{port}" for h in (service.get("hosts") or [service.get("host")]) if h]


def discover_runtime_service_addresses(global_variables, runtime_type: str, service_name: Optional[str] = None,
                                       config: Optional[Dict[str, Any]] = None, consumer: Optional[str] = None,
                                       feature: Optional[str] = None) -> List[str]:
    """Addresses of the first matching workspace service (clusters sorted by name)."""
    sel = _selector(config or {}, consumer, runtime_type)
    if service_name:
        sel.setdefault("services", [service_name])
    if feature:
        sel.setdefault("features", [feature])
    found = discover_runtime_services(global_variables, sel)
    return service_addresses(found[0]) if found else []


def _workspace_global_variables(config: Dict[str, Any]) -> Dict[str, str]:
    from cloudtik_amd.core.provider_factory import get_workspace_provider
    try:
        wp = get_workspace_provider(config["provider"], config.get("workspace_name", "default"))
        return wp.subscribe_global_variables(config) or {}
    except Exception:  # noqa: BLE001 -- providers without a workspace provider
        return {}


def _from_workspace(runtime_type: str, config: Dict[str, Any], consumer: Optional[str],
                    global_variables: Optional[Dict[str, str]]) -> Optional[str]:
    name, _, fmt = _KNOWN[runtime_type]
    gv = global_variables if global_variables is not None else _workspace_global_variables(config)
    addrs = discover_runtime_service_addresses(gv, runtime_type, name, config, consumer)
    return fmt(addrs) if addrs else None


def _on_head(runtime_type: str, config: Dict[str, Any], head_ip: str,
             worker_ips: Optional[List[str]] = None) -> Optional[str]:
    if runtime_type not in _runtime_types(config):
        return None
    _, port, fmt = _KNOWN[runtime_type]
    from cloudtik_amd.runtime.catalog import A, W, SPEC_BY_NAME
    spec = SPEC_BY_NAME.get(runtime_type)
    kind = spec.services[0].node_kind if spec and spec.services else None
    if kind == W:
        hosts = list(worker_ips or [])
    elif kind == A:
        hosts = [head_ip] + list(worker_ips or [])
    else:
        hosts = [head_ip]
    return fmt([f"{h}:{port}" for h in hosts]) if hosts else None


def _make(runtime_type: str):
    def from_workspace(config, consumer: Optional[str] = None, global_variables=None):
        return _from_workspace(runtime_type, config, consumer, global_variables)

    def on_head(config, head_ip: str, worker_ips: Optional[List[str]] = None):
        return _on_head(runtime_type, config, head_ip, worker_ips)

    from_workspace.__name__ = f"discover_{runtime_type}_from_workspace"
    on_head.__name__ = f"discover_{runtime_type}_on_head"
    return from_workspace, on_head


discover_hdfs_from_workspace, discover_hdfs_on_head = _make("hdfs")
discover_minio_from_workspace, discover_minio_on_head = _make("minio")
discover_metastore_from_workspace, discover_metastore_on_head = _make("metastore")
discover_zookeeper_from_workspace, discover_zookeeper_on_head = _make("zookeeper")
discover_etcd_from_workspace, discover_etcd_on_head = _make("etcd")
discover_consul_from_workspace, discover_consul_on_head = _make("consul")


def discover_database_from_workspace(config, consumer: Optional[str] = None,
                                     global_variables=None) -> Optional[Dict[str, Any]]:
    """First MySQL / Postgres service in the workspace as ``{engine, address, port}``."""
    gv = global_variables if global_variables is not None else _workspace_global_variables(config)
    for engine in DATABASE_RUNTIMES:
        addrs = discover_runtime_service_addresses(gv, engine, engine, config, consumer)
        if addrs:
            host, _, port = addrs[0].rpartition(":")
            return {"engine": engine, "address": host, "port": int(port)}
    return None


def discover_database_on_head(config, head_ip: str) -> Optional[Dict[str, Any]]:
    for engine in DATABASE_RUNTIMES:
        if engine in _runtime_types(config):
            return {"engine": engine, "address": head_ip, "port": _KNOWN[engine][1]}
    return None


def is_service_discovery(config: Dict[str, Any], consumer: Optional[str], runtime_type: str) -> bool:
    """``<consumer>.<runtime_type>_service_discovery`` (default on)."""
    if not consumer:
        return True
    rc = (config.get("runtime", {}) or {}).get(consumer, {}) or {}
    return bool(rc.get(f"{runtime_type}_service_discovery", True))


def discover_from_consul(runtime_type: str, config: Dict[str, Any], consumer: Optional[str] = None,
                         consul_address: Optional[str] = None, client=None) -> Optional[str]:
    """Healthy instances of the runtime's service known to the node's Consul agent."""
    if runtime_type not in _KNOWN:
        return None
    import os
    addr = consul_address or os.environ.get("CONSUL_HTTP_ADDR")
    if client is None:
        if not addr:
            return None
        from cloudtik_amd.runtime.common.consul import ConsulClient
        client = ConsulClient(addr)
    name, _, fmt = _KNOWN[runtime_type]
    sel = _selector(config, consumer, runtime_type)
    sel.pop("exclude_clusters", None)         # the same cluster's instances are fine through Consul
    try:
        insts = [i for i in client.select_services(sel) if i.get("name", "").endswith(name)]
    except Exception:  # noqa: BLE001 - no agent on this node
        return None
    addrs = sorted(f"{i['host']}:{i['port']}" for i in insts)
    return fmt(addrs) if addrs else None


def discover_service(runtime_type: str, config: Dict[str, Any], head_ip: Optional[str] = None,
                     consumer: Optional[str] = None, global_variables=None,
                     worker_ips: Optional[List[str]] = None, consul_address: Optional[str] = None):
    """Same cluster first, then Consul (when an agent address is known), then the workspace
    (the order the reference runtimes use); nothing when the consumer turned discovery of
    this dependency off."""
    if not is_service_discovery(config, consumer, runtime_type):
        return None
    on_head: Callable = globals()[f"discover_{runtime_type}_on_head"]
    from_ws: Callable = globals()[f"discover_{runtime_type}_from_workspace"]
    if head_ip:
        r = on_head(config, head_ip) if runtime_type == "database" else on_head(config, head_ip, worker_ips)
        if r:
            return r
    if runtime_type != "database":
        r = discover_from_consul(runtime_type, config, consumer, consul_address)
        if r:
            return r
    return from_ws(config, consumer, global_variables)


def discover_hdfs_name(config: Dict[str, Any], head_ip: Optional[str] = None, consumer: Optional[str] = None,
                       global_variables=None) -> Optional[str]:
    """The HDFS URI a consumer writes into fs.defaultFS: the HA nameservice
    (``hdfs://<cluster>``) when the cluster's HDFS runs ``cluster_mode: ha_cluster``, else the
    single NameNode's address."""
    hdfs = (config.get("runtime", {}) or {}).get("hdfs", {}) or {}
    if "hdfs" in _runtime_types(config) and hdfs.get("cluster_mode") == "ha_cluster":
        return f"hdfs://{(hdfs.get('ha_cluster') or {}).get('name_service') or config.get('cluster_name', 'cloudtik')}"
    return discover_service("hdfs", config, head_ip, consumer, global_variables)


def with_database_environment_variables(config: Dict[str, Any], consumer: str, head_ip: Optional[str] = None,
                                        global_variables=None) -> Dict[str, str]:
    """``CLOUDTIK_DATABASE_{ENGINE,HOST,PORT,USERNAME,PASSWORD}`` for the consumer runtime's
    database: its explicit ``database`` section, else discovery (same cluster, workspace)."""
    rc = (config.get("runtime", {}) or {}).get(consumer, {}) or {}
    db = dict(rc.get("database") or {})
    if not db.get("address") and not db.get("host"):
        found = None
        if is_service_discovery(config, consumer, "database"):
            found = (discover_database_on_head(config, head_ip) if head_ip else None) or \
                discover_database_from_workspace(config, consumer, global_variables)
        if not found:
            return {}
        db = dict(found, **{k: v for k, v in db.items() if v})
    engine = db.get("engine", "mysql")
    return {"CLOUDTIK_DATABASE_ENGINE": engine,
            "CLOUDTIK_DATABASE_HOST": str(db.get("address") or db.get("host")),
            "CLOUDTIK_DATABASE_PORT": str(db.get("port") or (3306 if engine == "mysql" else 5432)),
            "CLOUDTIK_DATABASE_USERNAME": str(db.get("username") or db.get("user") or
                                              ("root" if engine == "mysql" else "postgres")),
            "CLOUDTIK_DATABASE_PASSWORD": str(db.get("password") or "cloudtik")}
