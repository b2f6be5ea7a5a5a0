"""Generate the runtime / workspace / storage / database JSON schemas from compact tables.

    python -m cloudtik_amd.schema.build        # rewrites runtime.json, workspace.json, ...

Every runtime section lists its keys with a type shorthand; a section rejects unknown keys
(typos fail at ``cloudtik start`` instead of silently doing nothing) except ``config`` /
``envs`` pass-through objects and ``with_*`` feature flags.  Key names follow the reference
schema (python/cloudtik/schema/runtime.json) so existing cluster YAML validates; keys this
framework adds are marked ``# +``.
"""
from __future__ import annotations

import json
import os
from typing import Any, Dict

HERE = os.path.dirname(os.path.abspath(__file__))

T = {"b": {"type": "boolean"}, "i": {"type": "integer", "minimum": 0}, "n": {"type": "number"},
     "s": {"type": "string"}, "o": {"type": "object"}, "a": {"type": "array"},
     "bs": {"type": ["boolean", "string"]}, "sel": {"$ref": "#/definitions/service_selector"},
     "db": {"$ref": "#/definitions/database_connect"}, "port": {"type": "integer", "minimum": 1, "maximum": 65535}}


def _sd(prefix: str) -> Dict[str, str]:
    """service discovery switch + selector for a dependency (``<dep>_service_discovery``)."""
    return {f"{prefix}_service_discovery": "b", f"{prefix}_service_selector": "sel"}


_METASTORE = dict(_sd("metastore"), hive_metastore_uri="s")
_DATABASE = dict(_sd("database"), database="db")

RUNTIMES: Dict[str, Dict[str, Any]] = {
    "ai": dict(_DATABASE, with_gpu="bs", with_oneapi="b", mlflow="o", rccl="o", miopen_find_mode="s",
               hdfs_namenode_uri="s"),                                                    # + rccl/miopen/hdfs
    "apisix": dict(_sd("etcd"), port="port", admin_port="port", admin_key="s", etcd_uri="s", backend="o"),
    "bind": dict(port="port", dnssec_validation="s", default_resolver="b"),
    "consul": dict(server="b", data_center="s", disable_cluster_node_name="b", rpc_port="port", http_port="port",
                   dns_port="port"),
    "coredns": dict(port="port", default_resolver="b"),
    "dnsmasq": dict(port="port", default_resolver="b"),
    "elasticsearch": dict(port="port", transport_port="port", cluster_mode={"enum": ["none", "cluster"]},
                          security="b", password="s", snapshot_repository="b", clustering="o"),
    "etcd": dict(port="port", peer_port="port"),
    "flink": dict(_METASTORE, config="o"),
    "grafana": dict(port="port", high_availability="b",
                    data_sources_scope={"enum": ["none", "local", "workspace"]}, data_sources="a",
                    data_sources_services="sel", discovery_interval="i", consul_address="s", admin_user="s",
                    admin_password="s"),
    "hadoop": dict(_sd("hdfs"), **_sd("minio"), hadoop_default_cluster="b", hdfs_namenode_uri="s",
                   minio_endpoint_uri="s", minio_storage="o", default_storage="s"),               # + default_storage
    "haproxy": dict(port="port", protocol="s", app_mode="s", high_availability="b", backend="o"),
    "hdfs": dict(cluster_mode={"enum": ["simple", "ha_cluster"]}, ha_cluster="o", force_clean="b",
                 health_check_port="port", dfs_replication="i", dfs_blocksize="i"),              # + dfs_*
    "kafka": dict(_sd("zookeeper"), config="o", zookeeper_connect="s"),
    "kong": dict(_DATABASE, port="port", ssl_port="port", backend="o"),
    "loadbalancer": dict(high_availability="b", provider="o", backend="o"),
    "metastore": dict(_DATABASE, high_availability="b"),
    "minio": dict(port="port", console_port="port", server_pool_size="i", service_on_head="b"),
    "mongodb": dict(port="port", cluster_mode={"enum": ["none", "replication", "sharding"]}, root_user="s",
                    root_password="s", database="o", replication_set_name="s", replication_set_key="s",
                    sharding="o"),
    "mount": dict(hdfs_mount_method={"enum": ["fuse", "nfs"]}),
    "mysql": dict(port="port", cluster_mode={"enum": ["none", "replication", "group_replication"]},
                  root_password="s", health_check_port="port", database="o", group_replication="o"),
    "nginx": dict(port="port", app_mode="s", high_availability="b", backend="o"),
    "nodex": dict(port="port"),
    "pgbouncer": dict(port="port", high_availability="b", admin_user="s", admin_password="s", pool="o", backend="o"),
    "pgpool": dict(port="port", high_availability="b", admin_user="s", admin_password="s", postgres_admin_user="s",
                   postgres_admin_password="s", replication_user="s", replication_password="s", max_pool="i",
                   pcp_port="port", backend="o"),
    "postgres": dict(port="port", cluster_mode={"enum": ["none", "replication"]}, admin_user="s",
                     admin_password="s", replication_user="s", replication_password="s", archive_mode="b",
                     replication_slot="b", health_check_port="port", replication_synchronous="o", database="o",
                     repmgr="o"),
    "presto": dict(_METASTORE, config="o", catalogs="o"),
    "prometheus": dict(port="port", high_availability="b",
                       scrape_scope={"enum": ["local", "workspace", "federation"]}, scrape_services="sel",
                       service_discovery={"enum": ["file", "consul"]}, federation_targets="a",
                       pull_services="o", pull_interval="i", consul_address="s", use_consul="b"),
    "ray": dict(scaling="o"),
    "redis": dict(port="port", cluster_mode={"enum": ["none", "replication", "sharding"]}, password="s",
                  health_check_port="port", replication="o", sharding="o"),
    "spark": dict(_METASTORE, config="o", spark_executor_resource="o",                           # + sizing
                  optimizations={"type": ["object", "array", "string", "boolean"]}, optimized_build="b"),  # +
    "sshserver": dict(port="port"),
    "trino": dict(_METASTORE, catalogs="o"),
    "yarn": dict(scaling={"$ref": "#/definitions/yarn_scaling"}, yarn_resource_memory_ratio="n",
                 yarn_scheduler={"enum": ["capacity", "fair"]}, yarn_container_maximum="o"),  # + container max
    "zookeeper": dict(config="o"),
}

# keys the self-configuring runtimes add (runtime/configured*.py; node sizing overrides, rendered
# file settings)                                                                            # +
_NODE = dict(node_memory_mb="i", node_cpus="i")
_ADDED: Dict[str, Dict[str, Any]] = {
    "apisix": dict(etcd_hosts="a"),
    "bind": dict(domain="s", upstream="a"),
    "dnsmasq": dict(domain="s", upstream="a"),
    "elasticsearch": dict(_NODE, master_nodes="i", data_dir="s", heap_mb="i", config="o"),
    "flink": dict(_NODE, taskmanager_slots="i", taskmanager_memory_mb="i", jobmanager_memory_mb="i",
                  parallelism="i", execution_target="s", state_backend="s", checkpoints_dir="s",
                  high_availability_zookeeper="s"),
    "kong": dict(config="o"),
    "loadbalancer": dict(consul_address="s", use_consul="b"),
    "metastore": dict(warehouse_dir="s", config="o"),
    "minio": dict(access_key="s", secret_key="s", data_disks="i"),
    "mount": dict(mount_path="s", storage="o"),
    "nginx": dict(web_root="s"),
    "pgbouncer": dict(postgres_host="s", postgres_port="port", databases="o", pool_mode="s", max_client_conn="i",
                      default_pool_size="i"),
    "pgpool": dict(num_init_children="i", user="s", primary_no_reads="b"),
    "presto": dict(_NODE, jvm_max_memory_mb="i", query_max_memory_per_node_mb="i", query_max_memory_gb="i",
                   environment="s", data_dir="s", hive="o"),
    "ray": dict(_NODE, node_gpus="i", object_store_ratio="n", resources="o", auto_scaling="b"),
    "sshserver": dict(authorized_keys="s"),
    "trino": dict(_NODE, jvm_max_memory_mb="i", query_max_memory_per_node_mb="i", query_max_memory_gb="i",
                  environment="s", data_dir="s", hive="o", config="o"),
    "xinetd": dict(services="o"),
    "redis": dict(health_check_user="s"), "mysql": dict(health_check_user="s"),
    "postgres": dict(health_check_user="s"),
}
for _rt, _keys in _ADDED.items():
    RUNTIMES.setdefault(_rt, {}).update(_keys)

SCALING = dict(scaling_policy_class="s", scaling_policy={"enum": ["scaling-with-resources", "scaling-with-load",
                                                                   "scaling-with-time"]},
               scaling_policy_by_node_type="o", scaling_step="i", scaling_resource="s", cpu_load_threshold="n",
               memory_load_threshold="n", gpu_busy_threshold="n", in_use_cpu_load_threshold="n",
               scaling_periodic={"enum": ["daily", "weekly", "monthly"]},
               scaling_math_base={"enum": ["on-min-workers", "on-previous-time"]}, scaling_time_table="o",
               scaling_with_load="o", scaling_with_time="o")
YARN_SCALING = dict(scaling_mode={"enum": ["none", "apps-pending", "aggressive"]}, scaling_step="i",
                    scaling_resource={"enum": ["memory", "CPU"]}, apps_pending_threshold="i",
                    apps_pending_free_cores_threshold="n", apps_pending_free_memory_threshold="n",
                    aggressive_free_ratio_threshold="n")


def _expand(spec):
    if isinstance(spec, str):
        return dict(T[spec])
    return spec


# keys every runtime section accepts: the quorum manager's minimal node count (quorum
# runtimes wait for it before configuring, core/head/quorum_manager.py)
COMMON = {"minimal_nodes": "i"}


def _section(keys: Dict[str, Any], strict: bool = True) -> Dict[str, Any]:
    out = {"type": "object", "properties": {k: _expand(v) for k, v in dict(COMMON, **keys).items()}}
    if strict:
        out["patternProperties"] = {"^with_": {"type": ["boolean", "string"]}}
        out["additionalProperties"] = False
    return out


DEFINITIONS = {
    "service_selector": {"type": "object", "properties": {
        "runtimes": {"type": "array", "items": {"type": "string"}}, "services": {"type": "array"},
        "tags": {"type": "array"}, "labels": {"type": "object"}, "exclude_runtimes": {"type": "array"},
        "exclude_labels": {"type": "object"}, "clusters": {"type": "array"}, "exclude_clusters": {"type": "array"},
        "exclude_services": {"type": "array"}, "service_types": {"type": "array"},             # +
        "exclude_service_types": {"type": "array"}, "features": {"type": "array"}},            # +
        "additionalProperties": False},
    "database_connect": {"type": "object", "properties": {
        "engine": {"enum": ["mysql", "postgres"]}, "address": {"type": "string"}, "port": T["port"],
        "username": {"type": "string"}, "password": {"type": "string"}}},
    "yarn_scaling": _section(YARN_SCALING),
}


def runtime_schema() -> Dict[str, Any]:
    props = {"types": {"type": "array", "items": {"type": "string"}}, "envs": {"type": "object"},
             "scaling": _section(SCALING)}
    for name, keys in RUNTIMES.items():
        props[name] = _section(keys)
    return {"$schema": "http://json-schema.org/draft-07/schema#",
            "description": "cluster `runtime:` section (generated by cloudtik_amd/schema/build.py)",
            "type": "object", "definitions": DEFINITIONS, "properties": props,
            # runtimes registered by plugins (core.runtime_factory.register_runtime) stay open
            "additionalProperties": {"type": "object"}}


def _object_schema(name_key: str, extra: Dict[str, Any]) -> Dict[str, Any]:
    props = {"from": {"type": "string"}, name_key: {"type": "string", "pattern": "^[a-z0-9][a-z0-9-]{0,62}$"},
             "provider": {"type": "object", "required": ["type"],
                          "properties": {"type": {"type": "string"}, "region": {"type": "string"},
                                         "location": {"type": "string"}, "project_id": {"type": "string"},
                                         "availability_zone": {"type": "string"}}}}
    props.update(extra)
    return {"$schema": "http://json-schema.org/draft-07/schema#", "type": "object",
            "required": [name_key, "provider"], "properties": props}


def workspace_schema():
    return _object_schema("workspace_name", {
        "managed_cloud_storage": T["b"], "managed_cloud_database": T["b"], "allowed_ssh_sources": {
            "type": "array", "items": {"type": "string"}}, "use_internal_ips": T["b"], "use_working_vpc": T["b"],
        "public_ip_bandwidth": T["i"]})


def storage_schema():
    return _object_schema("storage_name", {"workspace_name": T["s"], "storage": {
        "type": "object", "properties": {"bucket": T["s"], "container": T["s"], "account": T["s"],
                                         "uri": T["s"], "class": T["s"]}}})


def database_schema():
    return _object_schema("database_name", {"workspace_name": T["s"], "database": {
        "type": "object", "properties": {"engine": {"enum": ["mysql", "postgres"]}, "instance_type": T["s"],
                                         "storage_size": T["i"], "admin_user": T["s"], "admin_password": T["s"],
                                         "high_availability": T["b"], "port": T["port"]}}})


def write_all(out_dir: str = HERE) -> Dict[str, str]:
    out = {}
    for name, fn in (("runtime", runtime_schema), ("workspace", workspace_schema), ("storage", storage_schema),
                     ("database", database_schema)):
        path = os.path.join(out_dir, f"{name}.json")
        with open(path, "w") as f:
            json.dump(fn(), f, indent=2, sort_keys=False)
            f.write("\n")
        out[name] = path
    return out


if __name__ == "__main__":
    for k, v in write_all().items():
        print(k, v)
