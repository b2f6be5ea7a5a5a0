"""Self-configuring runtimes, part 2: query engines, stream / compute frameworks, object and
search stores, gateways, DNS, database poolers and node utilities (reference
runtime/{metastore,presto,trino,flink,ray,minio,elasticsearch,nginx,kong,apisix,dnsmasq,bind,
pgbouncer,pgpool,mount,sshserver,xinetd,nodex}/scripts/configure.* + conf templates).

Same model as runtime/configured.py: membership and service wiring come from the provider at
environment time, ``files()`` renders each node's configuration from that environment and the
cluster's ``runtime.<name>`` section, ``node_configure`` writes the files and runs the steps.
JVM / engine memory is sized from the node (80 % of physical memory for the JVM, half of that
per query on Presto / Trino, the rest split between Flink's task slots) unless the config
says otherwise; Ray is started with the node's AMD GPUs as ``GPU`` resources.
"""
from __future__ import annotations

import json
import os
from typing import Any, Dict, List

import yaml

from cloudtik_amd.runtime.catalog import SPEC_BY_NAME
from cloudtik_amd.runtime.configured import DiscoveryBackedRuntime, ConfiguredRuntime, _extra, _props, parse_members


def _node_memory_mb(cfg: Dict[str, Any]) -> int:
    if cfg.get("node_memory_mb"):
        return int(cfg["node_memory_mb"])
    try:
        with open("/proc/meminfo") as f:
            for line in f:
                if line.startswith("MemTotal:"):
                    return int(line.split()[1]) // 1024
    except OSError:
        pass
    return 8192


def _node_cpus(cfg: Dict[str, Any]) -> int:
    return int(cfg.get("node_cpus") or os.cpu_count() or 1)


def _node_gpus(cfg: Dict[str, Any]) -> int:
    if "node_gpus" in cfg:
        return int(cfg["node_gpus"])
    from cloudtik_amd.core.resources import detect_amd_gpu_count
    return detect_amd_gpu_count()


def _xml(props: Dict[str, Any]) -> str:
    rows = "".join(f"  <property>\n    <name>{k}</name>\n    <value>{v}</value>\n  </property>\n"
                   for k, v in props.items())
    return f'<?xml version="1.0"?>\n<configuration>\n{rows}</configuration>\n'


def _db_of(cfg: Dict[str, Any], env_head: str) -> Dict[str, Any]:
    """The metastore / gateway database: ``database`` section, else the cluster's MySQL /
    Postgres runtime on the head."""
    db = dict(cfg.get("database") or {})
    # schema keys (database_connect: address / username) or the short forms
    if "address" in db:
        db.setdefault("host", db["address"])
    if "username" in db:
        db.setdefault("user", db["username"])
    db.setdefault("engine", "mysql")
    db.setdefault("host", env_head)
    db.setdefault("port", 3306 if db["engine"] == "mysql" else 5432)
    db.setdefault("user", "cloudtik")
    db.setdefault("password", "cloudtik")
    return db


# ----------------------------------------------------------------------------- Hive metastore
class MetastoreRuntime(ConfiguredRuntime):
    spec = SPEC_BY_NAME["metastore"]

    def files(self, c):
        if not c["head"]:
            return {}
        cfg = c["cfg"]
        db = _db_of(cfg, c["head_ip"])
        name = db.get("name", "hive_metastore")
        if db["engine"] == "mysql":
            url, driver = (f"jdbc:mysql://{db['host']}:{db['port']}/{name}?createDatabaseIfNotExist=true"
                           "&useSSL=false", "com.mysql.cj.jdbc.Driver")
        else:
            url, driver = f"jdbc:postgresql://{db['host']}:{db['port']}/{name}", "org.postgresql.Driver"
        warehouse = cfg.get("warehouse_dir") or "/shared/warehouse"
        props = {"javax.jdo.option.ConnectionURL": url, "javax.jdo.option.ConnectionDriverName": driver,
                 "javax.jdo.option.ConnectionUserName": db["user"],
                 "javax.jdo.option.ConnectionPassword": db["password"],
                 "hive.metastore.warehouse.dir": warehouse, "metastore.thrift.port": 9083,
                 "metastore.thrift.uris": f"thrift://{c['ip']}:9083",
                 "hive.metastore.event.db.notification.api.auth": "false",
                 "metastore.task.threads.always": "org.apache.hadoop.hive.metastore.events.EventCleanerTask",
                 "metastore.expression.proxy": "org.apache.hadoop.hive.metastore.DefaultPartitionExpressionProxy"}
        props.update(_extra(cfg))
        return {os.path.join(c["home"], "conf", "metastore-site.xml"): _xml(props)}

    def configure_steps(self, head):
        if not head:
            return []
        # schematool is idempotent with -initOrUpgradeSchema (first start creates the schema)
        engine = _db_of(self.runtime_config or {}, "")["engine"]
        return ["mkdir -p $RUNTIME_PATH/metastore/logs",
                f"[ -x $METASTORE_HOME/bin/schematool ] && $METASTORE_HOME/bin/schematool -dbType {engine} "
                "-initOrUpgradeSchema >> $RUNTIME_PATH/metastore/logs/schematool.log 2>&1 || true"]

    def with_environment_variables(self, config, provider, node_id):
        env = super().with_environment_variables(config, provider, node_id)
        env["METASTORE_URI"] = "thrift://$CLOUDTIK_HEAD_IP:9083"
        # the backing database: explicit section, the cluster's MySQL / Postgres, or the workspace
        from cloudtik_amd.runtime.common.discovery import with_database_environment_variables
        env.update(with_database_environment_variables(config or {}, "metastore", "$CLOUDTIK_HEAD_IP"))
        return env


# ----------------------------------------------------------------------------- Presto / Trino
class _SQLEngineRuntime(ConfiguredRuntime):
    port = 8081
    discovery_key = "discovery.uri"

    def _memory(self, cfg) -> Dict[str, int]:
        jvm = int(cfg.get("jvm_max_memory_mb") or _node_memory_mb(cfg) * 0.8)
        return {"jvm": jvm, "query_per_node": int(cfg.get("query_max_memory_per_node_mb") or jvm * 0.5),
                "headroom": int(jvm * 0.25)}

    def config_properties(self, c, mem) -> Dict[str, Any]:
        raise NotImplementedError

    def files(self, c):
        cfg = c["cfg"]
        mem = self._memory(cfg)
        etc = os.path.join(c["home"], "etc")
        node = {"node.environment": cfg.get("environment", "cloudtik"), "node.id": f"{c['cluster']}-{c['seq']}",
                "node.data-dir": cfg.get("data_dir") or os.path.join(c["dir"], "data")}
        jvm = ["-server", f"-Xmx{mem['jvm']}M", "-XX:+UseG1GC", "-XX:G1HeapRegionSize=32M",
               "-XX:+ExplicitGCInvokesConcurrent", "-XX:+ExitOnOutOfMemoryError", "-XX:+HeapDumpOnOutOfMemoryError",
               "-XX:ReservedCodeCacheSize=512M", "-Djdk.attach.allowAttachSelf=true", "-Djdk.nio.maxCachedBufferSize=2000000"]
        metastore = cfg.get("hive_metastore_uri") or f"thrift://{c['head_ip']}:9083"
        hive = {"connector.name": "hive-hadoop2" if self.name == "presto" else "hive", "hive.metastore.uri": metastore}
        hive.update(cfg.get("hive") or {})
        out = {os.path.join(etc, "node.properties"): _props(node),
               os.path.join(etc, "jvm.config"): "\n".join(jvm) + "\n",
               os.path.join(etc, "config.properties"): _props(self.config_properties(c, mem)),
               os.path.join(etc, "catalog", "hive.properties"): _props(hive)}
        for name, props in (cfg.get("catalogs") or {}).items():
            out[os.path.join(etc, "catalog", f"{name}.properties")] = _props(props)
        return out


class PrestoRuntime(_SQLEngineRuntime):
    spec = SPEC_BY_NAME["presto"]

    def config_properties(self, c, mem):
        p = {"coordinator": str(c["head"]).lower(), "http-server.http.port": self.port,
             "query.max-memory": f"{int(c['cfg'].get('query_max_memory_gb', 50))}GB",
             "query.max-memory-per-node": f"{mem['query_per_node']}MB",
             "query.max-total-memory-per-node": f"{int(mem['query_per_node'] * 1.2)}MB",
             "memory.heap-headroom-per-node": f"{mem['headroom']}MB",
             "discovery.uri": f"http://{c['head_ip']}:{self.port}"}
        if c["head"]:
            p["node-scheduler.include-coordinator"] = "false"
            p["discovery-server.enabled"] = "true"
        p.update(_extra(c["cfg"]))
        return p


class TrinoRuntime(_SQLEngineRuntime):
    spec = SPEC_BY_NAME["trino"]

    def config_properties(self, c, mem):
        p = {"coordinator": str(c["head"]).lower(), "http-server.http.port": self.port,
             "query.max-memory": f"{int(c['cfg'].get('query_max_memory_gb', 50))}GB",
             "query.max-memory-per-node": f"{mem['query_per_node']}MB",
             "memory.heap-headroom-per-node": f"{mem['headroom']}MB",
             "discovery.uri": f"http://{c['head_ip']}:{self.port}"}
        if c["head"]:
            p["node-scheduler.include-coordinator"] = "false"
        p.update(_extra(c["cfg"]))
        return p


# ----------------------------------------------------------------------------- Flink
class FlinkRuntime(ConfiguredRuntime):
    spec = SPEC_BY_NAME["flink"]

    def files(self, c):
        cfg = c["cfg"]
        mem = _node_memory_mb(cfg)
        cpus = _node_cpus(cfg)
        slots = int(cfg.get("taskmanager_slots") or max(1, cpus // 2))
        tm_mem = int(cfg.get("taskmanager_memory_mb") or mem * 0.8)
        conf = {"jobmanager.rpc.address": c["head_ip"], "jobmanager.rpc.port": 6123,
                "jobmanager.memory.process.size": f"{int(cfg.get('jobmanager_memory_mb', 4096))}m",
                "taskmanager.memory.process.size": f"{tm_mem}m", "taskmanager.numberOfTaskSlots": slots,
                "parallelism.default": int(cfg.get("parallelism", slots)),
                "execution.target": cfg.get("execution_target", "yarn-per-job"),
                "state.backend": cfg.get("state_backend", "rocksdb"),
                "state.checkpoints.dir": cfg.get("checkpoints_dir", "hdfs:///flink/checkpoints"),
                "jobmanager.archive.fs.dir": "hdfs:///flink/completed-jobs",
                "historyserver.archive.fs.dir": "hdfs:///flink/completed-jobs",
                "historyserver.web.address": "0.0.0.0", "historyserver.web.port": 8082}
        if cfg.get("high_availability_zookeeper"):
            conf.update({"high-availability": "zookeeper",
                         "high-availability.zookeeper.quorum": cfg["high_availability_zookeeper"],
                         "high-availability.storageDir": "hdfs:///flink/ha"})
        conf.update(_extra(cfg))
        return {os.path.join(c["home"], "conf", "flink-conf.yaml"): yaml.safe_dump(conf, sort_keys=False)}


# ----------------------------------------------------------------------------- Ray
class RayRuntime(ConfiguredRuntime):
    """Ray with the node's AMD GPUs as ``GPU`` resources (one Ray GPU = one MI355X) and the
    object store sized for 288 GB-HBM nodes' host memory (30 % of RAM by default)."""

    spec = SPEC_BY_NAME["ray"]

    def _args(self, head: bool) -> List[str]:
        cfg = self.runtime_config or {}
        args = [f"--num-gpus={_node_gpus(cfg)}", f"--num-cpus={_node_cpus(cfg)}",
                f"--object-store-memory={int(_node_memory_mb(cfg) * float(cfg.get('object_store_ratio', 0.3))) << 20}"]
        if cfg.get("resources"):
            args.append(f"--resources='{json.dumps(cfg['resources'])}'")
        if head:
            return ["ray", "start", "--head", "--port=6379", "--dashboard-host=0.0.0.0"] + args
        return ["ray", "start", "--address=$CLOUDTIK_HEAD_IP:6379"] + args

    def start_steps(self, head):
        return [" ".join(self._args(head))]

    def stop_steps(self, head):
        return ["ray stop --force || true"]

    def get_scaling_policy(self, cluster_config, head_ip):
        from cloudtik_amd.runtime.ray_scaling import RayScalingPolicy
        rc = (cluster_config.get("runtime") or {}).get("ray") or {}
        if not (rc.get("auto_scaling") or (rc.get("scaling") or {}).get("auto_scaling")):
            return None
        return RayScalingPolicy(cluster_config, head_ip)


# ----------------------------------------------------------------------------- MinIO
class MinIORuntime(ConfiguredRuntime):
    """Distributed MinIO over the quorum workers: every member serves the same server pool
    (``MINIO_VOLUMES`` = each member's drives), erasure-coded across them."""

    spec = SPEC_BY_NAME["minio"]
    members_env = "MINIO_MEMBERS"

    def with_environment_variables(self, config, provider, node_id):
        env = super().with_environment_variables(config, provider, node_id)
        rc = (config or {}).get("runtime", {}).get("minio", {}) or {}
        disks = int(rc.get("data_disks", 1))
        drives = [f"/mnt/cloudtik/data_disk_{k}/minio" for k in range(1, disks + 1)]
        members = [ip for _, ip in parse_members(env.get("MINIO_MEMBERS", ""))]
        env["MINIO_VOLUMES"] = " ".join(f"http://{ip}:9000{d}" for ip in members for d in drives) or \
            "$RUNTIME_PATH/minio/data"
        return env

    def files(self, c):
        if c["head"]:
            return {}
        cfg = c["cfg"]
        env = {"MINIO_ROOT_USER": cfg.get("access_key", "cloudtik"),
               "MINIO_ROOT_PASSWORD": cfg.get("secret_key", "cloudtik-minio"),
               "MINIO_OPTS": f"--address :9000 --console-address :{int(cfg.get('console_port', 9001))}"}
        return {os.path.join(c["dir"], "minio.env"): "".join(f'{k}="{v}"\n' for k, v in env.items())}


# ----------------------------------------------------------------------------- Elasticsearch
class ElasticsearchRuntime(ConfiguredRuntime):
    spec = SPEC_BY_NAME["elasticsearch"]
    members_env = "ELASTICSEARCH_MEMBERS"
    quorum_members = False

    def files(self, c):
        cfg = c["cfg"]
        hosts = [ip for _, ip in c["members"]]
        if c["head_ip"] not in hosts:
            hosts = [c["head_ip"]] + hosts
        masters = [f"{c['cluster']}-{'head' if ip == c['head_ip'] else 'node-' + str(s)}"
                   for s, ip in ([(0, c["head_ip"])] + c["members"])][: int(cfg.get("master_nodes", 3))]
        me = f"{c['cluster']}-head" if c["head"] else f"{c['cluster']}-node-{c['seq']}"
        conf = {"cluster.name": c["cluster"], "node.name": me, "network.host": c["ip"], "http.port": 9200,
                "path.data": cfg.get("data_dir") or "/mnt/cloudtik/data_disk_1/elasticsearch",
                "path.logs": os.path.join(c["dir"], "logs"), "discovery.seed_hosts": hosts,
                "cluster.initial_master_nodes": masters,
                "xpack.security.enabled": bool(cfg.get("security", False))}
        conf.update(_extra(cfg))
        heap = int(cfg.get("heap_mb") or min(31 * 1024, _node_memory_mb(cfg) // 2))
        return {os.path.join(c["home"], "config", "elasticsearch.yml"): yaml.safe_dump(conf, sort_keys=False),
                os.path.join(c["home"], "config", "jvm.options.d", "cloudtik.options"): f"-Xms{heap}m\n-Xmx{heap}m\n"}


# ----------------------------------------------------------------------------- NGINX
class NginxRuntime(DiscoveryBackedRuntime):
    """Web server (``config_mode: web``), load balancer over static backends (``backend.
    services`` with ``route_path`` per service), or over discovered services
    (``backend.config_mode: dynamic`` / a ``backend.selector``: ``DiscoverNginxBackends``
    rewrites nginx.conf and reloads when they change)."""

    spec = SPEC_BY_NAME["nginx"]
    discovery_class = "DiscoverNginxBackends"

    def files(self, c):
        cfg = c["cfg"]
        port = int(cfg.get("port", 80))
        lines = ["worker_processes auto;", "events { worker_connections 4096; }", "http {",
                 "  sendfile on;", "  keepalive_timeout 65;"]
        services = (cfg.get("backend") or {}).get("services") or {}
        for name, s in sorted(services.items()):
            lines.append(f"  upstream {name} {{")
            lines += [f"    server {srv};" for srv in s.get("servers", [])]
            lines.append("  }")
        lines += ["  server {", f"    listen {port};"]
        for name, s in sorted(services.items(), key=lambda kv: -len(kv[1].get("route_path", "/" + kv[0]))):
            route = s.get("route_path") or ("/" if s.get("default_service") else f"/{name}")
            target = f"http://{name}" + (s.get("service_path", "") + "/" if route != "/" else "")
            lines += [f"    location {route.rstrip('/') + '/' if route != '/' else '/'} {{",
                      f"      proxy_pass {target};", "      proxy_set_header Host $host;", "    }"]
        if not services:
            lines += [f"    root {cfg.get('web_root', os.path.join(c['dir'], 'html'))};"]
        lines += ["  }", "}"]
        out = {os.path.join(c["dir"], "nginx.conf"): "\n".join(lines) + "\n"}
        out.update(self._discovery_files(c))
        return out

    def discovery_config(self, c):
        d = super().discovery_config(c)
        conf = os.path.join(c["dir"], "nginx.conf")
        d.update(conf_path=conf, port=int(c["cfg"].get("port", 80)),
                 balance=(c["cfg"].get("backend") or {}).get("balance"),
                 reload_cmd=f"[ -d /etc/nginx ] && sudo cp {conf} /etc/nginx/nginx.conf; sudo nginx -s reload")
        return d

    def configure_steps(self, head):
        return ["mkdir -p $RUNTIME_PATH/nginx/html",
                "[ -d /etc/nginx ] && sudo cp $RUNTIME_PATH/nginx/nginx.conf /etc/nginx/nginx.conf || true"]


# ----------------------------------------------------------------------------- Kong / APISIX
class KongRuntime(DiscoveryBackedRuntime):
    """Kong on Postgres; discovered services become upstreams / services / routes through
    the admin API (``DiscoverKongBackends``)."""
    spec = SPEC_BY_NAME["kong"]
    discovery_class = "DiscoverKongBackends"

    def files(self, c):
        cfg = c["cfg"]
        db = _db_of(dict(cfg, database=dict({"engine": "postgres"}, **(cfg.get("database") or {}))), c["head_ip"])
        conf = {"database": "postgres", "pg_host": db["host"], "pg_port": db["port"], "pg_user": db["user"],
                "pg_password": db["password"], "pg_database": db.get("name", "kong"),
                "proxy_listen": "0.0.0.0:8000", "admin_listen": f"{c['ip']}:8001"}
        conf.update(_extra(cfg))
        out = {os.path.join(c["dir"], "kong.conf"): "".join(f"{k} = {v}\n" for k, v in conf.items())}
        out.update(self._discovery_files(c))
        return out

    def discovery_config(self, c):
        d = super().discovery_config(c)
        d["admin_url"] = f"http://{c['ip']}:8001"
        return d

    def configure_steps(self, head):
        # migrations once, on the head (kong migrations bootstrap is idempotent)
        return ["mkdir -p $RUNTIME_PATH/kong/logs"] + \
            (["kong migrations bootstrap -c $RUNTIME_PATH/kong/kong.conf >/dev/null 2>&1 || true"] if head else [])


class APISIXRuntime(DiscoveryBackedRuntime):
    """APISIX on etcd; discovered services become upstreams + routes through the admin API
    (``DiscoverAPISIXBackends``)."""
    spec = SPEC_BY_NAME["apisix"]
    discovery_class = "DiscoverAPISIXBackends"

    def files(self, c):
        cfg = c["cfg"]
        etcd = cfg.get("etcd_hosts") or [f"http://{ip}:2379" for _, ip in c["members"]] or \
            [f"http://{c['head_ip']}:2379"]
        conf = {"apisix": {"node_listen": 9080, "enable_admin": True},
                "deployment": {"role": "traditional", "role_traditional": {"config_provider": "etcd"},
                               "admin": {"admin_key": [{"name": "admin", "role": "admin",
                                                        "key": cfg.get("admin_key", "cloudtik-apisix")}],
                                         "allow_admin": ["0.0.0.0/0"]},
                               "etcd": {"host": etcd, "prefix": f"/apisix/{c['cluster']}"}}}
        out = {os.path.join(c["dir"], "conf", "config.yaml"): yaml.safe_dump(conf, sort_keys=False)}
        out.update(self._discovery_files(c))
        return out

    def discovery_config(self, c):
        d = super().discovery_config(c)
        d.update(admin_url="http://127.0.0.1:9180/apisix/admin", admin_key=c["cfg"].get("admin_key", "cloudtik-apisix"),
                 balance=(c["cfg"].get("backend") or {}).get("balance"))
        return d

    members_env = "APISIX_ETCD_MEMBERS"
    quorum_members = False


# ----------------------------------------------------------------------------- DNS
class DnsmasqRuntime(ConfiguredRuntime):
    """Local DNS: ``*.cloudtik`` / ``*.consul`` names to Consul's DNS, the rest upstream."""

    spec = SPEC_BY_NAME["dnsmasq"]

    def files(self, c):
        cfg = c["cfg"]
        lines = ["no-resolv", "listen-address=127.0.0.1," + c["ip"], "bind-interfaces",
                 f"server=/{cfg.get('domain', 'cloudtik')}/127.0.0.1#8600", "server=/consul/127.0.0.1#8600"]
        lines += [f"server={u}" for u in cfg.get("upstream", ["8.8.8.8"])]
        return {os.path.join(c["dir"], "cloudtik.conf"): "\n".join(lines) + "\n"}

    def configure_steps(self, head):
        return ["[ -d /etc/dnsmasq.d ] && sudo cp $RUNTIME_PATH/dnsmasq/cloudtik.conf /etc/dnsmasq.d/cloudtik.conf "
                "|| true"]


class BindRuntime(ConfiguredRuntime):
    spec = SPEC_BY_NAME["bind"]

    def files(self, c):
        cfg = c["cfg"]
        domain = cfg.get("domain", "cloudtik")
        fwd = "; ".join(cfg.get("upstream", ["8.8.8.8"]))
        text = (f'options {{\n  directory "/var/cache/bind";\n  listen-on {{ 127.0.0.1; {c["ip"]}; }};\n'
                f"  forwarders {{ {fwd}; }};\n  dnssec-validation no;\n  allow-query {{ any; }};\n}};\n"
                f'zone "{domain}" {{\n  type forward;\n  forward only;\n  forwarders {{ 127.0.0.1 port 8600; }};\n}};\n'
                'zone "consul" {\n  type forward;\n  forward only;\n  forwarders { 127.0.0.1 port 8600; };\n};\n')
        return {os.path.join(c["dir"], "named.conf.cloudtik"): text}

    def configure_steps(self, head):
        return ["[ -d /etc/bind ] && sudo cp $RUNTIME_PATH/bind/named.conf.cloudtik /etc/bind/named.conf.options "
                "|| true"]


# ----------------------------------------------------------------------------- Postgres poolers
def _cluster_runtimes() -> List[str]:
    return [r.strip() for r in os.environ.get("CLOUDTIK_RUNTIMES", "").split(",") if r.strip()]


class _PoolerRuntime(ConfiguredRuntime):
    """``backend.config_mode`` static / local / dynamic (runtime/pooler_discovery.py): dynamic
    starts a service daemon that rewrites the pooler's backends from the discovered Postgres
    services and reloads it."""

    static_key = "databases"
    discovery_class = ""
    conf_name = ""

    def _backend(self, cfg) -> Dict[str, Any]:
        return dict(cfg.get("backend") or {})

    def mode(self, cfg) -> str:
        from cloudtik_amd.runtime.pooler_discovery import resolve_config_mode
        b = self._backend(cfg)
        if self.static_key == "databases" and cfg.get("databases") and "databases" not in b:
            b["databases"] = cfg["databases"]            # the older top-level form
        return resolve_config_mode(b, _cluster_runtimes(), self.static_key)

    def discovery_files(self, c) -> Dict[str, str]:
        cfg = c["cfg"]
        if self.mode(cfg) != "dynamic":
            return {}
        b = self._backend(cfg)
        d = {"interval": b.get("interval", 15), "service_selector": b.get("service_selector") or {},
             "consul_address": b.get("consul_address") or f"{c['head_ip']}:8500",
             "conf_path": os.path.join(c["dir"], self.conf_name)}
        if b.get("reload_cmd"):
            d["reload_cmd"] = b["reload_cmd"]
        d.update(self.extra_discovery(c))
        return {os.path.join(c["dir"], "discovery.json"): json.dumps(d, indent=1)}

    def extra_discovery(self, c) -> Dict[str, Any]:
        return {}

    def start_steps(self, head):
        steps = super().start_steps(head)
        c = self.ctx(head, self.node_env(head))
        if self.mode(c["cfg"]) == "dynamic":
            steps.append(f"cloudtik node service-daemon start {self.name}-discovery "
                         f"--service-class cloudtik_amd.runtime.pooler_discovery.{self.discovery_class} "
                         f"config_file={os.path.join(c['dir'], 'discovery.json')}")
        return steps

    def stop_steps(self, head):
        steps = []
        if self.mode(self.runtime_config or {}) == "dynamic":
            steps.append(f"cloudtik node service-daemon stop {self.name}-discovery")
        return steps + super().stop_steps(head)


class PgBouncerRuntime(_PoolerRuntime):
    """PgBouncer in front of Postgres.  static: ``backend.databases`` ({name: {host, port,
    dbname, user, ...}} or ready ``host=.. port=..`` strings); local: every database of this
    cluster's Postgres (head); dynamic: one entry per discovered Postgres service
    (``DiscoverPgBouncerBackends``; ``backend.database`` gives the user / dbname / auth_user of
    those entries)."""
    spec = SPEC_BY_NAME["pgbouncer"]
    discovery_class = "DiscoverPgBouncerBackends"
    conf_name = "pgbouncer.ini"

    def _static_databases(self, cfg) -> Dict[str, Any]:
        b = self._backend(cfg)
        return dict(b.get("databases") or cfg.get("databases") or {})

    def files(self, c):
        from cloudtik_amd.runtime.pooler_discovery import pgbouncer_ini
        cfg = c["cfg"]
        mode = self.mode(cfg)
        pool = cfg.get("pool") or {}
        if mode == "static":
            dbs = self._static_databases(cfg)
        elif mode == "local":
            host = cfg.get("postgres_host") or c["head_ip"]
            dbs = {"*": f"host={host} port={int(cfg.get('postgres_port', 5432))}"}
        else:
            dbs = self._static_databases(cfg)        # the job adds the discovered ones
        settings = {"listen_addr": "0.0.0.0", "listen_port": int(cfg.get("port", 6432)), "auth_type": "md5",
                    "auth_file": "/etc/pgbouncer/userlist.txt",
                    "admin_users": cfg.get("admin_user", "cloudtik"),
                    "pool_mode": pool.get("pool_mode", cfg.get("pool_mode", "transaction")),
                    "max_client_conn": int(pool.get("max_client_conn", cfg.get("max_client_conn", 1000))),
                    "default_pool_size": int(pool.get("default_pool_size", cfg.get("default_pool_size", 20))),
                    "pidfile": os.path.join(c["dir"], "pgbouncer.pid")}
        out = {os.path.join(c["dir"], "pgbouncer.ini"): pgbouncer_ini(dbs, settings)}
        out.update(self.discovery_files(c))
        return out

    def extra_discovery(self, c):
        cfg = c["cfg"]
        b = self._backend(cfg)
        return {"database": b.get("database") or {}, "static_databases": self._static_databases(cfg),
                "reload_cmd": b.get("reload_cmd") or
                f"([ -d /etc/pgbouncer ] && sudo cp {os.path.join(c['dir'], 'pgbouncer.ini')} /etc/pgbouncer/ || true) "
                f"&& (kill -HUP $(cat {os.path.join(c['dir'], 'pgbouncer.pid')}) 2>/dev/null || "
                "sudo systemctl reload pgbouncer)"}

    def configure_steps(self, head):
        return ["[ -d /etc/pgbouncer ] && sudo cp $RUNTIME_PATH/pgbouncer/pgbouncer.ini /etc/pgbouncer/ || true"]


class PgpoolRuntime(_PoolerRuntime):
    """pgpool-II, streaming-replication mode with load-balanced reads.  static:
    ``backend.servers`` (the first is the primary); local: this cluster's Postgres primary
    (head) and replicas (workers); dynamic: the discovered Postgres servers, new ones appended
    as backends by ``DiscoverPgpoolBackends`` and pgpool reloaded."""

    spec = SPEC_BY_NAME["pgpool"]
    members_env = "PGPOOL_BACKENDS"
    quorum_members = False
    static_key = "servers"
    discovery_class = "DiscoverPgpoolBackends"
    conf_name = "pgpool.conf"

    def files(self, c):
        from cloudtik_amd.runtime.pooler_discovery import pgpool_backend_lines
        cfg = c["cfg"]
        mode = self.mode(cfg)
        if mode == "static":
            backends = []
            for srv in self._backend(cfg)["servers"]:
                h, _, p = str(srv).rpartition(":") if ":" in str(srv) else (str(srv), "", "5432")
                backends.append((h, int(p or 5432)))
        elif mode == "local":
            backends = [(ip, 5432) for ip in [c["head_ip"]] + [ip for _, ip in c["members"]]]
        else:
            backends = []                            # filled by the discovery job
        lines = ["listen_addresses = '*'", f"port = {int(cfg.get('port', 6432))}",
                 "backend_clustering_mode = 'streaming_replication'", "load_balance_mode = on",
                 f"num_init_children = {int(cfg.get('num_init_children', 32))}",
                 f"max_pool = {int(cfg.get('max_pool', 4))}", "sr_check_period = 10",
                 f"sr_check_user = '{cfg.get('user', 'cloudtik')}'", "health_check_period = 10",
                 f"health_check_user = '{cfg.get('user', 'cloudtik')}'"]
        for i, (ip, port) in enumerate(backends):
            primary = i == 0 and mode != "dynamic"
            lines += pgpool_backend_lines(i, ip, port, 0 if primary and cfg.get("primary_no_reads") else 1,
                                          "ALWAYS_PRIMARY" if primary else "ALLOW_TO_FAILOVER")
        out = {os.path.join(c["dir"], "pgpool.conf"): "\n".join(lines) + "\n"}
        out.update(self.discovery_files(c))
        return out

    def extra_discovery(self, c):
        b = self._backend(c["cfg"])
        return {"reload_cmd": b.get("reload_cmd") or
                f"([ -d /etc/pgpool2 ] && sudo cp {os.path.join(c['dir'], 'pgpool.conf')} /etc/pgpool2/pgpool.conf "
                "|| true) && sudo pgpool reload"}

    def configure_steps(self, head):
        return ["[ -d /etc/pgpool2 ] && sudo cp $RUNTIME_PATH/pgpool/pgpool.conf /etc/pgpool2/pgpool.conf || true"]


# ----------------------------------------------------------------------------- node utilities
class MountRuntime(ConfiguredRuntime):
    """Mounts the workspace's storage on every node: the cluster's HDFS through the FUSE
    client, or cloud buckets through s3fs / gcsfuse / blobfuse2 (``storage`` section)."""

    spec = SPEC_BY_NAME["mount"]

    def files(self, c):
        cfg = c["cfg"]
        mount = cfg.get("mount_path", "/cloudtik/fs")
        st = cfg.get("storage") or {}
        kind = st.get("type", "hdfs")
        if kind == "hdfs":
            cmd = f"hadoop-fuse-dfs dfs://{st.get('namenode', c['head_ip'] + ':9000')} {mount}"
        elif kind == "s3":
            cmd = f"s3fs {st['bucket']} {mount} -o iam_role=auto -o allow_other"
        elif kind == "gcs":
            cmd = f"gcsfuse --implicit-dirs {st['bucket']} {mount}"
        elif kind == "azure":
            cmd = f"blobfuse2 mount {mount} --config-file={os.path.join(c['dir'], 'blobfuse2.yaml')}"
        else:
            raise ValueError(f"mount: unknown storage type {kind}")
        script = ("#!/bin/bash\nset -e\n"
                  f"mountpoint -q {mount} && exit 0\nsudo mkdir -p {mount} && sudo chmod 777 {mount}\n{cmd}\n")
        out = {os.path.join(c["dir"], "cloudtik-mount-storage.sh"): script}
        if kind == "azure":
            out[os.path.join(c["dir"], "blobfuse2.yaml")] = yaml.safe_dump({
                "components": ["libfuse", "file_cache", "attr_cache", "azstorage"],
                "azstorage": {"type": "adls", "account-name": st["account"], "container": st["container"],
                              "mode": "msi"}, "file_cache": {"path": "/tmp/blobfuse2"}})
        return out

    def start_steps(self, head):
        return ["bash $RUNTIME_PATH/mount/cloudtik-mount-storage.sh"]

    def stop_steps(self, head):
        mount = (self.runtime_config or {}).get("mount_path", "/cloudtik/fs")
        return [f"mountpoint -q {mount} && sudo umount -l {mount} || true"]


class SSHServerRuntime(ConfiguredRuntime):
    spec = SPEC_BY_NAME["sshserver"]

    def files(self, c):
        cfg = c["cfg"]
        text = (f"Port {int(cfg.get('port', 22022))}\nPasswordAuthentication no\nPermitRootLogin prohibit-password\n"
                f"AuthorizedKeysFile {cfg.get('authorized_keys', os.path.join(c['dir'], 'authorized_keys'))}\n"
                f"HostKey {os.path.join(c['dir'], 'ssh_host_ed25519_key')}\nUsePAM yes\nX11Forwarding no\n"
                "AllowTcpForwarding yes\nClientAliveInterval 60\n")
        return {os.path.join(c["dir"], "sshd_config"): text}

    def configure_steps(self, head):
        return ["[ -f $RUNTIME_PATH/sshserver/ssh_host_ed25519_key ] || "
                "ssh-keygen -q -t ed25519 -N '' -f $RUNTIME_PATH/sshserver/ssh_host_ed25519_key"]


class XinetdRuntime(ConfiguredRuntime):
    """xinetd services: the role-aware health checks of the cluster's replicated runtimes
    (every runtime with a ``health_check_port``, runtime/common/health_check.py -- what HAProxy
    probes to find the primary) plus any explicit ``services``."""

    spec = SPEC_BY_NAME["xinetd"]

    def with_environment_variables(self, config, provider, node_id):
        env = super().with_environment_variables(config, provider, node_id)
        from cloudtik_amd.runtime.common.health_check import xinetd_services
        checks = xinetd_services((config or {}).get("runtime") or {}, python="/usr/bin/python3")
        if checks:
            env["XINETD_HEALTH_CHECKS"] = json.dumps(checks, sort_keys=True)
        return env

    def ctx(self, head, env):
        c = super().ctx(head, env)
        c["health_checks"] = json.loads(env.get("XINETD_HEALTH_CHECKS") or "{}")
        return c

    def files(self, c):
        out = {}
        services = dict(c.get("health_checks") or {})
        services.update(c["cfg"].get("services") or {})
        for name, s in sorted(services.items()):
            args = f"  server_args = {s['server_args']}\n" if s.get("server_args") else ""
            out[os.path.join(c["dir"], name)] = (
                f"service {name}\n{{\n  type = UNLISTED\n  port = {int(s['port'])}\n  socket_type = stream\n"
                f"  protocol = tcp\n  wait = no\n  user = {s.get('user', 'nobody')}\n  server = {s['server']}\n"
                f"{args}  only_from = {s.get('only_from', '0.0.0.0/0')}\n  disable = no\n}}\n")
        return out

    def configure_steps(self, head):
        return ["[ -d /etc/xinetd.d ] && ls $RUNTIME_PATH/xinetd/* >/dev/null 2>&1 && "
                "sudo cp $RUNTIME_PATH/xinetd/* /etc/xinetd.d/ || true"]


class NodexRuntime(ConfiguredRuntime):
    """node_exporter with the textfile collector pointed at the AMD GPU metrics the node
    monitor writes (core/node/metrics.py: utilisation, HBM, power, RAS error counts)."""

    spec = SPEC_BY_NAME["nodex"]

    def files(self, c):
        tdir = os.path.join(c["dir"], "textfile")
        args = [f"--web.listen-address=:{int(c['cfg'].get('port', 9100))}",
                f"--collector.textfile.directory={tdir}"]
        return {os.path.join(c["dir"], "nodex.args"): " ".join(args) + "\n",
                os.path.join(tdir, ".keep"): ""}

    def start_steps(self, head):
        return ["mkdir -p $RUNTIME_PATH/pids $RUNTIME_PATH/nodex/logs; nohup $NODEX_HOME/node_exporter "
                "$(cat $RUNTIME_PATH/nodex/nodex.args) > $RUNTIME_PATH/nodex/logs/node_exporter.out 2>&1 & "
                "echo $! > $RUNTIME_PATH/pids/node_exporter.pid"]


CONFIGURED_MORE = {
    "metastore": MetastoreRuntime, "presto": PrestoRuntime, "trino": TrinoRuntime, "flink": FlinkRuntime,
    "ray": RayRuntime, "minio": MinIORuntime, "elasticsearch": ElasticsearchRuntime, "nginx": NginxRuntime,
    "kong": KongRuntime, "apisix": APISIXRuntime, "dnsmasq": DnsmasqRuntime, "bind": BindRuntime,
    "pgbouncer": PgBouncerRuntime, "pgpool": PgpoolRuntime, "mount": MountRuntime, "sshserver": SSHServerRuntime,
    "xinetd": XinetdRuntime, "nodex": NodexRuntime,
}
