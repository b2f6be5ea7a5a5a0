"""Declarative catalog of the service runtimes (reference: python/cloudtik/runtime/*).

The reference ships 37 runtime plugins, each a Runtime subclass + bash
install/configure/services scripts + conf templates.  Here every non-AI runtime is one
``RuntimeSpec``: version + download location, the services it exposes (ports, head /
worker placement, discovery scope and features), the daemon processes it runs (for
``cloudtik process-status`` / the node agent), its runtime dependencies / required
runtimes (reference ``get_dependencies`` / ``get_required``), quorum constraints (ZooKeeper,
etcd, Consul, MinIO, MongoDB, Kafka need a minimal node set before setup proceeds) and the
node-side shell steps.  ``CatalogRuntime`` turns a spec into a full ``Runtime``.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

from cloudtik_amd.core import service_discovery as sd
from .common.runtime_base import RuntimeBase, standard_commands


@dataclass
class ServiceSpec:
    name: str
    port: int
    node_kind: str = sd.SERVICE_DISCOVERY_NODE_KIND_HEAD
    protocol: str = sd.SERVICE_DISCOVERY_PROTOCOL_TCP
    scope: str = sd.SERVICE_SCOPE_WORKSPACE
    features: Tuple[str, ...] = ()
    metrics: bool = False


@dataclass
class RuntimeSpec:
    name: str
    description: str
    version: str = ""
    home_env: str = ""
    download: str = ""                     # tarball URL template ({version})
    services: List[ServiceSpec] = field(default_factory=list)
    head_processes: List[str] = field(default_factory=list)
    worker_processes: List[str] = field(default_factory=list)
    logs: Dict[str, str] = field(default_factory=dict)
    dependencies: List[str] = field(default_factory=list)
    required: List[str] = field(default_factory=list)
    quorum: bool = False                   # needs minimal nodes before configure
    head_only: bool = False
    defaults: Dict[str, Any] = field(default_factory=dict)
    apt: List[str] = field(default_factory=list)
    start: Dict[str, str] = field(default_factory=dict)   # {"head": cmd, "worker": cmd}
    stop: Dict[str, str] = field(default_factory=dict)
    env: Dict[str, str] = field(default_factory=dict)


W = sd.SERVICE_DISCOVERY_NODE_KIND_WORKER
H = sd.SERVICE_DISCOVERY_NODE_KIND_HEAD
A = sd.SERVICE_DISCOVERY_NODE_KIND_NODE
HTTP = sd.SERVICE_DISCOVERY_PROTOCOL_HTTP
LOCAL = sd.SERVICE_SCOPE_LOCAL


def _S(name, port, kind=H, **kw):
    return ServiceSpec(name, port, kind, **kw)


APACHE = "https://archive.apache.org/dist"


def _bg(name: str, cmd: str) -> str:
    """Start a foreground daemon in the background and record its pid (stopped by _kill)."""
    return (f"mkdir -p $RUNTIME_PATH/pids $RUNTIME_PATH/{name}/logs; "
            f"nohup {cmd} > $RUNTIME_PATH/{name}/logs/{name}.out 2>&1 & echo $! > $RUNTIME_PATH/pids/{name}.pid")


def _kill(name: str, sudo: bool = False) -> str:
    """Stop exactly the process recorded by _bg (never by name pattern)."""
    k = "sudo kill" if sudo else "kill"
    return f"P=$RUNTIME_PATH/pids/{name}.pid; [ -f $P ] && {k} $(cat $P) 2>/dev/null; rm -f $P; true"


# per-runtime quorum semantics: Kafka brokers need their minimal set but no quorum of their
# own (ZooKeeper holds it); a MinIO server pool is fixed at creation (erasure sets), so its
# quorum cannot grow by joining nodes; ZooKeeper / etcd / Consul servers / MongoDB replica
# sets reconfigure membership online
QUORUM_CONSTRAINTS: Dict[str, Tuple[bool, bool, bool]] = {
    "kafka": (True, False, True),
    "minio": (True, True, False),
    "zookeeper": (True, True, True), "etcd": (True, True, True), "consul": (True, True, True),
    "mongodb": (True, True, True),
}

SPECS: List[RuntimeSpec] = [
    RuntimeSpec("spark", "Apache Spark on YARN with history server and auto executor sizing",
                "3.3.1", "SPARK_HOME", APACHE + "/spark/spark-{version}/spark-{version}-bin-hadoop3.tgz",
                [_S("spark-history", 18080, protocol=HTTP, features=(sd.SERVICE_DISCOVERY_FEATURE_ANALYTICS,)),
                 _S("spark-jupyter", 8888, protocol=HTTP, scope=LOCAL)],
                ["HistoryServer"], [], {"spark": "$SPARK_HOME/logs"}, ["metastore", "yarn", "hadoop"], ["hadoop"],
                start={"head": "$SPARK_HOME/sbin/start-history-server.sh"},
                stop={"head": "$SPARK_HOME/sbin/stop-history-server.sh"}),
    RuntimeSpec("hadoop", "Hadoop client configuration (fs.defaultFS, cloud storage connectors)",
                "3.3.1", "HADOOP_HOME", APACHE + "/hadoop/common/hadoop-{version}/hadoop-{version}.tar.gz",
                dependencies=["hdfs"]),
    RuntimeSpec("hdfs", "HDFS NameNode / DataNodes (+ fuse / NFS mount)", "3.3.1", "HADOOP_HOME",
                APACHE + "/hadoop/common/hadoop-{version}/hadoop-{version}.tar.gz",
                [_S("hdfs-name", 9870, protocol=HTTP, features=(sd.SERVICE_DISCOVERY_FEATURE_STORAGE,)),
                 _S("hdfs-rpc", 8020, features=(sd.SERVICE_DISCOVERY_FEATURE_STORAGE,))],
                ["NameNode"], ["DataNode"], {"hdfs": "$HADOOP_HOME/logs"},
                start={"head": "$HADOOP_HOME/bin/hdfs --daemon start namenode",
                       "worker": "$HADOOP_HOME/bin/hdfs --daemon start datanode"},
                stop={"head": "$HADOOP_HOME/bin/hdfs --daemon stop namenode",
                      "worker": "$HADOOP_HOME/bin/hdfs --daemon stop datanode"}),
    RuntimeSpec("yarn", "YARN ResourceManager / NodeManagers (+ YARN scaling policy & job waiter)",
                "3.3.1", "HADOOP_HOME", APACHE + "/hadoop/common/hadoop-{version}/hadoop-{version}.tar.gz",
                [_S("yarn-rm", 8032, features=(sd.SERVICE_DISCOVERY_FEATURE_SCHEDULER,)),
                 _S("yarn-web", 8088, protocol=HTTP)],
                ["ResourceManager"], ["NodeManager"], {"yarn": "$HADOOP_HOME/logs"}, ["hdfs"],
                start={"head": "$HADOOP_HOME/bin/yarn --daemon start resourcemanager",
                       "worker": "$HADOOP_HOME/bin/yarn --daemon start nodemanager"},
                stop={"head": "$HADOOP_HOME/bin/yarn --daemon stop resourcemanager",
                      "worker": "$HADOOP_HOME/bin/yarn --daemon stop nodemanager"}),
    RuntimeSpec("mount", "Mount HDFS / cloud storage to a local path (fuse)", dependencies=["hadoop"],
                start={"head": "cloudtik-mount-storage.sh", "worker": "cloudtik-mount-storage.sh"},
                stop={"head": "fusermount -u /cloudtik/fs || true", "worker": "fusermount -u /cloudtik/fs || true"}),
    RuntimeSpec("metastore", "Hive metastore backed by MySQL / Postgres", "3.1.2", "METASTORE_HOME",
                APACHE + "/hive/hive-standalone-metastore-{version}/hive-standalone-metastore-{version}-bin.tar.gz",
                [_S("metastore", 9083, features=(sd.SERVICE_DISCOVERY_FEATURE_DATABASE,))],
                ["HiveMetaStore"], [], {"metastore": "$METASTORE_HOME/logs"}, ["mysql", "postgres"],
                start={"head": _bg("metastore", "$METASTORE_HOME/bin/start-metastore")},
                stop={"head": _kill("metastore")}),
    RuntimeSpec("presto", "Presto interactive SQL", "0.276", "PRESTO_HOME",
                "https://repo1.maven.org/maven2/com/facebook/presto/presto-server/{version}/presto-server-{version}.tar.gz",
                [_S("presto", 8081, protocol=HTTP, features=(sd.SERVICE_DISCOVERY_FEATURE_ANALYTICS,))],
                ["PrestoServer"], ["PrestoServer"], {"presto": "/tmp/presto/data/var/log"}, ["hdfs", "metastore"],
                start={"head": "$PRESTO_HOME/bin/launcher start", "worker": "$PRESTO_HOME/bin/launcher start"},
                stop={"head": "$PRESTO_HOME/bin/launcher stop", "worker": "$PRESTO_HOME/bin/launcher stop"}),
    RuntimeSpec("trino", "Trino interactive SQL", "389", "TRINO_HOME",
                "https://repo1.maven.org/maven2/io/trino/trino-server/{version}/trino-server-{version}.tar.gz",
                [_S("trino", 8081, protocol=HTTP, features=(sd.SERVICE_DISCOVERY_FEATURE_ANALYTICS,))],
                ["TrinoServer"], ["TrinoServer"], {"trino": "/tmp/trino/data/var/log"}, ["hdfs", "metastore"],
                start={"head": "$TRINO_HOME/bin/launcher start", "worker": "$TRINO_HOME/bin/launcher start"},
                stop={"head": "$TRINO_HOME/bin/launcher stop", "worker": "$TRINO_HOME/bin/launcher stop"}),
    RuntimeSpec("flink", "Apache Flink on YARN + history server", "1.14.5", "FLINK_HOME",
                APACHE + "/flink/flink-{version}/flink-{version}-bin-scala_2.12.tgz",
                [_S("flink-history", 8082, protocol=HTTP), _S("flink-jupyter", 8888, protocol=HTTP, scope=LOCAL)],
                ["HistoryServer"], [], {"flink": "$FLINK_HOME/log"}, ["metastore", "yarn", "hadoop"], ["hadoop"],
                start={"head": "$FLINK_HOME/bin/historyserver.sh start"},
                stop={"head": "$FLINK_HOME/bin/historyserver.sh stop"}),
    RuntimeSpec("kafka", "Apache Kafka brokers", "3.2.0", "KAFKA_HOME",
                APACHE + "/kafka/{version}/kafka_2.13-{version}.tgz",
                [_S("kafka", 9092, W)], [], ["kafka.Kafka"], {"kafka": "$KAFKA_HOME/logs"}, ["zookeeper"], ["zookeeper"],
                quorum=True,
                start={"worker": "$KAFKA_HOME/bin/kafka-server-start.sh -daemon $KAFKA_HOME/config/server.properties"},
                stop={"worker": "$KAFKA_HOME/bin/kafka-server-stop.sh"}),
    RuntimeSpec("zookeeper", "ZooKeeper ensemble (quorum)", "3.7.1", "ZOOKEEPER_HOME",
                APACHE + "/zookeeper/zookeeper-{version}/apache-zookeeper-{version}-bin.tar.gz",
                [_S("zookeeper", 2181, W)], [], ["QuorumPeerMain"], {"zookeeper": "$ZOOKEEPER_HOME/logs"},
                quorum=True,
                start={"worker": "$ZOOKEEPER_HOME/bin/zkServer.sh start"},
                stop={"worker": "$ZOOKEEPER_HOME/bin/zkServer.sh stop"}),
    RuntimeSpec("ray", "Ray cluster (+ Ray scaling policy)", "2.5.0",
                services=[_S("ray-gcs", 6379), _S("ray-dashboard", 8265, protocol=HTTP)],
                head_processes=["gcs_server", "raylet"], worker_processes=["raylet"],
                start={"head": "ray start --head --port=6379 --dashboard-host=0.0.0.0",
                       "worker": "ray start --address=$CLOUDTIK_HEAD_IP:6379"},
                stop={"head": "ray stop", "worker": "ray stop"}),
    RuntimeSpec("mysql", "MySQL server (replicated)", "8.0", services=[_S("mysql", 3306, features=(sd.SERVICE_DISCOVERY_FEATURE_DATABASE,))],
                head_processes=["mysqld"], apt=["mysql-server"],
                start={"head": "sudo service mysql start"}, stop={"head": "sudo service mysql stop"}),
    RuntimeSpec("postgres", "PostgreSQL server (replicated)", "15", services=[_S("postgres", 5432, features=(sd.SERVICE_DISCOVERY_FEATURE_DATABASE,))],
                head_processes=["postgres"], apt=["postgresql"],
                start={"head": "sudo service postgresql start"}, stop={"head": "sudo service postgresql stop"}),
    RuntimeSpec("pgpool", "Pgpool-II in front of PostgreSQL", "4.4", services=[_S("pgpool", 6432, A, features=(sd.SERVICE_DISCOVERY_FEATURE_DATABASE,))],
                head_processes=["pgpool"], worker_processes=["pgpool"], dependencies=["postgres"], apt=["pgpool2"],
                start={"head": "sudo service pgpool2 start", "worker": "sudo service pgpool2 start"},
                stop={"head": "sudo service pgpool2 stop", "worker": "sudo service pgpool2 stop"}),
    RuntimeSpec("pgbouncer", "PgBouncer connection pooler", "1.19", services=[_S("pgbouncer", 6432, A, features=(sd.SERVICE_DISCOVERY_FEATURE_DATABASE,))],
                head_processes=["pgbouncer"], worker_processes=["pgbouncer"], dependencies=["postgres"], apt=["pgbouncer"],
                start={"head": "sudo service pgbouncer start", "worker": "sudo service pgbouncer start"},
                stop={"head": "sudo service pgbouncer stop", "worker": "sudo service pgbouncer stop"}),
    RuntimeSpec("redis", "Redis (replication / cluster)", "7.0", services=[_S("redis", 6379, A, features=(sd.SERVICE_DISCOVERY_FEATURE_KEY_VALUE,))],
                head_processes=["redis-server"], worker_processes=["redis-server"], apt=["redis-server"],
                start={"head": "redis-server $RUNTIME_PATH/redis/redis.conf --daemonize yes",
                       "worker": "redis-server $RUNTIME_PATH/redis/redis.conf --daemonize yes"},
                stop={"head": "redis-cli shutdown || true", "worker": "redis-cli shutdown || true"}),
    RuntimeSpec("mongodb", "MongoDB replica set / sharded", "6.0", services=[_S("mongodb", 27017, A, features=(sd.SERVICE_DISCOVERY_FEATURE_DATABASE,))],
                head_processes=["mongod"], worker_processes=["mongod"], quorum=True,
                start={"head": "mongod --fork --config $RUNTIME_PATH/mongodb/mongod.conf",
                       "worker": "mongod --fork --config $RUNTIME_PATH/mongodb/mongod.conf"},
                stop={"head": "mongod --shutdown --dbpath $RUNTIME_PATH/mongodb/data || true",
                      "worker": "mongod --shutdown --dbpath $RUNTIME_PATH/mongodb/data || true"}),
    RuntimeSpec("elasticsearch", "Elasticsearch cluster", "8.8.1", "ELASTICSEARCH_HOME",
                "https://artifacts.elastic.co/downloads/elasticsearch/elasticsearch-{version}-linux-x86_64.tar.gz",
                [_S("elasticsearch", 9200, A, protocol=HTTP)], ["Elasticsearch"], ["Elasticsearch"],
                dependencies=["mount"],
                start={"head": "mkdir -p $RUNTIME_PATH/pids; $ELASTICSEARCH_HOME/bin/elasticsearch -d -p $RUNTIME_PATH/pids/elasticsearch.pid",
                       "worker": "mkdir -p $RUNTIME_PATH/pids; $ELASTICSEARCH_HOME/bin/elasticsearch -d -p $RUNTIME_PATH/pids/elasticsearch.pid"},
                stop={"head": _kill("elasticsearch"), "worker": _kill("elasticsearch")}),
    RuntimeSpec("consul", "Consul service registry / KV (quorum)", "1.15.2",
                download="https://releases.hashicorp.com/consul/{version}/consul_{version}_linux_amd64.zip",
                services=[_S("consul", 8500, A, protocol=HTTP, features=(sd.SERVICE_DISCOVERY_FEATURE_KEY_VALUE,))],
                head_processes=["consul"], worker_processes=["consul"], quorum=True,
                start={"head": "nohup consul agent -config-dir=$RUNTIME_PATH/consul/consul.d > $RUNTIME_PATH/consul/consul.log 2>&1 &",
                       "worker": "nohup consul agent -config-dir=$RUNTIME_PATH/consul/consul.d > $RUNTIME_PATH/consul/consul.log 2>&1 &"},
                stop={"head": "consul leave || true", "worker": "consul leave || true"}),
    RuntimeSpec("etcd", "etcd key-value store (quorum)", "3.5.9",
                download="https://github.com/etcd-io/etcd/releases/download/v{version}/etcd-v{version}-linux-amd64.tar.gz",
                services=[_S("etcd", 2379, W, features=(sd.SERVICE_DISCOVERY_FEATURE_KEY_VALUE,)), _S("etcd-peer", 2380, W, scope=LOCAL)],
                worker_processes=["etcd"], quorum=True,
                start={"worker": _bg("etcd", "etcd --config-file $RUNTIME_PATH/etcd/etcd.yaml")},
                stop={"worker": _kill("etcd")}),
    RuntimeSpec("dnsmasq", "dnsmasq DNS forwarder (consul-backed)", services=[_S("dnsmasq", 53, A, features=(sd.SERVICE_DISCOVERY_FEATURE_DNS,))],
                head_processes=["dnsmasq"], worker_processes=["dnsmasq"], dependencies=["consul"], apt=["dnsmasq"],
                start={"head": "sudo service dnsmasq start", "worker": "sudo service dnsmasq start"},
                stop={"head": "sudo service dnsmasq stop", "worker": "sudo service dnsmasq stop"}),
    RuntimeSpec("bind", "BIND DNS server (consul forwarding)", services=[_S("bind", 53, A, features=(sd.SERVICE_DISCOVERY_FEATURE_DNS,))],
                head_processes=["named"], worker_processes=["named"], dependencies=["consul"], apt=["bind9"],
                start={"head": "sudo service named start", "worker": "sudo service named start"},
                stop={"head": "sudo service named stop", "worker": "sudo service named stop"}),
    RuntimeSpec("coredns", "CoreDNS (consul forwarding)", "1.10.1",
                download="https://github.com/coredns/coredns/releases/download/v{version}/coredns_{version}_linux_amd64.tgz",
                services=[_S("coredns", 53, A, features=(sd.SERVICE_DISCOVERY_FEATURE_DNS,))],
                head_processes=["coredns"], worker_processes=["coredns"], dependencies=["consul"],
                start={"head": _bg("coredns", "coredns -conf $RUNTIME_PATH/coredns/Corefile"),
                       "worker": _bg("coredns", "coredns -conf $RUNTIME_PATH/coredns/Corefile")},
                stop={"head": _kill("coredns"), "worker": _kill("coredns")}),
    RuntimeSpec("haproxy", "HAProxy L4/L7 load balancer (service-discovery backends)",
                services=[_S("haproxy", 80, A, protocol=HTTP, features=(sd.SERVICE_DISCOVERY_FEATURE_LOAD_BALANCER,))],
                head_processes=["haproxy"], worker_processes=["haproxy"], apt=["haproxy"],
                start={"head": "sudo service haproxy start", "worker": "sudo service haproxy start"},
                stop={"head": "sudo service haproxy stop", "worker": "sudo service haproxy stop"}),
    RuntimeSpec("nginx", "NGINX web server / load balancer", services=[_S("nginx", 80, A, protocol=HTTP, features=(sd.SERVICE_DISCOVERY_FEATURE_LOAD_BALANCER,))],
                head_processes=["nginx"], worker_processes=["nginx"], apt=["nginx"],
                start={"head": "sudo service nginx start", "worker": "sudo service nginx start"},
                stop={"head": "sudo service nginx stop", "worker": "sudo service nginx stop"}),
    RuntimeSpec("kong", "Kong API gateway", "3.3.0", services=[_S("kong", 8000, A, protocol=HTTP, features=(sd.SERVICE_DISCOVERY_FEATURE_LOAD_BALANCER,)),
                                                                _S("kong-admin", 8001, A, protocol=HTTP, scope=LOCAL)],
                head_processes=["nginx: master"], worker_processes=["nginx: master"], dependencies=["postgres"],
                start={"head": "kong start", "worker": "kong start"}, stop={"head": "kong stop", "worker": "kong stop"}),
    RuntimeSpec("apisix", "Apache APISIX API gateway", "3.3.0", services=[_S("apisix", 9080, A, protocol=HTTP, features=(sd.SERVICE_DISCOVERY_FEATURE_LOAD_BALANCER,))],
                head_processes=["apisix"], worker_processes=["apisix"], dependencies=["etcd"],
                start={"head": "apisix start", "worker": "apisix start"}, stop={"head": "apisix stop", "worker": "apisix stop"}),
    RuntimeSpec("loadbalancer", "Cloud load-balancer driver (LoadBalancerProvider) with service groups",
                head_processes=["cloudtik_load_balancer"], head_only=True,
                start={"head": "cloudtik node run load-balancer-controller"}, stop={"head": "true"}),
    RuntimeSpec("prometheus", "Prometheus with cluster / workspace service-discovery scrape", "2.45.0",
                "PROMETHEUS_HOME", "https://github.com/prometheus/prometheus/releases/download/v{version}/prometheus-{version}.linux-amd64.tar.gz",
                [_S("prometheus", 9090, protocol=HTTP, features=(sd.SERVICE_DISCOVERY_FEATURE_METRICS,))], ["prometheus"],
                start={"head": _bg("prometheus", "$PROMETHEUS_HOME/prometheus --config.file=$PROMETHEUS_HOME/prometheus.yml")},
                stop={"head": _kill("prometheus")}),
    RuntimeSpec("grafana", "Grafana dashboards (prometheus data source)", "10.0.3", "GRAFANA_HOME",
                "https://dl.grafana.com/oss/release/grafana-{version}.linux-amd64.tar.gz",
                [_S("grafana", 3000, protocol=HTTP)], ["grafana"],
                start={"head": _bg("grafana", "$GRAFANA_HOME/bin/grafana server --homepath $GRAFANA_HOME")},
                stop={"head": _kill("grafana")}),
    RuntimeSpec("nodex", "Node exporter (+ AMD GPU metrics textfile collector)", "1.6.1", "NODEX_HOME",
                "https://github.com/prometheus/node_exporter/releases/download/v{version}/node_exporter-{version}.linux-amd64.tar.gz",
                [_S("nodex", 9100, A, protocol=HTTP, features=(sd.SERVICE_DISCOVERY_FEATURE_METRICS,), metrics=True)],
                ["node_exporter"], ["node_exporter"],
                start={"head": _bg("node_exporter", "$NODEX_HOME/node_exporter"), "worker": _bg("node_exporter", "$NODEX_HOME/node_exporter")},
                stop={"head": _kill("node_exporter"), "worker": _kill("node_exporter")}),
    RuntimeSpec("sshserver", "In-cluster passwordless SSH server (port 22022) used by MPI / rsh launchers",
                services=[_S("sshserver", 22022, A, scope=LOCAL)], head_processes=["sshd"], worker_processes=["sshd"],
                start={"head": "mkdir -p $RUNTIME_PATH/pids; sudo /usr/sbin/sshd -f $RUNTIME_PATH/sshserver/sshd_config "
                               "-o PidFile=$RUNTIME_PATH/pids/sshserver.pid",
                       "worker": "mkdir -p $RUNTIME_PATH/pids; sudo /usr/sbin/sshd -f $RUNTIME_PATH/sshserver/sshd_config "
                               "-o PidFile=$RUNTIME_PATH/pids/sshserver.pid"},
                stop={"head": _kill("sshserver", sudo=True), "worker": _kill("sshserver", sudo=True)}),
    RuntimeSpec("xinetd", "xinetd health-check endpoints for load balancers", head_processes=["xinetd"], worker_processes=["xinetd"],
                apt=["xinetd"],
                start={"head": "sudo service xinetd start", "worker": "sudo service xinetd start"},
                stop={"head": "sudo service xinetd stop", "worker": "sudo service xinetd stop"}),
    RuntimeSpec("minio", "MinIO object storage (distributed, quorum)", "RELEASE.2023-07-21",
                download="https://dl.min.io/server/minio/release/linux-amd64/minio",
                services=[_S("minio", 9000, W, protocol=HTTP, features=(sd.SERVICE_DISCOVERY_FEATURE_STORAGE,))],
                worker_processes=["minio"], quorum=True,
                start={"worker": _bg("minio", "minio server $MINIO_VOLUMES")},
                stop={"worker": _kill("minio")}),
]

SPEC_BY_NAME = {s.name: s for s in SPECS}


class CatalogRuntime(RuntimeBase):
    spec: RuntimeSpec = None

    def __init__(self, runtime_config):
        super().__init__(runtime_config)
        self.name = self.spec.name

    def get_runtime_commands(self, cluster_config):
        return standard_commands(self.name)

    def get_defaults_config(self, cluster_config):
        return dict(self.spec.defaults)

    def with_environment_variables(self, config, provider, node_id):
        env = dict(self.spec.env)
        if self.spec.home_env:
            env[self.spec.home_env] = f"$RUNTIME_PATH/{self.name}"
        rc = (config or {}).get("runtime", {}).get(self.name, {}) or {}
        for k, v in rc.items():
            if k.startswith("with_"):
                env[f"{self.name.upper()}_{k.upper()}"] = str(v).lower() if isinstance(v, bool) else str(v)
        return env

    def get_runtime_services(self, cluster_config):
        cluster = cluster_config.get("cluster_name", "default")
        out = {}
        for s in self.spec.services:
            name = f"{cluster}-{s.name}"
            out[name] = sd.define_runtime_service(self.name, s.name, s.port, s.protocol, s.node_kind,
                                                  s.scope, list(s.features), s.metrics)
        return out

    def get_head_service_ports(self):
        return {s.name: {"protocol": s.protocol, "port": s.port}
                for s in self.spec.services if s.node_kind in (H, A)}

    def get_runtime_endpoints(self, cluster_config, cluster_head_ip):
        return {s.name: {"url": f"{'http://' if s.protocol == HTTP else ''}{cluster_head_ip}:{s.port}"}
                for s in self.spec.services if s.node_kind in (H, A)}

    def get_node_constraints(self, cluster_config, node_type=None):
        """(require minimal nodes before setup, manage a quorum of them, quorum can grow at
        runtime) -- reference Runtime.get_node_constraints."""
        if not self.spec.quorum:
            return None
        return QUORUM_CONSTRAINTS.get(self.name, (True, True, True))

    def node_constraints_reached(self, cluster_config, node_type, head_info, nodes_info, quorum_id=None):
        """Called on the head when the node type's minimal membership (or a quorum join) is
        complete: the ensemble -- member addresses in sequence order -- is registered in the
        workspace registry as ``<cluster>-<runtime>-ensemble`` so other clusters discover the
        servers of THIS quorum (reference zookeeper/utils.py:66 _handle_node_constraints_reached)."""
        if not self.spec.services:
            return None
        members = sorted(nodes_info.values(), key=lambda i: i.get("node_seq_id", 0))
        hosts = [m["node_ip"] for m in members if m.get("node_ip")]
        svc = self.spec.services[0]
        rec = sd.define_runtime_service(self.name, f"{svc.name}-ensemble", svc.port, svc.protocol, svc.node_kind,
                                        svc.scope, list(svc.features), svc.metrics)
        rec.update(quorum_id=quorum_id, node_type=node_type)
        key = sd.service_global_key(cluster_config.get("cluster_name", "default"), f"{self.name}-ensemble")
        gv = {key: sd.encode_service_address(rec, hosts[0] if hosts else None, hosts)}
        try:
            from cloudtik_amd.core.provider_factory import get_workspace_provider
            get_workspace_provider(cluster_config["provider"], cluster_config.get("workspace_name", "default")) \
                .publish_global_variables(cluster_config, gv)
        except Exception as e:  # noqa: BLE001 - discovery falls back to the members' tags
            import logging
            logging.getLogger(__name__).warning("%s: could not register the ensemble: %s", self.name, e)
        return gv

    def get_logs(self):
        return dict(self.spec.logs)

    def get_processes(self):
        out = []
        for p in self.spec.head_processes:
            out.append([p, False, p, "head"])
        for p in self.spec.worker_processes:
            out.append([p, False, p, "worker"])
        return out

    def get_dependencies(self):
        return list(self.spec.dependencies)

    def get_required(self):
        return list(self.spec.required)

    # ---------------------------------------------------------- node-side shell steps
    def install_steps(self, head):
        s = self.spec
        steps = []
        if s.apt:
            steps.append("which apt-get >/dev/null && (sudo apt-get -qq update -y && "
                         f"sudo DEBIAN_FRONTEND=noninteractive apt-get -qq install -y {' '.join(s.apt)} >/dev/null) || true")
        if s.download:
            url = s.download.format(version=s.version)
            dest = f"$RUNTIME_PATH/{s.name}"
            steps.append(f"mkdir -p $RUNTIME_PATH && ( [ -d {dest} ] || ( cd $RUNTIME_PATH && "
                         f"wget -q -O /tmp/{s.name}.pkg {url} && mkdir -p {dest} && "
                         f"(tar -xf /tmp/{s.name}.pkg -C {dest} --strip-components=1 2>/dev/null || "
                         f"(cp /tmp/{s.name}.pkg {dest}/{s.name} && chmod +x {dest}/{s.name})) ) )")
        return steps

    def configure_steps(self, head):
        return [f"mkdir -p $RUNTIME_PATH/{self.name}/logs"]

    def start_steps(self, head):
        c = self.spec.start.get("head" if head else "worker")
        return [c] if c else []

    def stop_steps(self, head):
        c = self.spec.stop.get("head" if head else "worker")
        return [c] if c else []


def make_runtime_class(name: str):
    spec = SPEC_BY_NAME[name]
    cls_name = "".join(p.capitalize() for p in name.split("_")) + "Runtime"
    return type(cls_name, (CatalogRuntime,), {"spec": spec, "__doc__": spec.description})
