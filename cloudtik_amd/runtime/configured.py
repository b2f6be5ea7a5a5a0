"""Self-configuring service runtimes: the configuration files the catalogue's start commands
expect, rendered per node at ``cloudtik runtime configure`` time (reference
runtime/{zookeeper,kafka,redis,mongodb,consul,etcd,coredns,mysql,postgres,prometheus,grafana,
haproxy}/scripts/configure.{sh,py} + conf templates -- server ensembles from the quorum
members, broker / server ids from node sequence ids, replication wiring to the head).

Membership comes from the provider while the node's setup environment is built
(``with_environment_variables``: the workers of this cluster -- of the same quorum when the
runtime forms one -- sorted by sequence id, as ``<NAME>_MEMBERS=seq@ip,...``), so every member
of a quorum is configured with the same ensemble.  Settings come from the cluster's
``runtime.<name>`` section (same keys as the reference schema, see schema/build.py).  Each
runtime's ``files()`` maps absolute paths to file contents; ``node_configure`` writes them and
then runs the catalogue's configure steps.
"""
from __future__ import annotations

import json
import os
import shlex
from typing import Any, Dict, List, Optional, Tuple

from cloudtik_amd.core import tags as T
from cloudtik_amd.runtime.catalog import SPEC_BY_NAME, CatalogRuntime

DATA_DISK_GLOB = "/mnt/cloudtik/data_disk_*"


def members_of(provider, node_id: Optional[str], quorum: bool) -> List[Tuple[int, str]]:
    """(seq id, internal ip) of the cluster's workers (same quorum id as ``node_id`` when it
    has one), in sequence order."""
    qid = provider.node_tags(node_id).get(T.CLOUDTIK_TAG_QUORUM_ID) if (quorum and node_id) else None
    out = []
    for n in provider.non_terminated_nodes({T.CLOUDTIK_TAG_NODE_KIND: T.NODE_KIND_WORKER}):
        t = provider.node_tags(n)
        if qid and t.get(T.CLOUDTIK_TAG_QUORUM_ID) != qid:
            continue
        seq = t.get(T.CLOUDTIK_TAG_NODE_SEQ_ID) or "0"
        out.append((int(seq) if str(seq).isdigit() else 0, provider.internal_ip(n)))
    return sorted(out)


def parse_members(s: str) -> List[Tuple[int, str]]:
    out = []
    for item in (s or "").split(","):
        if "@" in item:
            seq, ip = item.split("@", 1)
            out.append((int(seq), ip))
    return out


def _props(d: Dict[str, Any]) -> str:
    return "".join(f"{k}={v}\n" for k, v in d.items())


class ConfiguredRuntime(CatalogRuntime):
    """Catalogue runtime + rendered configuration files."""

    members_env = ""           # e.g. ZOOKEEPER_MEMBERS; "" = no membership needed
    quorum_members = True      # restrict membership to this node's quorum

    def with_environment_variables(self, config, provider, node_id):
        env = super().with_environment_variables(config, provider, node_id)
        if self.members_env and provider is not None:
            m = members_of(provider, node_id, self.quorum_members)
            env[self.members_env] = ",".join(f"{s}@{ip}" for s, ip in m)
        return env

    # ---------------------------------------------------------------- node side
    def ctx(self, head: bool, env: Dict[str, str]) -> Dict[str, Any]:
        rp = env.get("RUNTIME_PATH", "")
        home = env.get(self.spec.home_env) if self.spec.home_env else None
        seq = env.get("CLOUDTIK_NODE_SEQ_ID") or "1"
        return {"head": head, "rp": rp, "dir": os.path.join(rp, self.name), "home": home or os.path.join(rp, self.name),
                "ip": env.get("CLOUDTIK_NODE_IP") or "127.0.0.1",
                "head_ip": env.get("CLOUDTIK_HEAD_IP") or env.get("CLOUDTIK_NODE_IP") or "127.0.0.1",
                "seq": int(seq) if str(seq).isdigit() else 1, "cluster": env.get("CLOUDTIK_CLUSTER", "cloudtik"),
                "members": parse_members(env.get(self.members_env, "")) if self.members_env else [],
                "cfg": self.runtime_config or {}}

    def files(self, c: Dict[str, Any]) -> Dict[str, str]:
        return {}

    def render(self, head: bool) -> Dict[str, str]:
        env = self.node_env(head)
        out = self.files(self.ctx(head, env))
        for path, text in out.items():
            os.makedirs(os.path.dirname(path), exist_ok=True)
            with open(path, "w") as f:
                f.write(text)
        return out

    def node_configure(self, head: bool):
        self.render(head)
        return self._run_steps(self.configure_steps(head), head)


def _extra(cfg: Dict[str, Any]) -> Dict[str, Any]:
    return dict(cfg.get("config", {}) or {})


# ----------------------------------------------------------------------------- ZooKeeper
class ZooKeeperRuntime(ConfiguredRuntime):
    spec = SPEC_BY_NAME["zookeeper"]
    members_env = "ZOOKEEPER_MEMBERS"

    def files(self, c):
        if c["head"]:
            return {}
        data = os.path.join(c["dir"], "data")
        conf = {"tickTime": 2000, "initLimit": 10, "syncLimit": 5, "dataDir": data, "clientPort": 2181,
                "4lw.commands.whitelist": "srvr,ruok,mntr,stat", "admin.enableServer": "false"}
        conf.update(_extra(c["cfg"]))
        servers = "".join(f"server.{s}={ip}:2888:3888\n" for s, ip in c["members"])
        return {os.path.join(c["home"], "conf", "zoo.cfg"): _props(conf) + servers,
                os.path.join(data, "myid"): f"{c['seq']}\n"}


# ----------------------------------------------------------------------------- Kafka
class KafkaRuntime(ConfiguredRuntime):
    spec = SPEC_BY_NAME["kafka"]
    members_env = "KAFKA_MEMBERS"
    quorum_members = False

    def with_environment_variables(self, config, provider, node_id):
        env = super().with_environment_variables(config, provider, node_id)
        rc = (config or {}).get("runtime", {}) or {}
        zk = (rc.get("kafka", {}) or {}).get("zookeeper_connect")
        if not zk and "zookeeper" in (rc.get("types") or []) and provider is not None:
            # ZooKeeper of the same cluster: its members (all workers run it)
            zk = ",".join(f"{ip}:2181" for _, ip in members_of(provider, node_id, False))
        if zk:
            env["KAFKA_ZOOKEEPER_CONNECT"] = zk
        return env

    def ctx(self, head, env):
        c = super().ctx(head, env)
        c["zk"] = env.get("KAFKA_ZOOKEEPER_CONNECT") or c["cfg"].get("zookeeper_connect") or f"{c['head_ip']}:2181"
        return c

    def files(self, c):
        if c["head"]:
            return {}
        import glob
        disks = sorted(glob.glob(DATA_DISK_GLOB))
        logs = ",".join(os.path.join(d, "kafka-logs") for d in disks) or os.path.join(c["dir"], "kafka-logs")
        rf = max(1, min(3, len(c["members"]) or 1))
        conf = {"broker.id": c["seq"], "listeners": f"PLAINTEXT://{c['ip']}:9092",
                "advertised.listeners": f"PLAINTEXT://{c['ip']}:9092", "log.dirs": logs,
                "zookeeper.connect": c["zk"], "num.partitions": 8, "default.replication.factor": rf,
                "offsets.topic.replication.factor": rf, "transaction.state.log.replication.factor": rf,
                "transaction.state.log.min.isr": max(1, rf - 1), "log.retention.hours": 168,
                "num.network.threads": 8, "num.io.threads": 16}
        conf.update(_extra(c["cfg"]))
        return {os.path.join(c["home"], "config", "server.properties"): _props(conf)}


# ----------------------------------------------------------------------------- Redis
class RedisRuntime(ConfiguredRuntime):
    """``cluster_mode``: ``replication`` (workers replicate the head; with ``sentinel.enabled``
    a sentinel on every node fails the master over) or ``sharding`` (a Redis Cluster: the head
    bootstraps the slots, every worker meets it and takes a master share or a replica role --
    runtime/redis_cluster.py)."""
    spec = SPEC_BY_NAME["redis"]
    members_env = "REDIS_MEMBERS"
    quorum_members = False

    def files(self, c):
        cfg = c["cfg"]
        mode = cfg.get("cluster_mode", "none")
        port = int(cfg.get("port", 6379))
        lines = ["bind 0.0.0.0", f"port {port}", f"dir {os.path.join(c['dir'], 'data')}", "appendonly yes",
                 f"logfile {os.path.join(c['dir'], 'logs', 'redis.log')}", "protected-mode no"]
        if cfg.get("password"):
            lines += [f"requirepass {cfg['password']}", f"masterauth {cfg['password']}"]
        if mode == "replication" and not c["head"]:
            lines.append(f"replicaof {c['head_ip']} {port}")
        elif mode == "sharding":
            lines += ["cluster-enabled yes", f"cluster-config-file {os.path.join(c['dir'], 'data', 'nodes.conf')}",
                      "cluster-node-timeout 5000", f"cluster-announce-ip {c['ip']}"]
        lines += [f"{k} {v}" for k, v in _extra(cfg).items()]
        out = {os.path.join(c["dir"], "redis.conf"): "\n".join(lines) + "\n"}
        if mode == "replication" and (cfg.get("sentinel") or {}).get("enabled"):
            from cloudtik_amd.runtime.replication import redis_sentinel_conf
            out[os.path.join(c["dir"], "sentinel.conf")] = redis_sentinel_conf(c)
        return out

    def configure_steps(self, head):
        return [f"mkdir -p $RUNTIME_PATH/redis/data $RUNTIME_PATH/redis/logs"]

    def start_steps(self, head):
        import sys
        c = self.ctx(head, self.node_env(head))
        cfg = c["cfg"]
        mode = cfg.get("cluster_mode", "none")
        port = int(cfg.get("port", 6379))
        steps = super().start_steps(head)
        if mode == "replication" and (cfg.get("sentinel") or {}).get("enabled"):
            steps.append(f"redis-sentinel {c['dir']}/sentinel.conf --daemonize yes")
        elif mode == "sharding":
            seeds = [c["head_ip"]] + [ip for _, ip in c["members"] if ip != c["ip"]]
            # the join speaks RESP to every member: with requirepass set it must AUTH (the
            # password goes by environment, not argv, so it stays out of the process table)
            auth = f"REDIS_PASSWORD={shlex.quote(str(cfg['password']))} " if cfg.get("password") else ""
            steps.append(f"{auth}{sys.executable} -m cloudtik_amd.runtime.redis_cluster join --node-ip {c['ip']} "
                         f"--port {port} --seeds {','.join(seeds)}"
                         f" --replicas-per-master {int((cfg.get('sharding') or {}).get('replicas_per_master', 0))}"
                         f" --marker {c['dir']}/data/.cluster-initialized" + (" --head" if head else ""))
        return steps

    def stop_steps(self, head):
        steps = super().stop_steps(head)
        if (self.runtime_config or {}).get("cluster_mode") == "replication" and \
                ((self.runtime_config or {}).get("sentinel") or {}).get("enabled"):
            sp = int(((self.runtime_config or {}).get("sentinel") or {}).get("port", 26379))
            steps.append(f"redis-cli -p {sp} shutdown || true")
        return steps


# ----------------------------------------------------------------------------- MongoDB
class MongoDBRuntime(ConfiguredRuntime):
    """``cluster_mode``: ``replication`` (one replica set: the head initiates it, workers are
    added from the primary) or ``sharding`` (config-server replica set + mongos router on the
    head, the workers grouped into shard replica sets of ``shard_size`` members;
    runtime/replication.py)."""
    spec = SPEC_BY_NAME["mongodb"]
    members_env = "MONGODB_MEMBERS"
    quorum_members = False

    @staticmethod
    def _mongod(c, port, db, log, extra=None):
        conf = {"storage": {"dbPath": os.path.join(c["dir"], db)},
                "net": {"port": port, "bindIp": "0.0.0.0"},
                "systemLog": {"destination": "file", "path": os.path.join(c["dir"], "logs", log), "logAppend": True},
                "processManagement": {"fork": True}}
        conf.update(extra or {})
        return conf

    def files(self, c):
        import yaml
        cfg = c["cfg"]
        mode = cfg.get("cluster_mode", "none")
        port = int(cfg.get("port", 27017))
        if mode == "sharding":
            cfg_port = int(cfg.get("config_server_port", 27019))
            shard_port = int(cfg.get("shard_server_port", 27018))
            if c["head"]:
                cfg_rs = f"{c['cluster']}-cfg"
                cs = self._mongod(c, cfg_port, "data-cfg", "mongod-cfg.log",
                                  {"replication": {"replSetName": cfg_rs}, "sharding": {"clusterRole": "configsvr"}})
                mongos = {"net": {"port": port, "bindIp": "0.0.0.0"},
                          "systemLog": {"destination": "file", "path": os.path.join(c["dir"], "logs", "mongos.log"),
                                        "logAppend": True},
                          "processManagement": {"fork": True},
                          "sharding": {"configDB": f"{cfg_rs}/{c['head_ip']}:{cfg_port}"}}
                return {os.path.join(c["dir"], "mongod-cfg.conf"): yaml.safe_dump(cs, sort_keys=False),
                        os.path.join(c["dir"], "mongos.conf"): yaml.safe_dump(mongos, sort_keys=False)}
            from cloudtik_amd.runtime.replication import mongo_shard_layout
            layout = mongo_shard_layout(c["members"], cfg.get("shard_size", 1), c["cluster"])
            rs = next((s["name"] for s in layout if c["ip"] in s["members"]), f"{c['cluster']}-shard0")
            conf = self._mongod(c, shard_port, "data", "mongod.log",
                                {"replication": {"replSetName": rs}, "sharding": {"clusterRole": "shardsvr"}})
            return {os.path.join(c["dir"], "mongod.conf"): yaml.safe_dump(conf, sort_keys=False)}
        conf = self._mongod(c, port, "data", "mongod.log")
        if mode == "replication":
            conf["replication"] = {"replSetName": cfg.get("replication_set_name") or f"{c['cluster']}-rs"}
        return {os.path.join(c["dir"], "mongod.conf"): yaml.safe_dump(conf, sort_keys=False)}

    def configure_steps(self, head):
        return ["mkdir -p $RUNTIME_PATH/mongodb/data $RUNTIME_PATH/mongodb/data-cfg $RUNTIME_PATH/mongodb/logs"]

    def start_steps(self, head):
        from cloudtik_amd.runtime.replication import mongodb_bootstrap_steps
        c = self.ctx(head, self.node_env(head))
        if c["cfg"].get("cluster_mode", "none") == "sharding" and head:
            steps = [f"mongod --fork --config {c['dir']}/mongod-cfg.conf"]
        else:
            steps = super().start_steps(head)
        return steps + mongodb_bootstrap_steps(c)

    def stop_steps(self, head):
        if head and (self.runtime_config or {}).get("cluster_mode") == "sharding":
            return ["pkill -f 'mongos --config' || true",
                    "mongod --shutdown --dbpath $RUNTIME_PATH/mongodb/data-cfg || true"]
        return super().stop_steps(head)


# ----------------------------------------------------------------------------- Consul
class ConsulRuntime(ConfiguredRuntime):
    spec = SPEC_BY_NAME["consul"]
    members_env = "CONSUL_MEMBERS"

    def files(self, c):
        cfg = c["cfg"]
        servers_on_workers = bool(cfg.get("server", False))
        server = (not c["head"]) if servers_on_workers else c["head"]
        join = [ip for _, ip in c["members"]] if servers_on_workers else [c["head_ip"]]
        conf = {"datacenter": cfg.get("data_center") or c["cluster"], "data_dir": os.path.join(c["dir"], "data"),
                "bind_addr": c["ip"], "client_addr": "0.0.0.0", "server": server,
                "retry_join": [ip for ip in join if ip != c["ip"]] or join,
                "ports": {"http": int(cfg.get("http_port", 8500)), "dns": int(cfg.get("dns_port", 8600))},
                "ui_config": {"enabled": bool(server)}}
        if server:
            conf["bootstrap_expect"] = len(join) if servers_on_workers else 1
        if not cfg.get("disable_cluster_node_name"):
            conf["node_name"] = f"{c['cluster']}-{c['seq']}"
        return {os.path.join(c["dir"], "consul.d", "consul.json"): json.dumps(conf, indent=2) + "\n"}


# ----------------------------------------------------------------------------- etcd
class EtcdRuntime(ConfiguredRuntime):
    spec = SPEC_BY_NAME["etcd"]
    members_env = "ETCD_MEMBERS"

    def files(self, c):
        if c["head"]:
            return {}
        import yaml
        peers = ",".join(f"etcd{s}=http://{ip}:2380" for s, ip in c["members"])
        conf = {"name": f"etcd{c['seq']}", "data-dir": os.path.join(c["dir"], "data"),
                "listen-peer-urls": f"http://{c['ip']}:2380",
                "listen-client-urls": f"http://{c['ip']}:2379,http://127.0.0.1:2379",
                "initial-advertise-peer-urls": f"http://{c['ip']}:2380",
                "advertise-client-urls": f"http://{c['ip']}:2379", "initial-cluster": peers,
                "initial-cluster-token": f"cloudtik-{c['cluster']}", "initial-cluster-state": "new"}
        return {os.path.join(c["dir"], "etcd.yaml"): yaml.safe_dump(conf, sort_keys=False)}


# ----------------------------------------------------------------------------- CoreDNS
class CoreDNSRuntime(ConfiguredRuntime):
    spec = SPEC_BY_NAME["coredns"]

    def files(self, c):
        port = int(c["cfg"].get("port", 53))
        text = (f"consul:{port} {{\n    forward . 127.0.0.1:8600\n    cache 30\n}}\n"
                f".:{port} {{\n    forward . /etc/resolv.conf\n    cache 30\n    errors\n}}\n")
        return {os.path.join(c["dir"], "Corefile"): text}


# ----------------------------------------------------------------------------- MySQL / PostgreSQL
class MySQLRuntime(ConfiguredRuntime):
    """``cluster_mode``: ``replication`` (GTID source on the head, every worker a replica of
    it) or ``group_replication`` (single- or multi-primary group bootstrapped by the head);
    runtime/replication.py issues the replication statements after the server is up."""
    spec = SPEC_BY_NAME["mysql"]
    members_env = "MYSQL_MEMBERS"
    quorum_members = False

    def files(self, c):
        cfg = c["cfg"]
        mode = cfg.get("cluster_mode", "none")
        port = int(cfg.get("port", 3306))
        lines = ["[mysqld]", f"server-id = {c['seq']}", "bind-address = 0.0.0.0",
                 f"port = {port}", "max_connections = 1000", f"report_host = {c['ip']}"]
        if mode in ("replication", "group_replication"):
            lines += ["log_bin = mysql-bin", "binlog_format = ROW", "gtid_mode = ON",
                      "enforce_gtid_consistency = ON", "log_replica_updates = ON"]
            if mode == "replication" and not c["head"]:
                lines += ["read_only = ON", "super_read_only = ON", "skip_replica_start = OFF"]
            if mode == "group_replication":
                from cloudtik_amd.runtime.replication import mysql_group_conf
                lines += mysql_group_conf(c, port)
        return {os.path.join(c["dir"], "conf.d", "cloudtik.cnf"): "\n".join(lines) + "\n"}

    def configure_steps(self, head):
        # the packaged server reads /etc/mysql/mysql.conf.d
        return ["mkdir -p $RUNTIME_PATH/mysql/logs",
                "[ -d /etc/mysql/mysql.conf.d ] && sudo cp $RUNTIME_PATH/mysql/conf.d/cloudtik.cnf "
                "/etc/mysql/mysql.conf.d/zz-cloudtik.cnf || true"]

    def _clustered(self) -> bool:
        return (self.runtime_config or {}).get("cluster_mode", "none") in ("replication", "group_replication")

    def start_steps(self, head):
        from cloudtik_amd.runtime.replication import mysql_bootstrap_steps
        if not head and not self._clustered():
            return []
        c = self.ctx(head, self.node_env(head))
        return ["sudo service mysql start"] + mysql_bootstrap_steps(c)

    def stop_steps(self, head):
        return ["sudo service mysql stop"] if (head or self._clustered()) else []


class PostgresRuntime(ConfiguredRuntime):
    """``cluster_mode: replication``: streaming replication from the head; a worker's data
    directory is replaced by a base backup of the primary before its server starts (so it comes
    up as a hot standby, not a second primary); with ``repmgr.enabled`` the nodes register with
    repmgr and ``repmgrd`` promotes a standby when the primary fails (runtime/replication.py)."""
    spec = SPEC_BY_NAME["postgres"]

    def _data_dir(self, cfg):
        return cfg.get("data_dir") or f"/var/lib/postgresql/{self.spec.version}/main"

    def files(self, c):
        from cloudtik_amd.runtime.replication import postgres_repmgr_enabled, repmgr_conf
        cfg = c["cfg"]
        repl = cfg.get("cluster_mode", "none") == "replication"
        repmgr = postgres_repmgr_enabled(cfg)
        conf = [f"listen_addresses = '*'", f"port = {int(cfg.get('port', 5432))}", "max_connections = 500"]
        if repl:
            conf += ["wal_level = replica", "max_wal_senders = 16", "max_replication_slots = 16",
                     "hot_standby = on", "wal_keep_size = 2048", "wal_log_hints = on",
                     f"archive_mode = {'on' if cfg.get('archive_mode') else 'off'}"]
            if repmgr:
                conf.append("shared_preload_libraries = 'repmgr'")
            if not c["head"]:
                user = cfg.get("replication_user", "repl_user")
                conf.append(f"primary_conninfo = 'host={c['head_ip']} port={int(cfg.get('port', 5432))} "
                            f"user={user} application_name={c['cluster']}-{c['seq']}'")
        hba = ["host all all 0.0.0.0/0 scram-sha-256"]
        if repl:
            hba.append("host replication all 0.0.0.0/0 scram-sha-256")
        out = {os.path.join(c["dir"], "conf.d", "cloudtik.conf"): "\n".join(conf) + "\n",
               os.path.join(c["dir"], "conf.d", "pg_hba.cloudtik.conf"): "\n".join(hba) + "\n"}
        if repmgr:
            out[os.path.join(c["dir"], "repmgr.conf")] = repmgr_conf(c, self._data_dir(cfg))
        return out

    def configure_steps(self, head):
        # packaged server: include dir conf.d + hba rules appended once
        return ["mkdir -p $RUNTIME_PATH/postgres/logs",
                "for d in /etc/postgresql/*/main; do [ -d $d ] || continue; sudo mkdir -p $d/conf.d && "
                "sudo cp $RUNTIME_PATH/postgres/conf.d/cloudtik.conf $d/conf.d/zz-cloudtik.conf && "
                "(sudo grep -q cloudtik-hba $d/pg_hba.conf || (echo '# cloudtik-hba' | sudo tee -a $d/pg_hba.conf "
                ">/dev/null && sudo tee -a $d/pg_hba.conf < $RUNTIME_PATH/postgres/conf.d/pg_hba.cloudtik.conf "
                ">/dev/null)); done; true"]

    def _replicated(self) -> bool:
        return (self.runtime_config or {}).get("cluster_mode", "none") == "replication"

    def start_steps(self, head):
        from cloudtik_amd.runtime.replication import postgres_bootstrap_steps, postgres_pre_start_steps
        if not head and not self._replicated():
            return []
        c = self.ctx(head, self.node_env(head))
        return postgres_pre_start_steps(c) + ["sudo service postgresql start"] + postgres_bootstrap_steps(c)

    def stop_steps(self, head):
        if not head and not self._replicated():
            return []
        steps = ["pkill -f 'repmgrd -f' || true"] if (self.runtime_config or {}).get("repmgr") else []
        return steps + ["sudo service postgresql stop"]


# ----------------------------------------------------------------------------- Prometheus / Grafana
class PrometheusRuntime(ConfiguredRuntime):
    """``scrape_scope`` local (default) / workspace / federation and ``service_discovery``
    file / consul (auto: consul when the cluster runs it), runtime/monitoring_discovery.py.
    File-based local scrape: the head's ``DiscoverLocalTargets`` pull job keeps
    ``conf/local-targets.yaml`` current from the live nodes (``pull_services``, default every
    node's exporter :9100 and training metrics :9500); federation from ``federation_targets``
    is a static ``conf/federation-targets.yaml``."""
    spec = SPEC_BY_NAME["prometheus"]
    members_env = "PROMETHEUS_MEMBERS"
    quorum_members = False

    @staticmethod
    def _consul(cfg) -> bool:
        if "use_consul" in cfg:
            return bool(cfg["use_consul"])
        return "consul" in [r.strip() for r in os.environ.get("CLOUDTIK_RUNTIMES", "").split(",")]

    def _plan(self, c):
        from cloudtik_amd.runtime import monitoring_discovery as MD
        cfg = c["cfg"]
        scope, sd = MD.resolve_discovery(cfg, self._consul(cfg))
        return MD, scope, sd, os.path.join(c["home"], "conf")

    def files(self, c):
        import yaml
        MD, scope, sd, conf_dir = self._plan(c)
        cfg = c["cfg"]
        consul = cfg.get("consul_address") or f"{c['head_ip']}:8500"
        workspace = os.environ.get("CLOUDTIK_WORKSPACE", "default")
        scrape = MD.scrape_configs(scope, sd, conf_dir, c["cluster"], workspace, consul, cfg.get("scrape_services"))
        conf = {"global": {"scrape_interval": "30s", "evaluation_interval": "15s",
                           "external_labels": {"monitor": "cloudtik"}}, "scrape_configs": scrape}
        out = {os.path.join(c["home"], "prometheus.yml"): yaml.safe_dump(conf, sort_keys=False)}
        if scope == "federation" and sd == "file":
            out[os.path.join(conf_dir, "federation-targets.yaml")] = yaml.safe_dump(
                MD.federation_targets_file(cfg.get("federation_targets") or []), sort_keys=False)
        if self._pulls_local(c, scope, sd):
            out[os.path.join(c["dir"], "local-targets.json")] = json.dumps(
                {"interval": cfg.get("pull_interval", 15), "pull_services": cfg.get("pull_services") or
                 MD.DEFAULT_PULL_SERVICES, "targets_file": os.path.join(conf_dir, "local-targets.yaml"),
                 "state_address": f"{c['head_ip']}:{os.environ.get('CLOUDTIK_DEFAULT_PORT', '6789')}"}, indent=1)
        return out

    @staticmethod
    def _pulls_local(c, scope, sd) -> bool:
        # the file-based local scrape needs the live-node pull job, on the head (or on every
        # Prometheus node with high_availability)
        return sd == "file" and scope in ("local", "federation") and (
            c["head"] or bool(c["cfg"].get("high_availability")))

    def start_steps(self, head):
        steps = super().start_steps(head)
        c = self.ctx(head, self.node_env(head))
        _, scope, sd, _ = self._plan(c)
        if self._pulls_local(c, scope, sd):
            steps.append("cloudtik node service-daemon start prometheus-local-targets "
                         "--service-class cloudtik_amd.runtime.monitoring_discovery.DiscoverLocalTargets "
                         f"config_file={os.path.join(c['dir'], 'local-targets.json')}")
        return steps

    def stop_steps(self, head):
        return ["cloudtik node service-daemon stop prometheus-local-targets"] + super().stop_steps(head)


class GrafanaRuntime(ConfiguredRuntime):
    """``data_sources_scope`` (reference grafana/utils.py:95-110):

    * ``local`` (default): this cluster's Prometheus as the default data source (provisioned);
    * ``workspace``: every Prometheus server of the workspace, kept current by the
      ``DiscoverDataSources`` pull job through the admin API (``data_sources_services``
      narrows the service selector; needs Consul) -- runtime/monitoring_discovery.py;
    * ``none``: only the static ``data_sources``."""
    spec = SPEC_BY_NAME["grafana"]

    def _scope(self, cfg) -> str:
        scope = cfg.get("data_sources_scope") or "local"
        if scope not in ("none", "local", "workspace"):
            raise ValueError(f"grafana.data_sources_scope must be none / local / workspace, not {scope!r}")
        if scope == "workspace" and not PrometheusRuntime._consul(cfg):
            raise ValueError("grafana.data_sources_scope 'workspace' needs a service discovery runtime (consul)")
        return scope

    def files(self, c):
        import yaml
        cfg = c["cfg"]
        scope = self._scope(cfg)
        sources = [dict(s) for s in cfg.get("data_sources") or []]
        if scope == "local" and not any(s.get("type") == "prometheus" for s in sources):
            port = int((cfg.get("prometheus") or {}).get("port", 9090))
            sources.append({"name": "cloudtik-prometheus", "type": "prometheus",
                            "url": f"http://{c['head_ip']}:{port}", "isDefault": True})
        conf = {"apiVersion": 1, "datasources": [dict({"access": "proxy"}, **s) for s in sources]}
        # $GRAFANA_HOME/conf/provisioning is where a tarball install looks by default
        out = {os.path.join(c["home"], "conf", "provisioning", "datasources", "cloudtik.yaml"):
               yaml.safe_dump(conf, sort_keys=False)}
        if scope == "workspace":
            out[os.path.join(c["dir"], "data-sources.json")] = json.dumps(
                {"interval": cfg.get("discovery_interval", 15),
                 "admin_endpoint": f"http://127.0.0.1:{int(cfg.get('port', 3000))}",
                 "service_selector": cfg.get("data_sources_services") or {},
                 "consul_address": cfg.get("consul_address") or f"{c['head_ip']}:8500",
                 "user": cfg.get("admin_user", "cloudtik"), "password": cfg.get("admin_password", "cloudtik")},
                indent=1)
        return out

    def start_steps(self, head):
        steps = super().start_steps(head)
        c = self.ctx(head, self.node_env(head))
        if self._scope(c["cfg"]) == "workspace":
            steps.append("cloudtik node service-daemon start grafana-data-sources "
                         "--service-class cloudtik_amd.runtime.monitoring_discovery.DiscoverDataSources "
                         f"config_file={os.path.join(c['dir'], 'data-sources.json')}")
        return steps

    def stop_steps(self, head):
        steps = []
        if (self.runtime_config or {}).get("data_sources_scope") == "workspace":
            steps.append("cloudtik node service-daemon stop grafana-data-sources")
        return steps + super().stop_steps(head)


# ----------------------------------------------------------------------------- HAProxy
class DiscoveryBackedRuntime(ConfiguredRuntime):
    """A load balancer / gateway whose backends come from service discovery when
    ``backend.config_mode`` is ``dynamic`` (the default once a ``backend.selector`` is given):
    a pull job (runtime/gateway_discovery.py) started as a service daemon on every node that
    runs the gateway updates it as services come and go."""

    discovery_class = ""

    def dynamic(self, cfg) -> bool:
        backend = cfg.get("backend") or {}
        mode = backend.get("config_mode") or ("dynamic" if backend.get("selector") else "static")
        return mode == "dynamic"

    def discovery_config(self, c) -> Dict[str, Any]:
        cfg = c["cfg"]
        backend = cfg.get("backend") or {}
        selector = backend.get("selector") or {"clusters": [c["cluster"]], "tags": ["cloudtik-f-load-balancer"]}
        consul = cfg.get("consul_address") or f"{c['head_ip']}:8500"
        return {"service_selector": selector, "consul_address": consul, "interval": backend.get("interval", 15)}

    def _discovery_files(self, c) -> Dict[str, str]:
        if not self.dynamic(c["cfg"]):
            return {}
        return {os.path.join(c["dir"], "discovery.json"): json.dumps(self.discovery_config(c), indent=1)}

    def start_steps(self, head):
        steps = super().start_steps(head)
        c = self.ctx(head, self.node_env(head))
        if self.dynamic(c["cfg"]):
            steps.append(f"cloudtik node service-daemon start {self.name}-discovery "
                         f"--service-class cloudtik_amd.runtime.gateway_discovery.{self.discovery_class} "
                         f"config_file={os.path.join(c['dir'], 'discovery.json')}")
        return steps

    def stop_steps(self, head):
        steps = []
        if self.dynamic(self.runtime_config or {}):
            steps.append(f"cloudtik node service-daemon stop {self.name}-discovery")
        return steps + super().stop_steps(head)


class HAProxyRuntime(DiscoveryBackedRuntime):
    """Static backends (``backend.servers``) or dynamic ones: the runtime API socket is
    opened and the backend gets a pool of server slots that the discovery job fills
    (``DiscoverHAProxyBackends``)."""
    spec = SPEC_BY_NAME["haproxy"]
    discovery_class = "DiscoverHAProxyBackends"
    API_PORT = 19999

    def files(self, c):
        from cloudtik_amd.runtime.gateway_discovery import haproxy_config
        cfg = c["cfg"]
        backend = cfg.get("backend") or {}
        dyn = self.dynamic(cfg)
        text = haproxy_config(int(cfg.get("port", 80)), cfg.get("protocol", "http"),
                              [] if dyn else list(backend.get("servers") or []),
                              backend.get("health_check_port"), backend.get("health_check_path", "/"),
                              api_port=self.API_PORT if dyn else None)
        out = {os.path.join(c["dir"], "haproxy.cfg"): text}
        out.update(self._discovery_files(c))
        return out

    def discovery_config(self, c):
        cfg = c["cfg"]
        backend = cfg.get("backend") or {}
        d = super().discovery_config(c)
        d.update(backend_name="cloudtik-servers", api_addresses=[f"127.0.0.1:{self.API_PORT}"],
                 conf_path=os.path.join(c["dir"], "haproxy.cfg"),
                 haproxy={"port": int(cfg.get("port", 80)), "protocol": cfg.get("protocol", "http"),
                          "health_check_port": backend.get("health_check_port"),
                          "health_check_path": backend.get("health_check_path", "/"), "api_port": self.API_PORT})
        return d

    def configure_steps(self, head):
        return ["mkdir -p $RUNTIME_PATH/haproxy/logs",
                "[ -d /etc/haproxy ] && sudo cp $RUNTIME_PATH/haproxy/haproxy.cfg /etc/haproxy/haproxy.cfg || true"]


# ----------------------------------------------------------------------------- load balancer
class LoadBalancerRuntime(ConfiguredRuntime):
    """Head-only driver of the workspace's load balancers (reference runtime/loadbalancer).
    ``backend.config_mode: static`` -> the load balancers for ``backend.services`` are
    reconciled once at configure time; ``dynamic`` (default) -> the controller pull job
    (core/load_balancer.py ``LoadBalancerController``) discovers the services matching
    ``backend.selector`` (default: this cluster's services with the load-balancer feature)
    and reconciles on every change, under Consul leader election when Consul runs."""

    spec = SPEC_BY_NAME["loadbalancer"]

    def _controller_config(self, c) -> Dict[str, Any]:
        cfg = c["cfg"]
        backend = cfg.get("backend") or {}
        selector = backend.get("selector") or {"clusters": [c["cluster"]], "tags": ["cloudtik-f-load-balancer"]}
        provider = dict(cfg.get("provider") or {})
        provider.setdefault("type", os.environ.get("CLOUDTIK_PROVIDER_TYPE", "haproxy"))
        consul = cfg.get("consul_address") or (f"{c['head_ip']}:8500" if cfg.get("use_consul", True) else None)
        return {"provider_config": provider, "workspace_name": os.environ.get("CLOUDTIK_WORKSPACE", "default"),
                "service_selector": selector, "interval": backend.get("interval", 15), "consul_address": consul,
                "config_mode": backend.get("config_mode", "dynamic"), "services": backend.get("services") or {}}

    def files(self, c):
        if not c["head"]:
            return {}
        return {os.path.join(c["dir"], "controller.json"): json.dumps(self._controller_config(c), indent=1)}

    def node_configure(self, head: bool):
        out = self.render(head)
        if head:
            cc = json.loads(next(iter(out.values())))
            if cc["config_mode"] == "static":
                from cloudtik_amd.core.load_balancer import LoadBalancerManager, backend_services_from_config
                LoadBalancerManager(cc["provider_config"], cc["workspace_name"]).update(
                    backend_services_from_config({"services": cc["services"]}))
        return self._run_steps(self.configure_steps(head), head)

    def start_steps(self, head):
        if not head:
            return []
        c = self.ctx(head, self.node_env(head))
        cc = self._controller_config(c)
        if cc["config_mode"] == "static":
            return []
        return [f"cloudtik node service-daemon start loadbalancer "
                f"--service-class cloudtik_amd.core.load_balancer.LoadBalancerController "
                f"config_file={os.path.join(c['dir'], 'controller.json')}"]

    def stop_steps(self, head):
        return ["cloudtik node service-daemon stop loadbalancer"] if head else []


CONFIGURED = {"zookeeper": ZooKeeperRuntime, "kafka": KafkaRuntime, "redis": RedisRuntime,
              "mongodb": MongoDBRuntime, "consul": ConsulRuntime, "etcd": EtcdRuntime, "coredns": CoreDNSRuntime,
              "mysql": MySQLRuntime, "postgres": PostgresRuntime, "prometheus": PrometheusRuntime,
              "grafana": GrafanaRuntime, "haproxy": HAProxyRuntime, "loadbalancer": LoadBalancerRuntime}
