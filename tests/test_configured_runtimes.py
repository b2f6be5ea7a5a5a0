"""Service runtimes that render their own configuration (runtime/configured.py; reference
runtime/<name>/scripts/configure.* and conf templates): membership from the provider at
environment time (quorum-scoped), files rendered per node from that environment and the
cluster's runtime section."""
import json
import os

import yaml

from cloudtik_amd.core import runtime_factory as rf
from cloudtik_amd.core import tags as T
from cloudtik_amd.runtime.configured import members_of


class FakeProvider:
    def __init__(self):
        self.nodes = {
            "h": {T.CLOUDTIK_TAG_NODE_KIND: "head", T.CLOUDTIK_TAG_NODE_SEQ_ID: "1", "ip": "10.0.0.1"},
            "w3": {T.CLOUDTIK_TAG_NODE_KIND: "worker", T.CLOUDTIK_TAG_NODE_SEQ_ID: "3", T.CLOUDTIK_TAG_QUORUM_ID: "q1",
                   "ip": "10.0.0.13"},
            "w2": {T.CLOUDTIK_TAG_NODE_KIND: "worker", T.CLOUDTIK_TAG_NODE_SEQ_ID: "2", T.CLOUDTIK_TAG_QUORUM_ID: "q1",
                   "ip": "10.0.0.12"},
            "w4": {T.CLOUDTIK_TAG_NODE_KIND: "worker", T.CLOUDTIK_TAG_NODE_SEQ_ID: "4", T.CLOUDTIK_TAG_QUORUM_ID: "q1",
                   "ip": "10.0.0.14"},
            "w9": {T.CLOUDTIK_TAG_NODE_KIND: "worker", T.CLOUDTIK_TAG_NODE_SEQ_ID: "9", T.CLOUDTIK_TAG_QUORUM_ID: "q2",
                   "ip": "10.0.0.19"},      # a later quorum attempt: not part of q1's ensemble
        }

    def non_terminated_nodes(self, tag_filters):
        return [n for n, t in self.nodes.items() if all(t.get(k) == v for k, v in tag_filters.items())]

    def node_tags(self, n):
        return {k: v for k, v in self.nodes[n].items() if k != "ip"}

    def internal_ip(self, n):
        return self.nodes[n]["ip"]


def _render(name, rc, env, head=False, monkeypatch=None, tmp_path=None):
    rt = rf.get_runtime(name, rc)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("RUNTIME_PATH", str(tmp_path))
    if rt.spec.home_env:
        monkeypatch.setenv(rt.spec.home_env, str(tmp_path / name))
    out = rt.render(head)
    return {os.path.relpath(p, tmp_path): open(p).read() for p in out}


def test_membership_is_quorum_scoped_and_sequence_ordered():
    p = FakeProvider()
    assert members_of(p, "w3", quorum=True) == [(2, "10.0.0.12"), (3, "10.0.0.13"), (4, "10.0.0.14")]
    assert [s for s, _ in members_of(p, "w3", quorum=False)] == [2, 3, 4, 9]
    env = rf.get_runtime("zookeeper", {}).with_environment_variables({"runtime": {}}, p, "w2")
    assert env["ZOOKEEPER_MEMBERS"] == "2@10.0.0.12,3@10.0.0.13,4@10.0.0.14"


def test_zookeeper_and_kafka(tmp_path, monkeypatch):
    p = FakeProvider()
    cfg = {"runtime": {"types": ["zookeeper", "kafka"], "zookeeper": {"config": {"maxClientCnxns": 200}}}}
    env = rf.get_runtime("zookeeper", {}).with_environment_variables(cfg, p, "w3")
    env.update(CLOUDTIK_NODE_SEQ_ID="3", CLOUDTIK_NODE_IP="10.0.0.13", CLOUDTIK_HEAD_IP="10.0.0.1")
    files = _render("zookeeper", cfg["runtime"]["zookeeper"], env, monkeypatch=monkeypatch, tmp_path=tmp_path)
    zoo = files["zookeeper/conf/zoo.cfg"]
    assert "server.2=10.0.0.12:2888:3888\nserver.3=10.0.0.13:2888:3888\nserver.4=10.0.0.14:2888:3888" in zoo
    assert "maxClientCnxns=200" in zoo and "clientPort=2181" in zoo
    assert files["zookeeper/data/myid"] == "3\n"
    kenv = rf.get_runtime("kafka", {}).with_environment_variables(cfg, p, "w3")
    assert kenv["KAFKA_ZOOKEEPER_CONNECT"].startswith("10.0.0.12:2181,10.0.0.13:2181")
    kenv.update(CLOUDTIK_NODE_SEQ_ID="3", CLOUDTIK_NODE_IP="10.0.0.13")
    props = _render("kafka", {}, kenv, monkeypatch=monkeypatch, tmp_path=tmp_path)["kafka/config/server.properties"]
    kv = dict(line.split("=", 1) for line in props.splitlines())
    assert kv["broker.id"] == "3" and kv["listeners"] == "PLAINTEXT://10.0.0.13:9092"
    assert kv["default.replication.factor"] == "3" and kv["zookeeper.connect"] == kenv["KAFKA_ZOOKEEPER_CONNECT"]
    assert _render("zookeeper", {}, env, head=True, monkeypatch=monkeypatch, tmp_path=tmp_path) == {}


def test_etcd_consul_redis_mongodb(tmp_path, monkeypatch):
    p = FakeProvider()
    env = rf.get_runtime("etcd", {}).with_environment_variables({"runtime": {}}, p, "w4")
    env.update(CLOUDTIK_NODE_SEQ_ID="4", CLOUDTIK_NODE_IP="10.0.0.14", CLOUDTIK_CLUSTER="c1")
    etcd = yaml.safe_load(_render("etcd", {}, env, monkeypatch=monkeypatch, tmp_path=tmp_path)["etcd/etcd.yaml"])
    assert etcd["name"] == "etcd4" and etcd["initial-cluster"] == (
        "etcd2=http://10.0.0.12:2380,etcd3=http://10.0.0.13:2380,etcd4=http://10.0.0.14:2380")
    assert etcd["initial-cluster-token"] == "cloudtik-c1"
    # consul: servers on the quorum workers, head is a client
    cenv = rf.get_runtime("consul", {}).with_environment_variables({"runtime": {}}, p, "w2")
    cenv.update(CLOUDTIK_NODE_SEQ_ID="2", CLOUDTIK_NODE_IP="10.0.0.12", CLOUDTIK_HEAD_IP="10.0.0.1")
    srv = json.loads(_render("consul", {"server": True}, cenv, monkeypatch=monkeypatch,
                             tmp_path=tmp_path)["consul/consul.d/consul.json"])
    assert srv["server"] is True and srv["bootstrap_expect"] == 3 and "10.0.0.12" not in srv["retry_join"]
    cli = json.loads(_render("consul", {"server": True}, cenv, head=True, monkeypatch=monkeypatch,
                             tmp_path=tmp_path)["consul/consul.d/consul.json"])
    assert cli["server"] is False and "bootstrap_expect" not in cli
    # redis replication: workers follow the head; password on both sides
    renv = {"CLOUDTIK_NODE_IP": "10.0.0.12", "CLOUDTIK_HEAD_IP": "10.0.0.1"}
    conf = _render("redis", {"cluster_mode": "replication", "password": "pw"}, renv, monkeypatch=monkeypatch,
                   tmp_path=tmp_path)["redis/redis.conf"]
    assert "replicaof 10.0.0.1 6379" in conf and "masterauth pw" in conf
    head_conf = _render("redis", {"cluster_mode": "replication"}, renv, head=True, monkeypatch=monkeypatch,
                        tmp_path=tmp_path)["redis/redis.conf"]
    assert "replicaof" not in head_conf
    shard = _render("redis", {"cluster_mode": "sharding"}, renv, monkeypatch=monkeypatch,
                    tmp_path=tmp_path)["redis/redis.conf"]
    assert "cluster-enabled yes" in shard
    mongo = yaml.safe_load(_render("mongodb", {"cluster_mode": "replication"}, {"CLOUDTIK_CLUSTER": "c1"},
                                   monkeypatch=monkeypatch, tmp_path=tmp_path)["mongodb/mongod.conf"])
    assert mongo["replication"]["replSetName"] == "c1-rs" and mongo["net"]["bindIp"] == "0.0.0.0"


def test_databases_and_observability(tmp_path, monkeypatch):
    env = {"CLOUDTIK_NODE_SEQ_ID": "5", "CLOUDTIK_HEAD_IP": "10.0.0.1", "CLOUDTIK_CLUSTER": "c1"}
    my = _render("mysql", {"cluster_mode": "replication"}, env, monkeypatch=monkeypatch,
                 tmp_path=tmp_path)["mysql/conf.d/cloudtik.cnf"]
    assert "server-id = 5" in my and "gtid_mode = ON" in my and "read_only = ON" in my
    pg = _render("postgres", {"cluster_mode": "replication", "replication_user": "r"}, env, monkeypatch=monkeypatch,
                 tmp_path=tmp_path)
    assert "primary_conninfo = 'host=10.0.0.1 port=5432 user=r" in pg["postgres/conf.d/cloudtik.conf"]
    assert "host replication all" in pg["postgres/conf.d/pg_hba.cloudtik.conf"]
    p = FakeProvider()
    penv = rf.get_runtime("prometheus", {}).with_environment_variables({"runtime": {}}, p, "h")
    penv.update(CLOUDTIK_HEAD_IP="10.0.0.1")
    pf = _render("prometheus", {"scrape_scope": "federation", "federation_targets": ["10.9.0.1:9090"]}, penv,
                 head=True, monkeypatch=monkeypatch, tmp_path=tmp_path)
    prom = yaml.safe_load(pf["prometheus/prometheus.yml"])
    # this cluster from the live-node targets file (no consul), the others through /federate
    assert prom["scrape_configs"][0]["file_sd_configs"][0]["files"][0].endswith("conf/local-*targets.yaml")
    assert prom["scrape_configs"][-1]["metrics_path"] == "/federate"
    assert yaml.safe_load(pf["prometheus/conf/federation-targets.yaml"])[0]["targets"] == ["10.9.0.1:9090"]
    graf = yaml.safe_load(_render("grafana", {}, {"CLOUDTIK_HEAD_IP": "10.0.0.1"}, head=True, monkeypatch=monkeypatch,
                                  tmp_path=tmp_path)["grafana/conf/provisioning/datasources/cloudtik.yaml"])
    assert graf["datasources"][0]["url"] == "http://10.0.0.1:9090"
    ha = _render("haproxy", {"backend": {"servers": ["10.0.0.12:8080", "10.0.0.13:8080"]}}, {}, head=True,
                 monkeypatch=monkeypatch, tmp_path=tmp_path)["haproxy/haproxy.cfg"]
    assert "server s1 10.0.0.13:8080 check" in ha
    core = _render("coredns", {}, {}, monkeypatch=monkeypatch, tmp_path=tmp_path)["coredns/Corefile"]
    assert "forward . 127.0.0.1:8600" in core


def test_node_configure_writes_files_then_runs_steps(tmp_path, monkeypatch):
    monkeypatch.setenv("RUNTIME_PATH", str(tmp_path))
    monkeypatch.setenv("CLOUDTIK_NODE_IP", "10.0.0.12")
    rt = rf.get_runtime("redis", {"port": 6380})
    assert rt.node_configure(False)
    assert (tmp_path / "redis" / "redis.conf").read_text().startswith("bind 0.0.0.0\nport 6380")
    assert (tmp_path / "redis" / "data").is_dir()
