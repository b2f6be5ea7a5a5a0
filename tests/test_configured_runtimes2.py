"""Self-configuring runtimes, part 2 (runtime/configured_more.py; reference
runtime/<name>/scripts/configure.* + conf templates): rendered files per node for the query
engines, frameworks, stores, gateways, DNS, poolers and node utilities, with membership from
the provider and sizing from the node."""
import json
import os

import yaml

from test_configured_runtimes import FakeProvider, _render

from cloudtik_amd.core import runtime_factory as rf
from cloudtik_amd.runtime.catalog import SPEC_BY_NAME


def _kv(text):
    return dict(line.split("=", 1) for line in text.splitlines() if "=" in line)


def test_every_catalogue_runtime_is_configurable():
    for name in SPEC_BY_NAME:
        cls = rf.get_runtime_cls(name)
        assert hasattr(cls, "files") or name in ("ai", "hadoop", "hdfs", "yarn", "spark"), name


def test_metastore_presto_trino(tmp_path, monkeypatch):
    env = {"CLOUDTIK_HEAD_IP": "10.0.0.1", "CLOUDTIK_NODE_IP": "10.0.0.1", "CLOUDTIK_CLUSTER": "c1",
           "CLOUDTIK_NODE_SEQ_ID": "1"}
    ms = _render("metastore", {"database": {"engine": "postgres", "password": "pw"}}, env, head=True,
                 monkeypatch=monkeypatch, tmp_path=tmp_path)["metastore/conf/metastore-site.xml"]
    assert "jdbc:postgresql://10.0.0.1:5432/hive_metastore" in ms and "<value>pw</value>" in ms
    wenv = dict(env, CLOUDTIK_NODE_IP="10.0.0.12", CLOUDTIK_NODE_SEQ_ID="2")
    for name in ("presto", "trino"):
        head = _render(name, {"node_memory_mb": 10000}, env, head=True, monkeypatch=monkeypatch, tmp_path=tmp_path)
        worker = _render(name, {"node_memory_mb": 10000, "catalogs": {"tpch": {"connector.name": "tpch"}}}, wenv,
                         monkeypatch=monkeypatch, tmp_path=tmp_path)
        hc, wc = _kv(head[f"{name}/etc/config.properties"]), _kv(worker[f"{name}/etc/config.properties"])
        assert hc["coordinator"] == "true" and wc["coordinator"] == "false"
        assert wc["discovery.uri"] == "http://10.0.0.1:8081" and hc["query.max-memory-per-node"] == "4000MB"
        assert "-Xmx8000M" in head[f"{name}/etc/jvm.config"]
        assert _kv(worker[f"{name}/etc/catalog/hive.properties"])["hive.metastore.uri"] == "thrift://10.0.0.1:9083"
        assert _kv(worker[f"{name}/etc/node.properties"])["node.id"] == "c1-2"
        assert f"{name}/etc/catalog/tpch.properties" in worker
    assert _kv(_render("presto", {}, env, head=True, monkeypatch=monkeypatch, tmp_path=tmp_path)[
        "presto/etc/catalog/hive.properties"])["connector.name"] == "hive-hadoop2"


def test_flink_ray_minio(tmp_path, monkeypatch):
    env = {"CLOUDTIK_HEAD_IP": "10.0.0.1", "CLOUDTIK_NODE_IP": "10.0.0.12"}
    fl = yaml.safe_load(_render("flink", {"node_memory_mb": 20000, "node_cpus": 64}, env,
                                monkeypatch=monkeypatch, tmp_path=tmp_path)["flink/conf/flink-conf.yaml"])
    assert fl["jobmanager.rpc.address"] == "10.0.0.1" and fl["taskmanager.numberOfTaskSlots"] == 32
    assert fl["taskmanager.memory.process.size"] == "16000m"
    ray = rf.get_runtime("ray", {"node_gpus": 8, "node_cpus": 128, "node_memory_mb": 1000})
    head, worker = ray.start_steps(True)[0], ray.start_steps(False)[0]
    assert head.startswith("ray start --head") and "--num-gpus=8" in head and "--num-cpus=128" in head
    assert "--address=$CLOUDTIK_HEAD_IP:6379" in worker and f"--object-store-memory={300 << 20}" in worker
    p = FakeProvider()
    menv = rf.get_runtime("minio", {}).with_environment_variables(
        {"runtime": {"minio": {"data_disks": 2}}}, p, "w3")
    assert menv["MINIO_VOLUMES"].split() == [
        f"http://10.0.0.{ip}:9000/mnt/cloudtik/data_disk_{d}/minio" for ip in (12, 13, 14) for d in (1, 2)]
    menv.update(CLOUDTIK_NODE_IP="10.0.0.13")
    files = _render("minio", {"access_key": "ak"}, menv, monkeypatch=monkeypatch, tmp_path=tmp_path)
    assert 'MINIO_ROOT_USER="ak"' in files["minio/minio.env"]


def test_elasticsearch_nginx_gateways(tmp_path, monkeypatch):
    p = FakeProvider()
    env = rf.get_runtime("elasticsearch", {}).with_environment_variables({"runtime": {}}, p, "w2")
    env.update(CLOUDTIK_HEAD_IP="10.0.0.1", CLOUDTIK_NODE_IP="10.0.0.12", CLOUDTIK_NODE_SEQ_ID="2",
               CLOUDTIK_CLUSTER="c1")
    es = yaml.safe_load(_render("elasticsearch", {"node_memory_mb": 8192}, env, monkeypatch=monkeypatch,
                                tmp_path=tmp_path)["elasticsearch/config/elasticsearch.yml"])
    assert es["node.name"] == "c1-node-2" and es["discovery.seed_hosts"][0] == "10.0.0.1"
    assert es["cluster.initial_master_nodes"] == ["c1-head", "c1-node-2", "c1-node-3"]
    ng = _render("nginx", {"backend": {"services": {
        "api": {"servers": ["10.0.0.12:8080", "10.0.0.13:8080"], "route_path": "/api", "service_path": "/v1"},
        "web": {"servers": ["10.0.0.14:80"], "default_service": True}}}}, {}, head=True,
        monkeypatch=monkeypatch, tmp_path=tmp_path)["nginx/nginx.conf"]
    assert "upstream api {\n    server 10.0.0.12:8080;" in ng and "location /api/ {\n      proxy_pass http://api/v1/;" in ng
    assert "location / {\n      proxy_pass http://web;" in ng
    kong = _render("kong", {}, {"CLOUDTIK_HEAD_IP": "10.0.0.1", "CLOUDTIK_NODE_IP": "10.0.0.1"}, head=True,
                   monkeypatch=monkeypatch, tmp_path=tmp_path)["kong/kong.conf"]
    assert "pg_host = 10.0.0.1" in kong and "pg_port = 5432" in kong
    aenv = rf.get_runtime("apisix", {}).with_environment_variables({"runtime": {}}, p, "w2")
    ap = yaml.safe_load(_render("apisix", {}, dict(aenv, CLOUDTIK_CLUSTER="c1"), monkeypatch=monkeypatch,
                                tmp_path=tmp_path)["apisix/conf/config.yaml"])
    assert ap["deployment"]["etcd"]["host"][0] == "http://10.0.0.12:2379"


def test_dns_poolers_and_node_utilities(tmp_path, monkeypatch):
    env = {"CLOUDTIK_HEAD_IP": "10.0.0.1", "CLOUDTIK_NODE_IP": "10.0.0.12"}
    dm = _render("dnsmasq", {}, env, monkeypatch=monkeypatch, tmp_path=tmp_path)["dnsmasq/cloudtik.conf"]
    assert "server=/cloudtik/127.0.0.1#8600" in dm
    bind = _render("bind", {}, env, monkeypatch=monkeypatch, tmp_path=tmp_path)["bind/named.conf.cloudtik"]
    assert 'zone "consul"' in bind and "port 8600" in bind
    pgb = _render("pgbouncer", {"pool_mode": "session"}, env, monkeypatch=monkeypatch,
                  tmp_path=tmp_path)["pgbouncer/pgbouncer.ini"]
    assert "* = host=10.0.0.1 port=5432" in pgb and "pool_mode = session" in pgb
    p = FakeProvider()
    penv = rf.get_runtime("pgpool", {}).with_environment_variables({"runtime": {}}, p, "h")
    pp = _render("pgpool", {}, dict(penv, **env), head=True, monkeypatch=monkeypatch,
                 tmp_path=tmp_path)["pgpool/pgpool.conf"]
    assert "backend_hostname0 = '10.0.0.1'" in pp and "backend_flag0 = 'ALWAYS_PRIMARY'" in pp
    assert "backend_hostname4 = '10.0.0.19'" in pp
    mnt = _render("mount", {"storage": {"type": "s3", "bucket": "b1"}}, env, monkeypatch=monkeypatch,
                  tmp_path=tmp_path)["mount/cloudtik-mount-storage.sh"]
    assert "s3fs b1 /cloudtik/fs" in mnt
    assert "hadoop-fuse-dfs dfs://10.0.0.1:9000" in _render("mount", {}, env, monkeypatch=monkeypatch,
                                                           tmp_path=tmp_path)["mount/cloudtik-mount-storage.sh"]
    sshd = _render("sshserver", {"port": 2222}, env, monkeypatch=monkeypatch, tmp_path=tmp_path)["sshserver/sshd_config"]
    assert sshd.startswith("Port 2222") and "PasswordAuthentication no" in sshd
    xi = _render("xinetd", {"services": {"lbcheck": {"port": 9200, "server": "/usr/local/bin/check"}}}, env,
                 monkeypatch=monkeypatch, tmp_path=tmp_path)["xinetd/lbcheck"]
    assert "port = 9200" in xi and "server = /usr/local/bin/check" in xi
    nx = _render("nodex", {}, env, monkeypatch=monkeypatch, tmp_path=tmp_path)
    assert "--collector.textfile.directory=" in nx["nodex/nodex.args"]
    assert os.path.isdir(tmp_path / "nodex" / "textfile")
    assert json.dumps(rf.get_runtime("nodex", {}).start_steps(True)).count("nodex.args") == 1
