"""Process reaper, node naming and runtime service discovery (CPU)."""
import os
import signal
import subprocess
import sys
import time

from cloudtik_amd.core import naming
from cloudtik_amd.core import service_discovery as sd
from cloudtik_amd.runtime.common import discovery as disc


def _alive(pid):
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    # a zombie still answers kill(0): look at its state
    with open(f"/proc/{pid}/stat") as f:
        return f.read().split(")")[1].split()[0] != "Z"


def test_reaper_kills_children_when_launcher_dies(tmp_path):
    pidfile = tmp_path / "child.pid"
    launcher = tmp_path / "launcher.py"
    launcher.write_text(
        "import subprocess, sys, time\n"
        "from cloudtik_amd.core.node.reaper import Reaper\n"
        "r = Reaper()\n"
        "c = subprocess.Popen([sys.executable, '-c', 'import time; time.sleep(60)'], start_new_session=True)\n"
        "r.watch(c.pid)\n"
        f"open({str(pidfile)!r}, 'w').write(str(c.pid))\n"
        "time.sleep(60)\n")
    env = dict(os.environ, PYTHONPATH=os.getcwd())
    lp = subprocess.Popen([sys.executable, str(launcher)], env=env)
    try:
        for _ in range(200):
            if pidfile.exists() and pidfile.read_text():
                break
            time.sleep(0.05)
        child = int(pidfile.read_text())
        assert _alive(child)
        lp.send_signal(signal.SIGKILL)          # launcher dies without cleanup
        lp.wait()
        for _ in range(100):
            if not _alive(child):
                break
            time.sleep(0.05)
        assert not _alive(child)
    finally:
        if lp.poll() is None:
            lp.kill()


def test_reaper_release_leaves_children_alone():
    from cloudtik_amd.core.node.reaper import Reaper
    c = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(30)"], start_new_session=True)
    try:
        r = Reaper()
        r.watch(c.pid)
        r.release()
        time.sleep(0.2)
        assert c.poll() is None
    finally:
        c.kill()
        c.wait()


def test_naming():
    cfg = {"cluster_name": "train", "workspace_name": "ws", "runtime": {"types": ["ai"]}}
    assert naming.get_cluster_node_name("train", 3) == "train-3"
    assert naming.get_cluster_node_sqdn("train-3", "train") == "train-3.train.node"
    assert naming.get_cluster_head_host(cfg, "10.0.0.1") == "10.0.0.1"      # no DNS runtime
    cfg["runtime"]["types"].append("consul")
    assert naming.get_cluster_head_host(cfg, "10.0.0.1") == "train-1.train.ws.cloudtik"
    env = naming.with_node_host_environment_variables(cfg, 2, "10.0.0.2", {})
    assert env["CLOUDTIK_NODE_HOST"] == "train-2.train.ws.cloudtik"
    assert naming.get_address_type_of_hostname("::1") == "ipv6"
    assert naming.get_address_type_of_hostname("h.x") == "hostname"


def _publish(cluster, runtime, svc_name, port, kind, host, hosts=None, features=()):
    svc = sd.define_runtime_service(runtime, svc_name, port, node_kind=kind, features=list(features))
    return {sd.service_global_key(cluster, f"{cluster}-{svc_name}"): sd.encode_service_address(svc, host, hosts)}


def test_discovery_from_workspace_and_on_head():
    gv = {}
    gv.update(_publish("storage", "hdfs", "hdfs-rpc", 8020, "head", "10.1.0.1"))
    gv.update(_publish("zk", "zookeeper", "zookeeper", 2181, "worker", "10.2.0.1", ["10.2.0.2", "10.2.0.3"]))
    gv.update(_publish("db", "mysql", "mysql", 3306, "head", "10.3.0.1"))
    gv.update(_publish("meta", "metastore", "metastore", 9083, "head", "10.4.0.1"))
    cfg = {"cluster_name": "analytics", "runtime": {"types": ["spark"]}}
    assert disc.discover_hdfs_from_workspace(cfg, global_variables=gv) == "hdfs://10.1.0.1:8020"
    assert disc.discover_zookeeper_from_workspace(cfg, global_variables=gv) == "10.2.0.2:2181,10.2.0.3:2181"
    assert disc.discover_metastore_from_workspace(cfg, global_variables=gv) == "thrift://10.4.0.1:9083"
    assert disc.discover_database_from_workspace(cfg, global_variables=gv) == \
        {"engine": "mysql", "address": "10.3.0.1", "port": 3306}
    assert disc.discover_minio_from_workspace(cfg, global_variables=gv) is None
    # selector restricts the candidate clusters
    cfg["runtime"]["spark"] = {"hdfs_service_selector": {"clusters": ["other"]}}
    assert disc.discover_hdfs_from_workspace(cfg, consumer="spark", global_variables=gv) is None
    # a cluster never discovers itself through the workspace; it uses *_on_head
    own = {"cluster_name": "storage", "runtime": {"types": ["hdfs", "zookeeper"]}}
    assert disc.discover_hdfs_from_workspace(own, global_variables=gv) is None
    assert disc.discover_hdfs_on_head(own, "10.1.0.1") == "hdfs://10.1.0.1:8020"
    assert disc.discover_zookeeper_on_head(own, "10.1.0.1", ["10.1.0.5"]) == "10.1.0.5:2181"
    assert disc.discover_service("hdfs", own, head_ip="10.1.0.1") == "hdfs://10.1.0.1:8020"
    assert disc.discover_service("metastore", own, head_ip="10.1.0.1", global_variables=gv) == "thrift://10.4.0.1:9083"


def test_discovery_switches_consul_ha_name_and_database_env():
    from cloudtik_amd.runtime.common import discovery as D

    class FakeConsul:
        def select_services(self, sel):
            assert sel["runtimes"] == ["zookeeper"] and "exclude_clusters" not in sel
            return [{"name": "c2-zookeeper", "host": "10.1.0.3", "port": 2181},
                    {"name": "c2-zookeeper", "host": "10.1.0.2", "port": 2181}]

    cfg = {"cluster_name": "c1", "runtime": {"types": ["kafka"], "kafka": {}}}
    assert D.discover_from_consul("zookeeper", cfg, "kafka", client=FakeConsul()) == "10.1.0.2:2181,10.1.0.3:2181"
    off = {"cluster_name": "c1", "runtime": {"types": ["kafka"], "kafka": {"zookeeper_service_discovery": False}}}
    assert D.discover_service("zookeeper", off, "10.0.0.1", consumer="kafka", global_variables={}) is None
    ha = {"cluster_name": "c1", "runtime": {"types": ["hdfs"], "hdfs": {"cluster_mode": "ha_cluster"}}}
    assert D.discover_hdfs_name(ha) == "hdfs://c1"
    single = {"cluster_name": "c1", "runtime": {"types": ["hdfs"]}}
    assert D.discover_hdfs_name(single, "10.0.0.1") == "hdfs://10.0.0.1:8020"
    on_head = {"cluster_name": "c1", "runtime": {"types": ["postgres", "metastore"], "metastore": {}}}
    env = D.with_database_environment_variables(on_head, "metastore", "10.0.0.1", global_variables={})
    assert env["CLOUDTIK_DATABASE_ENGINE"] == "postgres" and env["CLOUDTIK_DATABASE_HOST"] == "10.0.0.1"
    assert env["CLOUDTIK_DATABASE_PORT"] == "5432" and env["CLOUDTIK_DATABASE_USERNAME"] == "postgres"
    explicit = {"runtime": {"types": ["metastore"], "metastore": {"database": {
        "engine": "mysql", "address": "db.example", "username": "hive", "password": "pw"}}}}
    env = D.with_database_environment_variables(explicit, "metastore")
    assert env["CLOUDTIK_DATABASE_HOST"] == "db.example" and env["CLOUDTIK_DATABASE_PORT"] == "3306"
    assert D.with_database_environment_variables({"runtime": {"types": []}}, "metastore", global_variables={}) == {}


def test_workspace_global_variables_through_the_provider(tmp_path, monkeypatch):
    """The registry is head-node tags behind the node provider (reference
    providers/_private/local/workspace_provider.py:54-80): a service published by cluster c1's
    head is discovered from ANOTHER CLI home (fresh workspace-provider instance, own state dir)
    through the provider, a long value survives the tag-size split, and the entries vanish
    with the head."""
    from cloudtik_amd.runtime.common import discovery as D
    from cloudtik_amd.providers.local import workspace_provider as lwp
    from cloudtik_amd.core import tags as T
    from cloudtik_amd.core.provider_factory import get_workspace_provider, get_node_provider
    from cloudtik_amd.providers.mock.node_provider import MockProvider
    MockProvider.reset()
    monkeypatch.setattr(lwp, "STATE_DIR", str(tmp_path / "home1"))
    pc = {"type": "mock"}
    heads = {}
    for c, ws in (("c1", "w"), ("c2", "w"), ("c3", "other")):
        p = get_node_provider(pc, c, use_cache=False)
        heads[c] = next(iter(p.create_node({}, {T.CLOUDTIK_TAG_CLUSTER_NAME: c, T.CLOUDTIK_TAG_NODE_KIND: "head",
                                                T.CLOUDTIK_TAG_WORKSPACE_NAME: ws}, 1)))
    long_value = '{"hosts": [' + ",".join(f'"10.0.{i // 250}.{i % 250}"' for i in range(60)) + "]}"
    cfg1 = {"provider": pc, "workspace_name": "w", "cluster_name": "c1"}
    get_workspace_provider(pc, "w").publish_global_variables(cfg1, {"service.c1.x": "{}", "service.c1.big": long_value})
    get_workspace_provider(pc, "w").publish_global_variables(
        {"provider": pc, "workspace_name": "w", "cluster_name": "c2"}, {"service.c2.y": "{}"})
    get_workspace_provider(pc, "other").publish_global_variables(
        {"provider": pc, "workspace_name": "other", "cluster_name": "c3"}, {"service.c3.z": "{}"})
    tags = get_node_provider(pc, "c1", use_cache=False).node_tags(heads["c1"])
    assert all(len(v) <= lwp.TAG_VALUE_MAX for k, v in tags.items() if k.startswith("x-"))
    # a second CLI home: nothing shared but the provider
    monkeypatch.setattr(lwp, "STATE_DIR", str(tmp_path / "home2"))
    cfg_other_host = {"provider": pc, "workspace_name": "w", "cluster_name": "c9"}
    gv = D._workspace_global_variables(cfg_other_host)
    assert gv["service.c1.x"] == "{}" and gv["service.c2.y"] == "{}" and gv["service.c1.big"] == long_value
    assert "service.c3.z" not in gv                            # another workspace
    assert sorted(get_workspace_provider(pc, "w").list_clusters(cfg_other_host)) == ["c1", "c2"]
    get_node_provider(pc, "c1", use_cache=False).terminate_node(heads["c1"])
    gv = D._workspace_global_variables(cfg_other_host)
    assert "service.c1.x" not in gv and "service.c2.y" in gv
    MockProvider.reset()


def test_local_provider_workspace_heads_span_cluster_state_files(tmp_path, monkeypatch):
    """Local clusters keep one state file each and share this host as head: the workspace
    listing scans every file (the same IP heads several clusters)."""
    from cloudtik_amd.core import tags as T
    from cloudtik_amd.providers.local import node_provider as lnp, workspace_provider as lwp
    monkeypatch.setattr(lnp, "STATE_DIR", str(tmp_path))
    monkeypatch.setattr(lwp, "STATE_DIR", str(tmp_path))
    pc = {"type": "local", "nodes": ["10.1.0.1"]}
    for c in ("a", "b"):
        p = lnp.LocalNodeProvider(pc, c)
        (h,) = p.create_node({}, {T.CLOUDTIK_TAG_CLUSTER_NAME: c, T.CLOUDTIK_TAG_NODE_KIND: "head",
                                  T.CLOUDTIK_TAG_WORKSPACE_NAME: "w"}, 1)
        lwp.LocalWorkspaceProvider(pc, "w").publish_global_variables(
            {"provider": pc, "cluster_name": c}, {f"service.{c}.s": c})
    heads = lnp.LocalNodeProvider(pc, "zz").workspace_head_nodes("w")
    assert sorted(heads) == ["a/10.1.0.1", "b/10.1.0.1"]
    gv = lwp.LocalWorkspaceProvider(pc, "w").subscribe_global_variables({"provider": pc, "cluster_name": "zz"})
    assert gv == {"service.a.s": "a", "service.b.s": "b"}


def test_cloud_listing_drops_cluster_filter_only_in_workspace_scope():
    """EC2 filters: the cluster tag in normal listings, the workspace + head tags inside
    workspace_scope (how a cloud provider finds every head of a workspace)."""
    from cloudtik_amd.core import tags as T
    from cloudtik_amd.providers.cloud import node_provider as NP
    p = NP.AWSNodeProvider({"region": "nowhere", "_client_factory": lambda svc: None}, "c1")
    names = {f["Name"] for f in p._filters({})}
    assert f"tag:{T.CLOUDTIK_TAG_CLUSTER_NAME}" in names
    with p.workspace_scope():
        f = p._filters({T.CLOUDTIK_TAG_WORKSPACE_NAME: "w"})
    assert {x["Name"] for x in f} == {"instance-state-name", f"tag:{T.CLOUDTIK_TAG_WORKSPACE_NAME}"}
    assert f"tag:{T.CLOUDTIK_TAG_CLUSTER_NAME}" in {x["Name"] for x in p._filters({})}


def test_service_selectors_tags_labels_and_exclusions():
    """Selector semantics of the workspace registry (reference
    tests/unit/runtime/test_service_discovery.py scenarios, over this registry's records)."""
    from cloudtik_amd.core import service_discovery as sd
    gv = {}
    for cluster, rt, name, host in (("cluster-1", "runtime-1", "runtime-1", "127.0.0.1"),
                                    ("cluster-1", "runtime-2", "runtime-2", "127.0.0.2"),
                                    ("cluster-2", "runtime-1", "service-1", "127.0.0.3"),
                                    ("cluster-2", "runtime-3", "service-1", "127.0.0.4")):
        rec = {"name": name, "service_type": rt, "cluster": cluster, "port": 80}
        gv[sd.service_global_key(cluster, f"{rt}-{name}")] = sd.encode_service_address(rec, host)

    def hosts(sel):
        return sorted(s["host"] for s in sd.discover_services(gv, sel))

    assert hosts({"clusters": ["cluster-1"], "runtimes": ["runtime-1"]}) == ["127.0.0.1"]
    assert hosts({"clusters": ["cluster-2"], "runtimes": ["runtime-1"], "services": ["service-1"]}) == ["127.0.0.3"]
    assert hosts({"clusters": ["cluster-1"]}) == ["127.0.0.1", "127.0.0.2"]
    assert hosts({"tags": ["cloudtik-c-cluster-2"]}) == ["127.0.0.3", "127.0.0.4"]
    assert hosts({"labels": {"cloudtik-runtime": "runtime-1"}}) == ["127.0.0.1", "127.0.0.3"]
    assert hosts({"exclude_labels": {"cloudtik-runtime": "runtime-1"}}) == ["127.0.0.2", "127.0.0.4"]
    assert hosts({"exclude_runtimes": ["runtime-1", "runtime-2"]}) == ["127.0.0.4"]
    assert hosts({"clusters": ["cluster-2"], "runtimes": ["runtime-3"], "services": ["service-1"],
                  "tags": ["cloudtik-c-cluster-2"], "labels": {"cloudtik-runtime": "runtime-3"},
                  "exclude_labels": {"cloudtik-runtime": "runtime-1"}}) == ["127.0.0.4"]
