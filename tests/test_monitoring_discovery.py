"""Prometheus scrape scopes / live targets and Grafana data-source discovery
(runtime/monitoring_discovery.py; reference runtime/prometheus/utils.py:142-186,
prometheus/discovery.py:62-106, conf/scrape-config-*.yaml, grafana/discovery.py:63-153,
grafana/admin_api.py:8-29).  Discovery sources and the Grafana admin API are fakes; the live
node table is the in-tree state server."""
import json
import os
import socket
import time

import pytest
import yaml

from cloudtik_amd.core import runtime_factory as rf
from cloudtik_amd.runtime import monitoring_discovery as MD


def _env(monkeypatch, tmp_path, runtimes="prometheus", **kw):
    env = {"RUNTIME_PATH": str(tmp_path), "CLOUDTIK_NODE_IP": "10.0.0.1", "CLOUDTIK_HEAD_IP": "10.0.0.1",
           "CLOUDTIK_CLUSTER": "c1", "CLOUDTIK_WORKSPACE": "ws", "CLOUDTIK_RUNTIMES": runtimes}
    env.update(kw)
    for k, v in env.items():
        monkeypatch.setenv(k, v)


def _prom(cfg, monkeypatch, tmp_path, head=True, runtimes="prometheus"):
    _env(monkeypatch, tmp_path, runtimes)
    rt = rf.get_runtime("prometheus", cfg)
    files = {os.path.relpath(p, tmp_path): t for p, t in rt.render(head).items()}
    return rt, files, yaml.safe_load(files["prometheus/prometheus.yml"])


def test_resolve_scope_and_discovery():
    assert MD.resolve_discovery({}, False) == ("local", "file")
    assert MD.resolve_discovery({}, True) == ("local", "consul")
    assert MD.resolve_discovery({"service_discovery": "file"}, True) == ("local", "file")
    assert MD.resolve_discovery({"scrape_scope": "workspace"}, True) == ("workspace", "consul")
    assert MD.resolve_discovery({"scrape_scope": "federation", "federation_targets": ["a:9090"]}, True) == \
        ("federation", "file")
    assert MD.resolve_discovery({"scrape_scope": "federation"}, True) == ("federation", "consul")
    for bad, consul in [({"scrape_scope": "workspace"}, False), ({"scrape_scope": "federation"}, False),
                        ({"scrape_scope": "cluster"}, True), ({"service_discovery": "consul"}, False)]:
        with pytest.raises(ValueError):
            MD.resolve_discovery(bad, consul)


def test_scrape_scope_is_honoured(tmp_path, monkeypatch):
    """Each scope renders its own jobs: scrape_scope is no longer a silently ignored key."""
    rt, files, local_file = _prom({}, monkeypatch, tmp_path / "a")
    assert [j["job_name"] for j in local_file["scrape_configs"]] == ["local"]
    job = local_file["scrape_configs"][0]
    assert job["file_sd_configs"][0]["files"][0].endswith("prometheus/conf/local-*targets.yaml")
    assert {"target_label": "cluster", "replacement": "c1"} in job["relabel_configs"]
    pull = json.loads(files["prometheus/local-targets.json"])
    assert pull["targets_file"].endswith("prometheus/conf/local-targets.yaml")
    assert pull["state_address"] == "10.0.0.1:6789"
    assert any("DiscoverLocalTargets" in s for s in rt.start_steps(True))

    rt, files, local_consul = _prom({"scrape_services": {"runtimes": ["spark", "ai"]}}, monkeypatch, tmp_path / "b",
                                    runtimes="consul,prometheus")
    job = local_consul["scrape_configs"][0]
    assert job["consul_sd_configs"][0]["tags"] == ["cloudtik-c-c1", "cloudtik-f-metrics"]
    assert job["consul_sd_configs"][0]["server"] == "10.0.0.1:8500"
    assert {"source_labels": ["__meta_consul_service_metadata_cloudtik_runtime"], "regex": "(spark|ai)",
            "action": "keep"} in job["relabel_configs"]
    assert "prometheus/local-targets.json" not in files
    assert not any("DiscoverLocalTargets" in s for s in rt.start_steps(True))

    _, _, ws = _prom({"scrape_scope": "workspace"}, monkeypatch, tmp_path / "c", runtimes="consul,prometheus")
    assert [j["job_name"] for j in ws["scrape_configs"]] == ["workspace"]
    assert ws["scrape_configs"][0]["consul_sd_configs"][0]["tags"] == ["cloudtik-f-metrics"]

    _, _, fed = _prom({"scrape_scope": "federation"}, monkeypatch, tmp_path / "d", runtimes="consul,prometheus")
    names = [j["job_name"] for j in fed["scrape_configs"]]
    assert names == ["local", "federation"]
    f = fed["scrape_configs"][1]
    assert f["metrics_path"] == "/federate" and f["consul_sd_configs"][0]["services"] == ["prometheus"]
    assert f["relabel_configs"][0] == {"source_labels": ["__meta_consul_service_metadata_cloudtik_cluster"],
                                       "regex": "c1", "action": "drop"}          # not itself

    with pytest.raises(ValueError):
        _prom({"scrape_scope": "workspace"}, monkeypatch, tmp_path / "e")          # no consul in the cluster


def test_local_targets_follow_live_nodes(tmp_path):
    nodes = [{"node_ip": "10.0.0.1", "node_type": "head"}, {"node_ip": "10.0.0.2", "node_type": "worker"},
             {"node_ip": "10.0.0.3", "node_type": "gpu-worker"}]
    out = tmp_path / "conf" / "local-targets.yaml"
    job = MD.DiscoverLocalTargets(services="node-exporter:9100,train:9500:gpu-worker", nodes=lambda: list(nodes),
                                  targets_file=str(out))
    job.pull()
    t = yaml.safe_load(out.read_text())
    assert t == [{"labels": {"service": "node-exporter"},
                  "targets": ["10.0.0.1:9100", "10.0.0.2:9100", "10.0.0.3:9100"]},
                 {"labels": {"service": "train"}, "targets": ["10.0.0.3:9500"]}]
    m0 = out.stat().st_mtime_ns
    time.sleep(0.01)
    job.pull()
    assert out.stat().st_mtime_ns == m0                                  # unchanged: not rewritten
    nodes.pop(1)
    nodes.append({"node_ip": "10.0.0.4", "node_type": "gpu-worker"})
    job.pull()
    t = yaml.safe_load(out.read_text())
    assert t[0]["targets"] == ["10.0.0.1:9100", "10.0.0.3:9100", "10.0.0.4:9100"]
    assert t[1]["targets"] == ["10.0.0.3:9500", "10.0.0.4:9500"]


def test_local_targets_from_the_state_server_node_table(tmp_path):
    """End to end against the native state server: nodes that heartbeat are targets, a node
    whose heartbeat is older than the timeout drops out."""
    from cloudtik_amd.core.state.state_client import ControlState, StateNodeManager, StateServer
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    srv = StateServer(port=port, data_dir=str(tmp_path / "st"), password="pw").start()
    try:
        mgr = StateNodeManager(ControlState(f"127.0.0.1:{port}", "pw").tables)
        mgr.register_node("n1", {"node_ip": "10.0.0.1", "node_type": "head"})
        mgr.register_node("n2", {"node_ip": "10.0.0.2", "node_type": "worker"})
        cfgf = tmp_path / "local-targets.json"
        cfgf.write_text(json.dumps({"pull_services": {"node-exporter": {"port": 9100}},
                                    "targets_file": str(tmp_path / "conf" / "local-targets.yaml"),
                                    "state_address": f"127.0.0.1:{port}", "state_password": "pw",
                                    "node_timeout_s": 0.5}))
        job = MD.DiscoverLocalTargets(config_file=str(cfgf))
        job.pull()
        t = yaml.safe_load((tmp_path / "conf" / "local-targets.yaml").read_text())
        assert t[0]["targets"] == ["10.0.0.1:9100", "10.0.0.2:9100"]
        time.sleep(0.7)
        mgr.heartbeat("n1")                                              # n2 stops heart-beating
        job.pull()
        t = yaml.safe_load((tmp_path / "conf" / "local-targets.yaml").read_text())
        assert t[0]["targets"] == ["10.0.0.1:9100"]
    finally:
        srv.stop()


class FakeGrafana:
    def __init__(self):
        self.ds = {"manual": {"name": "manual", "type": "loki", "url": "http://x"}}   # not ours
        self.calls, self.auth = [], set()

    def __call__(self, method, url, body=None, headers=None):
        self.calls.append((method, url))
        self.auth.add((headers or {}).get("Authorization"))
        path = url.split("://", 1)[1].split("/", 1)[1]
        if method == "GET" and path == "api/datasources":
            return list(self.ds.values())
        if method == "POST" and path == "api/datasources":
            self.ds[body["name"]] = dict(body)
            return {"datasource": body}
        if method == "DELETE" and path.startswith("api/datasources/name/"):
            del self.ds[path.rsplit("/", 1)[1]]
            return {"message": "deleted"}
        raise AssertionError((method, url))


def _svc(name, host, port, cluster):
    return {"name": name, "host": host, "port": port, "meta": {"cloudtik-cluster": cluster,
                                                                "cloudtik-runtime": "prometheus"}}


def test_grafana_data_sources_follow_prometheus_servers():
    rows = [_svc("prometheus", "10.0.0.1", 9090, "c1"), _svc("prometheus", "10.1.0.1", 9090, "c2")]
    seen_sel = []

    def query():
        return list(rows)

    g = FakeGrafana()
    job = MD.DiscoverDataSources(admin_endpoint="http://127.0.0.1:3000", query=query, http=g,
                                 service_selector={"clusters": ["c1", "c2"]})
    assert job.selector["runtimes"] == ["prometheus"] and job.selector["clusters"] == ["c1", "c2"]
    job.pull()
    assert set(g.ds) == {"manual", "prometheus-c1", "prometheus-c2"}
    assert g.ds["prometheus-c2"]["url"] == "http://10.1.0.1:9090" and g.ds["prometheus-c2"]["type"] == "prometheus"
    assert g.auth == {"Basic Y2xvdWR0aWs6Y2xvdWR0aWs="}                      # cloudtik:cloudtik
    rows.pop()                                                            # c2's server goes away
    job.pull()
    assert set(g.ds) == {"manual", "prometheus-c1"}                       # ours deleted, 'manual' kept
    n = len(g.calls)
    job.pull()
    assert [c[0] for c in g.calls[n:]] == ["GET"]                         # steady: only the listing
    rows[0] = _svc("prometheus", "10.0.0.9", 9090, "c1")                  # c1's server moved
    job.pull()
    assert g.ds["prometheus-c1"]["url"] == "http://10.0.0.9:9090" and "manual" in g.ds
    g.ds["manual"]["url"] = "http://y"
    rows.append(_svc("manual", "10.2.0.1", 9090, None))                    # same name as a data source not ours
    job.pull()
    assert g.ds["manual"]["url"] == "http://y"                            # never replaced


def test_grafana_scopes(tmp_path, monkeypatch):
    _env(monkeypatch, tmp_path, "consul,prometheus,grafana")
    local = rf.get_runtime("grafana", {})
    files = {os.path.relpath(p, tmp_path): t for p, t in local.render(True).items()}
    prov = yaml.safe_load(files["grafana/conf/provisioning/datasources/cloudtik.yaml"])
    assert prov["datasources"][0]["url"] == "http://10.0.0.1:9090" and "grafana/data-sources.json" not in files
    assert not any("DiscoverDataSources" in s for s in local.start_steps(True))
    ws = rf.get_runtime("grafana", {"data_sources_scope": "workspace",
                                    "data_sources_services": {"clusters": ["c2"]}})
    files = {os.path.relpath(p, tmp_path): t for p, t in ws.render(True).items()}
    d = json.loads(files["grafana/data-sources.json"])
    assert d["service_selector"] == {"clusters": ["c2"]} and d["admin_endpoint"] == "http://127.0.0.1:3000"
    assert any("service-daemon start grafana-data-sources" in s and "DiscoverDataSources" in s
               for s in ws.start_steps(True))
    none = rf.get_runtime("grafana", {"data_sources_scope": "none"})
    files = {os.path.relpath(p, tmp_path): t for p, t in none.render(True).items()}
    assert yaml.safe_load(files["grafana/conf/provisioning/datasources/cloudtik.yaml"])["datasources"] == []
    monkeypatch.setenv("CLOUDTIK_RUNTIMES", "grafana")
    with pytest.raises(ValueError):
        rf.get_runtime("grafana", {"data_sources_scope": "workspace"}).render(True)
