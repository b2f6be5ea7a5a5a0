"""Monitoring wiring that follows the cluster as it changes: Prometheus scrape scopes and
targets, and Grafana data sources.

Reference behaviour (what, not how):

* Prometheus (runtime/prometheus/utils.py:142-186, conf/scrape-config-*.yaml,
  scripting.py:195-230, discovery.py:62-106) scrapes in one of three scopes:

  - ``local``: this cluster's metrics endpoints.  With Consul, a ``consul_sd`` job selecting
    the services tagged ``cloudtik-c-<cluster>`` + ``cloudtik-f-metrics``; without it, a
    ``file_sd`` job over ``local-*targets.yaml``, which the ``DiscoverLocalTargets`` pull job
    on the head rewrites from the live nodes of the cluster (node table of the state server,
    grouped by node type, one target group per pull service);
  - ``workspace``: every metrics service of the workspace through Consul (required);
  - ``federation``: this cluster (as ``local``) plus the ``/federate`` endpoint of the other
    clusters' Prometheus servers: a static ``federation_targets`` list (``file_sd``) or, from
    Consul, the ``prometheus`` services of other clusters (its own cluster dropped).

* Grafana (runtime/grafana/discovery.py:63-153, admin_api.py:8-29): a pull job queries the
  Prometheus services through service discovery and adds a data source per server through
  the HTTP admin API (``POST /api/datasources``), deleting the ones it created earlier whose
  server is gone (``DELETE /api/datasources/name/<name>``); data sources it did not create
  are never touched.

Both jobs take injected sources (node table / service query / HTTP transport), which is what
the tests use; in a cluster they run as service daemons (``cloudtik node service-daemon``).
"""
from __future__ import annotations

import base64
import json
import logging
import os
import time
from typing import Any, Callable, Dict, List, Optional, Tuple

from cloudtik_amd.core.load_balancer import json_hash
from cloudtik_amd.core.service_daemon import PullJob

logger = logging.getLogger(__name__)

SCOPES = ("local", "workspace", "federation")
METRICS_TAG = "cloudtik-f-metrics"
AUTO_CREATED = "cloudtik_auto_created"
# what the local file-based scrape pulls when nothing is configured: every node's exporter
# (node metrics, amdgpu sysfs / RAS) and the training metrics endpoint (utils/metrics)
DEFAULT_PULL_SERVICES = {"node-exporter": {"port": 9100}, "training": {"port": 9500}}


# =============================================================================== Prometheus
def resolve_discovery(cfg: Dict[str, Any], consul_available: bool) -> Tuple[str, str]:
    """(scrape_scope, service discovery 'file' | 'consul') of a Prometheus runtime config;
    raises on a scope the cluster cannot serve (the reference's configure-time checks)."""
    scope = cfg.get("scrape_scope") or "local"
    if scope not in SCOPES:
        raise ValueError(f"prometheus.scrape_scope must be one of {SCOPES}, not {scope!r}")
    sd = cfg.get("service_discovery") or ("consul" if consul_available else "file")
    if sd not in ("file", "consul"):
        raise ValueError(f"prometheus.service_discovery must be 'file' or 'consul', not {sd!r}")
    if scope == "workspace":
        if not consul_available:
            raise ValueError("prometheus.scrape_scope 'workspace' needs a service discovery runtime (consul)")
        sd = "consul"
    elif scope == "federation":
        if cfg.get("federation_targets"):
            sd = "file"
        elif not consul_available:
            raise ValueError("prometheus.scrape_scope 'federation' needs federation_targets or consul")
        else:
            sd = "consul"
    if sd == "consul" and not consul_available:
        raise ValueError("prometheus.service_discovery 'consul' needs the consul runtime")
    return scope, sd


def _consul_sd(consul: str, tags: List[str], services: Optional[List[str]] = None) -> Dict[str, Any]:
    sd: Dict[str, Any] = {"server": consul, "tags": tags, "refresh_interval": "30s"}
    if services:
        sd["services"] = services
    return sd


_CONSUL_LABELS = [{"source_labels": ["__meta_consul_dc"], "target_label": "workspace"},
                  {"source_labels": ["__meta_consul_service_metadata_cloudtik_cluster"], "target_label": "cluster"},
                  {"source_labels": ["__meta_consul_service"], "target_label": "service"}]


def _selector_relabels(sel: Dict[str, Any]) -> List[Dict[str, Any]]:
    """``scrape_services`` selector (consul scopes): keep only the matching services /
    runtimes / clusters (the reference's relabel 'keep' rules on the consul meta)."""
    out = []
    for key, label in (("services", "__meta_consul_service"),
                       ("runtimes", "__meta_consul_service_metadata_cloudtik_runtime"),
                       ("clusters", "__meta_consul_service_metadata_cloudtik_cluster")):
        vals = sel.get(key)
        if vals:
            out.append({"source_labels": [label], "regex": "(" + "|".join(map(str, vals)) + ")", "action": "keep"})
    for k, v in (sel.get("labels") or {}).items():
        out.append({"source_labels": [f"__meta_consul_service_metadata_{k.replace('-', '_')}"],
                    "regex": str(v), "action": "keep"})
    return out


def scrape_configs(scope: str, sd: str, conf_dir: str, cluster: str, workspace: str,
                   consul: str = "127.0.0.1:8500", selector: Optional[Dict[str, Any]] = None) -> List[Dict[str, Any]]:
    """The scrape jobs of a scope.  ``conf_dir`` holds the ``*targets.yaml`` files of the
    file-based jobs."""
    sel = selector or {}
    jobs = []
    if scope in ("local", "federation"):
        if sd == "consul":
            jobs.append({"job_name": "local", "scrape_interval": "10s",
                         "consul_sd_configs": [_consul_sd(consul, [f"cloudtik-c-{cluster}", METRICS_TAG])],
                         "relabel_configs": _CONSUL_LABELS + _selector_relabels(sel)})
        else:
            jobs.append({"job_name": "local", "scrape_interval": "10s",
                         "file_sd_configs": [{"files": [os.path.join(conf_dir, "local-*targets.yaml")],
                                              "refresh_interval": "5m"}],
                         "relabel_configs": [{"target_label": "workspace", "replacement": workspace},
                                             {"target_label": "cluster", "replacement": cluster}]})
    if scope == "workspace":
        jobs.append({"job_name": "workspace", "scrape_interval": "10s",
                     "consul_sd_configs": [_consul_sd(consul, [METRICS_TAG])],
                     "relabel_configs": _CONSUL_LABELS + _selector_relabels(sel)})
    if scope == "federation":
        fed = {"job_name": "federation", "scrape_interval": "15s", "metrics_path": "/federate",
               "honor_labels": True, "params": {"match[]": ['{job=~".+"}']}}
        if sd == "consul":
            fed["consul_sd_configs"] = [_consul_sd(consul, [METRICS_TAG], services=["prometheus"])]
            fed["relabel_configs"] = [{"source_labels": ["__meta_consul_service_metadata_cloudtik_cluster"],
                                       "regex": cluster, "action": "drop"}]
        else:
            fed["file_sd_configs"] = [{"files": [os.path.join(conf_dir, "federation-*targets.yaml")],
                                       "refresh_interval": "1d"}]
        jobs.append(fed)
    return jobs


def federation_targets_file(targets: List[str]) -> List[Dict[str, Any]]:
    return [{"labels": {"service": "prometheus"}, "targets": [str(t) for t in targets]}]


def parse_pull_services(spec) -> Dict[str, Tuple[int, Optional[List[str]]]]:
    """``{name: {port, node_types}}`` (config) or ``"name:port[:type...],..."`` (the
    reference's command-line form) -> {name: (port, node_types or None = every node)}."""
    out: Dict[str, Tuple[int, Optional[List[str]]]] = {}
    if not spec:
        return out
    if isinstance(spec, str):
        for part in (p.strip() for p in spec.split(",") if p.strip()):
            f = [x.strip() for x in part.split(":")]
            if len(f) < 2:
                raise ValueError(f"pull service {part!r}: expected name:port[:node_type...]")
            out[f[0]] = (int(f[1]), f[2:] or None)
        return out
    for name, v in spec.items():
        v = v if isinstance(v, dict) else {"port": v}
        out[name] = (int(v["port"]), list(v["node_types"]) if v.get("node_types") else None)
    return out


def _save_yaml_atomic(path: str, data) -> None:
    import yaml
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    tmp = path + ".cloudtik-new"
    with open(tmp, "w") as f:
        yaml.safe_dump(data, f, sort_keys=False)
    os.replace(tmp, path)


def _state_live_nodes(address: str, password: Optional[str], timeout_s: float):
    """Live nodes from the head's node table: heartbeat within ``timeout_s``."""
    from cloudtik_amd.core.state.state_client import ControlState, StateNodeManager

    def query():
        cs = ControlState(address, password)
        now = time.time()
        rows = StateNodeManager(cs.tables).get_node_table()
        return [r for r in rows.values() if now - float(r.get("last_heartbeat_time", 0)) <= timeout_s]
    return query


class DiscoverLocalTargets(PullJob):
    """Head-side pull job of the file-based local scrape: writes ``local-targets.yaml`` (one
    target group per pull service: its port on every live node of its node types) whenever
    the set of live nodes changes."""

    def __init__(self, interval=None, services=None, config_file=None, state_address=None, state_password=None,
                 node_timeout_s=30.0, nodes: Optional[Callable[[], List[Dict[str, Any]]]] = None, targets_file=None):
        fc = {}
        if config_file:
            with open(config_file) as f:
                fc = json.load(f)
        super().__init__(float(interval or fc.get("interval") or 15.0))
        self.services = parse_pull_services(services or fc.get("pull_services") or DEFAULT_PULL_SERVICES)
        self.targets_file = targets_file or fc["targets_file"]
        if nodes is None:
            nodes = _state_live_nodes(state_address or fc.get("state_address"),
                                      state_password or fc.get("state_password") or os.environ.get(
                                          "CLOUDTIK_STATE_PASSWORD"), float(fc.get("node_timeout_s", node_timeout_s)))
        self.nodes = nodes
        self.last_hash: Optional[str] = None

    def targets(self) -> List[Dict[str, Any]]:
        by_type: Dict[str, List[str]] = {}
        for n in self.nodes():
            ip = n.get("node_ip")
            if ip:
                by_type.setdefault(str(n.get("node_type") or ""), []).append(ip)
        out = []
        for name, (port, types) in sorted(self.services.items()):
            ips = sorted({ip for t, lst in by_type.items() if types is None or t in types for ip in lst})
            if ips:
                out.append({"labels": {"service": name}, "targets": [f"{ip}:{port}" for ip in ips]})
        return out

    def pull(self):
        t = self.targets()
        h = json_hash(t)
        if h == self.last_hash:
            return
        _save_yaml_atomic(self.targets_file, t)
        self.last_hash = h


# =============================================================================== Grafana
def _basic(user: str, password: str) -> Dict[str, str]:
    return {"Authorization": "Basic " + base64.b64encode(f"{user}:{password}".encode()).decode()}


def _http_json(method: str, url: str, body=None, headers=None):
    import urllib.request
    data = json.dumps(body).encode() if body is not None else None
    req = urllib.request.Request(url, data=data, method=method,
                                 headers=dict({"Content-Type": "application/json"}, **(headers or {})))
    with urllib.request.urlopen(req, timeout=10) as r:
        raw = r.read()
    return json.loads(raw) if raw else None


def data_source_name(service: str, cluster: Optional[str]) -> str:
    return f"{service}-{cluster}" if cluster else service


def prometheus_data_source(name: str, url: str, is_default: bool = False) -> Dict[str, Any]:
    return {"name": name, "type": "prometheus", "access": "proxy", "url": url, "isDefault": is_default,
            "jsonData": {AUTO_CREATED: True}}


class DiscoverDataSources(PullJob):
    """Grafana data sources for every discovered Prometheus server, through the admin API."""

    def __init__(self, interval=None, admin_endpoint=None, service_selector=None, consul_address=None,
                 query=None, http=None, user="cloudtik", password="cloudtik", config_file=None):
        fc = {}
        if config_file:
            with open(config_file) as f:
                fc = json.load(f)
        super().__init__(float(interval or fc.get("interval") or 15.0))
        self.admin = (admin_endpoint or fc.get("admin_endpoint") or "").rstrip("/")
        if not self.admin:
            raise ValueError("DiscoverDataSources needs the Grafana admin endpoint")
        sel = dict(service_selector or fc.get("service_selector") or {})
        rts = list(sel.get("runtimes") or [])
        if "prometheus" not in rts:
            rts.append("prometheus")            # only Prometheus data sources are discovered
        sel["runtimes"] = rts
        self.selector = sel
        if query is None:
            from cloudtik_amd.runtime.common.consul import ConsulClient
            client = ConsulClient(consul_address or fc.get("consul_address") or "127.0.0.1:8500")
            query = lambda: client.select_services(self.selector)  # noqa: E731
        self.query = query
        self.http = http or _http_json
        self.headers = _basic(fc.get("user", user), fc.get("password", password))

    def wanted(self) -> Dict[str, Dict[str, Any]]:
        out = {}
        for inst in sorted(self.query(), key=lambda i: (i["name"], i["host"], int(i["port"]))):
            meta = inst.get("meta") or {}
            name = data_source_name(inst["name"], meta.get("cloudtik-cluster"))
            if name in out:            # several servers of one cluster: the first (sorted) wins
                continue
            out[name] = prometheus_data_source(name, f"http://{inst['host']}:{int(inst['port'])}")
        return out

    def pull(self):
        want = self.wanted()
        have = {d["name"]: d for d in (self.http("GET", f"{self.admin}/api/datasources", None, self.headers) or [])}
        for name in sorted(want):
            old = have.get(name)
            if old is not None:
                if old.get("url") == want[name]["url"] or not (old.get("jsonData") or {}).get(AUTO_CREATED):
                    continue            # up to date, or not ours
                # ours, but the server moved: replace it
                self.http("DELETE", f"{self.admin}/api/datasources/name/{name}", None, self.headers)
            self.http("POST", f"{self.admin}/api/datasources", want[name], self.headers)
            logger.info("grafana data source %s added: %s", name, want[name]["url"])
        for name, d in sorted(have.items()):
            if name in want or not (d.get("jsonData") or {}).get(AUTO_CREATED):
                continue                # still there, or not ours
            self.http("DELETE", f"{self.admin}/api/datasources/name/{name}", None, self.headers)
            logger.info("grafana data source %s deleted", name)
