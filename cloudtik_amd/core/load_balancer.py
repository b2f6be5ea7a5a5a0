"""Load balancers for a workspace's services (reference core/load_balancer_provider.py,
runtime/loadbalancer/{provider_api,controller,scripting}.py).

Three pieces:

* ``BackendService`` -- one service to expose: its backend servers (address, port, node id,
  seq id), its protocol / port, and the front-end it asks for (load balancer name, scheme,
  protocol, port, HTTP route path / service path / default service).  Built from a static
  ``backend.services`` config (``backend_services_from_config``) or from service discovery
  (``backend_services_from_instances`` over Consul ``select_services`` rows).
* ``LoadBalancerManager`` -- turns the backend services into load balancer configs and
  reconciles them against the provider: create the new ones, update the changed ones (a
  JSON hash per load balancer skips no-op updates), delete auto-created ones that lost all
  services.  Planning: services that name a load balancer go to it (one type per load
  balancer; a network load balancer serves one service per listener); unnamed TCP/TLS/UDP
  services share the workspace's default network load balancer ``<ws>-n`` and unnamed
  HTTP/HTTPS services the default application load balancer ``<ws>-a`` -- or, when the
  provider has single-service-group load balancers (or ``anonymous_prefer_default`` is
  off), one network load balancer per service and one application load balancer per
  ``<ws>-<protocol>-<port>``.  A service group is keyed by (listener protocol, port).
* ``LoadBalancerController`` -- the pull job the ``loadbalancer`` runtime starts on the head:
  every interval, discover the selected services, rebuild the backend services and, when the
  set changed, call the manager.  With a Consul address it runs under Consul leader election
  so that only one head of a multi-head deployment drives the cloud API.

Providers: ``HAProxyLoadBalancerProvider`` (here: on-premise / local -- renders and reloads
an HAProxy config on the node, frontends per listener, backends per service, path ACLs for
application load balancers) and the cloud ones in providers/cloud/load_balancer.py.
"""
from __future__ import annotations

import hashlib
import json
import logging
import os
import subprocess
from dataclasses import dataclass
from typing import Any, Callable, Dict, List, Optional, Tuple

from cloudtik_amd.core.provider_api import LoadBalancerProvider
from cloudtik_amd.core.service_daemon import PullJob

logger = logging.getLogger(__name__)

TYPE_NETWORK = "network"
TYPE_APPLICATION = "application"
PROTOCOL_TCP, PROTOCOL_TLS, PROTOCOL_UDP = "TCP", "TLS", "UDP"
PROTOCOL_HTTP, PROTOCOL_HTTPS = "HTTP", "HTTPS"
SCHEME_INTERNET_FACING = "internet-facing"
SCHEME_INTERNAL = "internal"
AUTO_CREATED_TAG = "cloudtik-auto-create"
NETWORK_DEFAULT = "{}-n"
APPLICATION_DEFAULT = "{}-a"

# service-discovery meta labels a service sets to ask for a front-end
LABEL_LB_NAME = "cloudtik-load-balancer-name"
LABEL_LB_SCHEME = "cloudtik-load-balancer-scheme"
LABEL_LB_PROTOCOL = "cloudtik-load-balancer-protocol"
LABEL_LB_PORT = "cloudtik-load-balancer-port"
LABEL_PROTOCOL = "cloudtik-protocol"
LABEL_ROUTE_PATH = "cloudtik-route-path"
LABEL_SERVICE_PATH = "cloudtik-service-path"
LABEL_DEFAULT_SERVICE = "cloudtik-default-service"


def is_application(protocol: Optional[str]) -> bool:
    return (protocol or "").upper() in (PROTOCOL_HTTP, PROTOCOL_HTTPS)


def _port(v) -> int:
    p = int(v)
    if not 0 < p < 65536:
        raise ValueError(f"invalid port {v}")
    return p


def json_hash(obj: Any) -> str:
    return hashlib.sha1(json.dumps(obj, sort_keys=True, default=str).encode()).hexdigest()


@dataclass
class BackendService:
    service_name: str
    backend_servers: Dict[Tuple[str, int], Dict[str, Any]]
    protocol: Optional[str] = None
    port: Optional[int] = None
    load_balancer_name: Optional[str] = None
    load_balancer_scheme: Optional[str] = None
    load_balancer_protocol: Optional[str] = None
    load_balancer_port: Optional[int] = None
    route_path: Optional[str] = None
    service_path: Optional[str] = None
    default_service: bool = False

    def __post_init__(self):
        if not self.backend_servers:
            raise ValueError(f"service {self.service_name} has no backend servers")
        self.protocol = (self.protocol or PROTOCOL_TCP).upper()
        if not self.port:
            self.port = next(iter(self.backend_servers.values()))["port"]
        self.port = _port(self.port)
        self.load_balancer_protocol = (self.load_balancer_protocol or self.protocol).upper()
        self.load_balancer_port = _port(self.load_balancer_port or self.port)
        # route path "/abc" matches /abc and /abc/*, "/abc/" only /abc/*, "/" everything (lowest
        # priority); default "/<name>", or "/" for the default service.  The service path
        # replaces the route prefix on the way to the backend ("/" or "" strips it).
        if self.route_path and not self.route_path.startswith("/"):
            self.route_path = "/" + self.route_path
        if self.service_path is not None:
            self.service_path = "/" + self.service_path.strip("/") if self.service_path.strip("/") else ""

    def get_route_path(self) -> str:
        return self.route_path or ("/" if self.default_service else f"/{self.service_name}")

    def get_service_path(self) -> Optional[str]:
        return self.service_path

    def to_dict(self) -> Dict[str, Any]:
        d = {k: v for k, v in self.__dict__.items() if k != "backend_servers"}
        d["servers"] = sorted((a, p) for a, p in self.backend_servers)
        return d


def _address(s: str) -> Tuple[str, int]:
    host, _, port = s.rpartition(":")
    return host, int(port)


def backend_services_from_config(backend_config: Dict[str, Any]) -> Dict[str, BackendService]:
    """``backend.services: {name: {servers: ["ip:port"], protocol, port, load_balancer_name,
    load_balancer_scheme, load_balancer_protocol, load_balancer_port, route_path,
    service_path, default_service}}`` (static mode)."""
    out = {}
    for name, sc in (backend_config.get("services") or {}).items():
        servers = {}
        for s in sc.get("servers") or []:
            a, p = _address(s)
            servers[(a, p)] = {"address": a, "port": p}
        if not servers:
            continue
        out[name] = BackendService(
            name, servers, sc.get("protocol"), sc.get("port"), sc.get("load_balancer_name"),
            sc.get("load_balancer_scheme"), sc.get("load_balancer_protocol"), sc.get("load_balancer_port"),
            sc.get("route_path"), sc.get("service_path"), bool(sc.get("default_service", False)))
    return out


def backend_services_from_instances(instances: List[Dict[str, Any]]) -> Dict[str, BackendService]:
    """Group discovered instances (``ConsulClient.select_services`` rows: name, host, port,
    meta, node) into backend services; front-end wishes come from the service meta."""
    by_name: Dict[str, List[Dict[str, Any]]] = {}
    for i in instances:
        by_name.setdefault(i["name"], []).append(i)
    out = {}
    for name, insts in sorted(by_name.items()):
        servers = {}
        meta: Dict[str, str] = {}
        for i in insts:
            m = i.get("meta") or {}
            meta.update(m)
            srv = {"address": i["host"], "port": int(i["port"])}
            if i.get("node"):
                srv["node_id"] = i["node"]
            if m.get("cloudtik-seq-id"):
                srv["seq_id"] = m["cloudtik-seq-id"]
            servers[(i["host"], int(i["port"]))] = srv
        out[name] = BackendService(
            name, servers, meta.get(LABEL_PROTOCOL), None, meta.get(LABEL_LB_NAME), meta.get(LABEL_LB_SCHEME),
            meta.get(LABEL_LB_PROTOCOL), meta.get(LABEL_LB_PORT), meta.get(LABEL_ROUTE_PATH),
            meta.get(LABEL_SERVICE_PATH), meta.get(LABEL_DEFAULT_SERVICE, "").lower() == "true")
    return out


class LoadBalancerManager:
    def __init__(self, provider_config: Dict[str, Any], workspace_name: str,
                 provider: Optional[LoadBalancerProvider] = None):
        self.provider_config = provider_config
        self.workspace_name = workspace_name
        self.provider = provider or get_load_balancer_provider(provider_config, workspace_name)
        self.hashes: Dict[str, str] = {}
        self.default_network = provider_config.get("default_network_load_balancer_name") or \
            NETWORK_DEFAULT.format(workspace_name)
        self.default_application = provider_config.get("default_application_load_balancer_name") or \
            APPLICATION_DEFAULT.format(workspace_name)
        self.error_abort = bool(provider_config.get("error_abort", False))
        self.default_scheme = provider_config.get("load_balancer_scheme", SCHEME_INTERNET_FACING)
        self.delete_auto_empty = provider_config.get("delete_auto_empty", True)
        self.prefer_default = provider_config.get("anonymous_prefer_default", True)

    # ------------------------------------------------------------------ planning
    @staticmethod
    def _groups(services: List[BackendService]) -> Dict[Tuple[str, int], List[BackendService]]:
        g: Dict[Tuple[str, int], List[BackendService]] = {}
        for s in services:
            g.setdefault((s.load_balancer_protocol, s.load_balancer_port), []).append(s)
        return g

    def plan(self, backend_services: Dict[str, BackendService]) -> Dict[str, Dict[Tuple[str, int], List[BackendService]]]:
        named: Dict[str, List[BackendService]] = {}
        for s in backend_services.values():
            named.setdefault(s.load_balancer_name or "", []).append(s)
        multi = self.provider.support_multi_service_group()
        plan: Dict[str, Dict[Tuple[str, int], List[BackendService]]] = {}
        for lb, svcs in named.items():
            if lb:
                try:
                    types = {is_application(s.load_balancer_protocol) for s in svcs}
                    if len(types) > 1:
                        raise ValueError("services mix network and application protocols")
                    groups = self._groups(svcs)
                    if not multi and len(groups) > 1:
                        raise ValueError("provider has single-service-group load balancers")
                    if not types.pop() and any(len(v) > 1 for v in groups.values()):
                        raise ValueError("a network listener serves one service")
                    plan[lb] = groups
                except ValueError as e:
                    logger.warning("load balancer %s not planned: %s", lb, e)
                continue
            net = [s for s in svcs if not is_application(s.load_balancer_protocol)]
            app = [s for s in svcs if is_application(s.load_balancer_protocol)]
            split = not multi or not self.prefer_default
            if net:
                groups = self._groups(net)
                if split:
                    for key, ss in groups.items():
                        for s in ss:
                            plan[s.service_name] = {key: [s]}
                else:
                    plan[self.default_network] = groups
            if app:
                groups = self._groups(app)
                if split:
                    for key, ss in groups.items():
                        plan[f"{self.workspace_name}-{key[0]}-{key[1]}"] = {key: ss}
                else:
                    plan[self.default_application] = groups
        return plan

    def load_balancers(self, backend_services: Dict[str, BackendService]) -> Dict[str, Dict[str, Any]]:
        out = {}
        for name, groups in self.plan(backend_services).items():
            lb_type = TYPE_APPLICATION if is_application(next(iter(groups))[0]) else TYPE_NETWORK
            schemes = {s.load_balancer_scheme for ss in groups.values() for s in ss if s.load_balancer_scheme}
            lb = {"name": name, "type": lb_type,
                  "scheme": schemes.pop() if len(schemes) == 1 else self.default_scheme,
                  "tags": {AUTO_CREATED_TAG: "true"}, "service_groups": []}
            for (proto, port), ss in sorted(groups.items()):
                services = []
                for s in sorted(ss, key=lambda s: s.service_name):
                    targets = sorted(s.backend_servers.values(), key=lambda t: (t["address"], t["port"]))
                    svc = {"name": s.service_name, "protocol": s.protocol, "port": s.port, "targets": targets}
                    if lb_type == TYPE_APPLICATION:
                        svc["route_path"] = s.get_route_path()
                        if s.service_path is not None:
                            svc["service_path"] = s.service_path
                        if s.default_service:
                            svc["default"] = True
                    services.append(svc)
                lb["service_groups"].append({"listeners": [{"protocol": proto, "port": port}], "services": services})
            out[name] = lb
        return out

    # ------------------------------------------------------------------ reconcile
    def _do(self, what: str, name: str, fn: Callable[[], None]) -> bool:
        try:
            fn()
            return True
        except Exception as e:  # noqa: BLE001 - one bad load balancer must not stop the others
            logger.error("%s load balancer %s failed: %s", what, name, e)
            if self.error_abort:
                raise
            return False

    def update(self, backend_services: Dict[str, BackendService]) -> Dict[str, List[str]]:
        wanted = self.load_balancers(backend_services)
        existing = self.provider.list()
        done: Dict[str, List[str]] = {"created": [], "updated": [], "deleted": []}
        for name, lb in wanted.items():
            h = json_hash(lb)
            if name not in existing:
                if self._do("creating", name, lambda: self.provider.create(lb)):
                    self.hashes[name] = h
                    done["created"].append(name)
            elif self.hashes.get(name) != h:
                if self._do("updating", name, lambda: self.provider.update(existing[name], lb)):
                    self.hashes[name] = h
                    done["updated"].append(name)
        for name, cur in existing.items():
            auto = str((cur.get("tags") or {}).get(AUTO_CREATED_TAG, "")).lower() == "true"
            if name not in wanted and auto and self.delete_auto_empty:
                if self._do("deleting", name, lambda: self.provider.delete(cur)):
                    self.hashes.pop(name, None)
                    done["deleted"].append(name)
        return done


class LoadBalancerController(PullJob):
    """Head-side pull job of the ``loadbalancer`` runtime (see module doc).  ``query`` returns
    discovered instances (default: Consul ``select_services(selector)``)."""

    def __init__(self, provider_config=None, workspace_name: str = "default", service_selector=None,
                 interval: Optional[float] = None, consul_address: Optional[str] = None,
                 query: Optional[Callable[[], List[Dict[str, Any]]]] = None,
                 manager: Optional[LoadBalancerManager] = None, leader_ttl_s: int = 10,
                 config_file: Optional[str] = None):
        if config_file:                     # written by the loadbalancer runtime at configure time
            with open(config_file) as f:
                fc = json.load(f)
            provider_config = provider_config or fc.get("provider_config")
            workspace_name = fc.get("workspace_name", workspace_name)
            service_selector = service_selector or fc.get("service_selector")
            interval = interval or fc.get("interval")
            consul_address = consul_address or fc.get("consul_address")
        super().__init__(float(interval) if interval else 15.0)
        if isinstance(provider_config, str):
            provider_config = json.loads(provider_config)
        if isinstance(service_selector, str):
            service_selector = json.loads(service_selector)
        self.manager = manager or LoadBalancerManager(provider_config or {}, workspace_name)
        self.selector = service_selector or {}
        self._client = None
        if query is None:
            from cloudtik_amd.runtime.common.consul import ConsulClient
            self._client = ConsulClient(consul_address or os.environ.get("CONSUL_HTTP_ADDR", "127.0.0.1:8500"))
            query = lambda: self._client.select_services(self.selector)  # noqa: E731
        self.query = query
        self.election = None
        if consul_address:
            from cloudtik_amd.runtime.common.consul import ConsulClient, ConsulLeaderElection
            self.election = ConsulLeaderElection(self._client or ConsulClient(consul_address),
                                                 "load-balancer-controller", ttl_s=leader_ttl_s)
        self.last_hash: Optional[str] = None

    def pull(self):
        if self.election is not None and not self.election.step():
            self.last_hash = None           # a standby re-applies everything once it takes over
            return
        services = backend_services_from_instances(self.query())
        h = json_hash({k: v.to_dict() for k, v in services.items()})
        if h != self.last_hash:
            self.manager.update(services)
            self.last_hash = h


# =============================================================================== HAProxy
class HAProxyLoadBalancerProvider(LoadBalancerProvider):
    """Load balancers as HAProxy frontends on this node (local / on-premise workspaces, where
    there is no cloud load-balancer API).  All load balancers of the workspace live in one
    config file (``config_file``; state beside it as JSON); every change re-renders it,
    validates it with ``haproxy -c`` when HAProxy is installed, and runs ``reload_command``."""

    def __init__(self, provider_config: Dict[str, Any], workspace_name: str):
        super().__init__(provider_config, workspace_name)
        home = os.environ.get("HAPROXY_HOME") or os.path.expanduser("~/.cloudtik/haproxy")
        self.config_file = provider_config.get("config_file") or os.path.join(home, f"{workspace_name}-lb.cfg")
        self.state_file = self.config_file + ".json"
        self.reload_command = provider_config.get("reload_command")

    def _state(self) -> Dict[str, Dict[str, Any]]:
        if not os.path.exists(self.state_file):
            return {}
        with open(self.state_file) as f:
            return json.load(f)

    def _save(self, state: Dict[str, Dict[str, Any]]):
        os.makedirs(os.path.dirname(self.config_file) or ".", exist_ok=True)
        text = self.render(state)
        tmp = self.config_file + ".tmp"
        with open(tmp, "w") as f:
            f.write(text)
        exe = self.provider_config.get("haproxy_bin", "haproxy")
        from shutil import which
        if which(exe):
            r = subprocess.run([exe, "-c", "-f", tmp], capture_output=True, text=True)
            if r.returncode != 0:
                os.unlink(tmp)
                raise RuntimeError(f"haproxy rejected the config: {r.stderr.strip()[:400]}")
        os.replace(tmp, self.config_file)
        with open(self.state_file, "w") as f:
            json.dump(state, f, indent=1, sort_keys=True)
        if self.reload_command:
            subprocess.run(self.reload_command, shell=True, check=True)

    @staticmethod
    def render(state: Dict[str, Dict[str, Any]]) -> str:
        out = ["global", "    maxconn 20000", "", "defaults", "    timeout connect 5s", "    timeout client 60s",
               "    timeout server 60s", ""]
        for name in sorted(state):
            lb = state[name]
            http = lb["type"] == TYPE_APPLICATION
            bind = "0.0.0.0" if lb.get("scheme", SCHEME_INTERNET_FACING) == SCHEME_INTERNET_FACING else "127.0.0.1"
            for g in lb["service_groups"]:
                for ls in g["listeners"]:
                    fe = f"{name}-{ls['protocol'].lower()}-{ls['port']}"
                    out += [f"frontend {fe}", f"    bind {bind}:{ls['port']}", f"    mode {'http' if http else 'tcp'}"]
                    default = None
                    routed = sorted(g["services"], key=lambda s: -len(s.get("route_path", "")))
                    for s in routed:
                        be = f"{name}-{s['name']}"
                        if not http:
                            default = be
                            continue
                        rp = s.get("route_path", "/")
                        if s.get("default") or rp == "/":
                            default = be
                            if rp == "/":
                                continue
                        acl = f"path_{s['name']}".replace("-", "_")
                        if not rp.endswith("/"):
                            out.append(f"    acl {acl} path {rp}")
                        out += [f"    acl {acl} path_beg {rp.rstrip('/')}/", f"    use_backend {be} if {acl}"]
                    if default:
                        out.append(f"    default_backend {default}")
                    out.append("")
            for g in lb["service_groups"]:
                for s in g["services"]:
                    out += [f"backend {name}-{s['name']}", f"    mode {'http' if http else 'tcp'}",
                            "    balance roundrobin"]
                    if http and s.get("service_path") is not None:
                        prefix = s.get("route_path", "/").rstrip("/")
                        out.append(f"    http-request replace-path ^{prefix}/?(.*)$ {s['service_path']}/\\1")
                    for i, t in enumerate(s["targets"]):
                        out.append(f"    server s{i} {t['address']}:{t['port']} check")
                    out.append("")
        return "\n".join(out)

    def list(self):
        return {n: {k: lb[k] for k in ("name", "type", "scheme", "tags")} for n, lb in self._state().items()}

    def create(self, load_balancer_config):
        st = self._state()
        st[load_balancer_config["name"]] = load_balancer_config
        self._save(st)

    def update(self, load_balancer, load_balancer_config):
        self.create(load_balancer_config)

    def delete(self, load_balancer):
        st = self._state()
        st.pop(load_balancer["name"], None)
        self._save(st)


def get_load_balancer_provider(provider_config: Dict[str, Any], workspace_name: str,
                               transport=None) -> LoadBalancerProvider:
    """By ``provider_config['type']``: aws / gcp / azure -> the cloud load balancers;
    local / onpremise / virtual / haproxy (default) -> HAProxy on the node; a
    ``provider_class`` dotted path -> that class."""
    cls = provider_config.get("provider_class")
    if cls:
        mod, _, name = cls.rpartition(".")
        import importlib
        return getattr(importlib.import_module(mod), name)(provider_config, workspace_name)
    t = provider_config.get("type", "haproxy")
    if t in ("aws", "gcp", "azure"):
        from cloudtik_amd.providers.cloud.load_balancer import cloud_load_balancer_provider
        return cloud_load_balancer_provider(provider_config, workspace_name, transport)
    return HAProxyLoadBalancerProvider(provider_config, workspace_name)
