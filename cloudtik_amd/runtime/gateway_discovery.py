"""Service-discovery pull jobs that keep the load balancers and API gateways of a cluster in
step with the services that come and go (``backend.config_mode: dynamic``).

Reference behaviour (runtime/haproxy/discovery.py:20-119 + admin_api.py:80-143,
runtime/nginx/discovery.py:18-118, runtime/kong/discovery.py, runtime/apisix/discovery.py):

* **HAProxy** -- changed live through its runtime API, no reload: a backend keeps a pool of
  server *slots*; a new server takes a free (maintenance) slot (``set server .. addr`` +
  ``state ready``), a vanished one is put back into maintenance, slots are added with
  ``add server`` when the pool is exhausted and the surplus beyond a few spare ones is deleted
  (``del server``).  The configuration file is re-rendered too, so a restart comes back with
  the same servers.
* **NGINX** -- upstreams rendered into nginx.conf; written and reloaded only when the set of
  servers changed (hash of the discovered backends).
* **Kong** -- admin API (``:8001``): one upstream + targets, service and route per discovered
  service; targets added / deleted by diff, services this job created (tag ``cloudtik``) that
  are no longer discovered are deleted.
* **APISIX** -- admin API (``:9180/apisix/admin``): an upstream (``nodes``) and a route per
  service, removed when the service goes away (label ``cloudtik``).

Discovery is the same query as the ``loadbalancer`` runtime's controller
(core/load_balancer.py): Consul ``select_services(selector)`` rows grouped into
``BackendService`` objects by ``backend_services_from_instances``; every job takes an injected
``query`` (and admin transport), which is what the tests use.
"""
from __future__ import annotations

import csv
import io
import json
import logging
import os
import socket
import subprocess
from typing import Any, Callable, Dict, List, Optional, Tuple

from cloudtik_amd.core.load_balancer import BackendService, backend_services_from_instances, json_hash
from cloudtik_amd.core.service_daemon import PullJob

logger = logging.getLogger(__name__)

Server = Tuple[str, int]
FREE_SLOTS = 4                    # spare maintenance slots kept per HAProxy backend
MANAGED_TAG = "cloudtik"


def slot_name(i: int) -> str:
    return f"server{i}"


def _consul_query(selector, consul_address):
    from cloudtik_amd.runtime.common.consul import ConsulClient
    client = ConsulClient(consul_address or os.environ.get("CONSUL_HTTP_ADDR", "127.0.0.1:8500"))
    return lambda: client.select_services(selector or {})


def _load_config(config_file: Optional[str]) -> Dict[str, Any]:
    if not config_file:
        return {}
    with open(config_file) as f:
        return json.load(f)


class DiscoveryJob(PullJob):
    """Common part: the discovery query and the change hash."""

    def __init__(self, interval=None, service_selector=None, consul_address=None, query=None, config_file=None):
        fc = _load_config(config_file)
        self.cfg = fc
        super().__init__(float(interval or fc.get("interval") or 15.0))
        sel = service_selector or fc.get("service_selector") or {}
        if isinstance(sel, str):
            sel = json.loads(sel)
        self.selector = sel
        self.query = query or _consul_query(sel, consul_address or fc.get("consul_address"))
        self.last_hash: Optional[str] = None

    def discover(self) -> Dict[str, BackendService]:
        return backend_services_from_instances(self.query())

    def pending(self, services: Dict[str, BackendService]) -> Optional[str]:
        """The hash of ``services`` when it differs from the last one APPLIED, else None.  The
        caller records it with ``commit`` only after every admin call / reload succeeded: a
        failed apply (an admin API not up yet at the first pull) is retried on the next pull
        even when the discovered set has not changed since."""
        h = json_hash({k: v.to_dict() for k, v in services.items()})
        return None if h == self.last_hash else h

    def commit(self, h: str) -> None:
        self.last_hash = h


# =============================================================================== HAProxy
class HAProxyRuntimeAPI:
    """The HAProxy runtime API over its stats socket (``stats socket ipv4@127.0.0.1:19999
    level admin``; a path = unix socket).  One command per connection."""

    def __init__(self, address: str = "127.0.0.1:19999", timeout: float = 5.0):
        self.address, self.timeout = address, timeout

    def send(self, command: str) -> str:
        if "/" in self.address:
            s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
            s.connect(self.address)
        else:
            host, _, port = self.address.rpartition(":")
            s = socket.create_connection((host, int(port)), timeout=self.timeout)
        try:
            s.sendall(command.rstrip("\n").encode() + b"\n")
            chunks = []
            while True:
                b = s.recv(65536)
                if not b:
                    break
                chunks.append(b)
            return b"".join(chunks).decode()
        finally:
            s.close()

    # ---- queries
    def _stat(self) -> List[Dict[str, str]]:
        text = self.send("show stat")
        if text.startswith("# "):
            text = text[2:]
        return list(csv.DictReader(io.StringIO(text)))

    def backends(self) -> List[str]:
        return sorted({r["pxname"] for r in self._stat() if r.get("svname") == "BACKEND"})

    def servers(self, backend: str) -> Tuple[Dict[Server, str], List[str]]:
        """({(addr, port): slot} of the active slots, [slot] of the ones in maintenance)."""
        active, inactive = {}, []
        text = self.send(f"show servers state {backend}")
        lines = [ln for ln in text.splitlines() if ln and not ln.startswith("#")]
        for ln in lines[1:] if lines and lines[0].strip().isdigit() else lines:
            f = ln.split()
            if len(f) < 19 or f[1] != backend:
                continue
            name, addr, admin = f[3], f[4], int(f[6])
            port = int(f[18])
            if admin & 0x1 or admin & 0x20:        # forced / inherited maintenance
                inactive.append(name)
            else:
                active[(addr, port)] = name
        inactive.sort(key=lambda n: int("".join(ch for ch in n if ch.isdigit()) or 0))
        return active, inactive

    # ---- changes
    def enable(self, backend: str, slot: str, server: Server):
        self.send(f"set server {backend}/{slot} addr {server[0]} port {server[1]}")
        self.send(f"set server {backend}/{slot} state ready")

    def disable(self, backend: str, slot: str):
        self.send(f"set server {backend}/{slot} state maint")

    def add(self, backend: str, slot: str, server: Server):
        self.send(f"add server {backend}/{slot} {server[0]}:{server[1]} check enabled")
        self.send(f"enable health {backend}/{slot}")

    def delete(self, backend: str, slot: str):
        self.send(f"del server {backend}/{slot}")


def haproxy_config(port: int, protocol: str = "http", servers: Optional[List] = None,
                   health_check_port: Optional[int] = None, health_check_path: str = "/",
                   api_port: Optional[int] = None, free_slots: int = FREE_SLOTS,
                   backend: str = "cloudtik-servers") -> str:
    """haproxy.cfg of a load balancer with one backend.  ``servers``: "ip:port" strings or
    (ip, port) pairs.  With ``api_port`` (dynamic mode) the runtime API socket is opened and
    the backend gets ``free_slots`` spare slots in maintenance (``server<i> 0.0.0.0:80
    disabled``) that the discovery job fills without a reload."""
    mode = "http" if protocol == "http" else "tcp"
    lines = ["global", "    maxconn 20000"]
    if api_port:
        lines.append(f"    stats socket ipv4@127.0.0.1:{int(api_port)} level admin expose-fd listeners")
    lines += ["defaults", f"    mode {mode}", "    timeout connect 5s", "    timeout client 60s",
              "    timeout server 60s", "frontend cloudtik", f"    bind *:{port}", f"    default_backend {backend}",
              f"backend {backend}", "    balance roundrobin"]
    # role-aware routing: probe the runtime's health check (runtime/common/health_check.py),
    # e.g. health_check_port 9201 + health_check_path /primary sends traffic to the primary only
    if health_check_port:
        lines.append(f"    option httpchk GET {health_check_path or '/'}")
    hc = f" port {int(health_check_port)}" if health_check_port else ""
    srv = [s if isinstance(s, str) else f"{s[0]}:{s[1]}" for s in (servers or [])]
    if api_port:
        for i, s in enumerate(srv, 1):
            lines.append(f"    server {slot_name(i)} {s} check{hc}")
        for i in range(len(srv) + 1, len(srv) + free_slots + 1):
            lines.append(f"    server {slot_name(i)} 0.0.0.0:80 check{hc} disabled")
    else:
        for i, s in enumerate(srv):
            lines.append(f"    server s{i} {s} check{hc}")
    return "\n".join(lines) + "\n"


def sync_haproxy_backend(api, backend: str, servers: List[Server], free_slots: int = FREE_SLOTS) -> Dict[str, int]:
    """Make ``backend``'s active slots exactly ``servers``.  Returns what was done."""
    active, inactive = api.servers(backend)
    total = len(active) + len(inactive)
    done = {"kept": 0, "enabled": 0, "disabled": 0, "added": 0, "deleted": 0}
    missing = []
    for srv in servers:
        if srv in active:
            del active[srv]
            done["kept"] += 1
        elif inactive:
            api.enable(backend, inactive.pop(0), srv)
            done["enabled"] += 1
        else:
            missing.append(srv)
    for srv, slot in active.items():                # still active but no longer discovered
        if missing:
            api.enable(backend, slot, missing.pop(0))
            done["enabled"] += 1
        else:
            api.disable(backend, slot)
            inactive.append(slot)
            done["disabled"] += 1
    for i, srv in enumerate(missing, start=total + 1):
        api.add(backend, slot_name(i), srv)
        done["added"] += 1
    if not missing:
        # delete surplus maintenance slots, highest numbers first, only from the tail so the
        # slot numbering stays dense
        extra = len(inactive) - free_slots
        n = total
        while extra > 0 and slot_name(n) in inactive:
            api.delete(backend, slot_name(n))
            inactive.remove(slot_name(n))
            n -= 1
            extra -= 1
            done["deleted"] += 1
    return done


class DiscoverHAProxyBackends(DiscoveryJob):
    """One backend fed by every discovered server (the load balancer mode), changed through
    the runtime API of each local HAProxy; the configuration file is re-rendered for restarts."""

    def __init__(self, interval=None, service_selector=None, consul_address=None, backend_name=None,
                 api_addresses=None, query=None, apis=None, config_file=None, render=None):
        super().__init__(interval, service_selector, consul_address, query, config_file)
        self.backend = backend_name or self.cfg.get("backend_name", "cloudtik-servers")
        addrs = api_addresses or self.cfg.get("api_addresses") or ["127.0.0.1:19999"]
        self.apis = apis or [HAProxyRuntimeAPI(a) for a in addrs]
        self.render = render            # servers -> None: rewrite haproxy.cfg (no reload)
        if render is None and self.cfg.get("conf_path"):
            hc = self.cfg.get("haproxy") or {}

            def _render(servers, path=self.cfg["conf_path"]):
                text = haproxy_config(hc.get("port", 80), hc.get("protocol", "http"), servers,
                                      hc.get("health_check_port"), hc.get("health_check_path", "/"),
                                      api_port=hc.get("api_port", 19999), backend=self.backend)
                with open(path + ".cloudtik-new", "w") as f:
                    f.write(text)
                os.replace(path + ".cloudtik-new", path)
            self.render = _render

    def pull(self):
        services = self.discover()
        servers = sorted({s for svc in services.values() for s in svc.backend_servers})
        if not servers:
            logger.warning("haproxy discovery: no live servers for the selector")
        for api in self.apis:
            sync_haproxy_backend(api, self.backend, servers)
        h = self.pending(services)
        if h is not None:
            if self.render is not None:
                self.render(servers)
            self.commit(h)


# =============================================================================== NGINX
def nginx_conf(services: Dict[str, BackendService], port: int = 80, balance: Optional[str] = None) -> str:
    """nginx.conf of a load balancer / gateway over the discovered services: one upstream per
    service, a location per route path (longest first; the default service at "/")."""
    lines = ["worker_processes auto;", "events { worker_connections 4096; }", "http {",
             "  sendfile on;", "  keepalive_timeout 65;"]
    for name, svc in sorted(services.items()):
        lines.append(f"  upstream {name} {{")
        if balance in ("least_conn", "ip_hash", "random"):
            lines.append(f"    {balance};")
        lines += [f"    server {a}:{p} max_fails=3 fail_timeout=10s;" for a, p in sorted(svc.backend_servers)]
        lines.append("  }")
    lines += ["  server {", f"    listen {port};"]
    for name, svc in sorted(services.items(), key=lambda kv: -len(kv[1].get_route_path())):
        route = svc.get_route_path()
        loc = "/" if route == "/" else route.rstrip("/") + "/"
        sp = svc.get_service_path()
        target = f"http://{name}" + ((sp or "") + "/" if loc != "/" else "")
        lines += [f"    location {loc} {{", f"      proxy_pass {target};", "      proxy_set_header Host $host;",
                  "    }"]
    lines += ["  }", "}"]
    return "\n".join(lines) + "\n"


class DiscoverNginxBackends(DiscoveryJob):
    """Rewrites nginx.conf and reloads NGINX when the discovered backends changed."""

    def __init__(self, interval=None, service_selector=None, consul_address=None, conf_path=None, port=None,
                 balance=None, query=None, reload_cmd=None, runner=None, config_file=None):
        super().__init__(interval, service_selector, consul_address, query, config_file)
        self.conf_path = conf_path or self.cfg.get("conf_path") or "/etc/nginx/nginx.conf"
        self.port = int(port or self.cfg.get("port") or 80)
        self.balance = balance or self.cfg.get("balance")
        self.reload_cmd = reload_cmd or self.cfg.get("reload_cmd") or "sudo nginx -s reload"
        self.runner = runner or (lambda cmd: subprocess.run(["bash", "-c", cmd], check=False))
        self.reloads = 0

    def pull(self):
        services = self.discover()
        h = self.pending(services)
        if h is None:
            return
        text = nginx_conf(services, self.port, self.balance)
        tmp = self.conf_path + ".cloudtik-new"
        with open(tmp, "w") as f:
            f.write(text)
        os.replace(tmp, self.conf_path)
        r = self.runner(self.reload_cmd)
        if getattr(r, "returncode", 0) not in (0, None):
            raise RuntimeError(f"nginx reload failed (rc {r.returncode}): {self.reload_cmd}")
        self.reloads += 1
        self.commit(h)


# =============================================================================== admin-API gateways
def _http_json(method: str, url: str, body: Optional[dict] = None, headers: Optional[dict] = None) -> Any:
    import urllib.request
    data = json.dumps(body).encode() if body is not None else None
    req = urllib.request.Request(url, data=data, method=method,
                                 headers=dict({"Content-Type": "application/json"}, **(headers or {})))
    with urllib.request.urlopen(req, timeout=10) as r:
        raw = r.read()
    return json.loads(raw) if raw else None


class DiscoverKongBackends(DiscoveryJob):
    """Kong admin API: upstream ``<svc>`` with one target per server, service ``<svc>`` on
    that upstream (path = the service path), route ``<svc>`` on the route path (prefix
    stripped).  Objects carry the tag ``cloudtik``; the ones of vanished services are deleted."""

    def __init__(self, interval=None, service_selector=None, consul_address=None, admin_url=None, query=None,
                 http=None, config_file=None):
        super().__init__(interval, service_selector, consul_address, query, config_file)
        self.admin = (admin_url or self.cfg.get("admin_url") or "http://127.0.0.1:8001").rstrip("/")
        self.http = http or _http_json

    def _get_all(self, path: str) -> List[dict]:
        out, url = [], f"{self.admin}{path}"
        while url:
            r = self.http("GET", url) or {}
            out += r.get("data") or []
            nxt = r.get("next")
            url = (nxt if nxt.startswith("http") else f"{self.admin}{nxt}") if nxt else None
        return out

    def pull(self):
        services = self.discover()
        h = self.pending(services)
        if h is None:
            return
        managed = {s["name"] for s in self._get_all(f"/services?tags={MANAGED_TAG}")}
        for name, svc in services.items():
            self.http("PUT", f"{self.admin}/upstreams/{name}", {"name": name, "tags": [MANAGED_TAG]})
            have = {t["target"]: t["id"] for t in self._get_all(f"/upstreams/{name}/targets")}
            want = {f"{a}:{p}" for a, p in svc.backend_servers}
            for t in sorted(want - set(have)):
                self.http("POST", f"{self.admin}/upstreams/{name}/targets", {"target": t, "weight": 100})
            for t in sorted(set(have) - want):
                self.http("DELETE", f"{self.admin}/upstreams/{name}/targets/{have[t]}")
            self.http("PUT", f"{self.admin}/services/{name}",
                      {"name": name, "host": name, "port": int(svc.port), "protocol": "http",
                       "path": svc.get_service_path() or None, "tags": [MANAGED_TAG]})
            self.http("PUT", f"{self.admin}/routes/{name}",
                      {"name": name, "paths": [svc.get_route_path()], "strip_path": True,
                       "service": {"name": name}, "tags": [MANAGED_TAG]})
        for name in sorted(managed - set(services)):
            self.http("DELETE", f"{self.admin}/routes/{name}")
            self.http("DELETE", f"{self.admin}/services/{name}")
            self.http("DELETE", f"{self.admin}/upstreams/{name}")
        self.commit(h)


class DiscoverAPISIXBackends(DiscoveryJob):
    """APISIX admin API: upstream + route per service (id = service name), label
    ``cloudtik``; routes / upstreams of vanished services are deleted."""

    def __init__(self, interval=None, service_selector=None, consul_address=None, admin_url=None, admin_key=None,
                 query=None, http=None, config_file=None, balance=None):
        super().__init__(interval, service_selector, consul_address, query, config_file)
        self.admin = (admin_url or self.cfg.get("admin_url") or "http://127.0.0.1:9180/apisix/admin").rstrip("/")
        self.key = admin_key or self.cfg.get("admin_key") or "cloudtik-apisix"
        self.balance = balance or self.cfg.get("balance") or "roundrobin"
        self.http = http or _http_json

    def _call(self, method, path, body=None):
        return self.http(method, f"{self.admin}{path}", body, {"X-API-KEY": self.key})

    def _managed(self, kind: str) -> List[str]:
        r = self._call("GET", f"/{kind}") or {}
        items = r.get("list") or r.get("node", {}).get("nodes") or []
        out = []
        for it in items:
            v = it.get("value") or it
            if (v.get("labels") or {}).get("managed-by") == MANAGED_TAG:
                out.append(str(v.get("id")))
        return out

    def pull(self):
        services = self.discover()
        h = self.pending(services)
        if h is None:
            return
        for name, svc in services.items():
            self._call("PUT", f"/upstreams/{name}",
                       {"id": name, "type": self.balance, "labels": {"managed-by": MANAGED_TAG},
                        "nodes": {f"{a}:{p}": 1 for a, p in sorted(svc.backend_servers)}})
            route = svc.get_route_path()
            uri = "/*" if route == "/" else route.rstrip("/") + "/*"
            body = {"id": name, "uri": uri, "upstream_id": name, "labels": {"managed-by": MANAGED_TAG}}
            if route != "/":
                sp = svc.get_service_path() or ""
                body["plugins"] = {"proxy-rewrite": {"regex_uri": [f"^{route.rstrip('/')}/(.*)", f"{sp}/$1"]}}
            self._call("PUT", f"/routes/{name}", body)
        for rid in sorted(set(self._managed("routes")) - set(services)):
            self._call("DELETE", f"/routes/{rid}")
        for uid in sorted(set(self._managed("upstreams")) - set(services)):
            self._call("DELETE", f"/upstreams/{uid}")
        self.commit(h)
