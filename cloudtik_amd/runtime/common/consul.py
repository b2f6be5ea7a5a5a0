"""Consul HTTP API client for service discovery (reference runtime/common/service_discovery/
consul.py: catalog queries used to resolve runtime services and DNS names).

Only the endpoints the platform uses, over urllib (no SDK):

* catalog: services, nodes of a service (by tag), healthy instances (``health/service`` with
  ``passing``), selector queries over CloudTik's service tags / meta (``select_services``:
  the same selector dict as the workspace registry -- runtimes, services, clusters, tags,
  labels and their exclusions);
* agent: register / deregister a local service with a TCP or HTTP health check, carrying the
  CloudTik tags (``cloudtik-c-<cluster>``, ``cloudtik-r-<runtime>``, ``cloudtik-f-<feature>``)
  and meta (cluster, runtime, service);
* KV: get / put / delete / keys, and session-based locks (``session/create`` with a TTL +
  ``kv?acquire=``), on which ``ConsulLock`` and ``ConsulLeaderElection`` give the Consul
  backend of core/state/lock.py's lock and leader election (reference
  core/_private/util/leader_election + runtime/common/service_discovery/consul.py).
"""
from __future__ import annotations

import base64
import json
import threading
import time
import urllib.error
import urllib.parse
import urllib.request
import uuid
from typing import Any, Dict, List, Optional, Tuple

DEFAULT_ADDRESS = "127.0.0.1:8500"


class ConsulClient:
    def __init__(self, address: str = DEFAULT_ADDRESS, token: Optional[str] = None, timeout: float = 10.0):
        self.base = address if address.startswith("http") else f"http://{address}"
        self.token, self.timeout = token, timeout

    def _req(self, method: str, path: str, query: Optional[Dict[str, Any]] = None, body: Any = None):
        url = f"{self.base}/v1/{path.lstrip('/')}"
        if query:
            url += "?" + urllib.parse.urlencode({k: v for k, v in query.items() if v is not None})
        data = None
        if body is not None:
            data = body if isinstance(body, bytes) else json.dumps(body).encode()
        req = urllib.request.Request(url, data=data, method=method)
        if self.token:
            req.add_header("X-Consul-Token", self.token)
        with urllib.request.urlopen(req, timeout=self.timeout) as r:
            raw = r.read()
        if not raw:
            return None
        try:
            return json.loads(raw)
        except ValueError:
            return raw.decode()

    # ---------------------------------------------------------------- catalog
    def services(self) -> Dict[str, List[str]]:
        return self._req("GET", "catalog/services") or {}

    def service_nodes(self, service: str, tag: Optional[str] = None) -> List[Dict[str, Any]]:
        return self._req("GET", f"catalog/service/{urllib.parse.quote(service)}", {"tag": tag}) or []

    def service_addresses(self, service: str, tag: Optional[str] = None) -> List[Tuple[str, int]]:
        out = []
        for n in self.service_nodes(service, tag):
            host = n.get("ServiceAddress") or n.get("Address")
            out.append((host, int(n.get("ServicePort") or 0)))
        return out

    def nodes(self) -> List[Dict[str, Any]]:
        return self._req("GET", "catalog/nodes") or []

    def healthy_instances(self, service: str, tag: Optional[str] = None) -> List[Dict[str, Any]]:
        """Instances whose every health check passes (``health/service?passing``)."""
        rows = self._req("GET", f"health/service/{urllib.parse.quote(service)}", {"tag": tag, "passing": "true"}) or []
        out = []
        for r in rows:
            svc, node = r.get("Service", {}), r.get("Node", {})
            out.append({"name": svc.get("Service"), "id": svc.get("ID"), "host": svc.get("Address") or
                        node.get("Address"), "port": int(svc.get("Port") or 0), "tags": svc.get("Tags") or [],
                        "meta": svc.get("Meta") or {}, "node": node.get("Node")})
        return out

    def select_services(self, selector: Optional[Dict[str, Any]] = None, passing: bool = True) -> List[Dict[str, Any]]:
        """Service instances matching a CloudTik service selector (runtimes / services /
        clusters / tags / labels, with exclude_* variants), healthy ones by default."""
        sel = selector or {}
        out = []
        for name, tags in sorted(self.services().items()):
            if sel.get("services") and name not in sel["services"]:
                continue
            insts = self.healthy_instances(name) if passing else [
                {"name": n.get("ServiceName"), "id": n.get("ServiceID"), "host": n.get("ServiceAddress") or
                 n.get("Address"), "port": int(n.get("ServicePort") or 0), "tags": n.get("ServiceTags") or [],
                 "meta": n.get("ServiceMeta") or {}, "node": n.get("Node")} for n in self.service_nodes(name)]
            for i in insts:
                if _matches(i, sel):
                    out.append(i)
        return out

    # ---------------------------------------------------------------- agent
    def register_service(self, name: str, port: int, address: Optional[str] = None, tags: Optional[List[str]] = None,
                         service_id: Optional[str] = None, check_http: Optional[str] = None,
                         check_interval: str = "10s", meta: Optional[Dict[str, str]] = None,
                         cluster: Optional[str] = None, runtime: Optional[str] = None,
                         features: Optional[List[str]] = None):
        tags = list(tags or [])
        meta = dict(meta or {})
        if cluster:
            tags.append(f"cloudtik-c-{cluster}")
            meta["cloudtik-cluster"] = cluster
        if runtime:
            tags.append(f"cloudtik-r-{runtime}")
            meta["cloudtik-runtime"] = runtime
        tags += [f"cloudtik-f-{f}" for f in features or []]
        body: Dict[str, Any] = {"Name": name, "ID": service_id or name, "Port": int(port), "Tags": tags,
                                "Meta": meta}
        if address:
            body["Address"] = address
        if check_http:
            body["Check"] = {"HTTP": check_http, "Interval": check_interval}
        else:
            body["Check"] = {"TCP": f"{address or '127.0.0.1'}:{port}", "Interval": check_interval}
        self._req("PUT", "agent/service/register", body=body)

    def deregister_service(self, service_id: str):
        self._req("PUT", f"agent/service/deregister/{urllib.parse.quote(service_id)}")

    # ---------------------------------------------------------------- KV
    def kv_get(self, key: str) -> Optional[bytes]:
        try:
            r = self._req("GET", f"kv/{key}")
        except urllib.error.HTTPError as e:
            if e.code == 404:
                return None
            raise
        if not r:
            return None
        v = r[0].get("Value")
        return base64.b64decode(v) if v is not None else b""

    def kv_put(self, key: str, value: bytes, acquire: Optional[str] = None, release: Optional[str] = None,
               cas: Optional[int] = None) -> bool:
        q = {"acquire": acquire, "release": release, "cas": cas}
        data = value if isinstance(value, bytes) else str(value).encode()
        return bool(self._req("PUT", f"kv/{key}", {k: v for k, v in q.items() if v is not None} or None, body=data))

    def kv_delete(self, key: str, recurse: bool = False) -> bool:
        return bool(self._req("DELETE", f"kv/{key}", {"recurse": "true"} if recurse else None))

    def kv_keys(self, prefix: str = "") -> List[str]:
        try:
            return self._req("GET", f"kv/{prefix}", {"keys": "true"}) or []
        except urllib.error.HTTPError as e:
            if e.code == 404:
                return []
            raise

    def kv_session(self, key: str) -> Optional[str]:
        """The session currently holding ``key`` (None if free / missing)."""
        try:
            r = self._req("GET", f"kv/{key}")
        except urllib.error.HTTPError as e:
            if e.code == 404:
                return None
            raise
        return (r or [{}])[0].get("Session") or None

    # ---------------------------------------------------------------- sessions
    def session_create(self, name: str, ttl_s: int = 15, behavior: str = "release") -> str:
        return self._req("PUT", "session/create", body={"Name": name, "TTL": f"{int(ttl_s)}s",
                                                        "Behavior": behavior, "LockDelay": "0s"})["ID"]

    def session_renew(self, session: str) -> bool:
        try:
            return bool(self._req("PUT", f"session/renew/{session}"))
        except urllib.error.HTTPError as e:
            if e.code == 404:
                return False
            raise

    def session_destroy(self, session: str) -> bool:
        return bool(self._req("PUT", f"session/destroy/{session}"))


def _matches(inst: Dict[str, Any], sel: Dict[str, Any]) -> bool:
    tags, meta = set(inst.get("tags") or []), inst.get("meta") or {}
    cluster, runtime = meta.get("cloudtik-cluster"), meta.get("cloudtik-runtime")
    if sel.get("runtimes") and runtime not in sel["runtimes"]:
        return False
    if sel.get("exclude_runtimes") and runtime in sel["exclude_runtimes"]:
        return False
    if sel.get("clusters") and cluster not in sel["clusters"]:
        return False
    if sel.get("exclude_clusters") and cluster in sel["exclude_clusters"]:
        return False
    if sel.get("tags") and not set(sel["tags"]) <= tags:
        return False
    for k, v in (sel.get("labels") or {}).items():
        if meta.get(k) != v:
            return False
    for k, v in (sel.get("exclude_labels") or {}).items():
        if meta.get(k) == v:
            return False
    return True


class ConsulLock:
    """A lock on a Consul KV key held by a TTL session (the Consul backend of
    core/state/lock.py's DistributedLock: same acquire / renew / release / owner calls)."""

    def __init__(self, client: ConsulClient, name: str, ttl_s: int = 15, owner: Optional[str] = None):
        self.c, self.key, self.ttl_s = client, f"cloudtik/locks/{name}", ttl_s
        self.owner_id = owner or uuid.uuid4().hex
        self.session: Optional[str] = None

    def acquire(self, blocking: bool = True, timeout: Optional[float] = None, poll: float = 0.1) -> bool:
        deadline = None if timeout is None else time.time() + timeout
        while True:
            if self.session is None or not self.c.session_renew(self.session):
                self.session = self.c.session_create(self.key, self.ttl_s)
            if self.c.kv_put(self.key, self.owner_id.encode(), acquire=self.session):
                return True
            if not blocking or (deadline is not None and time.time() > deadline):
                return False
            time.sleep(poll)

    def renew(self) -> bool:
        return self.session is not None and self.c.session_renew(self.session) and \
            self.c.kv_session(self.key) == self.session

    def release(self) -> bool:
        if self.session is None:
            return False
        ok = self.c.kv_put(self.key, b"", release=self.session)
        self.c.session_destroy(self.session)
        self.session = None
        return ok

    def owner(self) -> Optional[str]:
        if self.c.kv_session(self.key) is None:
            return None
        v = self.c.kv_get(self.key)
        return v.decode() if v else None

    def __enter__(self):
        self.acquire()
        return self

    def __exit__(self, *exc):
        self.release()


class ConsulLeaderElection:
    """Leader election over a ConsulLock: ``step()`` tries to take or keep leadership; a
    background loop (``start``) renews at a third of the TTL; a leader whose session expires
    (crash, partition) loses the key and another candidate takes it."""

    def __init__(self, client: ConsulClient, name: str, candidate_id: Optional[str] = None, ttl_s: int = 15,
                 on_elected=None, on_demoted=None):
        self.lock = ConsulLock(client, f"leader/{name}", ttl_s, candidate_id)
        self.on_elected, self.on_demoted = on_elected, on_demoted
        self._leader = False
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None

    @property
    def candidate_id(self) -> str:
        return self.lock.owner_id

    def is_leader(self) -> bool:
        return self._leader

    def leader(self) -> Optional[str]:
        return self.lock.owner()

    def step(self) -> bool:
        was = self._leader
        self._leader = self.lock.renew() if was else self.lock.acquire(blocking=False)
        if self._leader and not was and self.on_elected:
            self.on_elected()
        if was and not self._leader and self.on_demoted:
            self.on_demoted()
        return self._leader

    def start(self):
        def loop():
            while not self._stop.is_set():
                try:
                    self.step()
                except Exception:            # noqa: BLE001 - consul briefly unreachable: retry
                    pass
                self._stop.wait(max(0.05, self.lock.ttl_s / 3))
        self._thread = threading.Thread(target=loop, daemon=True)
        self._thread.start()

    def resign(self):
        self._stop.set()
        if self._thread:
            self._thread.join(5)
        if self._leader:
            # stop acting as leader before the lock is handed over
            self._leader = False
            if self.on_demoted:
                self.on_demoted()
            self.lock.release()


def service_dns_name(service: str, tag: Optional[str] = None, domain: str = "consul") -> str:
    """Consul DNS name of a service (``[tag.]service.service.<domain>``)."""
    return f"{tag + '.' if tag else ''}{service}.service.{domain}"
