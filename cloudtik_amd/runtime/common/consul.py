"""Consul HTTP API client for service discovery (reference runtime/common/service_discovery/
consul.py: catalog queries used to resolve runtime services and DNS names).

Only the agent/catalog/KV endpoints the platform uses, over urllib (no SDK): list services,
nodes of a service (optionally filtered by tag), register / deregister a local service with
a TCP or HTTP health check, and KV get / put.
"""
from __future__ import annotations

import base64
import json
import urllib.parse
import urllib.request
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

    # ---------------------------------------------------------------- agent
    def register_service(self, name: str, port: int, address: Optional[str] = None, tags: Optional[List[str]] = None,
                         service_id: Optional[str] = None, check_http: Optional[str] = None,
                         check_interval: str = "10s", meta: Optional[Dict[str, str]] = None):
        body: Dict[str, Any] = {"Name": name, "ID": service_id or name, "Port": int(port), "Tags": tags or [],
                                "Meta": meta or {}}
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

    def kv_put(self, key: str, value: bytes) -> bool:
        return bool(self._req("PUT", f"kv/{key}", body=value if isinstance(value, bytes) else str(value).encode()))


def service_dns_name(service: str, tag: Optional[str] = None, domain: str = "consul") -> str:
    """Consul DNS name of a service (``[tag.]service.service.<domain>``)."""
    return f"{tag + '.' if tag else ''}{service}.service.{domain}"
