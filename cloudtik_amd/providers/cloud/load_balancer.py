"""Cloud load balancers for a workspace (reference providers/_private/aws/load_balancer_*.py,
gcp/load_balancer_*.py, _azure/load_balancer_*.py; contract core/provider_api.py
``LoadBalancerProvider``; planning in core/load_balancer.py).

Every provider takes the load balancer config the manager plans (service groups of
listeners + services with IP targets) and makes the cloud match it -- create what is
missing, change what differs, remove what is no longer planned -- so ``update`` is the same
reconcile as ``create``:

* **AWS** (ELBv2 over a boto3 client): a network or application load balancer in the
  workspace subnets (public ones for internet-facing, private ones for internal); one IP
  target group per service (targets registered / deregistered by diff); one listener per
  service group; on application load balancers, path rules (``/abc`` -> ``/abc``,
  ``/abc/*``) in route-length order and the default service as the default action
  (else a fixed 404).  Target groups carry a per-load-balancer name prefix, so the ones a
  removed service leaves behind are found and deleted.
* **GCP** (Compute REST, regional managed proxies): per service a zonal NEG of
  ``GCE_VM_IP_PORT`` endpoints (attach / detach by diff), a regional health check and a
  regional backend service; per listener a forwarding rule onto a regional target TCP proxy
  (network) or a target HTTP proxy + URL map with path rules and prefix rewrite
  (application).  Load balancers are found by the forwarding rules' JSON description.
* **Azure** (ARM REST): network -> a Standard ``loadBalancers`` resource (frontend public IP
  or private subnet address, one IP-addressed backend pool + probe per service, one rule
  per listener); application -> an ``applicationGateways`` Standard_v2 resource (frontend
  port + HTTP listener per service group, pool + HTTP settings per service with the service
  path override, a URL path map per listener, path-based routing rules).  Found by tags.
"""
from __future__ import annotations

import hashlib
import json
import re
import time
from typing import Any, Dict, List, Optional, Tuple

from cloudtik_amd.core.load_balancer import SCHEME_INTERNET_FACING, TYPE_APPLICATION, TYPE_NETWORK
from cloudtik_amd.core.provider_api import LoadBalancerProvider
from cloudtik_amd.providers.cloud.rest_providers import CloudAPIError

WS_TAG = "cloudtik-workspace"
LB_TAG = "cloudtik-load-balancer"


def _h(*parts, n: int = 6) -> str:
    return hashlib.sha1("/".join(str(p) for p in parts).encode()).hexdigest()[:n]


def _paths(route: str) -> List[str]:
    """Path patterns of a route: "/" -> everything, "/abc/" -> only below it, "/abc" -> both."""
    if route == "/":
        return ["/*"]
    if route.endswith("/"):
        return [route + "*"]
    return [route, route + "/*"]


def _by_route(services: List[Dict[str, Any]]) -> Tuple[Optional[Dict[str, Any]], List[Dict[str, Any]]]:
    """(default service, the routed ones longest route first)."""
    default = next((s for s in services if s.get("default")), None) or \
        next((s for s in services if s.get("route_path", "/") == "/"), None)
    routed = [s for s in services if s is not default and s.get("route_path", "/") != "/"]
    return default, sorted(routed, key=lambda s: (-len(s["route_path"]), s["name"]))


# =============================================================================== AWS
class AWSLoadBalancerProvider(LoadBalancerProvider):
    def __init__(self, provider_config: Dict[str, Any], workspace_name: str, client_factory=None):
        super().__init__(provider_config, workspace_name)
        if client_factory is None:
            import boto3
            client_factory = lambda svc: boto3.client(svc, region_name=provider_config["region"])  # noqa: E731
        self.elb = client_factory("elbv2")
        self._factory = client_factory
        self._net: Optional[Dict[str, Any]] = None

    # -------------------------------------------------------------- workspace network
    def _network(self) -> Dict[str, Any]:
        if self._net is None:
            c = self.provider_config
            if c.get("vpc_id"):
                self._net = {"vpc": c["vpc_id"], "public": c.get("public_subnet_ids") or c.get("subnet_ids", []),
                             "private": c.get("private_subnet_ids") or c.get("subnet_ids", []),
                             "security_groups": c.get("security_group_ids", [])}
            else:
                from cloudtik_amd.providers.cloud.workspace import AWSWorkspace
                ws = AWSWorkspace(c, self.workspace_name, self._factory)

                def subnets(kind):
                    out = ws.ec2.describe_subnets(Filters=ws._filters([{"Name": "tag:cloudtik-subnet",
                                                                        "Values": [kind]}]))["Subnets"]
                    return [s["SubnetId"] for s in out]
                sg = ws._sg()
                self._net = {"vpc": ws._vpc_id(), "public": subnets("public"), "private": subnets("private"),
                             "security_groups": [sg] if sg else []}
        return self._net

    # -------------------------------------------------------------- helpers
    def _prefix(self, lb_name: str) -> str:
        return "ct" + _h(self.workspace_name, lb_name, n=8)

    def _tg_name(self, lb_name: str, svc: Dict[str, Any]) -> str:
        base = re.sub(r"[^A-Za-z0-9-]", "-", svc["name"])[:14].strip("-")
        return f"{self._prefix(lb_name)}-{base}-{_h(svc['name'], svc['protocol'], svc['port'], n=4)}"[:32]

    def _all(self, call, key, **kw):
        out, marker = [], None
        while True:
            r = call(**kw, **({"Marker": marker} if marker else {}))
            out += r.get(key, [])
            marker = r.get("NextMarker")
            if not marker:
                return out

    def _lb(self, name: str) -> Optional[Dict[str, Any]]:
        try:
            r = self.elb.describe_load_balancers(Names=[name])["LoadBalancers"]
        except Exception as e:  # noqa: BLE001 - LoadBalancerNotFound
            if "NotFound" in type(e).__name__ or "NotFound" in str(e):
                return None
            raise
        return r[0] if r else None

    # -------------------------------------------------------------- contract
    def list(self):
        lbs = self._all(self.elb.describe_load_balancers, "LoadBalancers")
        out = {}
        for i in range(0, len(lbs), 20):
            chunk = lbs[i:i + 20]
            descs = self.elb.describe_tags(ResourceArns=[lb["LoadBalancerArn"] for lb in chunk])["TagDescriptions"]
            tags = {d["ResourceArn"]: {t["Key"]: t["Value"] for t in d["Tags"]} for d in descs}
            for lb in chunk:
                t = tags.get(lb["LoadBalancerArn"], {})
                if t.get(WS_TAG) == self.workspace_name:
                    out[lb["LoadBalancerName"]] = {
                        "name": lb["LoadBalancerName"], "type": lb["Type"], "scheme": lb["Scheme"],
                        "tags": {k: v for k, v in t.items() if k != WS_TAG}, "id": lb["LoadBalancerArn"],
                        "dns_name": lb.get("DNSName")}
        return out

    def create(self, cfg):
        net = self._network()
        scheme = cfg.get("scheme", SCHEME_INTERNET_FACING)
        subnets = net["public" if scheme == SCHEME_INTERNET_FACING else "private"]
        tags = [{"Key": WS_TAG, "Value": self.workspace_name}] + \
            [{"Key": k, "Value": str(v)} for k, v in (cfg.get("tags") or {}).items()]
        kw = dict(Name=cfg["name"], Subnets=subnets, Scheme=scheme, Type=cfg["type"], Tags=tags)
        if cfg["type"] == TYPE_APPLICATION and net["security_groups"]:
            kw["SecurityGroups"] = net["security_groups"]
        arn = self.elb.create_load_balancer(**kw)["LoadBalancers"][0]["LoadBalancerArn"]
        self.elb.get_waiter("load_balancer_available").wait(LoadBalancerArns=[arn])
        self._sync(arn, cfg)

    def update(self, load_balancer, cfg):
        arn = load_balancer.get("id") or self._lb(cfg["name"])["LoadBalancerArn"]
        self._sync(arn, cfg)

    def delete(self, load_balancer):
        lb = self._lb(load_balancer["name"])
        if lb is None:
            return
        arn = lb["LoadBalancerArn"]
        for ls in self._all(self.elb.describe_listeners, "Listeners", LoadBalancerArn=arn):
            self.elb.delete_listener(ListenerArn=ls["ListenerArn"])
        self.elb.delete_load_balancer(LoadBalancerArn=arn)
        self.elb.get_waiter("load_balancers_deleted").wait(LoadBalancerArns=[arn])
        self._drop_target_groups(load_balancer["name"], keep=set())

    # -------------------------------------------------------------- reconcile
    def _target_group(self, lb_name: str, svc: Dict[str, Any]) -> str:
        name = self._tg_name(lb_name, svc)
        try:
            found = self.elb.describe_target_groups(Names=[name])["TargetGroups"]
        except Exception as e:  # noqa: BLE001 - TargetGroupNotFound
            if "NotFound" not in type(e).__name__ and "NotFound" not in str(e):
                raise
            found = []
        if found:
            arn = found[0]["TargetGroupArn"]
        else:
            arn = self.elb.create_target_group(
                Name=name, Protocol=svc["protocol"], Port=int(svc["port"]), VpcId=self._network()["vpc"],
                TargetType="ip", HealthCheckProtocol="TCP" if svc["protocol"] in ("TCP", "TLS", "UDP") else "HTTP",
                Tags=[{"Key": WS_TAG, "Value": self.workspace_name}, {"Key": LB_TAG, "Value": lb_name}],
            )["TargetGroups"][0]["TargetGroupArn"]
        want = {(t["address"], int(t["port"])) for t in svc["targets"]}
        have = {(d["Target"]["Id"], int(d["Target"]["Port"]))
                for d in self.elb.describe_target_health(TargetGroupArn=arn)["TargetHealthDescriptions"]}
        if want - have:
            self.elb.register_targets(TargetGroupArn=arn, Targets=[{"Id": a, "Port": p} for a, p in sorted(want - have)])
        if have - want:
            self.elb.deregister_targets(TargetGroupArn=arn,
                                        Targets=[{"Id": a, "Port": p} for a, p in sorted(have - want)])
        return arn

    def _drop_target_groups(self, lb_name: str, keep: set):
        prefix = self._prefix(lb_name) + "-"
        for tg in self._all(self.elb.describe_target_groups, "TargetGroups"):
            if tg["TargetGroupName"].startswith(prefix) and tg["TargetGroupArn"] not in keep:
                self.elb.delete_target_group(TargetGroupArn=tg["TargetGroupArn"])

    def _sync(self, arn: str, cfg: Dict[str, Any]):
        name = cfg["name"]
        listeners = {(ls["Protocol"], int(ls["Port"])): ls
                     for ls in self._all(self.elb.describe_listeners, "Listeners", LoadBalancerArn=arn)}
        used = set()
        for g in cfg["service_groups"]:
            tgs = {s["name"]: self._target_group(name, s) for s in g["services"]}
            used |= set(tgs.values())
            for ls in g["listeners"]:
                key = (ls["protocol"], int(ls["port"]))
                if cfg["type"] == TYPE_NETWORK:
                    default = {"Type": "forward", "TargetGroupArn": tgs[g["services"][0]["name"]]}
                    routed = []
                else:
                    dsvc, routed = _by_route(g["services"])
                    default = {"Type": "forward", "TargetGroupArn": tgs[dsvc["name"]]} if dsvc else \
                        {"Type": "fixed-response", "FixedResponseConfig": {"StatusCode": "404",
                                                                           "ContentType": "text/plain"}}
                if key in listeners:
                    la = listeners.pop(key)["ListenerArn"]
                    self.elb.modify_listener(ListenerArn=la, DefaultActions=[default])
                else:
                    la = self.elb.create_listener(LoadBalancerArn=arn, Protocol=key[0], Port=key[1],
                                                  DefaultActions=[default])["Listeners"][0]["ListenerArn"]
                self._sync_rules(la, [(s, tgs[s["name"]]) for s in routed])
        for ls in listeners.values():          # listeners of removed service groups
            self.elb.delete_listener(ListenerArn=ls["ListenerArn"])
        self._drop_target_groups(name, keep=used)

    def _sync_rules(self, listener_arn: str, routed: List[Tuple[Dict[str, Any], str]]):
        want = {}
        for prio, (s, tg) in enumerate(routed, 1):
            want[(prio, tuple(_paths(s["route_path"])), tg)] = s
        have = {}
        for r in self.elb.describe_rules(ListenerArn=listener_arn)["Rules"]:
            if r.get("IsDefault"):
                continue
            paths = tuple(v for c in r["Conditions"] if c["Field"] == "path-pattern" for v in c["Values"])
            tg = r["Actions"][0].get("TargetGroupArn")
            have[(int(r["Priority"]), paths, tg)] = r["RuleArn"]
        for k, rarn in have.items():
            if k not in want:
                self.elb.delete_rule(RuleArn=rarn)
        for (prio, paths, tg) in want:
            if (prio, paths, tg) not in have:
                self.elb.create_rule(ListenerArn=listener_arn, Priority=prio,
                                     Conditions=[{"Field": "path-pattern", "Values": list(paths)}],
                                     Actions=[{"Type": "forward", "TargetGroupArn": tg}])


# =============================================================================== GCP
_GCE = "https://compute.googleapis.com/compute/v1"


def _gname(*parts) -> str:
    n = re.sub(r"[^a-z0-9-]", "-", "-".join(str(p) for p in parts).lower()).strip("-")
    if len(n) > 63:
        n = n[:56].rstrip("-") + "-" + _h(n)
    return n if n[0].isalpha() else "lb-" + n[:60]


class GCPLoadBalancerProvider(LoadBalancerProvider):
    def __init__(self, provider_config: Dict[str, Any], workspace_name: str, call, poll_s: float = 2.0):
        super().__init__(provider_config, workspace_name)
        self.project = provider_config["project_id"]
        self.region = provider_config["region"]
        self.zone = provider_config.get("availability_zone") or f"{self.region}-a"
        self.call = call
        self.poll_s = float(provider_config.get("poll_interval_s", poll_s))
        from cloudtik_amd.providers.cloud.workspace import GCPWorkspace
        ws = GCPWorkspace(dict(provider_config, project_id=self.project, region=self.region), workspace_name, call)
        self.network = provider_config.get("network") or ws._vpc_link()
        self.subnets = {k: self._p(f"regions/{self.region}/subnetworks/{v}") for k, v in ws.subnets.items()}

    def _p(self, path: str) -> str:
        return f"{_GCE}/projects/{self.project}/{path}"

    def _n(self, lb: str, *parts) -> str:
        """Resource name: a per-load-balancer hashed prefix (so one load balancer's leftovers
        are found by prefix without matching another's) + readable parts."""
        return _gname("ct" + _h(self.workspace_name, lb, n=8), *parts)

    def _r(self, coll: str, name: str = "") -> str:
        return self._p(f"regions/{self.region}/{coll}" + (f"/{name}" if name else ""))

    def _wait(self, op):
        if not isinstance(op, dict) or "status" not in op or "selfLink" not in op:
            return op
        deadline = time.time() + 900
        while op.get("status") != "DONE":
            if time.time() > deadline:
                raise CloudAPIError(504, f"operation {op.get('name')} timed out")
            time.sleep(self.poll_s)
            op = self.call("GET", op["selfLink"], None, None)
        if op.get("error"):
            raise CloudAPIError(400, str(op["error"])[:500])
        return op

    def _get(self, url: str) -> Optional[Dict[str, Any]]:
        try:
            return self.call("GET", url, None, None)
        except CloudAPIError as e:
            if e.status == 404:
                return None
            raise

    def _items(self, url: str) -> List[Dict[str, Any]]:
        out, token = [], None
        while True:
            r = self.call("GET", url, {"pageToken": token} if token else None, None) or {}
            out += r.get("items", [])
            token = r.get("nextPageToken")
            if not token:
                return out

    def _ensure(self, coll_url: str, body: Dict[str, Any], compare: Tuple[str, ...] = ()) -> str:
        """Create ``body`` in the collection unless it exists; PATCH the ``compare`` fields
        that differ.  Returns the resource URL."""
        url = f"{coll_url}/{body['name']}"
        cur = self._get(url)
        if cur is None:
            self._wait(self.call("POST", coll_url, None, body))
        else:
            diff = {k: body[k] for k in compare if k in body and cur.get(k) != body[k]}
            if diff:
                if "fingerprint" in cur:
                    diff["fingerprint"] = cur["fingerprint"]
                self._wait(self.call("PATCH", url, None, diff))
        return url

    def _scheme(self, cfg) -> str:
        return "EXTERNAL_MANAGED" if cfg.get("scheme", SCHEME_INTERNET_FACING) == SCHEME_INTERNET_FACING \
            else "INTERNAL_MANAGED"

    def _desc(self, cfg) -> str:
        return json.dumps({WS_TAG: self.workspace_name, "load_balancer": cfg["name"], "type": cfg["type"],
                           "scheme": cfg.get("scheme", SCHEME_INTERNET_FACING), "tags": cfg.get("tags") or {}},
                          sort_keys=True)

    # -------------------------------------------------------------- contract
    def list(self):
        out = {}
        for fr in self._items(self._r("forwardingRules")):
            try:
                d = json.loads(fr.get("description") or "{}")
            except ValueError:
                continue
            if d.get(WS_TAG) == self.workspace_name and d.get("load_balancer"):
                out[d["load_balancer"]] = {"name": d["load_balancer"], "type": d["type"], "scheme": d["scheme"],
                                           "tags": d.get("tags", {})}
        return out

    def create(self, cfg):
        self._sync(cfg)

    def update(self, load_balancer, cfg):
        self._sync(cfg)

    def delete(self, load_balancer):
        self._sync({"name": load_balancer["name"], "type": load_balancer.get("type", TYPE_NETWORK),
                    "service_groups": []})

    # -------------------------------------------------------------- reconcile
    def _neg(self, lb: str, svc: Dict[str, Any]) -> str:
        coll = self._p(f"zones/{self.zone}/networkEndpointGroups")
        url = self._ensure(coll, {"name": self._n(lb, svc["name"], "neg"), "networkEndpointType": "GCE_VM_IP_PORT",
                                  "network": self.network, "subnetwork": self.subnets["private"],
                                  "defaultPort": int(svc["port"])})
        have = {}
        for e in self.call("POST", f"{url}/listNetworkEndpoints", None, {}).get("items", []):
            ep = e["networkEndpoint"]
            have[(ep["ipAddress"], int(ep["port"]))] = ep
        want = {}
        for t in svc["targets"]:
            ep = {"ipAddress": t["address"], "port": int(t["port"])}
            if t.get("node_id"):
                ep["instance"] = t["node_id"]
            want[(t["address"], int(t["port"]))] = ep
        if set(want) - set(have):
            self._wait(self.call("POST", f"{url}/attachNetworkEndpoints", None,
                                 {"networkEndpoints": [want[k] for k in sorted(set(want) - set(have))]}))
        if set(have) - set(want):
            self._wait(self.call("POST", f"{url}/detachNetworkEndpoints", None,
                                 {"networkEndpoints": [have[k] for k in sorted(set(have) - set(want))]}))
        return url

    def _backend_service(self, cfg, svc) -> str:
        lb = cfg["name"]
        http = svc["protocol"] in ("HTTP", "HTTPS")
        hc = {"name": self._n(lb, svc["name"], "hc"), "type": "HTTP" if http else "TCP"}
        hc["httpHealthCheck" if http else "tcpHealthCheck"] = {"portSpecification": "USE_SERVING_PORT"}
        hc_url = self._ensure(self._r("healthChecks"), hc)
        neg = self._neg(lb, svc)
        body = {"name": self._n(lb, svc["name"], "bs"), "protocol": svc["protocol"],
                "loadBalancingScheme": self._scheme(cfg), "healthChecks": [hc_url],
                "backends": [{"group": neg, "balancingMode": "RATE" if http else "CONNECTION",
                              ("maxRatePerEndpoint" if http else "maxConnectionsPerEndpoint"): 1000,
                              "capacityScaler": 1.0}]}
        return self._ensure(self._r("backendServices"), body, ("backends", "healthChecks", "protocol"))

    def _url_map(self, name: str, services: List[Dict[str, Any]], bs: Dict[str, str]) -> str:
        default, routed = _by_route(services)
        rules = []
        for s in routed:
            rule = {"paths": _paths(s["route_path"]), "service": bs[s["name"]]}
            if s.get("service_path") is not None:
                rule["routeAction"] = {"urlRewrite": {"pathPrefixRewrite": s["service_path"] or "/"}}
            rules.append(rule)
        fallback = bs[(default or services[0])["name"]]
        body = {"name": name, "defaultService": fallback,
                "hostRules": [{"hosts": ["*"], "pathMatcher": "paths"}],
                "pathMatchers": [{"name": "paths", "defaultService": fallback, "pathRules": rules}]}
        return self._ensure(self._r("urlMaps"), body, ("defaultService", "pathMatchers", "hostRules"))

    def _sync(self, cfg: Dict[str, Any]):
        lb = cfg["name"]
        keep: Dict[str, set] = {c: set() for c in ("forwardingRules", "targetTcpProxies", "targetHttpProxies",
                                                   "urlMaps", "backendServices", "healthChecks", "neg")}
        for g in cfg["service_groups"]:
            bs = {}
            for s in g["services"]:
                bs[s["name"]] = self._backend_service(cfg, s)
                keep["backendServices"].add(self._n(lb, s["name"], "bs"))
                keep["healthChecks"].add(self._n(lb, s["name"], "hc"))
                keep["neg"].add(self._n(lb, s["name"], "neg"))
            for ls in g["listeners"]:
                port = int(ls["port"])
                if cfg["type"] == TYPE_NETWORK:
                    pname = self._n(lb, port, "tp")
                    target = self._ensure(self._r("targetTcpProxies"),
                                          {"name": pname, "service": bs[g["services"][0]["name"]]}, ("service",))
                    keep["targetTcpProxies"].add(pname)
                else:
                    um = self._url_map(self._n(lb, port, "um"), g["services"], bs)
                    keep["urlMaps"].add(self._n(lb, port, "um"))
                    pname = self._n(lb, port, "hp")
                    target = self._ensure(self._r("targetHttpProxies"), {"name": pname, "urlMap": um}, ("urlMap",))
                    keep["targetHttpProxies"].add(pname)
                fr = {"name": self._n(lb, port, "fr"), "portRange": str(port), "IPProtocol": "TCP", "target": target,
                      "loadBalancingScheme": self._scheme(cfg), "network": self.network,
                      "networkTier": "PREMIUM" if cfg.get("scheme") == SCHEME_INTERNET_FACING else "STANDARD",
                      "description": self._desc(cfg)}
                if self._scheme(cfg) == "INTERNAL_MANAGED":
                    fr["subnetwork"] = self.subnets["private"]
                self._ensure(self._r("forwardingRules"), fr, ("target",))
                keep["forwardingRules"].add(fr["name"])
        # remove what this load balancer no longer uses, users before what they use
        prefix = "ct" + _h(self.workspace_name, lb, n=8) + "-"
        for coll in ("forwardingRules", "targetTcpProxies", "targetHttpProxies", "urlMaps", "backendServices",
                     "healthChecks"):
            for it in self._items(self._r(coll)):
                if it["name"].startswith(prefix) and it["name"] not in keep[coll]:
                    self._wait(self.call("DELETE", self._r(coll, it["name"]), None, None))
        negs = self._p(f"zones/{self.zone}/networkEndpointGroups")
        for it in self._items(negs):
            if it["name"].startswith(prefix) and it["name"] not in keep["neg"]:
                self._wait(self.call("DELETE", f"{negs}/{it['name']}", None, None))


# =============================================================================== Azure
_ARM = "https://management.azure.com"
_NET_API = "2023-04-01"


class AzureLoadBalancerProvider(LoadBalancerProvider):
    def __init__(self, provider_config: Dict[str, Any], workspace_name: str, call, poll_s: float = 5.0):
        super().__init__(provider_config, workspace_name)
        from cloudtik_amd.providers.cloud.workspace import AzureWorkspace
        ws = AzureWorkspace(provider_config, workspace_name, call)
        self.sub, self.rg, self.location = ws.sub, ws.rg, ws.location
        self.vnet_id = f"/subscriptions/{self.sub}/resourceGroups/{self.rg}/providers/Microsoft.Network/" \
                       f"virtualNetworks/{ws.vnet}"
        self.subnet_ids = {k: f"{self.vnet_id}/subnets/{v}" for k, v in ws.subnets.items()}
        self.gateway_subnet = f"{self.vnet_id}/subnets/" + provider_config.get(
            "application_gateway_subnet", f"cloudtik-{workspace_name}-appgw-subnet")
        self.call = call
        self.poll_s = float(provider_config.get("poll_interval_s", poll_s))

    def _id(self, kind: str, name: str) -> str:
        return f"/subscriptions/{self.sub}/resourceGroups/{self.rg}/providers/Microsoft.Network/{kind}/{name}"

    def _url(self, kind: str, name: str = "") -> str:
        return _ARM + (self._id(kind, name) if name else
                       f"/subscriptions/{self.sub}/resourceGroups/{self.rg}/providers/Microsoft.Network/{kind}")

    def _put(self, kind: str, name: str, body: Dict[str, Any]):
        url = self._url(kind, name)
        out = self.call("PUT", url, {"api-version": _NET_API}, body)
        deadline = time.time() + 1800
        while (out or {}).get("properties", {}).get("provisioningState") not in (None, "Succeeded"):
            if out["properties"]["provisioningState"] in ("Failed", "Canceled"):
                raise CloudAPIError(400, f"{url}: {out['properties']['provisioningState']}")
            if time.time() > deadline:
                raise CloudAPIError(504, f"{url}: provisioning timed out")
            time.sleep(self.poll_s)
            out = self.call("GET", url, {"api-version": _NET_API}, None)
        return out

    def _del(self, kind: str, name: str):
        try:
            self.call("DELETE", self._url(kind, name), {"api-version": _NET_API}, None)
        except CloudAPIError as e:
            if e.status != 404:
                raise

    def _tags(self, cfg) -> Dict[str, str]:
        return dict({k: str(v) for k, v in (cfg.get("tags") or {}).items()}, **{
            WS_TAG: self.workspace_name, "cloudtik-lb-type": cfg["type"],
            "cloudtik-lb-scheme": cfg.get("scheme", SCHEME_INTERNET_FACING)})

    def _frontend(self, cfg) -> Dict[str, Any]:
        if cfg.get("scheme", SCHEME_INTERNET_FACING) == SCHEME_INTERNET_FACING:
            ip = f"{cfg['name']}-ip"
            self._put("publicIPAddresses", ip, {"location": self.location, "sku": {"name": "Standard"},
                                                "properties": {"publicIPAllocationMethod": "Static"},
                                                "tags": {WS_TAG: self.workspace_name}})
            return {"publicIPAddress": {"id": self._id("publicIPAddresses", ip)}}
        return {"subnet": {"id": self.subnet_ids["private"]}, "privateIPAllocationMethod": "Dynamic"}

    # -------------------------------------------------------------- contract
    def list(self):
        out = {}
        for kind in ("loadBalancers", "applicationGateways"):
            for r in (self.call("GET", self._url(kind), {"api-version": _NET_API}, None) or {}).get("value", []):
                t = r.get("tags") or {}
                if t.get(WS_TAG) == self.workspace_name:
                    out[r["name"]] = {"name": r["name"], "type": t.get("cloudtik-lb-type"),
                                      "scheme": t.get("cloudtik-lb-scheme"), "id": r.get("id"),
                                      "tags": {k: v for k, v in t.items() if not k.startswith("cloudtik-lb-")
                                               and k != WS_TAG}}
        return out

    def create(self, cfg):
        if cfg["type"] == TYPE_NETWORK:
            self._put("loadBalancers", cfg["name"], self._network_body(cfg))
        else:
            self._put("applicationGateways", cfg["name"], self._gateway_body(cfg))

    def update(self, load_balancer, cfg):
        self.create(cfg)                       # ARM PUT is a full, idempotent replace

    def delete(self, load_balancer):
        kind = "loadBalancers" if load_balancer.get("type") == TYPE_NETWORK else "applicationGateways"
        self._del(kind, load_balancer["name"])
        if load_balancer.get("scheme", SCHEME_INTERNET_FACING) == SCHEME_INTERNET_FACING:
            self._del("publicIPAddresses", f"{load_balancer['name']}-ip")

    # -------------------------------------------------------------- bodies
    def _network_body(self, cfg) -> Dict[str, Any]:
        lb_id = self._id("loadBalancers", cfg["name"])
        pools, probes, rules = [], [], []
        for g in cfg["service_groups"]:
            for s in g["services"]:
                pools.append({"name": s["name"], "properties": {"loadBalancerBackendAddresses": [
                    {"name": f"{t['address']}-{t['port']}", "properties": {
                        "ipAddress": t["address"], "virtualNetwork": {"id": self.vnet_id}}}
                    for t in s["targets"]]}})
                probes.append({"name": f"{s['name']}-probe", "properties": {
                    "protocol": "Tcp", "port": int(s["port"]), "intervalInSeconds": 5, "numberOfProbes": 2}})
            s = g["services"][0]
            for ls in g["listeners"]:
                rules.append({"name": f"{s['name']}-{ls['port']}", "properties": {
                    "protocol": "Udp" if ls["protocol"] == "UDP" else "Tcp", "frontendPort": int(ls["port"]),
                    "backendPort": int(s["port"]), "enableFloatingIP": False, "idleTimeoutInMinutes": 4,
                    "frontendIPConfiguration": {"id": f"{lb_id}/frontendIPConfigurations/frontend"},
                    "backendAddressPool": {"id": f"{lb_id}/backendAddressPools/{s['name']}"},
                    "probe": {"id": f"{lb_id}/probes/{s['name']}-probe"}}})
        return {"location": self.location, "sku": {"name": "Standard"}, "tags": self._tags(cfg), "properties": {
            "frontendIPConfigurations": [{"name": "frontend", "properties": self._frontend(cfg)}],
            "backendAddressPools": pools, "probes": probes, "loadBalancingRules": rules}}

    def _gateway_body(self, cfg) -> Dict[str, Any]:
        gw = self._id("applicationGateways", cfg["name"])
        ports, listeners, pools, settings, maps, routing = [], [], [], [], [], []
        prio = 100
        for g in cfg["service_groups"]:
            for s in g["services"]:
                pools.append({"name": s["name"], "properties": {"backendAddresses": [
                    {"ipAddress": t["address"]} for t in s["targets"]]}})
                st = {"port": int(s["port"]), "protocol": "Https" if s["protocol"] == "HTTPS" else "Http",
                      "cookieBasedAffinity": "Disabled", "requestTimeout": 60}
                if s.get("service_path") is not None:
                    st["path"] = (s["service_path"] or "") + "/"
                settings.append({"name": f"{s['name']}-settings", "properties": st})
            default, routed = _by_route(g["services"])
            fallback = (default or g["services"][0])["name"]
            for ls in g["listeners"]:
                port = int(ls["port"])
                ports.append({"name": f"port-{port}", "properties": {"port": port}})
                listeners.append({"name": f"listener-{port}", "properties": {
                    "frontendIPConfiguration": {"id": f"{gw}/frontendIPConfigurations/frontend"},
                    "frontendPort": {"id": f"{gw}/frontendPorts/port-{port}"},
                    "protocol": "Https" if ls["protocol"] == "HTTPS" else "Http"}})
                maps.append({"name": f"paths-{port}", "properties": {
                    "defaultBackendAddressPool": {"id": f"{gw}/backendAddressPools/{fallback}"},
                    "defaultBackendHttpSettings": {"id": f"{gw}/backendHttpSettingsCollection/{fallback}-settings"},
                    "pathRules": [{"name": s["name"], "properties": {
                        "paths": _paths(s["route_path"]),
                        "backendAddressPool": {"id": f"{gw}/backendAddressPools/{s['name']}"},
                        "backendHttpSettings": {"id": f"{gw}/backendHttpSettingsCollection/{s['name']}-settings"}}}
                        for s in routed]}})
                routing.append({"name": f"rule-{port}", "properties": {
                    "ruleType": "PathBasedRouting", "priority": prio,
                    "httpListener": {"id": f"{gw}/httpListeners/listener-{port}"},
                    "urlPathMap": {"id": f"{gw}/urlPathMaps/paths-{port}"}}})
                prio += 10
        return {"location": self.location, "tags": self._tags(cfg), "properties": {
            "sku": {"name": "Standard_v2", "tier": "Standard_v2",
                    "capacity": int(self.provider_config.get("application_gateway_capacity", 2))},
            "gatewayIPConfigurations": [{"name": "gateway", "properties": {"subnet": {"id": self.gateway_subnet}}}],
            "frontendIPConfigurations": [{"name": "frontend", "properties": self._frontend(cfg)}],
            "frontendPorts": ports, "httpListeners": listeners, "backendAddressPools": pools,
            "backendHttpSettingsCollection": settings, "urlPathMaps": maps, "requestRoutingRules": routing}}


def cloud_load_balancer_provider(provider_config: Dict[str, Any], workspace_name: str, transport=None):
    t = provider_config.get("type")
    if t == "aws":
        return AWSLoadBalancerProvider(provider_config, workspace_name,
                                       transport or provider_config.get("_client_factory"))
    from cloudtik_amd.providers.cloud.rest_providers import requests_transport
    call = transport or provider_config.get("_transport")
    if t == "gcp":
        if call is None:
            from cloudtik_amd.providers.cloud.rest_providers import GCPNodeProvider
            tok = GCPNodeProvider.__new__(GCPNodeProvider)
            tok.provider_config = provider_config
            call = requests_transport(tok._token)
        return GCPLoadBalancerProvider(provider_config, workspace_name, call)
    if t == "azure":
        if call is None:
            from cloudtik_amd.providers.cloud.rest_providers import AzureNodeProvider
            tok = AzureNodeProvider.__new__(AzureNodeProvider)
            tok.provider_config = provider_config
            call = requests_transport(tok._token)
        return AzureLoadBalancerProvider(provider_config, workspace_name, call)
    raise ValueError(f"no cloud load balancer for provider type {t!r}")


__all__ = ["AWSLoadBalancerProvider", "GCPLoadBalancerProvider", "AzureLoadBalancerProvider",
           "cloud_load_balancer_provider"]
