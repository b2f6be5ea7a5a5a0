"""Load balancers (core/load_balancer.py, providers/cloud/load_balancer.py; reference
runtime/loadbalancer/{provider_api,controller}.py, providers/_private/{aws,gcp,_azure}/
load_balancer_*.py, tests/unit/runtime/test_load_balancer.py): planning of named / unnamed
services into network and application load balancers, reconcile (create / no-op / update /
delete-auto-empty), the HAProxy provider's rendered config, the AWS / GCP / Azure providers
against in-memory fakes of their APIs, the controller pull job and the runtime."""
import json
import os
import re

import pytest

from cloudtik_amd.core import load_balancer as LB
from cloudtik_amd.core.provider_api import LoadBalancerProvider
from cloudtik_amd.providers.cloud.load_balancer import (AWSLoadBalancerProvider, AzureLoadBalancerProvider,
                                                        GCPLoadBalancerProvider)
from cloudtik_amd.providers.cloud.rest_providers import CloudAPIError

SERVERS = ["10.0.0.1:1234", "10.0.0.2:1234", "10.0.0.3:1234"]


def svc(protocol, port, lb_port, lb_name=None, **kw):
    d = {"protocol": protocol, "port": port, "load_balancer_port": lb_port, "servers": list(SERVERS), **kw}
    if lb_name:
        d["load_balancer_name"] = lb_name
    return d


BACKEND = {"services": {
    "a-1": svc("TCP", 1000, 100, "lb-a"), "a-2": svc("TCP", 1000, 110, "lb-a"),
    "b-1": svc("HTTP", 8080, 80, "lb-b"), "b-2": svc("HTTP", 8090, 80, "lb-b"),
    "b-3": svc("HTTP", 8080, 81, "lb-b"), "b-4": svc("HTTP", 8090, 81, "lb-b"),
    "c-1": svc("TCP", 1000, 100), "c-2": svc("TCP", 1000, 110),
    "d-1": svc("HTTP", 8080, 80), "d-2": svc("HTTP", 8080, 80),
    "d-3": svc("HTTP", 8080, 81), "d-4": svc("HTTP", 8080, 81),
}}


class MemoryProvider(LoadBalancerProvider):
    def __init__(self, multi=True):
        super().__init__({}, "ws")
        self.multi = multi
        self.lbs = {}
        self.calls = []

    def support_multi_service_group(self):
        return self.multi

    def list(self):
        return {n: {k: v[k] for k in ("name", "type", "scheme", "tags")} for n, v in self.lbs.items()}

    def create(self, cfg):
        self.calls.append(("create", cfg["name"]))
        self.lbs[cfg["name"]] = cfg

    def update(self, lb, cfg):
        self.calls.append(("update", cfg["name"]))
        self.lbs[cfg["name"]] = cfg

    def delete(self, lb):
        self.calls.append(("delete", lb["name"]))
        self.lbs.pop(lb["name"])


def _shape(lb):
    return [len(g["services"]) for g in lb["service_groups"]]


def test_plan_multi_service_group():
    p = MemoryProvider()
    m = LB.LoadBalancerManager({}, "ws", provider=p)
    m.update(LB.backend_services_from_config(BACKEND))
    assert set(p.lbs) == {"lb-a", "lb-b", "ws-n", "ws-a"}
    assert p.lbs["lb-a"]["type"] == "network" and _shape(p.lbs["lb-a"]) == [1, 1]
    assert p.lbs["lb-b"]["type"] == "application" and _shape(p.lbs["lb-b"]) == [2, 2]
    assert p.lbs["ws-n"]["type"] == "network" and _shape(p.lbs["ws-n"]) == [1, 1]
    assert p.lbs["ws-a"]["type"] == "application" and _shape(p.lbs["ws-a"]) == [2, 2]
    g = p.lbs["lb-b"]["service_groups"][0]
    assert g["listeners"] == [{"protocol": "HTTP", "port": 80}]
    assert [s["route_path"] for s in g["services"]] == ["/b-1", "/b-2"]
    assert [t["address"] for t in g["services"][0]["targets"]] == ["10.0.0.1", "10.0.0.2", "10.0.0.3"]
    assert p.lbs["lb-a"]["tags"] == {LB.AUTO_CREATED_TAG: "true"}


def test_plan_single_service_group():
    cfg = {"services": {k: v for k, v in BACKEND["services"].items() if k not in ("a-2", "b-3", "b-4")}}
    p = MemoryProvider(multi=False)
    LB.LoadBalancerManager({}, "ws", provider=p).update(LB.backend_services_from_config(cfg))
    assert set(p.lbs) == {"lb-a", "lb-b", "c-1", "c-2", "ws-HTTP-80", "ws-HTTP-81"}
    assert _shape(p.lbs["lb-b"]) == [2] and _shape(p.lbs["c-1"]) == [1] and _shape(p.lbs["ws-HTTP-81"]) == [2]


def test_conflicting_named_lb_is_skipped_not_fatal():
    cfg = {"services": {"x": svc("TCP", 1, 100, "mix"), "y": svc("HTTP", 2, 80, "mix"),
                        "z": svc("TCP", 3, 200, "ok")}}
    p = MemoryProvider()
    LB.LoadBalancerManager({}, "ws", provider=p).update(LB.backend_services_from_config(cfg))
    assert set(p.lbs) == {"ok"}


def test_reconcile_noop_update_delete():
    p = MemoryProvider()
    m = LB.LoadBalancerManager({}, "ws", provider=p)
    cfg = {"services": {"web": svc("HTTP", 8080, 80, "site"), "db": svc("TCP", 5432, 5432)}}
    assert m.update(LB.backend_services_from_config(cfg))["created"] == ["site", "ws-n"]
    assert m.update(LB.backend_services_from_config(cfg)) == {"created": [], "updated": [], "deleted": []}
    cfg["services"]["web"]["servers"] = SERVERS[:2]
    assert m.update(LB.backend_services_from_config(cfg))["updated"] == ["site"]
    del cfg["services"]["db"]
    p.lbs["manual"] = {"name": "manual", "type": "network", "scheme": "internal", "tags": {}}
    done = m.update(LB.backend_services_from_config(cfg))
    assert done["deleted"] == ["ws-n"] and "manual" in p.lbs        # user-made load balancers are kept


def test_route_and_service_paths():
    s = LB.BackendService("api", {("h", 1): {"address": "h", "port": 1}}, "http", route_path="v1/",
                          service_path="/")
    assert s.protocol == "HTTP" and s.get_route_path() == "/v1/" and s.service_path == ""
    d = LB.BackendService("home", {("h", 1): {"address": "h", "port": 1}}, "HTTP", default_service=True)
    assert d.get_route_path() == "/"
    with pytest.raises(ValueError):
        LB.BackendService("x", {("h", 1): {"address": "h", "port": 1}}, port=70000)


def test_haproxy_provider_renders_routes(tmp_path):
    conf = tmp_path / "lb.cfg"
    m = LB.LoadBalancerManager({"type": "haproxy", "config_file": str(conf), "haproxy_bin": "no-such-haproxy"}, "ws")
    cfg = {"services": {
        "api": svc("HTTP", 8080, 80, "site", route_path="/api", service_path="/v2"),
        "home": svc("HTTP", 8000, 80, "site", default_service=True),
        "pg": svc("TCP", 5432, 15432, load_balancer_scheme="internal")}}
    m.update(LB.backend_services_from_config(cfg))
    text = conf.read_text()
    assert "frontend site-http-80\n    bind 0.0.0.0:80\n    mode http" in text
    assert "    acl path_api path /api\n    acl path_api path_beg /api/\n    use_backend site-api if path_api" in text
    assert "    default_backend site-home" in text
    assert "http-request replace-path ^/api/?(.*)$ /v2/\\1" in text
    assert "frontend ws-n-tcp-15432\n    bind 127.0.0.1:15432\n    mode tcp\n    default_backend ws-n-pg" in text
    assert text.count("server s") == 9
    assert set(m.provider.list()) == {"site", "ws-n"}
    del cfg["services"]["pg"]
    m.update(LB.backend_services_from_config(cfg))
    assert "ws-n" not in conf.read_text()


# ======================================================================= AWS ELBv2 fake
class NotFound(Exception):
    pass


class FakeELB:
    def __init__(self):
        self.lbs, self.tgs, self.listeners, self.rules, self.tags, self.n = {}, {}, {}, {}, {}, 0

    def _arn(self, kind):
        self.n += 1
        return f"arn:{kind}/{self.n}"

    def describe_load_balancers(self, Names=None, Marker=None):
        lbs = [lb for lb in self.lbs.values() if not Names or lb["LoadBalancerName"] in Names]
        if Names and not lbs:
            raise NotFound("LoadBalancerNotFound")
        return {"LoadBalancers": lbs}

    def describe_tags(self, ResourceArns):
        return {"TagDescriptions": [{"ResourceArn": a, "Tags": self.tags.get(a, [])} for a in ResourceArns]}

    def create_load_balancer(self, Name, Subnets, Scheme, Type, Tags, SecurityGroups=None):
        assert Subnets, "subnets required"
        arn = self._arn("lb")
        self.lbs[arn] = {"LoadBalancerArn": arn, "LoadBalancerName": Name, "Type": Type, "Scheme": Scheme,
                         "Subnets": Subnets, "SecurityGroups": SecurityGroups}
        self.tags[arn] = Tags
        return {"LoadBalancers": [self.lbs[arn]]}

    def get_waiter(self, name):
        class W:
            def wait(self, **kw):
                pass
        return W()

    def delete_load_balancer(self, LoadBalancerArn):
        assert not [ls for ls in self.listeners.values() if ls["LoadBalancerArn"] == LoadBalancerArn]
        del self.lbs[LoadBalancerArn]

    def describe_target_groups(self, Names=None, Marker=None):
        tgs = [t for t in self.tgs.values() if not Names or t["TargetGroupName"] in Names]
        if Names and not tgs:
            raise NotFound("TargetGroupNotFound")
        return {"TargetGroups": tgs}

    def create_target_group(self, Name, Protocol, Port, VpcId, TargetType, HealthCheckProtocol, Tags):
        assert len(Name) <= 32 and re.match(r"^[A-Za-z0-9][A-Za-z0-9-]*[A-Za-z0-9]$", Name)
        arn = self._arn("tg")
        self.tgs[arn] = {"TargetGroupArn": arn, "TargetGroupName": Name, "Protocol": Protocol, "Port": Port,
                         "Targets": set()}
        return {"TargetGroups": [self.tgs[arn]]}

    def delete_target_group(self, TargetGroupArn):
        for ls in self.listeners.values():
            assert ls["DefaultActions"][0].get("TargetGroupArn") != TargetGroupArn, "target group in use"
        for r in self.rules.values():
            assert r["Actions"][0]["TargetGroupArn"] != TargetGroupArn, "target group in use"
        del self.tgs[TargetGroupArn]

    def describe_target_health(self, TargetGroupArn):
        return {"TargetHealthDescriptions": [{"Target": {"Id": a, "Port": p}}
                                             for a, p in sorted(self.tgs[TargetGroupArn]["Targets"])]}

    def register_targets(self, TargetGroupArn, Targets):
        self.tgs[TargetGroupArn]["Targets"] |= {(t["Id"], t["Port"]) for t in Targets}

    def deregister_targets(self, TargetGroupArn, Targets):
        self.tgs[TargetGroupArn]["Targets"] -= {(t["Id"], t["Port"]) for t in Targets}

    def describe_listeners(self, LoadBalancerArn, Marker=None):
        return {"Listeners": [ls for ls in self.listeners.values() if ls["LoadBalancerArn"] == LoadBalancerArn]}

    def create_listener(self, LoadBalancerArn, Protocol, Port, DefaultActions):
        arn = self._arn("listener")
        self.listeners[arn] = {"ListenerArn": arn, "LoadBalancerArn": LoadBalancerArn, "Protocol": Protocol,
                               "Port": Port, "DefaultActions": DefaultActions}
        return {"Listeners": [self.listeners[arn]]}

    def modify_listener(self, ListenerArn, DefaultActions):
        self.listeners[ListenerArn]["DefaultActions"] = DefaultActions

    def delete_listener(self, ListenerArn):
        del self.listeners[ListenerArn]
        for k in [k for k, r in self.rules.items() if r["ListenerArn"] == ListenerArn]:
            del self.rules[k]

    def describe_rules(self, ListenerArn):
        rules = [dict(r, IsDefault=False) for r in self.rules.values() if r["ListenerArn"] == ListenerArn]
        return {"Rules": rules + [{"RuleArn": "default", "IsDefault": True, "Priority": "default"}]}

    def create_rule(self, ListenerArn, Priority, Conditions, Actions):
        assert not [r for r in self.rules.values() if r["ListenerArn"] == ListenerArn and r["Priority"] == str(Priority)]
        arn = self._arn("rule")
        self.rules[arn] = {"RuleArn": arn, "ListenerArn": ListenerArn, "Priority": str(Priority),
                           "Conditions": Conditions, "Actions": Actions}

    def delete_rule(self, RuleArn):
        del self.rules[RuleArn]


def test_aws_provider_lifecycle():
    elb = FakeELB()
    cfg = {"type": "aws", "region": "us-west-2", "vpc_id": "vpc-1", "public_subnet_ids": ["s-pub1", "s-pub2"],
           "private_subnet_ids": ["s-priv"], "security_group_ids": ["sg-1"]}
    prov = AWSLoadBalancerProvider(cfg, "ws", client_factory=lambda svc: elb)
    m = LB.LoadBalancerManager(cfg, "ws", provider=prov)
    backend = {"services": {
        "api": svc("HTTP", 8080, 80, "site", route_path="/api"),
        "home": svc("HTTP", 8000, 80, "site", default_service=True),
        "docs": svc("HTTP", 8001, 80, "site", route_path="/docs/"),
        "pg": svc("TCP", 5432, 5432, load_balancer_scheme="internal")}}
    m.update(LB.backend_services_from_config(backend))
    lbs = prov.list()
    assert set(lbs) == {"site", "ws-n"} and lbs["ws-n"]["scheme"] == "internal"
    site = next(lb for lb in elb.lbs.values() if lb["LoadBalancerName"] == "site")
    assert site["Subnets"] == ["s-pub1", "s-pub2"] and site["SecurityGroups"] == ["sg-1"]
    assert len(elb.tgs) == 4 and all(len(t["Targets"]) == 3 for t in elb.tgs.values())
    rules = sorted(elb.rules.values(), key=lambda r: int(r["Priority"]))
    assert [r["Conditions"][0]["Values"] for r in rules] == [["/docs/*"], ["/api", "/api/*"]]
    home_tg = next(a for a, t in elb.tgs.items() if "-home-" in t["TargetGroupName"])
    site_ls = next(ls for ls in elb.listeners.values() if ls["LoadBalancerArn"] == site["LoadBalancerArn"])
    assert site_ls["DefaultActions"] == [{"Type": "forward", "TargetGroupArn": home_tg}]
    # drop a backend server and the docs service: targets deregistered, rule + target group removed
    backend["services"]["api"]["servers"] = SERVERS[:1]
    del backend["services"]["docs"]
    assert m.update(LB.backend_services_from_config(backend))["updated"] == ["site"]
    assert len(elb.tgs) == 3 and len(elb.rules) == 1
    api_tg = next(t for t in elb.tgs.values() if "-api-" in t["TargetGroupName"])
    assert api_tg["Targets"] == {("10.0.0.1", 1234)}
    # no services left: both auto-created load balancers and everything under them go
    assert sorted(m.update({})["deleted"]) == ["site", "ws-n"]
    assert not elb.lbs and not elb.tgs and not elb.listeners and not elb.rules


# ======================================================================= GCP fake
class FakeGCP:
    """Compute REST resources keyed by URL; collections list their items; NEG actions."""

    def __init__(self):
        self.res = {}
        self.endpoints = {}

    def __call__(self, method, url, params, body):
        if method == "POST" and url.endswith("/listNetworkEndpoints"):
            neg = url.rsplit("/", 1)[0]
            return {"items": [{"networkEndpoint": e} for e in self.endpoints.get(neg, [])]}
        if method == "POST" and url.endswith("/attachNetworkEndpoints"):
            self.endpoints.setdefault(url.rsplit("/", 1)[0], []).extend(body["networkEndpoints"])
            return {"name": "op"}
        if method == "POST" and url.endswith("/detachNetworkEndpoints"):
            neg = url.rsplit("/", 1)[0]
            drop = {(e["ipAddress"], e["port"]) for e in body["networkEndpoints"]}
            self.endpoints[neg] = [e for e in self.endpoints[neg] if (e["ipAddress"], e["port"]) not in drop]
            return {"name": "op"}
        if method == "POST":
            assert re.match(r"^[a-z]([-a-z0-9]*[a-z0-9])?$", body["name"]) and len(body["name"]) <= 63
            self.res[f"{url}/{body['name']}"] = dict(body)
            return {"name": "op"}
        if method == "PATCH":
            self.res[url].update(body)
            return {"name": "op"}
        if method == "DELETE":
            for other in self.res.values():      # a resource in use cannot be deleted
                assert url not in json.dumps(other), f"{url} still referenced"
            del self.res[url]
            self.endpoints.pop(url, None)
            return {"name": "op"}
        if url in self.res:
            return self.res[url]
        items = [v for k, v in self.res.items() if k.rsplit("/", 1)[0] == url]
        if items or url.rsplit("/", 1)[1] in ("forwardingRules", "targetTcpProxies", "targetHttpProxies", "urlMaps",
                                              "backendServices", "healthChecks", "networkEndpointGroups"):
            return {"items": items}
        raise CloudAPIError(404, url)

    def kinds(self):
        return sorted(k.split("/")[-2] for k in self.res)


def test_gcp_provider_lifecycle():
    api = FakeGCP()
    cfg = {"type": "gcp", "project_id": "p", "region": "us-central1", "availability_zone": "us-central1-b"}
    prov = GCPLoadBalancerProvider(cfg, "ws", api)
    m = LB.LoadBalancerManager(cfg, "ws", provider=prov)
    backend = {"services": {
        "api": svc("HTTP", 8080, 80, "site", route_path="/api", service_path="/v2"),
        "home": svc("HTTP", 8000, 80, "site", default_service=True),
        "pg": svc("TCP", 5432, 5432)}}
    m.update(LB.backend_services_from_config(backend))
    assert set(prov.list()) == {"site", "ws-n"}
    um = next(v for k, v in api.res.items() if "/urlMaps/" in k)
    rules = um["pathMatchers"][0]["pathRules"]
    assert rules[0]["paths"] == ["/api", "/api/*"]
    assert rules[0]["routeAction"]["urlRewrite"]["pathPrefixRewrite"] == "/v2"
    assert "home" in um["defaultService"]
    assert api.kinds().count("backendServices") == 3 and api.kinds().count("forwardingRules") == 2
    assert all(len(v) == 3 for v in api.endpoints.values())
    backend["services"]["pg"]["servers"] = SERVERS[1:]
    m.update(LB.backend_services_from_config(backend))
    pg_neg = next(k for k in api.endpoints if "-pg-" in k)
    assert sorted(e["ipAddress"] for e in api.endpoints[pg_neg]) == ["10.0.0.2", "10.0.0.3"]
    del backend["services"]["api"]
    m.update(LB.backend_services_from_config(backend))
    assert api.kinds().count("backendServices") == 2
    m.update({})
    assert api.res == {}


# ======================================================================= Azure fake
class FakeARM:
    def __init__(self):
        self.res = {}

    def __call__(self, method, url, params, body):
        assert params and "api-version" in params
        if method == "PUT":
            self.res[url] = dict(body, name=url.rsplit("/", 1)[1], id=url.replace("https://management.azure.com", ""),
                                 properties=dict(body.get("properties", {}), provisioningState="Succeeded"))
            return self.res[url]
        if method == "DELETE":
            self.res.pop(url, None)
            return {}
        if url in self.res:
            return self.res[url]
        if url.endswith(("loadBalancers", "applicationGateways")):
            return {"value": [v for k, v in self.res.items() if k.rsplit("/", 1)[0] == url]}
        raise CloudAPIError(404, url)


def test_azure_provider_lifecycle():
    api = FakeARM()
    cfg = {"type": "azure", "subscription_id": "sub", "resource_group": "rg", "location": "westus"}
    prov = AzureLoadBalancerProvider(cfg, "ws", api)
    m = LB.LoadBalancerManager(cfg, "ws", provider=prov)
    backend = {"services": {
        "api": svc("HTTP", 8080, 80, "site", route_path="/api", service_path="/v2"),
        "home": svc("HTTP", 8000, 80, "site", default_service=True),
        "pg": svc("TCP", 5432, 15432, load_balancer_scheme="internal")}}
    m.update(LB.backend_services_from_config(backend))
    lbs = prov.list()
    assert lbs["site"]["type"] == "application" and lbs["ws-n"]["scheme"] == "internal"
    gw = next(v for k, v in api.res.items() if "/applicationGateways/" in k)["properties"]
    assert gw["urlPathMaps"][0]["properties"]["pathRules"][0]["properties"]["paths"] == ["/api", "/api/*"]
    assert gw["urlPathMaps"][0]["properties"]["defaultBackendAddressPool"]["id"].endswith("/home")
    assert {s["name"]: s["properties"].get("path") for s in gw["backendHttpSettingsCollection"]} == \
        {"api-settings": "/v2/", "home-settings": None}
    assert any(k.endswith("publicIPAddresses/site-ip") for k in api.res)
    nlb = next(v for k, v in api.res.items() if "/loadBalancers/" in k)["properties"]
    assert "subnet" in nlb["frontendIPConfigurations"][0]["properties"]
    rule = nlb["loadBalancingRules"][0]["properties"]
    assert (rule["frontendPort"], rule["backendPort"]) == (15432, 5432)
    assert len(nlb["backendAddressPools"][0]["properties"]["loadBalancerBackendAddresses"]) == 3
    m.update({})
    assert not [k for k in api.res if "/loadBalancers/" in k or "/applicationGateways/" in k or "site-ip" in k]


# ======================================================================= controller + runtime
def test_controller_discovers_and_reconciles_on_change():
    p = MemoryProvider()
    rows = [{"name": "web", "host": "10.0.0.5", "port": 8080, "node": "n5",
             "meta": {LB.LABEL_PROTOCOL: "http", LB.LABEL_LB_NAME: "site", LB.LABEL_ROUTE_PATH: "/web"}},
            {"name": "web", "host": "10.0.0.6", "port": 8080, "node": "n6", "meta": {}}]
    ctl = LB.LoadBalancerController(workspace_name="ws", query=lambda: list(rows),
                                    manager=LB.LoadBalancerManager({}, "ws", provider=p), interval=1)
    ctl.pull()
    ctl.pull()
    assert p.calls == [("create", "site")]
    svc0 = p.lbs["site"]["service_groups"][0]["services"][0]
    assert svc0["route_path"] == "/web" and [t["node_id"] for t in svc0["targets"]] == ["n5", "n6"]
    rows.pop()
    ctl.pull()
    assert p.calls[-1] == ("update", "site")


def test_loadbalancer_runtime_static_mode(tmp_path, monkeypatch):
    from cloudtik_amd.core import runtime_factory as rf
    conf = tmp_path / "lb.cfg"
    rc = {"provider": {"type": "haproxy", "config_file": str(conf), "haproxy_bin": "no-such-haproxy"},
          "backend": {"config_mode": "static", "services": {"web": svc("HTTP", 8080, 80)}}}
    monkeypatch.setenv("RUNTIME_PATH", str(tmp_path))
    monkeypatch.setenv("CLOUDTIK_WORKSPACE", "ws")
    rt = rf.get_runtime("loadbalancer", rc)
    assert rt.node_configure(True)
    cc = json.loads((tmp_path / "loadbalancer" / "controller.json").read_text())
    assert cc["config_mode"] == "static" and cc["workspace_name"] == "ws"
    assert "frontend ws-a-http-80" in conf.read_text()
    assert rt.start_steps(True) == []
    rt2 = rf.get_runtime("loadbalancer", {"backend": {}})
    step = rt2.start_steps(True)[0]
    assert "LoadBalancerController" in step and "config_file=" in step
    assert os.path.basename(step.split("config_file=")[1]) == "controller.json"
