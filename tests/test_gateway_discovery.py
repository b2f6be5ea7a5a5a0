"""Discovery-driven load-balancer / gateway backends (runtime/gateway_discovery.py; reference
runtime/haproxy/discovery.py:20-119 + admin_api.py:80-143, runtime/nginx/discovery.py:18-118,
runtime/kong/discovery.py, runtime/apisix/discovery.py).

A fake discovery source (the Consul ``select_services`` rows) is changed between pulls; each
test checks that the backends follow: HAProxy slots through a fake runtime API, nginx.conf +
reload, and the Kong / APISIX admin objects through fake admin APIs."""
import json
import os

import pytest

from cloudtik_amd.core import runtime_factory as rf
from cloudtik_amd.runtime import gateway_discovery as GD


def _inst(name, host, port, **meta):
    return {"name": name, "host": host, "port": port, "meta": {k.replace("_", "-"): v for k, v in meta.items()},
            "node": host}


class Source:
    def __init__(self, rows):
        self.rows = list(rows)

    def __call__(self):
        return list(self.rows)


# ------------------------------------------------------------------------------- HAProxy
class FakeHAProxy:
    """Server slots of one backend, changed by the runtime-API commands the job sends."""

    def __init__(self, backend, free=4):
        self.backend = backend
        self.slots = {GD.slot_name(i): {"addr": "0.0.0.0", "port": 80, "maint": True} for i in range(1, free + 1)}
        self.log = []

    def servers(self, backend):
        active, inactive = {}, []
        for n, s in self.slots.items():
            if s["maint"]:
                inactive.append(n)
            else:
                active[(s["addr"], s["port"])] = n
        inactive.sort(key=lambda n: int(n[6:]))
        return active, inactive

    def enable(self, b, slot, srv):
        self.log.append(("enable", slot, srv))
        self.slots[slot].update(addr=srv[0], port=srv[1], maint=False)

    def disable(self, b, slot):
        self.log.append(("disable", slot))
        self.slots[slot]["maint"] = True

    def add(self, b, slot, srv):
        assert slot not in self.slots
        self.log.append(("add", slot, srv))
        self.slots[slot] = {"addr": srv[0], "port": srv[1], "maint": False}

    def delete(self, b, slot):
        assert self.slots[slot]["maint"]
        self.log.append(("delete", slot))
        del self.slots[slot]

    def active(self):
        return sorted((s["addr"], s["port"]) for s in self.slots.values() if not s["maint"])


def test_haproxy_slots_follow_discovered_servers(tmp_path):
    src = Source([_inst("web", "10.0.0.2", 8080), _inst("web", "10.0.0.3", 8080), _inst("api", "10.0.0.4", 9000)])
    hp = FakeHAProxy("cloudtik-servers")
    rendered = []
    job = GD.DiscoverHAProxyBackends(query=src, apis=[hp], render=rendered.append)
    job.pull()
    assert hp.active() == [("10.0.0.2", 8080), ("10.0.0.3", 8080), ("10.0.0.4", 9000)]
    assert [e[0] for e in hp.log] == ["enable"] * 3 and len(rendered) == 1
    hp.log.clear()
    job.pull()                                                 # nothing changed: no command
    assert hp.log == [] and len(rendered) == 1
    src.rows = src.rows[1:]                                    # 10.0.0.2 went away
    job.pull()
    assert hp.active() == [("10.0.0.3", 8080), ("10.0.0.4", 9000)] and hp.log == [("disable", "server1")]
    src.rows += [_inst("web", f"10.0.1.{i}", 8080) for i in range(6)]   # more than the free slots
    hp.log.clear()
    job.pull()
    assert len(hp.active()) == 8
    assert sum(e[0] == "add" for e in hp.log) == 8 - 4 and ("enable", "server1", ("10.0.1.0", 8080)) in hp.log
    src.rows = src.rows[:1]                                    # shrink: spare slots beyond 4 deleted
    hp.log.clear()
    job.pull()
    assert hp.active() == [("10.0.0.3", 8080)]
    assert sum(e[0] == "delete" for e in hp.log) == 3 and len(hp.slots) == 5
    assert len(rendered) == 4 and rendered[-1] == [("10.0.0.3", 8080)]


def test_haproxy_runtime_api_parses_server_state(monkeypatch):
    api = GD.HAProxyRuntimeAPI("127.0.0.1:1")
    state = ("1\n# be_id be_name srv_id srv_name srv_addr srv_op_state srv_admin_state srv_uweight srv_iweight "
             "srv_time_since_last_change srv_check_status srv_check_result srv_check_health srv_check_state "
             "srv_agent_state bk_f_forced_id srv_f_forced_id srv_fqdn srv_port srvrecord\n"
             "3 b1 1 server1 10.0.0.2 2 0 1 1 5 6 3 4 6 0 0 0 - 8080 -\n"
             "3 b1 2 server2 0.0.0.0 0 1 1 1 5 6 3 4 6 0 0 0 - 80 -\n")
    sent = []
    monkeypatch.setattr(api, "send", lambda cmd: sent.append(cmd) or state)
    active, inactive = api.servers("b1")
    assert active == {("10.0.0.2", 8080): "server1"} and inactive == ["server2"]
    api.enable("b1", "server2", ("10.0.0.9", 81))
    assert sent[-2:] == ["set server b1/server2 addr 10.0.0.9 port 81", "set server b1/server2 state ready"]


def test_haproxy_runtime_dynamic_config_and_daemon(tmp_path, monkeypatch):
    rc = {"backend": {"selector": {"services": ["web"]}}, "port": 8000}
    rt = rf.get_runtime("haproxy", rc)
    for k, v in {"RUNTIME_PATH": str(tmp_path), "CLOUDTIK_NODE_IP": "10.0.0.1", "CLOUDTIK_HEAD_IP": "10.0.0.1",
                 "CLOUDTIK_CLUSTER": "c1"}.items():
        monkeypatch.setenv(k, v)
    files = {os.path.relpath(p, tmp_path): t for p, t in rt.render(True).items()}
    cfg = files["haproxy/haproxy.cfg"]
    assert "stats socket ipv4@127.0.0.1:19999 level admin" in cfg
    assert "server server1 0.0.0.0:80 check disabled" in cfg and "bind *:8000" in cfg
    d = json.loads(files["haproxy/discovery.json"])
    assert d["service_selector"] == {"services": ["web"]} and d["consul_address"] == "10.0.0.1:8500"
    start = rt.start_steps(True)
    assert any("service-daemon start haproxy-discovery" in s and "DiscoverHAProxyBackends" in s for s in start)
    # the job re-renders the same file from the discovery config
    job = GD.DiscoverHAProxyBackends(query=Source([_inst("web", "10.0.0.7", 80)]), apis=[FakeHAProxy("x")],
                                     config_file=str(tmp_path / "haproxy" / "discovery.json"))
    job.pull()
    assert "server server1 10.0.0.7:80 check" in (tmp_path / "haproxy" / "haproxy.cfg").read_text()


# ------------------------------------------------------------------------------- NGINX
def test_nginx_rewrites_and_reloads_only_on_change(tmp_path):
    src = Source([_inst("web", "10.0.0.2", 8080, cloudtik_route_path="/app"),
                  _inst("home", "10.0.0.3", 80, cloudtik_default_service="true")])
    reloads = []
    conf = tmp_path / "nginx.conf"
    job = GD.DiscoverNginxBackends(query=src, conf_path=str(conf), port=81, runner=reloads.append,
                                   reload_cmd="nginx -s reload")
    job.pull()
    job.pull()
    text = conf.read_text()
    assert reloads == ["nginx -s reload"]
    assert "upstream web {\n    server 10.0.0.2:8080" in text and "listen 81;" in text
    assert "location /app/ {\n      proxy_pass http://web/;" in text and "location / {\n      proxy_pass http://home;" in text
    assert text.index("location /app/") < text.index("location / {")     # longest route first
    src.rows.append(_inst("web", "10.0.0.5", 8080, cloudtik_route_path="/app"))
    job.pull()
    assert len(reloads) == 2 and "server 10.0.0.5:8080" in conf.read_text()


# ------------------------------------------------------------------------------- Kong / APISIX
class FakeKong:
    def __init__(self):
        self.objs = {"upstreams": {}, "services": {}, "routes": {}}
        self.targets = {}
        self.calls = []
        self._id = 0

    def __call__(self, method, url, body=None, headers=None):
        path = url.split("8001", 1)[1]
        self.calls.append((method, path))
        parts = [p for p in path.split("?")[0].split("/") if p]
        if method == "GET" and parts == ["services"]:
            return {"data": [v for v in self.objs["services"].values() if "cloudtik" in v.get("tags", [])]}
        if method == "GET" and len(parts) == 3 and parts[2] == "targets":
            return {"data": [{"target": t, "id": i} for t, i in self.targets.get(parts[1], {}).items()]}
        if method == "PUT":
            self.objs[parts[0]][parts[1]] = dict(body)
            return body
        if method == "POST" and parts[2] == "targets":
            self._id += 1
            self.targets.setdefault(parts[1], {})[body["target"]] = f"t{self._id}"
            return {}
        if method == "DELETE":
            if len(parts) == 4:
                tg = self.targets[parts[1]]
                del tg[next(t for t, i in tg.items() if i == parts[3])]
            else:
                del self.objs[parts[0]][parts[1]]
            return None
        raise AssertionError((method, path))


def test_kong_admin_objects_follow_services():
    src = Source([_inst("web", "10.0.0.2", 8080, cloudtik_route_path="/w", cloudtik_service_path="/v1"),
                  _inst("web", "10.0.0.3", 8080, cloudtik_route_path="/w", cloudtik_service_path="/v1"),
                  _inst("api", "10.0.0.4", 9000)])
    kong = FakeKong()
    job = GD.DiscoverKongBackends(query=src, http=kong, admin_url="http://127.0.0.1:8001")
    job.pull()
    assert set(kong.objs["services"]) == {"web", "api"}
    assert set(kong.targets["web"]) == {"10.0.0.2:8080", "10.0.0.3:8080"}
    assert kong.objs["routes"]["web"]["paths"] == ["/w"] and kong.objs["services"]["web"]["path"] == "/v1"
    assert kong.objs["services"]["web"]["host"] == "web"                 # through the upstream
    src.rows = [r for r in src.rows if r["host"] != "10.0.0.3"]
    job.pull()
    assert set(kong.targets["web"]) == {"10.0.0.2:8080"}
    src.rows = [r for r in src.rows if r["name"] != "api"]
    job.pull()
    assert set(kong.objs["services"]) == {"web"} and "api" not in kong.objs["routes"]
    assert "api" not in kong.objs["upstreams"]
    n = len(kong.calls)
    job.pull()                                                           # unchanged: no admin call
    assert len(kong.calls) == n


def test_failed_apply_is_retried_on_the_next_pull():
    """The admin API is not up yet at the first pull: the job must apply again on the next
    pull even though the discovered set did not change (the hash is recorded only after a
    successful apply)."""
    src = Source([_inst("web", "10.0.0.2", 8080)])
    kong = FakeKong()
    down = {"n": 1}

    def flaky(method, url, body=None, headers=None):
        if down["n"] > 0:
            down["n"] -= 1
            raise ConnectionRefusedError("admin API not up")
        return kong(method, url, body, headers)

    job = GD.DiscoverKongBackends(query=src, http=flaky, admin_url="http://127.0.0.1:8001")
    with pytest.raises(ConnectionRefusedError):
        job.pull()
    job.pull()                                                           # same services: retried
    assert set(kong.objs["services"]) == {"web"}
    n = len(kong.calls)
    job.pull()
    assert len(kong.calls) == n                                          # applied: now idle


def test_nginx_failed_reload_is_retried(tmp_path):
    src = Source([_inst("web", "10.0.0.2", 8080)])

    class R:
        def __init__(self, rc):
            self.returncode = rc

    rcs = [1, 0]
    ran = []
    job = GD.DiscoverNginxBackends(query=src, conf_path=str(tmp_path / "nginx.conf"),
                                   runner=lambda cmd: ran.append(cmd) or R(rcs.pop(0)))
    with pytest.raises(RuntimeError):
        job.pull()
    job.pull()
    assert len(ran) == 2 and job.reloads == 1
    job.pull()
    assert len(ran) == 2


class FakeAPISIX:
    def __init__(self):
        self.objs = {"upstreams": {}, "routes": {}}
        self.keys = set()

    def __call__(self, method, url, body=None, headers=None):
        self.keys.add((headers or {}).get("X-API-KEY"))
        kind, _, oid = url.split("/apisix/admin/", 1)[1].partition("/")
        if method == "GET":
            return {"list": [{"value": v} for v in self.objs[kind].values()]}
        if method == "PUT":
            self.objs[kind][oid] = dict(body)
        elif method == "DELETE":
            del self.objs[kind][oid]
        return {}


def test_apisix_routes_and_upstreams_follow_services():
    src = Source([_inst("web", "10.0.0.2", 8080, cloudtik_route_path="/w"), _inst("api", "10.0.0.4", 9000)])
    ax = FakeAPISIX()
    ax.objs["routes"]["manual"] = {"id": "manual", "uri": "/m/*"}        # not ours: never touched
    job = GD.DiscoverAPISIXBackends(query=src, http=ax, admin_key="k1")
    job.pull()
    assert ax.keys == {"k1"}
    assert ax.objs["upstreams"]["web"]["nodes"] == {"10.0.0.2:8080": 1}
    assert ax.objs["routes"]["web"]["uri"] == "/w/*" and ax.objs["routes"]["web"]["upstream_id"] == "web"
    assert ax.objs["routes"]["api"]["plugins"]["proxy-rewrite"]["regex_uri"][0] == "^/api/(.*)"
    src.rows = src.rows[:1]
    job.pull()
    assert set(ax.objs["routes"]) == {"web", "manual"} and set(ax.objs["upstreams"]) == {"web"}


@pytest.mark.parametrize("name,cls", [("nginx", "DiscoverNginxBackends"), ("kong", "DiscoverKongBackends"),
                                      ("apisix", "DiscoverAPISIXBackends")])
def test_gateway_runtimes_start_their_discovery_daemon(name, cls, tmp_path, monkeypatch):
    rt = rf.get_runtime(name, {"backend": {"selector": {"clusters": ["c2"]}}})
    for k, v in {"RUNTIME_PATH": str(tmp_path), "CLOUDTIK_NODE_IP": "10.0.0.3", "CLOUDTIK_HEAD_IP": "10.0.0.1",
                 "CLOUDTIK_CLUSTER": "c1"}.items():
        monkeypatch.setenv(k, v)
    files = rt.render(False)
    d = json.loads(next(t for p, t in files.items() if p.endswith("discovery.json")))
    assert d["service_selector"] == {"clusters": ["c2"]}
    assert any(f"service-daemon start {name}-discovery" in s and cls in s for s in rt.start_steps(False))
    static = rf.get_runtime(name, {})
    assert not any("service-daemon" in s for s in static.start_steps(False))
