"""Consul client depth (runtime/common/consul.py; reference runtime/common/service_discovery/
consul.py + core/_private/util leader election): healthy-instance queries, selector-based
service selection over CloudTik tags/meta, KV keys/delete, TTL sessions and session locks,
and leader election with failover -- against an in-process stand-in for Consul's HTTP API."""
import base64
import json
import threading
import time
import urllib.parse
import uuid
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pytest

from cloudtik_amd.runtime.common.consul import ConsulClient, ConsulLeaderElection, ConsulLock


class FakeConsul:
    """Just enough of /v1 for the client: agent register/deregister, catalog, health,
    KV (keys, recurse delete, acquire/release) and sessions with a real TTL."""

    def __init__(self):
        self.services = {}          # id -> body
        self.failing = set()        # service ids whose check fails
        self.kv = {}                # key -> {"Value": bytes, "Session": sid|None}
        self.sessions = {}          # sid -> expiry time
        self.ttl = {}
        self.lock = threading.Lock()

    def _expire(self):
        now = time.time()
        for sid in [s for s, exp in self.sessions.items() if exp < now]:
            self._destroy(sid)

    def _destroy(self, sid):
        self.sessions.pop(sid, None)
        for e in self.kv.values():
            if e["Session"] == sid:
                e["Session"] = None

    def handle(self, method, path, q, body):
        with self.lock:
            self._expire()
            p = path[len("/v1/"):]
            if p == "agent/service/register":
                b = json.loads(body)
                self.services[b["ID"]] = b
                return True
            if p.startswith("agent/service/deregister/"):
                self.services.pop(p.rsplit("/", 1)[1], None)
                return True
            if p == "catalog/services":
                out = {}
                for b in self.services.values():
                    out.setdefault(b["Name"], [])
                    out[b["Name"]] = sorted(set(out[b["Name"]]) | set(b["Tags"]))
                return out
            if p.startswith("catalog/service/"):
                name = p.rsplit("/", 1)[1]
                return [{"Node": "n-" + i, "Address": "10.0.0.1", "ServiceID": i, "ServiceName": b["Name"],
                         "ServiceAddress": b.get("Address", ""), "ServicePort": b["Port"], "ServiceTags": b["Tags"],
                         "ServiceMeta": b["Meta"]} for i, b in self.services.items() if b["Name"] == name]
            if p.startswith("health/service/"):
                name = p.rsplit("/", 1)[1]
                return [{"Node": {"Node": "n-" + i, "Address": "10.0.0.1"},
                         "Service": {"ID": i, "Service": b["Name"], "Address": b.get("Address", ""),
                                     "Port": b["Port"], "Tags": b["Tags"], "Meta": b["Meta"]}}
                        for i, b in self.services.items() if b["Name"] == name
                        and not ("passing" in q and i in self.failing)]
            if p == "session/create":
                b = json.loads(body)
                sid = uuid.uuid4().hex
                self.ttl[sid] = float(b["TTL"].rstrip("s"))
                self.sessions[sid] = time.time() + self.ttl[sid]
                return {"ID": sid}
            if p.startswith("session/renew/"):
                sid = p.rsplit("/", 1)[1]
                if sid not in self.sessions:
                    return 404
                self.sessions[sid] = time.time() + self.ttl[sid]
                return [{"ID": sid}]
            if p.startswith("session/destroy/"):
                self._destroy(p.rsplit("/", 1)[1])
                return True
            if p.startswith("kv/"):
                key = p[3:]
                if method == "GET" and "keys" in q:
                    return sorted(k for k in self.kv if k.startswith(key)) or 404
                if method == "GET":
                    e = self.kv.get(key)
                    if e is None:
                        return 404
                    return [{"Key": key, "Value": base64.b64encode(e["Value"]).decode(), "Session": e["Session"]}]
                if method == "DELETE":
                    for k in [k for k in self.kv if (k.startswith(key) if "recurse" in q else k == key)]:
                        del self.kv[k]
                    return True
                e = self.kv.setdefault(key, {"Value": b"", "Session": None})
                if "acquire" in q:
                    sid = q["acquire"]
                    if sid not in self.sessions or e["Session"] not in (None, sid):
                        return False
                    e["Session"] = sid
                elif "release" in q:
                    if e["Session"] != q["release"]:
                        return False
                    e["Session"] = None
                e["Value"] = body
                return True
            return 404


@pytest.fixture()
def consul():
    fake = FakeConsul()

    class H(BaseHTTPRequestHandler):
        def log_message(self, *a):
            pass

        def _do(self):
            u = urllib.parse.urlsplit(self.path)
            q = dict(urllib.parse.parse_qsl(u.query, keep_blank_values=True))
            n = int(self.headers.get("Content-Length") or 0)
            r = fake.handle(self.command, u.path, q, self.rfile.read(n) if n else b"")
            if r == 404 and not isinstance(r, bool):
                self.send_response(404)
                self.end_headers()
                return
            data = json.dumps(r).encode()
            self.send_response(200)
            self.send_header("Content-Length", str(len(data)))
            self.end_headers()
            self.wfile.write(data)

        do_GET = do_PUT = do_DELETE = _do

    srv = ThreadingHTTPServer(("127.0.0.1", 0), H)
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    yield fake, ConsulClient(f"127.0.0.1:{srv.server_address[1]}")
    srv.shutdown()
    srv.server_close()


def test_selectors_and_health(consul):
    fake, c = consul
    c.register_service("zookeeper", 2181, "10.0.0.2", service_id="zk-a", cluster="c1", runtime="zookeeper")
    c.register_service("zookeeper", 2181, "10.0.0.3", service_id="zk-b", cluster="c2", runtime="zookeeper")
    c.register_service("hdfs-name", 9000, "10.0.0.4", service_id="nn", cluster="c1", runtime="hdfs",
                       features=["storage"], meta={"role": "name"})
    assert "cloudtik-c-c1" in c.services()["zookeeper"]
    assert {i["id"] for i in c.select_services({"runtimes": ["zookeeper"]})} == {"zk-a", "zk-b"}
    assert [i["id"] for i in c.select_services({"runtimes": ["zookeeper"], "clusters": ["c2"]})] == ["zk-b"]
    assert [i["id"] for i in c.select_services({"exclude_clusters": ["c2"], "tags": ["cloudtik-f-storage"]})] == ["nn"]
    assert [i["id"] for i in c.select_services({"labels": {"role": "name"}})] == ["nn"]
    fake.failing.add("zk-a")
    assert [i["id"] for i in c.select_services({"services": ["zookeeper"]})] == ["zk-b"]
    assert {i["id"] for i in c.select_services({"services": ["zookeeper"]}, passing=False)} == {"zk-a", "zk-b"}
    assert c.healthy_instances("zookeeper")[0]["host"] == "10.0.0.3"
    c.deregister_service("zk-b")
    assert c.select_services({"services": ["zookeeper"]}) == []


def test_kv_keys_delete(consul):
    _, c = consul
    for k in ("app/a", "app/b", "other/x"):
        assert c.kv_put(k, k.encode())
    assert c.kv_keys("app/") == ["app/a", "app/b"]
    assert c.kv_get("app/a") == b"app/a"
    assert c.kv_delete("app/", recurse=True)
    assert c.kv_keys("app/") == [] and c.kv_get("app/a") is None and c.kv_get("other/x") == b"other/x"


def test_lock_mutual_exclusion_and_release(consul):
    _, c = consul
    a, b = ConsulLock(c, "job", ttl_s=5, owner="A"), ConsulLock(c, "job", ttl_s=5, owner="B")
    assert a.acquire(blocking=False) and a.owner() == "A" and a.renew()
    assert not b.acquire(blocking=False)
    assert not b.acquire(timeout=0.3)
    a.release()
    assert a.owner() is None
    with b:
        assert b.owner() == "B" and not a.acquire(blocking=False)
    assert a.acquire(blocking=False)


def test_session_expiry_frees_lock(consul):
    _, c = consul
    a, b = ConsulLock(c, "ttl", ttl_s=1, owner="A"), ConsulLock(c, "ttl", ttl_s=1, owner="B")
    assert a.acquire(blocking=False)
    time.sleep(1.3)                              # A stops renewing (crashed)
    assert not a.renew()
    assert b.acquire(timeout=2) and b.owner() == "B"


def test_leader_election_failover(consul):
    _, c = consul
    events = []
    e1 = ConsulLeaderElection(c, "head", "n1", ttl_s=1, on_elected=lambda: events.append("n1+"),
                              on_demoted=lambda: events.append("n1-"))
    e2 = ConsulLeaderElection(c, "head", "n2", ttl_s=1, on_elected=lambda: events.append("n2+"))
    assert e1.step() and not e2.step()
    assert e1.leader() == "n1" and e1.is_leader() and not e2.is_leader()
    e2.start()
    e1.resign()                                  # graceful handover
    deadline = time.time() + 5
    while not e2.is_leader() and time.time() < deadline:
        time.sleep(0.05)
    assert e2.is_leader() and e2.leader() == "n2"
    e2.resign()
    assert events == ["n1+", "n1-", "n2+"]
