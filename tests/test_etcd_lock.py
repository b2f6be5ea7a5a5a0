"""etcd-backed locks and leader election (runtime/common/etcd.py; reference
runtime/common/leader_election/etcd_leader_election.py) against an in-process stand-in for
etcd's v3 JSON gateway with real lease expiry; plus the coordinator-URL factory."""
import base64
import json
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pytest

from cloudtik_amd.runtime.common.etcd import EtcdClient, EtcdLeaderElection, EtcdLock, leader_election


class FakeEtcd:
    def __init__(self):
        self.kv = {}           # key(bytes) -> (value bytes, lease id or None, create_rev)
        self.leases = {}       # id -> (ttl, expiry)
        self.rev = 0
        self.lock = threading.Lock()

    def _expire(self):
        now = time.time()
        for lid in [l for l, (_, exp) in self.leases.items() if exp < now]:
            self._revoke(lid)

    def _revoke(self, lid):
        self.leases.pop(lid, None)
        for k in [k for k, v in self.kv.items() if v[1] == lid]:
            del self.kv[k]

    def handle(self, path, b):
        d = lambda s: base64.b64decode(s) if s else b""  # noqa: E731
        with self.lock:
            self._expire()
            if path == "/v3/lease/grant":
                self.rev += 1
                lid = str(7000 + self.rev)
                self.leases[lid] = (b["TTL"], time.time() + b["TTL"])
                return {"ID": lid, "TTL": str(b["TTL"])}
            if path == "/v3/lease/keepalive":
                if b["ID"] not in self.leases:
                    return {"result": {"ID": b["ID"]}}
                ttl = self.leases[b["ID"]][0]
                self.leases[b["ID"]] = (ttl, time.time() + ttl)
                return {"result": {"ID": b["ID"], "TTL": str(ttl)}}
            if path == "/v3/lease/revoke":
                self._revoke(b["ID"])
                return {}
            if path == "/v3/kv/put":
                self.rev += 1
                old = self.kv.get(d(b["key"]))
                self.kv[d(b["key"])] = (d(b.get("value")), b.get("lease"), old[2] if old else self.rev)
                return {}
            if path == "/v3/kv/range":
                k = d(b["key"])
                if "range_end" in b:
                    end = d(b["range_end"])
                    keys = sorted(x for x in self.kv if k <= x < end)
                else:
                    keys = [k] if k in self.kv else []
                return {"kvs": [{"key": base64.b64encode(x).decode(),
                                 "value": base64.b64encode(self.kv[x][0]).decode()} for x in keys]}
            if path == "/v3/kv/deleterange":
                n = 1 if self.kv.pop(d(b["key"]), None) is not None else 0
                return {"deleted": str(n)}
            if path == "/v3/kv/txn":
                c = b["compare"][0]
                cur = self.kv.get(d(c["key"]))
                if c["target"] == "CREATE":
                    ok = cur is None
                else:
                    ok = cur is not None and cur[0] == d(c["value"])
                if ok:
                    for op in b["success"]:
                        if "request_put" in op:
                            p = op["request_put"]
                            self.rev += 1
                            self.kv[d(p["key"])] = (d(p["value"]), p.get("lease"), self.rev)
                        if "request_delete_range" in op:
                            self.kv.pop(d(op["request_delete_range"]["key"]), None)
                return {"succeeded": ok}
            raise AssertionError(path)


@pytest.fixture()
def etcd():
    fake = FakeEtcd()

    class H(BaseHTTPRequestHandler):
        def log_message(self, *a):
            pass

        def do_POST(self):
            n = int(self.headers.get("Content-Length") or 0)
            out = json.dumps(fake.handle(self.path, json.loads(self.rfile.read(n) or b"{}"))).encode()
            self.send_response(200)
            self.send_header("Content-Length", str(len(out)))
            self.end_headers()
            self.wfile.write(out)

    srv = ThreadingHTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    yield fake, EtcdClient(f"127.0.0.1:{srv.server_address[1]}"), srv.server_address[1]
    srv.shutdown()
    srv.server_close()


def test_kv_and_prefix(etcd):
    _, c, _ = etcd
    c.put("/a/1", "x")
    c.put("/a/2", b"y")
    c.put("/b/1", "z")
    assert c.get("/a/1") == b"x" and c.get("/nope") is None
    assert c.get_prefix("/a/") == {"/a/1": b"x", "/a/2": b"y"}
    assert c.delete("/a/1") == 1 and c.get("/a/1") is None


def test_lock_exclusion_release_and_expiry(etcd):
    _, c, _ = etcd
    a, b = EtcdLock(c, "job", ttl_s=1, owner="A"), EtcdLock(c, "job", ttl_s=1, owner="B")
    assert a.acquire(blocking=False) and a.owner() == "A" and a.renew()
    assert not b.acquire(blocking=False)
    a.release()
    assert b.acquire(blocking=False) and b.owner() == "B"
    time.sleep(1.3)                                # B stops keeping its lease alive
    assert not b.renew() and a.acquire(timeout=2) and a.owner() == "A"


def test_leader_election_and_factory(etcd):
    _, c, port = etcd
    ev = []
    e1 = EtcdLeaderElection(c, "ctl", "n1", ttl_s=1, on_elected=lambda: ev.append("n1+"))
    e2 = leader_election(f"etcd://127.0.0.1:{port}", "ctl", "n2", ttl_s=1, on_elected=lambda: ev.append("n2+"))
    assert isinstance(e2, EtcdLeaderElection)
    assert e1.step() and not e2.step() and e2.leader() == "n1"
    e2.start()
    e1.resign()
    deadline = time.time() + 5
    while not e2.is_leader() and time.time() < deadline:
        time.sleep(0.05)
    assert e2.is_leader() and ev == ["n1+", "n2+"]
    e2.resign()
    with pytest.raises(ValueError):
        leader_election("zk://x:1", "n")


def test_leader_demotes_itself_when_etcd_unreachable(etcd):
    """A leader that cannot renew for a lease TTL stops acting as leader (its lease expires on
    the server and another candidate takes over): never two leaders at once."""
    _, c, port = etcd
    ev = []
    cut = threading.Event()
    partitioned = EtcdClient(f"127.0.0.1:{port}")
    real_post = partitioned._post

    def post(path, body):
        if cut.is_set():
            raise OSError("gateway unreachable")
        return real_post(path, body)

    partitioned._post = post
    e1 = EtcdLeaderElection(partitioned, "svc", "n1", ttl_s=1, on_elected=lambda: ev.append("n1+"),
                            on_demoted=lambda: ev.append("n1-"))
    e2 = EtcdLeaderElection(c, "svc", "n2", ttl_s=1, on_elected=lambda: ev.append("n2+"))
    e1.start()
    deadline = time.time() + 5
    while not e1.is_leader() and time.time() < deadline:
        time.sleep(0.02)
    assert e1.is_leader()
    cut.set()
    t_cut = time.time()
    while e1.is_leader() and time.time() < deadline + 5:
        time.sleep(0.02)
    assert not e1.is_leader() and time.time() - t_cut < 2.5
    e2.start()
    while not e2.is_leader() and time.time() < deadline + 10:
        time.sleep(0.02)
    assert e2.is_leader()
    assert ev.index("n1-") < ev.index("n2+")              # demoted before the other took over
    cut.clear()
    e1.resign()
    e2.resign()


def test_demotion_deadline_uses_send_time_and_precedes_server_expiry():
    """The renew's SEND time bounds the server-side lease start, so the leader must step
    down at sent + ttl - margin, strictly before the server can expire the lease -- also
    when the renew RPC itself is slow or hangs (fake clock, stub lock)."""
    now = [100.0]

    class StubLock:
        ttl_s, owner_id, lease = 10, "n1", "L1"

        def __init__(self):
            self.calls = []

        def acquire(self, blocking=True):
            now[0] += 0.5                         # the acquire RPC takes 0.5 s
            return True

        def renew(self, timeout=None):
            self.calls.append(timeout)
            now[0] += 2.0                         # a slow keepalive round trip
            return True

        def owner(self):
            return "n1"

    e = EtcdLeaderElection.__new__(EtcdLeaderElection)
    EtcdLeaderElection.__init__(e, EtcdClient("127.0.0.1:1"), "x", "n1", ttl_s=10, clock=lambda: now[0])
    e.lock = StubLock()
    sent = now[0]
    assert e.step() and e._last_renew == sent            # the send time, not the reply time
    sent = now[0]
    assert e.step() and e._last_renew == sent
    assert e.lock.calls == [e.rpc_timeout_s]              # renew carries an explicit timeout
    server_expiry = sent + e.lock.ttl_s                    # earliest possible server-side expiry
    # etcd now unreachable: the leader stays only until its deadline, before server expiry
    assert e.deadline() < server_expiry - e.poll_s
    now[0] = e.deadline() - 0.01
    assert e.is_leader()
    now[0] = e.deadline()
    assert not e.is_leader() and e.lock.lease is None
