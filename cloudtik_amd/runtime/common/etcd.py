"""etcd v3 client over the JSON gateway (``/v3/...``), with leases, a lease-bound lock and
leader election -- the etcd backend of the active-standby services (reference
runtime/common/leader_election/etcd_leader_election.py + the locks beside it; the other
backends are core/state/lock.py on the state server and runtime/common/consul.py).

Keys and values travel base64-encoded, as the gateway requires.  A lock is a key created in
a transaction only if it does not exist yet (``create_revision == 0``), attached to a lease
the holder keeps alive; when the holder dies the lease expires, etcd deletes the key and the
next candidate's transaction succeeds.
"""
from __future__ import annotations

import base64
import json
import threading
import time
import urllib.request
import uuid
from typing import Any, Dict, List, Optional


def _b64(s) -> str:
    return base64.b64encode(s if isinstance(s, bytes) else str(s).encode()).decode()


def _unb64(s: Optional[str]) -> bytes:
    return base64.b64decode(s) if s else b""


class EtcdClient:
    def __init__(self, endpoint: str = "127.0.0.1:2379", timeout: float = 10.0):
        self.base = endpoint if endpoint.startswith("http") else f"http://{endpoint}"
        self.timeout = timeout

    def _post(self, path: str, body: Dict[str, Any], timeout: Optional[float] = None) -> Dict[str, Any]:
        req = urllib.request.Request(f"{self.base}/v3/{path}", data=json.dumps(body).encode(), method="POST",
                                     headers={"Content-Type": "application/json"})
        with urllib.request.urlopen(req, timeout=timeout or self.timeout) as r:
            return json.loads(r.read() or b"{}")

    # ---------------------------------------------------------------- KV
    def put(self, key: str, value, lease: Optional[str] = None):
        body = {"key": _b64(key), "value": _b64(value)}
        if lease:
            body["lease"] = lease
        self._post("kv/put", body)

    def get(self, key: str, timeout: Optional[float] = None) -> Optional[bytes]:
        kvs = self._post("kv/range", {"key": _b64(key)}, timeout=timeout).get("kvs") or []
        return _unb64(kvs[0].get("value")) if kvs else None

    def get_prefix(self, prefix: str) -> Dict[str, bytes]:
        end = prefix[:-1] + chr(ord(prefix[-1]) + 1) if prefix else "\0"
        kvs = self._post("kv/range", {"key": _b64(prefix), "range_end": _b64(end)}).get("kvs") or []
        return {_unb64(kv["key"]).decode(): _unb64(kv.get("value")) for kv in kvs}

    def delete(self, key: str) -> int:
        return int(self._post("kv/deleterange", {"key": _b64(key)}).get("deleted", 0))

    def put_if_absent(self, key: str, value, lease: Optional[str] = None) -> bool:
        put = {"key": _b64(key), "value": _b64(value)}
        if lease:
            put["lease"] = lease
        r = self._post("kv/txn", {"compare": [{"key": _b64(key), "target": "CREATE", "result": "EQUAL",
                                               "create_revision": "0"}],
                                  "success": [{"request_put": put}]})
        return bool(r.get("succeeded"))

    def delete_if_value(self, key: str, value) -> bool:
        r = self._post("kv/txn", {"compare": [{"key": _b64(key), "target": "VALUE", "result": "EQUAL",
                                               "value": _b64(value)}],
                                  "success": [{"request_delete_range": {"key": _b64(key)}}]})
        return bool(r.get("succeeded"))

    # ---------------------------------------------------------------- leases
    def lease_grant(self, ttl_s: int) -> str:
        return str(self._post("lease/grant", {"TTL": int(ttl_s)})["ID"])

    def lease_keepalive(self, lease: str, timeout: Optional[float] = None) -> bool:
        r = self._post("lease/keepalive", {"ID": lease}, timeout=timeout)
        return int((r.get("result") or r).get("TTL", 0) or 0) > 0

    def lease_revoke(self, lease: str):
        self._post("lease/revoke", {"ID": lease})


class EtcdLock:
    """Same calls as core/state/lock.py ``DistributedLock`` (acquire / renew / release /
    owner), on an etcd key bound to a keep-alive lease."""

    def __init__(self, client: EtcdClient, name: str, ttl_s: int = 10, owner: Optional[str] = None):
        self.c, self.key, self.ttl_s = client, f"/cloudtik/locks/{name}", ttl_s
        self.owner_id = owner or uuid.uuid4().hex
        self.lease: Optional[str] = None

    def acquire(self, blocking: bool = True, timeout: Optional[float] = None, poll: float = 0.1) -> bool:
        deadline = None if timeout is None else time.time() + timeout
        while True:
            if self.lease is None or not self.c.lease_keepalive(self.lease):
                self.lease = self.c.lease_grant(self.ttl_s)
            if self.c.put_if_absent(self.key, self.owner_id, self.lease):
                return True
            if self.c.get(self.key) == self.owner_id.encode():
                return True                         # re-entrant for the same owner
            if not blocking or (deadline is not None and time.time() > deadline):
                return False
            time.sleep(poll)

    def renew(self, timeout: Optional[float] = None) -> bool:
        return self.lease is not None and self.c.lease_keepalive(self.lease, timeout=timeout) and \
            self.c.get(self.key, timeout=timeout) == self.owner_id.encode()

    def release(self) -> bool:
        ok = self.c.delete_if_value(self.key, self.owner_id)
        if self.lease is not None:
            self.c.lease_revoke(self.lease)
            self.lease = None
        return ok

    def owner(self) -> Optional[str]:
        v = self.c.get(self.key)
        return v.decode() if v else None

    def __enter__(self):
        self.acquire()
        return self

    def __exit__(self, *exc):
        self.release()


class EtcdLeaderElection:
    """Leader election on an EtcdLock (same interface as runtime/common/consul.py
    ``ConsulLeaderElection``: step / start / resign / is_leader / leader).

    Leadership is time-bounded: the server starts a lease's TTL when it HANDLES a keepalive,
    so the only safe local lower bound of the expiry is the time the keepalive was SENT.  A
    leader therefore stops acting as leader at ``sent + ttl - margin``, where the margin
    covers one loop poll plus the two RPC timeouts of a renew (keepalive + owner check), so
    the demotion lands before the server can expire the lease and hand the lock to another
    candidate -- even when an etcd call hangs (every call carries an explicit timeout, and
    ``is_leader()`` checks the deadline itself instead of trusting the loop)."""

    def __init__(self, client: EtcdClient, name: str, candidate_id: Optional[str] = None, ttl_s: int = 10,
                 on_elected=None, on_demoted=None, clock=time.monotonic):
        self.lock = EtcdLock(client, f"leader/{name}", ttl_s, candidate_id)
        self.on_elected, self.on_demoted = on_elected, on_demoted
        self.clock = clock
        self.poll_s = max(0.05, ttl_s / 5)
        self.rpc_timeout_s = max(0.05, ttl_s / 7)
        self.margin_s = self.poll_s + 2 * self.rpc_timeout_s
        self._leader = False
        self._last_renew = 0.0          # send time of the last renew / acquire that succeeded
        self._stop = threading.Event()
        self._mu = threading.Lock()
        self._thread: Optional[threading.Thread] = None

    @property
    def candidate_id(self) -> str:
        return self.lock.owner_id

    def deadline(self) -> float:
        """Local time after which this node must no longer act as leader."""
        return self._last_renew + self.lock.ttl_s - self.margin_s

    def is_leader(self) -> bool:
        if self._leader and self.clock() >= self.deadline():
            self._expire()
        return self._leader

    def leader(self) -> Optional[str]:
        return self.lock.owner()

    def _set(self, leader: bool, sent: Optional[float] = None):
        with self._mu:
            was, self._leader = self._leader, leader
            if leader and sent is not None:
                self._last_renew = sent
        if leader and not was and self.on_elected:
            self.on_elected()
        if was and not leader and self.on_demoted:
            self.on_demoted()

    def _expire(self):
        """The lease may already be gone server-side: stop leading, re-acquire with a new lease."""
        self.lock.lease = None
        self._set(False)

    def step(self) -> bool:
        if self._leader and self.clock() >= self.deadline():
            self._expire()
        sent = self.clock()
        if self._leader:
            ok = self.lock.renew(timeout=self.rpc_timeout_s)
        else:
            ok = self.lock.acquire(blocking=False)
        self._set(ok, sent)
        return self._leader

    def _on_error(self):
        """etcd unreachable: keep leading only until the send-time deadline."""
        if self._leader and self.clock() >= self.deadline():
            self._expire()

    def start(self):
        def loop():
            while not self._stop.is_set():
                try:
                    self.step()
                except Exception:  # noqa: BLE001 - etcd briefly unreachable: retry
                    self._on_error()
                wait = self.poll_s
                if self._leader:
                    wait = min(wait, max(0.0, self.deadline() - self.clock()))
                self._stop.wait(max(0.01, wait))
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


def leader_election(url: str, name: str, candidate_id: Optional[str] = None, ttl_s: int = 10, **kw):
    """A leader election for a coordinator URL: ``consul://host:port``, ``etcd://host:port``
    or ``state://host:port`` (the cluster's state server) -- how active-standby services (load
    balancer controller, metrics pullers) pick their backend from config."""
    scheme, _, addr = url.partition("://")
    if scheme == "consul":
        from cloudtik_amd.runtime.common.consul import ConsulClient, ConsulLeaderElection
        return ConsulLeaderElection(ConsulClient(addr), name, candidate_id, ttl_s, **kw)
    if scheme == "etcd":
        return EtcdLeaderElection(EtcdClient(addr), name, candidate_id, ttl_s, **kw)
    if scheme in ("state", "redis"):
        from cloudtik_amd.core.state.lock import LeaderElection
        from cloudtik_amd.core.state.state_client import StateClient
        return LeaderElection(StateClient.create(addr), name, candidate_id, ttl_ms=ttl_s * 1000, **kw)
    raise ValueError(f"unknown coordinator url {url!r}")


__all__: List[str] = ["EtcdClient", "EtcdLock", "EtcdLeaderElection", "leader_election"]
