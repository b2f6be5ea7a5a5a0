"""Distributed locks and leader election on the native state server (reference
runtime/common/lock/* and leader_election/* -- Consul / etcd / redis backed -- and
active_standby_service.py).

* :class:`DistributedLock`: ``SET key token NX PX ttl`` to acquire, the server-side
  ``DELIFEQ`` to release only our own lease, ``PEXPIREIFEQ`` to renew -- atomic because the
  state server executes commands one at a time;
* :class:`LeaderElection`: a renewing lease under ``leader/<name>`` with
  ``on_elected`` / ``on_demoted`` callbacks, for active-standby head services;
* :class:`ActiveStandbyService`: runs ``start()`` only while this instance is the leader.
"""
from __future__ import annotations

import threading
import time
import uuid
from typing import Callable, Optional

from cloudtik_amd.core.state.state_client import StateClient

LOCK_NAMESPACE = "lock"


class DistributedLock:
    def __init__(self, client: StateClient, name: str, ttl_ms: int = 10000, token: Optional[str] = None):
        self.client = client
        self.key = f"@namespace_{LOCK_NAMESPACE}:{name}"
        self.ttl_ms = int(ttl_ms)
        self.token = token or uuid.uuid4().hex

    def acquire(self, blocking: bool = True, timeout: Optional[float] = None, poll: float = 0.05) -> bool:
        deadline = time.time() + timeout if timeout is not None else None
        while True:
            if self.client.conn.execute("SET", self.key, self.token, "NX", "PX", self.ttl_ms) == "OK":
                return True
            if not blocking or (deadline is not None and time.time() >= deadline):
                return False
            time.sleep(poll)

    def renew(self) -> bool:
        return self.client.conn.execute("PEXPIREIFEQ", self.key, self.token, self.ttl_ms) == 1

    def release(self) -> bool:
        return self.client.conn.execute("DELIFEQ", self.key, self.token) == 1

    def owner(self) -> Optional[str]:
        v = self.client.conn.get(self.key)
        return v.decode() if v else None

    def __enter__(self):
        self.acquire()
        return self

    def __exit__(self, *exc):
        self.release()


class LeaderElection:
    def __init__(self, client: StateClient, name: str, candidate_id: Optional[str] = None, ttl_ms: int = 5000,
                 on_elected: Optional[Callable[[], None]] = None, on_demoted: Optional[Callable[[], None]] = None):
        self.lock = DistributedLock(client, f"leader/{name}", ttl_ms, token=candidate_id or uuid.uuid4().hex)
        self.on_elected, self.on_demoted = on_elected, on_demoted
        self._leader = False
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None

    @property
    def candidate_id(self) -> str:
        return self.lock.token

    def is_leader(self) -> bool:
        return self._leader

    def leader(self) -> Optional[str]:
        return self.lock.owner()

    def step(self):
        """One campaign / renewal round (the background thread calls this)."""
        if self._leader:
            if not self.lock.renew():
                self._leader = False
                if self.on_demoted:
                    self.on_demoted()
        elif self.lock.acquire(blocking=False):
            self._leader = True
            if self.on_elected:
                self.on_elected()

    def start(self):
        def loop():
            period = self.lock.ttl_ms / 3000.0
            while not self._stop.is_set():
                try:
                    self.step()
                except (ConnectionError, OSError):
                    if self._leader:
                        self._leader = False
                        if self.on_demoted:
                            self.on_demoted()
                self._stop.wait(period)
        self._thread = threading.Thread(target=loop, daemon=True, name="leader-election")
        self._thread.start()
        return self

    def resign(self):
        self._stop.set()
        if self._thread:
            self._thread.join(timeout=5)
        if self._leader:
            # stop acting as leader before the lock is handed over
            self._leader = False
            if self.on_demoted:
                self.on_demoted()
            self.lock.release()


class ActiveStandbyService:
    """Runs ``start_fn`` while this instance leads and ``stop_fn`` when it loses the lease."""

    def __init__(self, client: StateClient, name: str, start_fn: Callable[[], None], stop_fn: Callable[[], None],
                 ttl_ms: int = 5000):
        self.election = LeaderElection(client, name, ttl_ms=ttl_ms, on_elected=start_fn, on_demoted=stop_fn)

    def start(self):
        self.election.start()
        return self

    def stop(self):
        self.election.resign()
