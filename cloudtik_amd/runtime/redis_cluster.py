"""Redis sharded cluster bootstrap and growth (``redis.cluster_mode: sharding``).

Reference behaviour: runtime/redis/scripting.py:94-243 (``init_cluster_service``,
``_bootstrap_cluster``, ``_join_cluster_with_workers``, ``_meet_with_cluster``, role assignment
under a distributed lock, re-sharding on join).  Here the protocol is spoken directly over RESP
(``core.state.resp.RespConnection``: no redis-py dependency):

* a node that finds no running cluster bootstraps one: all 16384 hash slots on itself
  (``CLUSTER ADDSLOTSRANGE 0 16383``);
* a joining node is introduced by a live member (``CLUSTER MEET <ip> <port>`` sent to that
  member) and waits until the member's ``CLUSTER NODES`` lists it;
* under the cluster-wide role lock it then takes a role: while every master already has
  ``replicas_per_master`` replicas it becomes a MASTER and re-shards -- it takes an even share
  of the slots from the masters holding the most (``SETSLOT IMPORTING / MIGRATING``, keys moved
  with ``MIGRATE``, ``SETSLOT NODE`` on both ends); otherwise it becomes a REPLICA of the master
  with the fewest replicas (``CLUSTER REPLICATE``);
* a marker file in the data directory makes the whole thing a no-op on restart (the node's
  ``nodes.conf`` already carries its cluster state).

Run by the runtime's start step on every node after ``redis-server`` is up:
``python -m cloudtik_amd.runtime.redis_cluster join --node-ip IP --port P [--head] --seeds A,B``.
"""
from __future__ import annotations

import argparse
import contextlib
import os
import sys
import time
from typing import Callable, Dict, List, Optional, Sequence

SLOTS = 16384


class ClusterNode:
    __slots__ = ("id", "host", "port", "flags", "master_id", "slots", "connected")

    def __init__(self, line: str):
        parts = line.split()
        self.id = parts[0]
        addr = parts[1].split("@", 1)[0]
        self.host, _, port = addr.rpartition(":")
        self.port = int(port) if port.isdigit() else 0
        self.flags = set(parts[2].split(","))
        self.master_id = None if parts[3] == "-" else parts[3]
        self.connected = len(parts) > 7 and parts[7] == "connected"
        self.slots: List[int] = []
        for tok in parts[8:]:
            if tok.startswith("["):            # a slot being imported / migrated: not owned yet
                continue
            lo, _, hi = tok.partition("-")
            self.slots.extend(range(int(lo), int(hi or lo) + 1))

    @property
    def is_master(self) -> bool:
        return "master" in self.flags and "fail" not in self.flags

    @property
    def is_myself(self) -> bool:
        return "myself" in self.flags


def parse_nodes(text) -> List[ClusterNode]:
    if isinstance(text, bytes):
        text = text.decode()
    return [ClusterNode(line) for line in text.splitlines() if line.strip()]


def _s(v) -> str:
    return v.decode() if isinstance(v, bytes) else str(v)


class RedisClusterManager:
    """``connect(host, port)`` returns an object with ``execute(*args)`` (a RespConnection,
    or a fake in tests)."""

    def __init__(self, connect: Callable[[str, int], object], port: int = 6379,
                 replicas_per_master: int = 0, lock: Optional[Callable[[], contextlib.AbstractContextManager]] = None,
                 wait: float = 30.0, poll: float = 0.2, migrate_timeout_ms: int = 5000,
                 password: Optional[str] = None):
        self.connect = connect
        self.password = password or None      # MIGRATE authenticates to the target itself
        self.port = int(port)
        self.replicas = max(0, int(replicas_per_master))
        self.lock = lock or contextlib.nullcontext
        self.wait, self.poll = wait, poll
        self.migrate_timeout_ms = migrate_timeout_ms
        self._conns: Dict[tuple, object] = {}

    def _c(self, host: str, port: Optional[int] = None):
        key = (host, int(port or self.port))
        c = self._conns.get(key)
        if c is None:
            c = self._conns[key] = self.connect(*key)
        return c

    def nodes(self, host: str, port: Optional[int] = None) -> List[ClusterNode]:
        return parse_nodes(self._c(host, port).execute("CLUSTER", "NODES"))

    def myid(self, host: str) -> str:
        return _s(self._c(host).execute("CLUSTER", "MYID"))

    # ------------------------------------------------------------------ roles
    def bootstrap(self, host: str) -> None:
        """A one-node cluster owning every slot."""
        self._c(host).execute("CLUSTER", "ADDSLOTSRANGE", 0, SLOTS - 1)

    def meet(self, my_ip: str, seeds: Sequence[str]) -> str:
        """Introduce this node through the first live seed; returns that seed.  Waits until the
        seed's view lists this node."""
        me = self.myid(my_ip)
        last = None
        for seed in seeds:
            try:
                self._c(seed).execute("CLUSTER", "MEET", my_ip, self.port)
            except Exception as e:  # noqa: BLE001 - try the next seed
                last = e
                self._conns.pop((seed, self.port), None)
                continue
            deadline = time.time() + self.wait
            while time.time() < deadline:
                if any(n.id == me for n in self.nodes(seed)):
                    return seed
                time.sleep(self.poll)
            last = TimeoutError(f"{my_ip} not visible from {seed} after {self.wait}s")
        raise RuntimeError(f"could not join the redis cluster through {list(seeds)}: {last}")

    def assign_role(self, my_ip: str, seed: str) -> str:
        """'master' (after taking its share of the slots) or 'replica'."""
        with self.lock():
            view = [n for n in self.nodes(seed) if "fail" not in n.flags]
            me = self.myid(my_ip)
            masters = [n for n in view if n.is_master and n.slots and n.id != me]
            replicas_of = {m.id: 0 for m in masters}
            for n in view:
                if n.master_id in replicas_of and n.id != me:
                    replicas_of[n.master_id] += 1
            if not masters:
                self.bootstrap(my_ip)
                return "master"
            short = sorted((cnt, mid) for mid, cnt in replicas_of.items())
            if self.replicas and short and short[0][0] < self.replicas:
                target = short[0][1]
                self._c(my_ip).execute("CLUSTER", "REPLICATE", target)
                return "replica"
            self.reshard_to(me, my_ip, masters)
            return "master"

    def reshard_to(self, dst_id: str, dst_ip: str, masters: List[ClusterNode]) -> int:
        """Move an even share of the slots to the new master (from the richest masters first);
        returns the number of slots moved."""
        want = SLOTS // (len(masters) + 1)
        owned = {m.id: sorted(m.slots) for m in masters}
        plan, moved = [], 0
        while moved < want:
            d = max(masters, key=lambda m: len(owned[m.id]))
            excess = len(owned[d.id]) - want
            if excess <= 0:
                break
            take = min(excess, want - moved)
            plan.append((d, owned[d.id][-take:]))
            owned[d.id] = owned[d.id][:-take]
            moved += take
        dst = self._c(dst_ip)
        for src_node, slots in plan:
            src = self._c(src_node.host, src_node.port)
            for s in slots:
                dst.execute("CLUSTER", "SETSLOT", s, "IMPORTING", src_node.id)
                src.execute("CLUSTER", "SETSLOT", s, "MIGRATING", dst_id)
                while True:
                    keys = src.execute("CLUSTER", "GETKEYSINSLOT", s, 100) or []
                    if not keys:
                        break
                    auth = ("AUTH", self.password) if self.password else ()
                    src.execute("MIGRATE", dst_ip, self.port, "", 0, self.migrate_timeout_ms, *auth, "KEYS", *keys)
                dst.execute("CLUSTER", "SETSLOT", s, "NODE", dst_id)
                src.execute("CLUSTER", "SETSLOT", s, "NODE", dst_id)
        return moved

    # ------------------------------------------------------------------ entry
    def join(self, my_ip: str, seeds: Sequence[str], head: bool = False) -> str:
        """Bootstrap (no live seed) or meet + take a role.  Returns 'bootstrap', 'master' or
        'replica'."""
        live = [s for s in seeds if s != my_ip and self._alive(s)]
        if not live:
            if head:
                self.bootstrap(my_ip)
                return "bootstrap"
            raise RuntimeError(f"no live redis cluster member among {list(seeds)}")
        seed = self.meet(my_ip, live)
        return self.assign_role(my_ip, seed)

    def _alive(self, host: str) -> bool:
        try:
            view = self.nodes(host)
        except Exception:  # noqa: BLE001
            self._conns.pop((host, self.port), None)
            return False
        return any(n.is_myself and n.slots for n in view) or any(n.slots for n in view)


def _state_lock(name: str):
    """The cluster-wide role lock on the head's state server (core/state/lock.py); a no-op
    when the head is not reachable (single-node tests)."""
    @contextlib.contextmanager
    def cm():
        head = os.environ.get("CLOUDTIK_HEAD_IP")
        lk = None
        if head:
            try:
                from cloudtik_amd.core import constants as C
                from cloudtik_amd.core.state.lock import DistributedLock
                from cloudtik_amd.core.state.state_client import StateClient
                pw = os.environ.get("CLOUDTIK_STATE_PASSWORD") or C.CLOUDTIK_STATE_PASSWORD
                lk = DistributedLock(StateClient.create(f"{head}:{C.CLOUDTIK_DEFAULT_PORT}", pw, timeout=5),
                                     name, ttl_ms=120000)
                lk.acquire(timeout=300)
            except Exception:  # noqa: BLE001 - no state server: run unlocked
                lk = None
        try:
            yield
        finally:
            if lk is not None:
                lk.release()
    return cm


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m cloudtik_amd.runtime.redis_cluster")
    ap.add_argument("command", choices=["join"])
    ap.add_argument("--node-ip", required=True)
    ap.add_argument("--port", type=int, default=6379)
    ap.add_argument("--password", default=os.environ.get("REDIS_PASSWORD"))
    ap.add_argument("--head", action="store_true")
    ap.add_argument("--seeds", default="", help="comma list of member IPs to join through")
    ap.add_argument("--replicas-per-master", type=int, default=0)
    ap.add_argument("--marker", default=None, help="file marking this node as initialised")
    a = ap.parse_args(argv)
    if a.marker and os.path.exists(a.marker):
        return 0
    from cloudtik_amd.core.state.resp import RespConnection

    def connect(host, port):
        return RespConnection(host, port, a.password or None, timeout=10, connect_retries=30).connect()

    cluster = os.environ.get("CLOUDTIK_CLUSTER", "cloudtik")
    mgr = RedisClusterManager(connect, a.port, a.replicas_per_master, lock=_state_lock(f"{cluster}.redis.role"),
                              password=a.password or None)
    role = mgr.join(a.node_ip, [s for s in a.seeds.split(",") if s], head=a.head)
    print(f"redis cluster: {a.node_ip} -> {role}")
    if a.marker:
        os.makedirs(os.path.dirname(a.marker) or ".", exist_ok=True)
        open(a.marker, "w").close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
