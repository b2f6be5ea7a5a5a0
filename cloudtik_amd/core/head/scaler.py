"""Head-side cluster scaler (reference core/_private/cluster/cluster_scaler.py:ClusterScaler,
node_launcher.py:NodeLauncher, node_tracker / node_availability_tracker).

One :meth:`ClusterScaler.update` round:

1. reload the cluster config if its file changed (``cloudtik start`` on an existing cluster);
2. collect worker nodes, their tags, the heartbeats and free resources from the state
   service;
3. terminate workers that are outdated (launch-config hash changed), over ``max_workers``,
   failed to set up, or idle longer than ``idle_timeout_minutes`` above ``min_workers``;
4. ask :class:`ResourceDemandScheduler` what to launch for ``min_workers``, the resource
   demands published in the state service and ``cloudtik scale`` requests, and launch them
   in batches (:class:`NodeLauncher`), backing off node types that recently failed to
   launch (:class:`NodeAvailabilityTracker`);
5. start :class:`NodeUpdaterThread` s for uninitialized nodes, and recovery updaters for
   up-to-date nodes whose heartbeat is older than ``CLOUDTIK_HEARTBEAT_TIMEOUT_S``;
6. publish a scaling status summary (nodes by status, launching, failures, demands).
"""
from __future__ import annotations

import json
import logging
import threading
import time
from collections import Counter, defaultdict
from typing import Any, Dict, List, Optional

from cloudtik_amd.core import constants as C
from cloudtik_amd.core import tags as T
from cloudtik_amd.core.cluster_utils import create_updater, get_head_node, next_seq_id, node_tags
from cloudtik_amd.core.head.resource_demand_scheduler import ResourceDemandScheduler, subtract
from cloudtik_amd.core.node_provider import NodeLaunchException

logger = logging.getLogger(__name__)

SCALING_NAMESPACE = C.KV_NAMESPACE_SCALING
KEY_RESOURCE_DEMANDS = b"resource_demands"      # JSON list of bundles, written by runtimes/jobs
KEY_CLUSTER_REQUESTS = b"cluster_requests"      # JSON {"bundles": [...], "time": t}, `cloudtik scale`
KEY_SCALING_STATUS = b"scaling_status"


class NodeAvailabilityTracker:
    """Remembers launch failures per node type for a staleness window."""

    def __init__(self, staleness_s: float = C.CLOUDTIK_NODE_AVAILABILITY_MAX_STALENESS_S):
        self.staleness = staleness_s
        self.failures: Dict[str, tuple] = {}

    def record_failure(self, node_type: str, category: str, description: str):
        self.failures[node_type] = (time.time(), category, description)

    def record_success(self, node_type: str):
        self.failures.pop(node_type, None)

    def unavailable(self) -> Dict[str, tuple]:
        now = time.time()
        return {t: f for t, f in self.failures.items() if now - f[0] < min(self.staleness, 300)}


class NodeLauncher(threading.Thread):
    def __init__(self, provider, config, node_type: str, count: int, tracker: NodeAvailabilityTracker,
                 pending: Counter, lock: threading.Lock, extra_tags: Optional[Dict[str, str]] = None):
        super().__init__(daemon=True, name=f"launcher-{node_type}")
        self.provider, self.config = provider, config
        self.node_type, self.count = node_type, count
        self.extra_tags = dict(extra_tags or {})      # e.g. the quorum a joining node enters
        self.tracker, self.pending, self.lock = tracker, pending, lock
        self.error: Optional[BaseException] = None

    def run(self):
        try:
            nt = self.config["available_node_types"][self.node_type]
            for _ in range(self.count):
                with self.lock:
                    seq = next_seq_id(self.provider, self.config["cluster_name"])
                tags = node_tags(self.config, self.node_type, T.NODE_KIND_WORKER, seq, self.provider)
                tags.update(self.extra_tags)
                self.provider.create_node_with_resources(nt.get("node_config", {}), tags, 1,
                                                         nt.get("resources", {}))
            self.tracker.record_success(self.node_type)
        except NodeLaunchException as e:
            self.error = e
            self.tracker.record_failure(self.node_type, e.category, e.description)
            logger.warning("failed to launch %s x %d: %s", self.node_type, self.count, e)
        except Exception as e:  # noqa: BLE001
            self.error = e
            self.tracker.record_failure(self.node_type, "Unknown", str(e))
            logger.exception("failed to launch %s", self.node_type)
        finally:
            with self.lock:
                self.pending[self.node_type] -= self.count


class ClusterScaler:
    def __init__(self, config: Dict[str, Any], provider, state_client=None, head_ip: Optional[str] = None,
                 config_reader=None, synchronous: bool = False):
        self.config = config
        self.provider = provider
        self.state = state_client
        self.config_reader = config_reader
        self.synchronous = synchronous       # tests: launch + update inline
        self.head_ip = head_ip or self._head_ip()
        opts = config.get("options", {}) or {}
        self.scheduler = ResourceDemandScheduler(config["available_node_types"], config.get("max_workers", 0),
                                                 config["head_node_type"], opts.get("upscaling_speed", 1.0))
        self.idle_timeout_s = 60.0 * float(opts.get("idle_timeout_minutes", 5))
        self.tracker = NodeAvailabilityTracker()
        self.pending_launches: Counter = Counter()
        self.launch_lock = threading.Lock()
        self.updaters: Dict[str, Any] = {}
        self.failed_updates: Counter = Counter()
        self.gpu_unhealthy_since: Dict[str, float] = {}
        self.last_active: Dict[str, float] = {}
        self.num_failures = 0
        self.events: List[str] = []
        self.last_update_time = None
        from cloudtik_amd.core.head.quorum_manager import QuorumManager
        from cloudtik_amd.core.head.scaling_policies import create_scaling_policy
        self.quorum = QuorumManager(config, provider, state_client)
        self.policy = create_scaling_policy(config, self.head_ip, metrics_source=self.node_metrics)
        self.policy_requests: List[Dict[str, float]] = []

    # ------------------------------------------------------------------ inputs
    def _head_ip(self) -> Optional[str]:
        h = get_head_node(self.provider, self.config["cluster_name"])
        return self.provider.internal_ip(h) if h else None

    def workers(self) -> List[str]:
        return self.provider.non_terminated_nodes({T.CLOUDTIK_TAG_CLUSTER_NAME: self.config["cluster_name"],
                                                   T.CLOUDTIK_TAG_NODE_KIND: T.NODE_KIND_WORKER})

    def _kv_json(self, key):
        if self.state is None:
            return None
        v = self.state.kv_get(key, namespace=SCALING_NAMESPACE)
        return json.loads(v) if v else None

    def resource_demands(self) -> List[Dict[str, float]]:
        return list(self._kv_json(KEY_RESOURCE_DEMANDS) or [])

    def cluster_requests(self) -> List[Dict[str, float]]:
        """`cloudtik scale` requests, raised to what the scaling policy asks for."""
        r = self._kv_json(KEY_CLUSTER_REQUESTS) or {}
        user = list(r.get("bundles", []))
        return user if len(user) >= len(self.policy_requests) else list(self.policy_requests)

    def heartbeats(self) -> Dict[str, Dict]:
        if self.state is None:
            return {}
        from cloudtik_amd.core.state.state_client import NODE_TABLE
        return self.state.table_get_all(NODE_TABLE)

    def node_metrics(self) -> Dict[str, Dict]:
        if self.state is None:
            return {}
        from cloudtik_amd.core.state.state_client import NODE_METRICS_TABLE
        rows = self.state.table_get_all(NODE_METRICS_TABLE)
        # tag each row with its node type (scaling-by-node-type routes metrics by it)
        types = {}
        try:
            for n in self.workers():
                t = self.provider.node_tags(n).get(T.CLOUDTIK_TAG_USER_NODE_TYPE)
                types[n] = t
                ip = self.provider.internal_ip(n)
                if ip:
                    types[ip] = t
        except Exception:  # noqa: BLE001 - metrics stay usable without types
            return rows
        for nid, row in rows.items():
            if isinstance(row, dict) and "node_type" not in row:
                t = types.get(nid) or types.get(row.get("node_ip") or row.get("ip"))
                if t:
                    row["node_type"] = t
        return rows

    # ------------------------------------------------------------------ round
    def reset_config(self, config: Dict[str, Any]):
        self.config = config
        opts = config.get("options", {}) or {}
        self.scheduler.reset_config(config["available_node_types"], config.get("max_workers", 0),
                                    config["head_node_type"], opts.get("upscaling_speed", 1.0))
        self.idle_timeout_s = 60.0 * float(opts.get("idle_timeout_minutes", 5))
        self.quorum.reset(config, self.provider)
        if self.policy is not None:
            self.policy.reset(config)

    def update(self):
        try:
            self._update()
            self.num_failures = 0
        except Exception:  # noqa: BLE001
            self.num_failures += 1
            logger.exception("cluster scaler update failed (%d in a row)", self.num_failures)
            if self.num_failures > C.CLOUDTIK_MAX_NUM_FAILURES:
                raise

    def _update(self):
        if self.config_reader is not None:
            new = self.config_reader()
            if new is not None and new != self.config:
                self.reset_config(new)
        now = time.time()
        self.last_update_time = now
        if self.policy is not None:
            st = self.policy.get_scaling_state()
            self.policy_requests = list(((st.autoscaling_instructions or {}) if st else {}).get("resource_requests", []))
        workers = self.workers()
        tags = {n: self.provider.node_tags(n) for n in workers}
        types = self.config["available_node_types"]
        with self.launch_lock:
            self.quorum.update(workers, tags, dict(+self.pending_launches))

        # 3) terminations
        to_terminate: Dict[str, str] = {}
        for n in workers:
            t = tags[n]
            nt = t.get(T.CLOUDTIK_TAG_USER_NODE_TYPE)
            if nt not in types:
                to_terminate[n] = "unknown node type"
                continue
            if self.quorum.terminate_for_quorum(nt, n):
                to_terminate[n] = "member of a quorum that lost its majority"
                continue
            from cloudtik_amd.core.cluster_utils import launch_hash
            if t.get(T.CLOUDTIK_TAG_LAUNCH_CONFIG) != launch_hash(self.config, nt, self.provider):
                to_terminate[n] = "outdated launch config"
            elif t.get(T.CLOUDTIK_TAG_NODE_STATUS) == T.STATUS_UPDATE_FAILED and n not in self.updaters:
                to_terminate[n] = "setup failed"
        by_type = defaultdict(list)
        for n in workers:
            if n not in to_terminate:
                by_type[tags[n].get(T.CLOUDTIK_TAG_USER_NODE_TYPE)].append(n)
        for nt, nodes in by_type.items():
            mx = types.get(nt, {}).get("max_workers", 0)
            for n in sorted(nodes, key=lambda x: tags[x].get(T.CLOUDTIK_TAG_NODE_SEQ_ID, ""))[mx:]:
                to_terminate[n] = "over max_workers"
        self._terminate_idle(by_type, tags, to_terminate, now)
        for n, why in to_terminate.items():
            self._log(f"terminating {n}: {why}")
            self.updaters.pop(n, None)
        if to_terminate:
            self.provider.terminate_nodes(list(to_terminate))
            self.quorum.remove_terminating(list(to_terminate))
            workers = [n for n in workers if n not in to_terminate]

        # 4) launches
        existing = Counter(tags[n].get(T.CLOUDTIK_TAG_USER_NODE_TYPE) for n in workers)
        hb = self.heartbeats()
        unused = {}
        for nid, info in self.node_metrics().items():
            res = dict(info.get("resources") or {})
            unused[nid] = res
        with self.launch_lock:
            launching = dict(+self.pending_launches)
        to_launch, infeasible = self.scheduler.get_nodes_to_launch(
            dict(existing), launching, self.resource_demands(), self._free_resources(unused),
            self.cluster_requests(), running_count=len(workers))
        unavailable = self.tracker.unavailable()
        for nt, cnt in self._prioritize_launch(to_launch).items():
            if nt in unavailable:
                continue
            allowed, qid = self.quorum.is_launch_allowed(nt)
            if not allowed:
                continue
            if qid:
                cnt = 1                    # a running quorum grows one joining node at a time
            self._launch(nt, cnt, self.quorum.launch_tags(qid))
        self.infeasible = infeasible

        # 5) updates + recovery; held back while a constrained node type (quorum runtimes)
        # lacks its minimal membership
        workers = self.workers()
        to_replace = []
        if self.quorum.enabled:
            with self.launch_lock:
                pending = dict(+self.pending_launches)
            self.quorum.update(workers, {}, pending)
        if self.quorum.wait_for_update():
            self.publish_status()
            return
        for n in workers:
            t = self.provider.node_tags(n)
            status = t.get(T.CLOUDTIK_TAG_NODE_STATUS)
            u = self.updaters.get(n)
            if u is not None and (not hasattr(u, "is_alive") or not u.is_alive()):
                self.updaters.pop(n)
                if u.exitcode != 0:
                    self.failed_updates[n] += 1
                self.quorum.on_update_done(n, u.exitcode == 0)
                continue
            if u is not None:
                continue
            if status == T.STATUS_UNINITIALIZED:
                self._spawn_updater(n, recovery=False)
            elif status == T.STATUS_UP_TO_DATE and self.state is not None:
                beat = hb.get(n) or hb.get(self.provider.internal_ip(n) or "")
                last = (beat or {}).get("last_heartbeat_time")
                started = float(t.get("cloudtik-up-time", 0) or 0)
                if last is not None and now - last > C.CLOUDTIK_HEARTBEAT_TIMEOUT_S and now - started > C.CLOUDTIK_HEARTBEAT_TIMEOUT_S:
                    self._log(f"node {n} lost heartbeat for {now - last:.0f}s: recovering")
                    self._spawn_updater(n, recovery=True)
                    continue
                self._check_gpu_health(n, now, to_replace)
        if to_replace:
            # a GPU that keeps reporting uncorrectable errors / overheating is not fixed by
            # restarting services: terminate the node; the next pass launches a replacement
            self.provider.terminate_nodes(list(to_replace))
        self.publish_status()

    def _check_gpu_health(self, n: str, now: float, to_replace: List[str]):
        m = self.node_metrics().get(n) or self.node_metrics().get(self.provider.internal_ip(n) or "") or {}
        if m.get("gpu_healthy", True):
            self.gpu_unhealthy_since.pop(n, None)
            return
        since = self.gpu_unhealthy_since.setdefault(n, now)
        if now - since >= C.CLOUDTIK_GPU_UNHEALTHY_TIMEOUT_S:
            self._log(f"node {n} GPUs unhealthy for {now - since:.0f}s "
                      f"({'; '.join(m.get('gpu_health_issues') or [])}): replacing")
            self.gpu_unhealthy_since.pop(n, None)
            to_replace.append(n)

    def _free_resources(self, unused: Dict[str, Dict]) -> Dict[str, Dict]:
        # without per-task accounting the free capacity of a node is its static resources
        # minus what the runtime reported as used (``used_resources`` in the metrics row)
        out = {}
        for nid, res in unused.items():
            r = dict(res)
            m = self.node_metrics().get(nid, {}) if self.state is not None else {}
            subtract(r, m.get("used_resources", {}) or {})
            out[nid] = r
        return out

    def _terminate_idle(self, by_type, tags, to_terminate, now):
        if self.idle_timeout_s <= 0:
            return
        metrics = self.node_metrics()
        demands = self.resource_demands() or self.cluster_requests()
        for nt, nodes in by_type.items():
            mn = self.config["available_node_types"].get(nt, {}).get("min_workers", 0)
            candidates = []
            for n in nodes:
                ip = self.provider.internal_ip(n)
                m = metrics.get(n) or metrics.get(ip or "") or {}
                busy = (m.get("cpu_percent") or 0) > 10 or (m.get("gpu_busy_percent_avg") or 0) > 5
                if busy or demands or n not in self.last_active:
                    self.last_active[n] = now
                if now - self.last_active[n] > self.idle_timeout_s:
                    candidates.append(n)
            keep = max(0, len(nodes) - len(candidates))
            for n in candidates:
                if keep >= mn:
                    to_terminate[n] = "idle"
                else:
                    keep += 1

    def _prioritize_launch(self, to_launch: Dict[str, int]) -> Dict[str, int]:
        """Only the node types of the lowest ``launch_priority`` value launch this round
        (reference cluster_scaler.py:671 _prioritize_launch): storage / coordination types
        come up before the compute types that discover them."""
        if len(to_launch) <= 1:
            return dict(to_launch)
        types = self.config["available_node_types"]
        prio = {nt: int((types.get(nt) or {}).get("launch_priority", 0) or 0) for nt in to_launch}
        best = min(prio.values())
        return {nt: c for nt, c in to_launch.items() if prio[nt] == best}

    def _launch(self, node_type: str, count: int, extra_tags: Optional[Dict[str, str]] = None):
        count = min(count, C.CLOUDTIK_MAX_LAUNCH_BATCH * 4)
        with self.launch_lock:
            self.pending_launches[node_type] += count
        self._log(f"launching {count} x {node_type}" + (" (quorum join)" if extra_tags else ""))
        launcher = NodeLauncher(self.provider, self.config, node_type, count, self.tracker,
                                self.pending_launches, self.launch_lock, extra_tags)
        if self.synchronous:
            launcher.run()
        else:
            launcher.start()

    def _spawn_updater(self, node_id: str, recovery: bool):
        self.provider.set_node_tags(node_id, {"cloudtik-up-time": str(time.time())})
        u = create_updater(self.config, self.provider, node_id, is_head=False, head_ip=self.head_ip,
                           for_recovery=recovery, threaded=not self.synchronous)
        self.updaters[node_id] = u
        if self.synchronous:
            u.run()
            self.updaters.pop(node_id)
            if u.exitcode != 0:
                self.failed_updates[node_id] += 1
            self.quorum.on_update_done(node_id, u.exitcode == 0)
        else:
            u.start()

    def _log(self, msg: str):
        logger.info(msg)
        self.events.append(f"{time.strftime('%H:%M:%S')} {msg}")
        self.events = self.events[-100:]

    # ------------------------------------------------------------------ status
    def summary(self) -> Dict[str, Any]:
        workers = self.workers()
        by_status = defaultdict(list)
        by_type = Counter()
        for n in workers:
            t = self.provider.node_tags(n)
            by_status[t.get(T.CLOUDTIK_TAG_NODE_STATUS, "unknown")].append(n)
            by_type[t.get(T.CLOUDTIK_TAG_USER_NODE_TYPE)] += 1
        with self.launch_lock:
            launching = dict(+self.pending_launches)
        return {
            "time": time.time(),
            "head_ip": self.head_ip,
            "workers": len(workers),
            "nodes_by_status": {k: sorted(v) for k, v in by_status.items()},
            "nodes_by_type": dict(by_type),
            "launching": launching,
            "updating": sorted(self.updaters),
            "failed_launches": {k: list(v) for k, v in self.tracker.unavailable().items()},
            "resource_demands": self.resource_demands(),
            "cluster_requests": self.cluster_requests(),
            "infeasible": getattr(self, "infeasible", []),
            "events": self.events[-20:],
        }

    def publish_status(self):
        if self.state is not None:
            self.state.kv_put(KEY_SCALING_STATUS, json.dumps(self.summary()), namespace=SCALING_NAMESPACE)
