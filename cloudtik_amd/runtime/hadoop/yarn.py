"""YARN-driven scaling policy and job waiter (reference runtime/yarn/scaling_policy.py:48,
runtime/yarn/job_waiter.py:11).

The policy reads the ResourceManager REST API on the head (``/ws/v1/cluster/metrics``,
``/ws/v1/cluster/nodes``) every scaling round:

* ``scaling_mode: apps-pending`` -- applications are pending and the free vcores (or MB)
  dropped below a threshold -> request ``scaling_step`` more worker nodes;
* ``scaling_mode: aggressive`` -- the free share of vcores (or memory) dropped below
  ``aggressive_free_ratio_threshold`` -> request ``scaling_step`` more workers;
* per-node total / used resources come from the NodeManager reports, and NodeManagers that
  are not RUNNING are reported as lost nodes (the scaler's recovery path).

The job waiter blocks ``cloudtik submit --wait`` until no YARN application is pending or
running.  Both take a ``fetch(path) -> dict`` callable so tests drive them with canned
ResourceManager responses.
"""
from __future__ import annotations

import json
import logging
import socket
import time
import urllib.request
from typing import Any, Callable, Dict, List, Optional

from cloudtik_amd.core.provider_api import JobWaiter, ScalingPolicy, ScalingState

logger = logging.getLogger(__name__)

YARN_WEB_PORT = 8088
MODE_NONE, MODE_APPS_PENDING, MODE_AGGRESSIVE = "none", "apps-pending", "aggressive"
RESOURCE_MEMORY, RESOURCE_CPU = "memory", "CPU"


def _http_fetch(head_ip: str, port: int = YARN_WEB_PORT) -> Callable[[str], Dict[str, Any]]:
    def fetch(path: str) -> Dict[str, Any]:
        with urllib.request.urlopen(f"http://{head_ip}:{port}/{path.lstrip('/')}", timeout=10) as r:
            return json.loads(r.read() or b"{}")
    return fetch


def _worker_bundle(config: Dict[str, Any]) -> Dict[str, float]:
    types = config.get("available_node_types") or {}
    for name, t in types.items():
        if name != config.get("head_node_type"):
            res = t.get("resources") or {}
            return {k: float(v) for k, v in res.items() if isinstance(v, (int, float))}
    return {}


def _ip(host: str) -> Optional[str]:
    try:
        return socket.gethostbyname(host)
    except OSError:
        return None


class YarnScalingPolicy(ScalingPolicy):
    def __init__(self, config: Dict[str, Any], head_ip: str,
                 fetch: Optional[Callable[[str], Dict[str, Any]]] = None):
        super().__init__(config, head_ip)
        self.fetch = fetch or _http_fetch(head_ip)
        self.last_request_time = 0.0
        self.reset(config)

    def name(self) -> str:
        return "scaling-with-yarn"

    def reset(self, config):
        self.config = config
        sc = ((config.get("runtime") or {}).get("yarn") or {}).get("scaling") or {}
        self.mode = sc.get("scaling_mode", MODE_NONE) or MODE_NONE
        self.step = int(sc.get("scaling_step", 1))
        self.resource = sc.get("scaling_resource", RESOURCE_MEMORY)
        self.apps_pending_threshold = int(sc.get("apps_pending_threshold", 1))
        self.free_cores_threshold = float(sc.get("apps_pending_free_cores_threshold", 4))
        self.free_memory_threshold = float(sc.get("apps_pending_free_memory_threshold", 1024))
        self.free_ratio_threshold = float(sc.get("aggressive_free_ratio_threshold", 0.1))

    # ---------------------------------------------------------------- decisions
    def nodes_needed(self, m: Dict[str, Any]) -> int:
        cpu = self.resource == RESOURCE_CPU
        avail = float(m["availableVirtualCores"] if cpu else m["availableMB"])
        if self.mode == MODE_AGGRESSIVE:
            total = float(m["totalVirtualCores"] if cpu else m["totalMB"]) or 1.0
            return self.step if avail / total < self.free_ratio_threshold else 0
        if self.mode == MODE_APPS_PENDING:
            thr = self.free_cores_threshold if cpu else self.free_memory_threshold
            if int(m.get("appsPending", 0)) >= self.apps_pending_threshold and avail < thr:
                return self.step
        return 0

    def _requests(self) -> List[Dict[str, float]]:
        if self.mode == MODE_NONE:
            return []
        try:
            m = self.fetch("ws/v1/cluster/metrics").get("clusterMetrics") or {}
        except Exception as e:  # noqa: BLE001 - a scaling round never raises
            logger.warning("YARN cluster metrics unavailable: %s", e)
            return []
        n = self.nodes_needed(m) if m else 0
        if n:
            free = (f"{m['availableVirtualCores']}/{m['totalVirtualCores']} vcores" if self.resource == RESOURCE_CPU
                    else f"{m['availableMB']}/{m['totalMB']} MB")
            logger.info("YARN scaling: %s free, %s pending apps -> %d more worker(s)", free,
                        m.get("appsPending"), n)
            self.last_request_time = time.time()
        bundle = _worker_bundle(self.config)
        return [dict(bundle) for _ in range(n)] if bundle else []

    def _node_states(self):
        try:
            nodes = ((self.fetch("ws/v1/cluster/nodes").get("nodes") or {}).get("node")) or []
        except Exception as e:  # noqa: BLE001
            logger.warning("YARN node reports unavailable: %s", e)
            return {}, {}
        states, lost = {}, {}
        for nd in nodes:
            ip = _ip(nd.get("nodeHostName", ""))
            if ip is None:
                continue
            if nd.get("state") != "RUNNING":
                lost[ip] = ip
                continue
            mb = 1 << 20
            total = {"CPU": nd["availableVirtualCores"] + nd["usedVirtualCores"],
                     "memory": (nd["availMemoryMB"] + nd["usedMemoryMB"]) * mb}
            free = {"CPU": nd["availableVirtualCores"], "memory": nd["availMemoryMB"] * mb}
            states[ip] = {"total": total, "available": free,
                          "used": {k: total[k] - free[k] for k in total}}
        return states, lost

    def get_scaling_state(self) -> Optional[ScalingState]:
        states, lost = self._node_states()
        return ScalingState(autoscaling_instructions={"resource_requests": self._requests(), "time": time.time()},
                            node_resource_states=states, lost_nodes=lost)


class YarnJobWaiter(JobWaiter):
    def __init__(self, config: Dict[str, Any] = None, fetch: Optional[Callable[[str], Dict[str, Any]]] = None,
                 interval: float = 5.0):
        super().__init__(config)
        self.interval = interval
        self._fetch = fetch

    def _fetch_metrics(self) -> Dict[str, Any]:
        if self._fetch is not None:
            return self._fetch("ws/v1/cluster/metrics")
        from cloudtik_amd.core.cluster_tunnel_request import _request_rest_to_head
        return json.loads(_request_rest_to_head(self.config, "ws/v1/cluster/metrics", YARN_WEB_PORT) or b"{}")

    def ongoing(self):
        m = self._fetch_metrics().get("clusterMetrics") or {}
        return int(m.get("appsPending", 0)), int(m.get("appsRunning", 0))

    def wait_for_completion(self, node_id: str, cmd: str, session_name: str = None, timeout: int = None):
        deadline = time.time() + (timeout if timeout is not None else 7 * 24 * 3600)
        pending, running = self.ongoing()
        while pending or running:
            if time.time() >= deadline:
                raise TimeoutError(f"YARN jobs still active: {pending} pending, {running} running")
            logger.info("waiting for YARN jobs: %d pending, %d running", pending, running)
            time.sleep(self.interval)
            pending, running = self.ongoing()
        return True
