"""Built-in scaling policies (reference core/_private/cluster/scaling_policies.py:43-724,
resource_scaling_policy.py; runtime-provided policies via ``Runtime.get_scaling_policy``).

A policy turns node metrics into resource *requests* the scaler packs against the cluster
(plus per-node resource states):

* ``scaling-with-resources``: reports node resource usage, requests nothing;
* ``scaling-with-load``: when the cluster's CPU load (load-avg / cores), memory use or --
  MI355X addition -- average GPU busy %% stays above its threshold, request
  ``scaling_step`` more worker nodes' worth of resources;
* ``scaling-with-time``: a daily / weekly / monthly table of worker counts
  (``"09:00": 4``, ``"Mon 18:00": "+2"``, ``"20:00": "*0.5"``) relative to min_workers or the
  previous entry;
* ``scaling-by-node-type`` (reference scaling_policies.py:595): ``scaling_policy_by_node_type``
  maps worker node types to their own load / time policy and scaling parameters (e.g. CPU
  ETL nodes scale with load, MI355X GPU nodes on a time table); each sees only the metrics of
  its own nodes and requests bundles of its own type, and the requests are concatenated.

Configured under ``runtime.scaling`` (``scaling_policy: scaling-with-load`` ...).
"""
from __future__ import annotations

import math
import time
from typing import Any, Dict, List, Optional

from cloudtik_amd.core.provider_api import ScalingPolicy, ScalingState

SCALING_WITH_RESOURCES = "scaling-with-resources"
SCALING_WITH_LOAD = "scaling-with-load"
SCALING_WITH_TIME = "scaling-with-time"
SCALING_BY_NODE_TYPE = "scaling-by-node-type"

WEEKDAYS = ["mon", "tue", "wed", "thu", "fri", "sat", "sun"]


def _worker_type(config) -> Optional[str]:
    types = [t for t in config.get("available_node_types", {}) if t != config.get("head_node_type")]
    return types[0] if types else None


def _node_bundle(config, node_type) -> Dict[str, float]:
    res = config["available_node_types"].get(node_type, {}).get("resources") or {}
    return {k: float(v) for k, v in res.items() if isinstance(v, (int, float)) and k in ("CPU", "GPU", "memory")}


class ScalingWithResources(ScalingPolicy):
    def __init__(self, config: Dict[str, Any], head_ip: str, metrics_source=None, node_type: Optional[str] = None,
                 scaling_config: Optional[Dict[str, Any]] = None):
        super().__init__(config, head_ip)
        self.metrics_source = metrics_source        # callable -> {node_id: metrics row}
        self.node_type = node_type                  # scale only this worker type (by-node-type)
        self._scaling_override = scaling_config
        self.reset(config)

    def name(self) -> str:
        return SCALING_WITH_RESOURCES

    def reset(self, config):
        self.config = config
        self.scaling_config = self._scaling_override if self._scaling_override is not None \
            else (config.get("runtime", {}).get("scaling") or {})

    def _wtype(self) -> Optional[str]:
        return self.node_type or _worker_type(self.config)

    def _metrics(self) -> Dict[str, Dict[str, Any]]:
        return self.metrics_source() if self.metrics_source else {}

    def node_resource_states(self, metrics) -> Dict[str, Dict[str, Any]]:
        out = {}
        for nid, m in metrics.items():
            total = dict(m.get("resources") or {})
            cpus = float(m.get("cpu_count") or total.get("CPU", 0) or 0)
            used_cpu = min(cpus, float((m.get("load_avg") or [0])[0]))
            used_gpu = round(len(m.get("gpus") or []) * float(m.get("gpu_busy_percent_avg") or 0) / 100.0, 2)
            out[nid] = {"total": total, "used": {"CPU": used_cpu, "GPU": used_gpu,
                                                   "memory": float(m.get("memory_used") or 0)}}
        return out

    def requests(self, metrics) -> List[Dict[str, float]]:
        return []

    def get_scaling_state(self) -> Optional[ScalingState]:
        metrics = self._metrics()
        return ScalingState(autoscaling_instructions={"resource_requests": self.requests(metrics),
                                                      "time": time.time()},
                            node_resource_states=self.node_resource_states(metrics))


class ScalingWithLoad(ScalingWithResources):
    def name(self) -> str:
        return SCALING_WITH_LOAD

    def reset(self, config):
        super().reset(config)
        c = self.scaling_config
        self.scaling_step = int(c.get("scaling_step", 1))
        self.scaling_resource = c.get("scaling_resource", "CPU")
        self.cpu_threshold = float(c.get("cpu_load_threshold", 0.85))
        self.memory_threshold = float(c.get("memory_load_threshold", 0.85))
        self.gpu_threshold = float(c.get("gpu_busy_threshold", 0.85))

    def _utilisation(self, metrics):
        cpus = sum(float(m.get("cpu_count") or 0) for m in metrics.values())
        load = sum(float((m.get("load_avg") or [0])[0]) for m in metrics.values())
        mem_t = sum(float(m.get("memory_total") or 0) for m in metrics.values())
        mem_u = sum(float(m.get("memory_used") or 0) for m in metrics.values())
        gpus = [g for m in metrics.values() for g in (m.get("gpus") or [])]
        gpu_busy = (sum(float(g.get("busy_percent") or 0) for g in gpus) / (100.0 * len(gpus))) if gpus else 0.0
        return {"cpu": load / cpus if cpus else 0.0, "memory": mem_u / mem_t if mem_t else 0.0, "gpu": gpu_busy,
                "nodes": len(metrics)}

    def requests(self, metrics) -> List[Dict[str, float]]:
        if not metrics:
            return []
        u = self._utilisation(metrics)
        res = self.scaling_resource.upper()
        hot = (res == "CPU" and u["cpu"] > self.cpu_threshold) or \
              (res == "MEMORY" and u["memory"] > self.memory_threshold) or \
              (res == "GPU" and u["gpu"] > self.gpu_threshold)
        if not hot:
            return []
        wt = self._wtype()
        if wt is None:
            return []
        bundle = _node_bundle(self.config, wt)
        # keep what runs now and add `scaling_step` nodes' worth
        return [dict(bundle) for _ in range(max(0, u["nodes"] - 1) + self.scaling_step)]


class ScalingWithTime(ScalingWithResources):
    def name(self) -> str:
        return SCALING_WITH_TIME

    def reset(self, config):
        super().reset(config)
        c = self.scaling_config
        self.periodic = c.get("scaling_periodic", "daily")
        self.math_base = c.get("scaling_math_base", "on-min-workers")
        self.table = self._expand(c.get("scaling_time_table", {}) or {})

    def _seconds(self, spec: str) -> int:
        """``[day ]HH:MM[:SS]`` -> seconds into the period (day: Mon..Sun weekly, 1..31
        monthly)."""
        parts = spec.strip().split()
        day = 0
        if self.periodic == "weekly" and len(parts) == 2:
            day = WEEKDAYS.index(parts[0][:3].lower())
        elif self.periodic == "monthly" and len(parts) == 2:
            day = int(parts[0]) - 1
        hh, mm, ss = (parts[-1].split(":") + ["0", "0"])[:3]
        return day * 86400 + int(hh) * 3600 + int(mm) * 60 + int(ss)

    def _period(self) -> int:
        return {"daily": 86400, "weekly": 7 * 86400, "monthly": 31 * 86400}[self.periodic]

    def _min_workers(self) -> int:
        wt = self._wtype()
        return int(self.config["available_node_types"].get(wt, {}).get("min_workers", 0)) if wt else 0

    @property
    def min_workers(self) -> int:
        return self._min_workers()

    @property
    def scaling_time_table(self) -> List:
        return self.table

    def _expand(self, table: Dict[str, Any]) -> List:
        """Absolute counts, ``+n`` / ``-n`` / ``*f`` relative to the base (min_workers, or the
        previous entry -- cyclically, so a leading relative entry follows the period's last
        one); 0 means min_workers."""
        entries = sorted((self._seconds(k), v) for k, v in table.items())
        mw = self._min_workers()

        def resolve(prev):
            out = []
            for sec, spec in entries:
                base = mw if self.math_base == "on-min-workers" else prev
                s = str(spec).strip()
                if s.startswith(("+", "-")):
                    n = base + int(float(s))
                elif s.startswith("*"):
                    n = int(math.ceil(base * float(s[1:])))
                else:
                    n = int(float(s)) or mw
                n = max(0, n)
                out.append((sec, n))
                prev = n
            return out
        out = resolve(mw)
        if out and self.math_base != "on-min-workers":
            out = resolve(out[-1][1])                # the period wraps: start from its last value
        return out

    def _get_nodes_request(self, seconds: int) -> Optional[int]:
        """Workers wanted ``seconds`` into the period (the last entry before it, wrapping)."""
        if not self.table:
            return None
        current = self.table[-1][1]
        for sec, n in self.table:
            if sec <= seconds:
                current = n
        return current

    def _get_resource_requests_at_seconds(self, seconds: int) -> List[Dict[str, float]]:
        """The whole cluster's resource request at that point: the head plus the workers."""
        n = self._get_nodes_request(seconds)
        wt = self._wtype()
        if n is None or wt is None:
            return []
        head = self.config.get("head_node_type")
        reqs = [_node_bundle(self.config, head)] if head else []
        return reqs + [_node_bundle(self.config, wt) for _ in range(n)]

    def nodes_at(self, t: Optional[float] = None) -> Optional[int]:
        if not self.table:
            return None
        lt = time.localtime(t if t is not None else time.time())
        if self.periodic == "weekly":
            now = lt.tm_wday * 86400
        elif self.periodic == "monthly":
            now = (lt.tm_mday - 1) * 86400
        else:
            now = 0
        now += lt.tm_hour * 3600 + lt.tm_min * 60 + lt.tm_sec
        return self._get_nodes_request(now)

    def requests(self, metrics) -> List[Dict[str, float]]:
        n = self.nodes_at()
        wt = self._wtype()
        if n is None or wt is None:
            return []
        return [_node_bundle(self.config, wt) for _ in range(n)]


class ScalingByNodeType(ScalingWithResources):
    """One sub-policy per worker node type; metrics rows are routed by their ``node_type``
    and rows of other types are still reported as node resource states."""

    def __init__(self, config, head_ip, metrics_source=None, policies: Optional[Dict[str, ScalingPolicy]] = None):
        self.policies = dict(policies or {})
        super().__init__(config, head_ip, metrics_source)

    def name(self) -> str:
        return SCALING_BY_NODE_TYPE

    def reset(self, config):
        super().reset(config)
        for p in getattr(self, "policies", {}).values():
            p.reset(config)

    def get_scaling_state(self) -> Optional[ScalingState]:
        metrics = self._metrics()
        by_type: Dict[str, Dict[str, Any]] = {t: {} for t in self.policies}
        other = {}
        for nid, row in metrics.items():
            t = row.get("node_type")
            (by_type[t] if t in by_type else other)[nid] = row
        requests: List[Dict[str, float]] = []
        states = self.node_resource_states(other)
        for t, p in self.policies.items():
            requests += p.requests(by_type[t])
            states.update(p.node_resource_states(by_type[t]))
        return ScalingState(autoscaling_instructions={"resource_requests": requests, "time": time.time()},
                            node_resource_states=states)


POLICIES = {SCALING_WITH_RESOURCES: ScalingWithResources, SCALING_WITH_LOAD: ScalingWithLoad,
            SCALING_WITH_TIME: ScalingWithTime}


def _by_node_type(config, head_ip, metrics_source, table) -> Optional[ScalingPolicy]:
    types = config.get("available_node_types") or {}
    policies = {}
    for t, sc in (table or {}).items():
        if t == config.get("head_node_type") or t not in types or not sc:
            continue
        name = sc.get("scaling_policy")
        if name not in (SCALING_WITH_LOAD, SCALING_WITH_TIME):
            raise ValueError(f"node type {t}: scaling_policy must be {SCALING_WITH_LOAD} or {SCALING_WITH_TIME}")
        policies[t] = POLICIES[name](config, head_ip, metrics_source, node_type=t, scaling_config=sc)
    return ScalingByNodeType(config, head_ip, metrics_source, policies) if policies else None


def create_scaling_policy(config: Dict[str, Any], head_ip: str, metrics_source=None) -> Optional[ScalingPolicy]:
    """Runtime-provided policy first (e.g. YARN pending containers), then the built-ins."""
    from cloudtik_amd.core import runtime_factory as rf
    from cloudtik_amd.core.cluster_config import get_runtime_types
    for t in get_runtime_types(config):
        p = rf.get_runtime(t, config.get("runtime", {}).get(t, {}) or {}).get_scaling_policy(config, head_ip)
        if p is not None:
            return p
    scaling = config.get("runtime", {}).get("scaling") or {}
    if scaling.get("scaling_policy_by_node_type"):
        return _by_node_type(config, head_ip, metrics_source, scaling["scaling_policy_by_node_type"])
    name = scaling.get("scaling_policy")
    if not name:
        return None
    if name not in POLICIES:
        raise ValueError(f"unknown scaling policy {name!r} (choices: {sorted(POLICIES)})")
    return POLICIES[name](config, head_ip, metrics_source)
