"""Ray-driven scaling policy (reference runtime/ray/scaling_policy.py:86 ``RayScalingPolicy``,
which reads the GCS resource usage over gRPC).

Here the policy reads the Ray dashboard's REST API on the head -- no ``ray`` package is needed
in the controller's environment:

* ``/api/cluster_status`` -> ``loadMetricsReport.resourceDemand`` (``[[shape, count], ...]``,
  queued + infeasible task / actor shapes) and ``pgDemand`` (placement-group bundles): the
  resource demands the scaler bin-packs onto node types (``scaling.auto_scaling: true``),
  clipped like the reference to 1000 waiting + 1000 infeasible bundles;
* ``/nodes?view=summary`` -> per node total / available resources and raylet state; DEAD
  raylets are reported as lost nodes (the scaler's recovery path).

A Ray ``GPU`` is one MI355X (the ray runtime starts raylets with ``--num-gpus`` = the node's
AMD GPUs), so GPU task demands become node launches of the GPU node type.  ``fetch(path)``
is injectable for tests.
"""
from __future__ import annotations

import json
import logging
import time
import urllib.request
from typing import Any, Callable, Dict, List, Optional, Tuple

from cloudtik_amd.core.provider_api import ScalingPolicy, ScalingState

logger = logging.getLogger(__name__)

RAY_DASHBOARD_PORT = 8265
MAX_DEMAND = 1000


def _http_fetch(head_ip: str, port: int = RAY_DASHBOARD_PORT) -> Callable[[str], Dict[str, Any]]:
    def fetch(path: str) -> Dict[str, Any]:
        with urllib.request.urlopen(f"http://{head_ip}:{port}/{path.lstrip('/')}", timeout=10) as r:
            return json.loads(r.read() or b"{}")
    return fetch


def resource_demands(report: Dict[str, Any]) -> List[Dict[str, float]]:
    """Expand ``[[shape, count], ...]`` demand entries (and placement-group bundles) into a
    bounded list of resource bundles."""
    out: List[Dict[str, float]] = []
    for shape, count in report.get("resourceDemand") or []:
        out += [{k: float(v) for k, v in shape.items()} for _ in range(min(int(count), MAX_DEMAND - len(out)))]
        if len(out) >= MAX_DEMAND:
            break
    pg: List[Dict[str, float]] = []
    for entry in report.get("pgDemand") or []:
        bundles = entry[0] if isinstance(entry, (list, tuple)) else entry.get("bundles", [])
        count = int(entry[1]) if isinstance(entry, (list, tuple)) and len(entry) > 1 else 1
        for _ in range(count):
            for b in bundles:
                if len(pg) < MAX_DEMAND:
                    pg.append({k: float(v) for k, v in (b.get("resources", b)).items()})
    return out + pg


class RayScalingPolicy(ScalingPolicy):
    def __init__(self, config: Dict[str, Any], head_ip: str,
                 fetch: Optional[Callable[[str], Dict[str, Any]]] = None):
        super().__init__(config, head_ip)
        self.fetch = fetch or _http_fetch(head_ip)
        rc = ((config.get("runtime") or {}).get("ray") or {})
        self.auto_scaling = bool(rc.get("auto_scaling") or (rc.get("scaling") or {}).get("auto_scaling"))

    def name(self) -> str:
        return "scaling-with-ray"

    def _demands(self) -> Optional[Dict[str, Any]]:
        if not self.auto_scaling:
            return None
        try:
            st = self.fetch("api/cluster_status?format=0")
            report = (((st.get("data") or {}).get("clusterStatus") or {}).get("loadMetricsReport")) or {}
        except Exception as e:  # noqa: BLE001 - a scaling round never raises
            logger.warning("Ray cluster status unavailable: %s", e)
            return None
        d = resource_demands(report)
        if d:
            logger.info("Ray scaling: %d pending resource bundles", len(d))
        return {"resource_demands": d, "time": time.time()}

    def _nodes(self) -> Tuple[Dict[str, Any], Dict[str, str]]:
        try:
            rows = ((self.fetch("nodes?view=summary").get("data") or {}).get("summary")) or []
        except Exception as e:  # noqa: BLE001
            logger.warning("Ray node summary unavailable: %s", e)
            return {}, {}
        states, lost = {}, {}
        for n in rows:
            r = n.get("raylet") or n
            ip = r.get("nodeManagerAddress") or n.get("ip")
            if not ip:
                continue
            if r.get("state", "ALIVE") != "ALIVE":
                lost[ip] = ip
                continue
            total = {k: float(v) for k, v in (r.get("resourcesTotal") or {}).items() if not k.startswith("node:")}
            avail = {k: float(v) for k, v in (r.get("resourcesAvailable") or total).items()
                     if not k.startswith("node:")}
            states[ip] = {"total": total, "available": avail,
                          "used": {k: total[k] - avail.get(k, 0.0) for k in total}}
        lost = {k: v for k, v in lost.items() if k not in states}
        return states, lost

    def get_scaling_state(self) -> Optional[ScalingState]:
        states, lost = self._nodes()
        return ScalingState(autoscaling_instructions=self._demands(), node_resource_states=states, lost_nodes=lost)
