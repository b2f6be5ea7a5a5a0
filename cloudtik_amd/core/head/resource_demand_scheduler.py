"""Which worker nodes to launch for a set of resource demands (reference
core/_private/cluster/resource_demand_scheduler.py:ResourceDemandScheduler.get_nodes_to_launch).

Inputs: the available node types (with their ``resources``, ``min_workers``,
``max_workers``), the current and launching nodes by type, the free resources of running
nodes, a list of resource demand bundles (e.g. ``[{"GPU": 8}, {"CPU": 4}]`` -- from
runtime scaling policies and job waiters), and an optional explicit minimum cluster size
(``cloudtik scale`` requests).

Algorithm:
1. every type is brought up to ``min_workers``;
2. demands are first-fit (largest first) bin-packed onto the free resources of running
   nodes, then onto the full resources of nodes already launching / being added;
3. for the remaining demands node types are added greedily by a utilization score: a
   type must fit at least one demand; GPU types are only chosen for demands that need a
   GPU when CPU-only types could serve them (``CLOUDTIK_CONSERVE_GPU_NODES`` -- an 8 x
   MI355X node is not launched to run a CPU task); among feasible types the one that
   places the most demands and wastes the least capacity wins;
4. the total is capped by per-type and global ``max_workers`` and by the upscaling speed
   (at most ``max(5, upscaling_speed * running)`` new nodes per round).

Demands that no node type can ever satisfy are returned as infeasible.
"""
from __future__ import annotations

import copy
import math
from typing import Dict, List, Optional, Tuple

from cloudtik_amd.core import constants as C

ResourceDict = Dict[str, float]


def fits(avail: ResourceDict, demand: ResourceDict) -> bool:
    return all(avail.get(k, 0.0) + 1e-9 >= v for k, v in demand.items() if v > 0)


def subtract(avail: ResourceDict, demand: ResourceDict) -> None:
    for k, v in demand.items():
        if v > 0:
            avail[k] = avail.get(k, 0.0) - v


def _demand_size(d: ResourceDict) -> Tuple:
    return (d.get("GPU", 0.0), d.get("CPU", 0.0), d.get("memory", 0.0), sum(d.values()))


def bin_pack(demands: List[ResourceDict], bins: List[ResourceDict]) -> List[ResourceDict]:
    """First-fit decreasing; mutates ``bins``; returns the demands that did not fit."""
    left = []
    for d in sorted(demands, key=_demand_size, reverse=True):
        for b in bins:
            if fits(b, d):
                subtract(b, d)
                break
        else:
            left.append(d)
    return left


class ResourceDemandScheduler:
    def __init__(self, node_types: Dict[str, Dict], max_workers: int, head_node_type: str,
                 upscaling_speed: float = 1.0, conserve_gpu_nodes: bool = bool(C.CLOUDTIK_CONSERVE_GPU_NODES)):
        self.node_types = node_types
        self.max_workers = max_workers
        self.head_node_type = head_node_type
        self.upscaling_speed = upscaling_speed
        self.conserve_gpu = conserve_gpu_nodes

    def reset_config(self, node_types, max_workers, head_node_type, upscaling_speed=1.0):
        self.__init__(node_types, max_workers, head_node_type, upscaling_speed, self.conserve_gpu)

    def _resources(self, t: str) -> ResourceDict:
        return {k: float(v) for k, v in (self.node_types[t].get("resources") or {}).items()
                if isinstance(v, (int, float))}

    def _worker_types(self) -> List[str]:
        return [t for t in self.node_types if t != self.head_node_type]

    def _score(self, t: str, demands: List[ResourceDict]) -> Optional[Tuple]:
        res = self._resources(t)
        b = [dict(res)]
        placed = len(demands) - len(bin_pack(list(demands), b))
        if placed == 0:
            return None
        is_gpu_type = res.get("GPU", 0) > 0
        wants_gpu = any(d.get("GPU", 0) > 0 for d in demands)
        gpu_penalty = 1 if (self.conserve_gpu and is_gpu_type and not wants_gpu) else 0
        used = [1.0 - (b[0].get(k, 0.0) / v) for k, v in res.items() if v > 0 and k in ("CPU", "GPU", "memory")]
        util = sum(used) / len(used) if used else 0.0
        return (-gpu_penalty, placed, util)

    def get_nodes_to_launch(self, existing: Dict[str, int], launching: Dict[str, int],
                            resource_demands: List[ResourceDict],
                            unused_resources: Dict[str, ResourceDict],
                            min_cluster_bundles: Optional[List[ResourceDict]] = None,
                            running_count: Optional[int] = None
                            ) -> Tuple[Dict[str, int], List[ResourceDict]]:
        counts = {t: existing.get(t, 0) + launching.get(t, 0) for t in self.node_types}
        total = sum(c for t, c in counts.items() if t != self.head_node_type)
        to_add: Dict[str, int] = {}

        def can_add(t):
            mx = self.node_types[t].get("max_workers", self.max_workers)
            return counts[t] + to_add.get(t, 0) < mx and total + sum(to_add.values()) < self.max_workers

        # 1) min_workers
        for t in self._worker_types():
            need = self.node_types[t].get("min_workers", 0) - counts[t]
            for _ in range(max(0, need)):
                if not can_add(t):
                    break
                to_add[t] = to_add.get(t, 0) + 1

        def capacity_bins(include_unused=True):
            bins = [dict(r) for r in unused_resources.values()] if include_unused else []
            for t, n in launching.items():
                bins += [self._resources(t) for _ in range(n)]
            for t, n in to_add.items():
                bins += [self._resources(t) for _ in range(n)]
            return bins

        # 2) explicit minimum cluster size: bundles against the TOTAL capacity of all nodes;
        # 3) pending demands against the FREE capacity -- two separate views of the same
        #    nodes (a request is a floor on cluster size, a demand is unplaced load)
        remaining = []
        if min_cluster_bundles:
            total_bins = [self._resources(t) for t, n in existing.items() for _ in range(n)]
            total_bins += capacity_bins(include_unused=False)
            remaining += bin_pack([dict(d) for d in min_cluster_bundles], total_bins)
        remaining += bin_pack([dict(d) for d in resource_demands], capacity_bins())
        infeasible = []
        while remaining:
            best, best_score = None, None
            for t in self._worker_types():
                if not can_add(t):
                    continue
                s = self._score(t, remaining)
                if s is not None and (best_score is None or s > best_score):
                    best, best_score = t, s
            if best is None:
                break
            to_add[best] = to_add.get(best, 0) + 1
            remaining = bin_pack(remaining, [self._resources(best)])
        for d in remaining:
            if not any(fits(self._resources(t), d) for t in self._worker_types()):
                infeasible.append(d)

        # 4) upscaling speed
        running = running_count if running_count is not None else total
        cap = max(5, int(math.ceil(self.upscaling_speed * max(1, running))))
        out, n = {}, 0
        for t, c in sorted(to_add.items()):
            take = min(c, cap - n)
            if take > 0:
                out[t] = take
                n += take
        return out, infeasible

    def node_type_resources(self, t: str) -> ResourceDict:
        return copy.deepcopy(self._resources(t))
