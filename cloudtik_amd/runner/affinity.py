"""GPU-aware CPU affinity for one-process-per-GPU jobs (MI355X replacement of the reference's
CPU-socket/core pinning in runtime/ai/runner/cpu/cpu_pool.py + cpu_launcher.py).

Each rank should run on the cores of the NUMA node its GPU hangs off (host<->device copies,
the data loader's pinned buffers and RCCL proxy threads stay local).  The GPU's NUMA node
is read from ``/sys/class/drm/cardN/device/numa_node`` and the node's cores from
``/sys/devices/system/node/nodeX/cpulist``; ranks that share a NUMA node split its cores
evenly.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

from cloudtik_amd.core.node.metrics import amd_gpu_cards


def parse_cpulist(s: str) -> List[int]:
    out = []
    for part in s.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def gpu_numa_nodes(drm_root: str = "/sys/class/drm") -> List[int]:
    out = []
    for card in amd_gpu_cards(drm_root):
        try:
            with open(os.path.join(card, "device", "numa_node")) as f:
                out.append(max(0, int(f.read().strip())))
        except (OSError, ValueError):
            out.append(0)
    return out


def numa_cpus(node: int, sys_root: str = "/sys/devices/system/node") -> List[int]:
    try:
        with open(os.path.join(sys_root, f"node{node}", "cpulist")) as f:
            return parse_cpulist(f.read())
    except OSError:
        return list(range(os.cpu_count() or 1))


def rank_cpu_sets(local_world: int, gpu_numa: Optional[List[int]] = None,
                  cpus_of_node=numa_cpus) -> Dict[int, List[int]]:
    """local_rank -> core list.  Rank r drives GPU r (one process per GPU)."""
    gpu_numa = gpu_numa if gpu_numa is not None else gpu_numa_nodes()
    if not gpu_numa:
        return {}
    ranks_by_node: Dict[int, List[int]] = {}
    for r in range(local_world):
        ranks_by_node.setdefault(gpu_numa[r % len(gpu_numa)], []).append(r)
    out = {}
    for node, ranks in ranks_by_node.items():
        cores = cpus_of_node(node)
        per = max(1, len(cores) // len(ranks))
        for i, r in enumerate(ranks):
            out[r] = cores[i * per:(i + 1) * per] or cores
    return out
