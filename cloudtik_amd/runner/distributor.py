"""Host / process distribution for ``cloudtik-run`` (reference
runtime/ai/runner/util/distributor.py:14-354 and util/hosts.py).

Hosts come from ``--hosts ip1,ip2:8`` or a ``--hostfile`` ("ip [slots=N]" or "ip:N" per
line).  Given any subset of (num_proc, nnodes, nproc_per_node, hosts) the distributor
resolves the rest.  On MI355X the natural default is one process per GPU, so an
unspecified ``nproc_per_node`` resolves to the node's visible GPU count (1 without GPUs).
"""
from __future__ import annotations

import os
import re
from dataclasses import dataclass
from typing import List, Optional


@dataclass
class HostSlots:
    host: str
    slots: Optional[int] = None

    def __str__(self):
        return f"{self.host}:{self.slots}" if self.slots else self.host


_HOST_RE = re.compile(r"^\s*([^\s:]+)(?::(\d+))?(?:\s+slots\s*=\s*(\d+))?\s*$")


def parse_host(spec: str) -> HostSlots:
    m = _HOST_RE.match(spec)
    if not m:
        raise ValueError(f"invalid host specification: {spec!r}")
    slots = m.group(2) or m.group(3)
    return HostSlots(m.group(1), int(slots) if slots else None)


def parse_hosts(hosts: str) -> List[HostSlots]:
    return [parse_host(h) for h in hosts.split(",") if h.strip()]


def parse_hostfile(path: str) -> List[HostSlots]:
    out = []
    with open(path) as f:
        for line in f:
            line = line.split("#", 1)[0].strip()
            if line:
                out.append(parse_host(line))
    return out


def local_gpu_count() -> int:
    from cloudtik_amd.core.resources import detect_amd_gpu_count
    try:
        return detect_amd_gpu_count()
    except Exception:  # noqa: BLE001
        return 0


class Distributor:
    def __init__(self, num_proc: int = 0, nnodes: int = 0, nproc_per_node: int = 0,
                 hosts: Optional[str] = None, hostfile: Optional[str] = None):
        self.hosts: List[HostSlots] = []
        if hosts:
            self.hosts = parse_hosts(hosts)
        elif hostfile:
            self.hosts = parse_hostfile(hostfile)
        self.num_proc = int(num_proc or 0)
        self.nnodes = int(nnodes or 0)
        self.nproc_per_node = int(nproc_per_node or 0)
        self.resolve()

    @property
    def distributed_with_hosts(self) -> bool:
        return len(self.hosts) > 0

    @property
    def distributed(self) -> bool:
        return self.nnodes > 1

    def resolve(self):
        if self.hosts:
            if self.nnodes and self.nnodes < len(self.hosts):
                self.hosts = self.hosts[:self.nnodes]
            self.nnodes = len(self.hosts)
            slots = [h.slots for h in self.hosts]
            if self.nproc_per_node == 0:
                if all(s for s in slots) and len(set(slots)) == 1:
                    self.nproc_per_node = slots[0]
                elif self.num_proc:
                    self.nproc_per_node = max(1, self.num_proc // self.nnodes)
                else:
                    self.nproc_per_node = local_gpu_count() or 1
            for h in self.hosts:
                h.slots = h.slots or self.nproc_per_node
        else:
            if self.nnodes == 0:
                # without hosts, extra nodes run their own `cloudtik-run --node-rank i`
                self.nnodes = -(-self.num_proc // self.nproc_per_node) if (self.num_proc and self.nproc_per_node) else 1
            if self.nproc_per_node == 0:
                self.nproc_per_node = (self.num_proc // self.nnodes) if self.num_proc else (local_gpu_count() or 1)
        if self.num_proc == 0:
            self.num_proc = sum(h.slots for h in self.hosts) if self.hosts else self.nnodes * self.nproc_per_node
        total = sum(h.slots for h in self.hosts) if self.hosts else self.nnodes * self.nproc_per_node
        if self.num_proc > total:
            raise ValueError(f"num_proc {self.num_proc} exceeds the {total} slots of {self.nnodes} node(s)")
        return self

    def host_ranks(self):
        """[(host, node_rank, local_world, first_global_rank)] in node order."""
        out, rank = [], 0
        hosts = self.hosts or [HostSlots("127.0.0.1", self.nproc_per_node)]
        for i, h in enumerate(hosts):
            n = min(h.slots or self.nproc_per_node, self.num_proc - rank)
            if n <= 0:
                break
            out.append((h.host, i, n, rank))
            rank += n
        return out

    def export_host_file(self, path: str, with_slots: bool = True):
        with open(path, "w") as f:
            for h in self.hosts or [HostSlots("127.0.0.1", self.nproc_per_node)]:
                f.write(f"{h.host} slots={h.slots}\n" if with_slots else f"{h.host}\n")

    def hosts_str(self) -> str:
        return ",".join(f"{h.host}:{h.slots}" for h in self.hosts)
