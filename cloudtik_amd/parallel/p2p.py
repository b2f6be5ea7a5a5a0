"""One-shot peer-to-peer all-reduce for small buckets ("custom one-shot
P2P all-reduce for <= ~1 M elements"; the reference only reaches NCCL / oneCCL / gloo
all-reduce, trainer.py:215-219 and run_pretrain_mlperf.py:565-567).

RCCL's ring all-reduce costs 2*(world-1) latency-bound steps; for the small buckets of a
step (metric scalars, LayerNorm / bias gradients, the tail bucket) that latency dominates.
On one MI355X node every GPU pair has a direct xGMI link, so a single kernel can read all
peers' buffers at once: ``P2PAllReducer`` keeps one IPC-exported staging buffer and one
uncached signal buffer per rank, maps every peer's pair once (``hipIpcOpenMemHandle``,
handles exchanged over the process group), and each ``all_reduce`` is

    copy input -> own staging buffer (hipMemcpyAsync);  one kernel (ops/csrc/p2p.hip): barrier-in on the
    signal buffers, sum all ranks' staging buffers in fixed rank order (fp32 accumulate,
    bit-identical on every rank), write the output, barrier-out.

Buckets larger than ``max_bytes`` (and non-fp32/bf16 or misaligned tensors) go to RCCL
through ``torch.distributed.all_reduce``.  Barrier waits are bounded in the kernel; a rank
that never arrives raises ``RuntimeError`` on ``check()`` instead of hanging the GPU.
Opt-in for the Trainer through ``CLOUDTIK_P2P_ALLREDUCE_BYTES`` (see parallel/ddp.py).
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.distributed as dist


class P2PAllReducer:
    def __init__(self, group=None, max_bytes: int = 4 << 20, blocks: int = 32, max_spin: int = 1 << 24,
                 device: Optional[torch.device] = None):
        from cloudtik_amd import ops
        ops.require_native()
        self._C = ops._C
        self.group = group
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        if self.world > 8:
            raise ValueError("the one-shot P2P all-reduce spans at most 8 ranks (one xGMI-connected node)")
        self.max_bytes = int(max_bytes)
        self.blocks, self.max_spin = int(blocks), int(max_spin)
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        with torch.cuda.device(self.device):
            self._staging = self._C.p2p_alloc(self.max_bytes, False)
            self._signal = self._C.p2p_alloc(0, True)
            mine = (self._C.ipc_get(self._staging), self._C.ipc_get(self._signal))
            handles: List = [None] * self.world
            dist.all_gather_object(handles, mine, group=group)
            self._opened: List[int] = []
            self._data, self._sig = [], []
            for r, (hd, hs) in enumerate(handles):
                if r == self.rank:
                    self._data.append(self._staging)
                    self._sig.append(self._signal)
                    continue
                d, s = self._C.ipc_open(hd), self._C.ipc_open(hs)
                self._opened += [d, s]
                self._data.append(d)
                self._sig.append(s)
        self._epoch = 0
        # every rank has mapped every peer before anyone signals into a peer's buffer
        dist.barrier(group=group)

    def supports(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.is_contiguous() and t.dtype in (torch.float32, torch.bfloat16)
                and t.numel() * t.element_size() <= self.max_bytes and t.data_ptr() % 16 == 0)

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        """In-place sum over the group (same contract as ``dist.all_reduce``)."""
        if not self.supports(t):
            dist.all_reduce(t, group=self.group)
            return t
        self._epoch = (self._epoch + 1) & 0xFFFFFFFF or 1
        self._C.p2p_allreduce(self._data, self._sig, t, self.max_bytes, self.rank, self.world, self._epoch,
                              self.max_spin, self.blocks)
        return t

    def check(self):
        """Synchronous: raise if any barrier of this rank timed out since construction."""
        if self._C.p2p_error(self._signal):
            raise RuntimeError(f"rank {self.rank}: P2P all-reduce barrier timed out (a peer did not arrive)")

    def close(self):
        if self._staging is None:
            return
        torch.cuda.synchronize(self.device)
        dist.barrier(group=self.group)  # no peer still reads our buffers
        for p in self._opened:
            self._C.ipc_close(p)
        self._C.p2p_free(self._staging)
        self._C.p2p_free(self._signal)
        self._staging = self._signal = None
        self._opened = []


def from_env(group=None) -> Optional[P2PAllReducer]:
    """``CLOUDTIK_P2P_ALLREDUCE_BYTES=<n>`` (> 0) enables the one-shot path for buckets up to n bytes."""
    n = int(os.environ.get("CLOUDTIK_P2P_ALLREDUCE_BYTES", "0") or 0)
    if n <= 0 or not torch.cuda.is_available() or not dist.is_initialized() or dist.get_world_size(group) > 8:
        return None
    return P2PAllReducer(group, max_bytes=n)
