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
through ``torch.distributed.all_reduce``.  Barrier waits are bounded in WALL-CLOCK time
(``timeout_s``, default ``CLOUDTIK_P2P_TIMEOUT_S`` or 300 s -- an RCCL-like timeout, so a
slow peer doing a first-step solver search or a checkpoint is waited for); a timed-out wait
sets a host-mapped error word that ``check()`` reads without a device sync.  The gradient
bucketer calls ``check()`` every step and raises, so a missing peer is fatal for the job
(restart from the last checkpoint) instead of silently diverging ranks.
Opt-in for the Trainer through ``CLOUDTIK_P2P_ALLREDUCE_BYTES`` (see parallel/ddp.py); only
enabled when every rank of the group runs on ONE host (xGMI domain), decided collectively.
Verified so far with two ranks sharing one MI355X (tests/test_p2p_gpu.py); the cross-GPU
xGMI path has not been measured yet.
"""
from __future__ import annotations

import os
import socket
from typing import List, Optional

import torch
import torch.distributed as dist


class P2PAllReducer:
    def __init__(self, group=None, max_bytes: int = 4 << 20, blocks: int = 32, timeout_s: Optional[float] = None,
                 device: Optional[torch.device] = None):
        from cloudtik_amd import ops
        ops.require_native()
        self._C = ops._C
        self.group = group
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        if self.world > 8:
            raise ValueError("the one-shot P2P all-reduce spans at most 8 ranks (one xGMI-connected node)")
        self.max_bytes = int(max_bytes)
        self.blocks = int(blocks)
        self.timeout_s = float(timeout_s if timeout_s is not None else os.environ.get("CLOUDTIK_P2P_TIMEOUT_S", 300))
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        with torch.cuda.device(self.device):
            self._staging = self._C.p2p_alloc(self.max_bytes, False)
            self._signal = self._C.p2p_alloc(0, True)
            self._err_host, self._err_dev = self._C.p2p_alloc_flag()
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
                              self.timeout_s, self._err_dev, self.blocks)
        return t

    def error(self) -> int:
        """Non-zero once a barrier of an already-finished kernel timed out (1 = barrier-in: the
        output is this rank's unreduced input; 2 = barrier-out).  No device sync."""
        return int(self._C.p2p_error(self._err_host)) if self._staging is not None else 0

    def check(self):
        """Raise if any barrier of this rank timed out (among kernels finished so far)."""
        e = self.error()
        if e:
            raise RuntimeError(f"rank {self.rank}: P2P all-reduce {'barrier-in' if e == 1 else 'barrier-out'} "
                               f"timed out after {self.timeout_s:.0f}s (a peer did not arrive); the reduced "
                               f"gradients are invalid -- restart from the last checkpoint")

    def close(self):
        if self._staging is None:
            return
        torch.cuda.synchronize(self.device)
        dist.barrier(group=self.group)  # no peer still reads our buffers
        for p in self._opened:
            self._C.ipc_close(p)
        self._C.p2p_free(self._staging)
        self._C.p2p_free(self._signal)
        self._C.p2p_free_flag(self._err_host)
        self._staging = self._signal = None
        self._opened = []


def from_env(group=None) -> Optional[P2PAllReducer]:
    """``CLOUDTIK_P2P_ALLREDUCE_BYTES=<n>`` (> 0) enables the one-shot path for buckets up to n bytes
    (0 disables it); unset, the crossover measured on this node at this world size
    (``parallel/comm_tuning.py``, written by ``bench/comm_bench.py --write-tuning``) decides, and
    with no measurement the path stays off.

    The decision is COLLECTIVE: every rank contributes (hostname, n, GPU available) and the
    path is enabled only if all ranks agree and share one host, so either every rank builds a
    reducer (whose constructor is itself collective) or none does -- a 2-node job never gets
    foreign IPC handles and never leaves ranks waiting in a barrier the others skipped."""
    if not dist.is_initialized():
        return None
    world = dist.get_world_size(group)
    env = os.environ.get("CLOUDTIK_P2P_ALLREDUCE_BYTES")
    if env is not None and env != "":
        n = int(env)
    else:
        from cloudtik_amd.parallel.comm_tuning import p2p_bytes
        n = p2p_bytes(world)
    mine = (socket.gethostname(), n, bool(torch.cuda.is_available()))
    votes: List = [None] * world
    dist.all_gather_object(votes, mine, group=group)
    if not decide(votes):
        return None
    return P2PAllReducer(group, max_bytes=n)


def decide(votes) -> bool:
    """Enable the one-shot path iff all ranks asked for the same n > 0, have a GPU, sit on
    one host, and there are at most 8 of them (one xGMI-connected node)."""
    if not votes or len(votes) > 8:
        return False
    hosts = {v[0] for v in votes}
    sizes = {v[1] for v in votes}
    return len(hosts) == 1 and len(sizes) == 1 and next(iter(sizes)) > 0 and all(v[2] for v in votes)
