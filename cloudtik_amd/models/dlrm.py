"""DLRM with hybrid parallelism (reference: applications/ai/quickstart DLRM
dlrm_s_pytorch.py:267-269,407-418 and extend_distributed.py:275-414; SURVEY.md §2.12,
§2.14 "Hybrid MP (embedding-table sharding, EP-like)").

* bottom MLP (dense features) and top MLP are data-parallel: their gradients go through the
  flat-buffer bucketed all-reduce;
* the sparse tables are model-parallel: rank r owns a contiguous block of tables (balanced
  by row count) stored as ONE fp32 EmbeddingBagCollection; every rank looks up its tables
  for the GLOBAL batch ([B_global, T_r, E], one HIP launch for all its tables), and one
  ``all_to_all_single`` turns that into [B_local, T_all, E] for the local batch slice
  (backward is the mirrored all-to-all).  Table gradients never leave their owner and are
  applied in the embedding backward kernel (fused sparse SGD), like the reference's
  IPEX SplitSGD path;
* the dot interaction is the fused HIP kernel.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist
import torch.nn as nn


@dataclass
class DLRMConfig:
    dense_features: int = 13
    embedding_dim: int = 64
    table_sizes: List[int] = field(default_factory=lambda: [100000] * 26)
    bottom_mlp: List[int] = field(default_factory=lambda: [512, 256, 64])
    top_mlp: List[int] = field(default_factory=lambda: [1024, 1024, 512, 256, 1])
    sparse_lr: float = 0.0           # > 0: fused sparse SGD in the embedding backward

    @classmethod
    def tiny(cls, **kw):
        c = cls(dense_features=13, embedding_dim=16, table_sizes=[50, 80, 30, 120, 60], bottom_mlp=[32, 16],
                top_mlp=[32, 1])
        for k, v in kw.items():
            setattr(c, k, v)
        return c


def _mlp(dims: Sequence[int], device, sigmoid_last=False) -> nn.ModuleList:
    return nn.ModuleList(nn.Linear(a, b, device=device) for a, b in zip(dims[:-1], dims[1:]))


def _run_mlp(layers, x, relu_last: bool):
    from cloudtik_amd import ops
    for i, l in enumerate(layers):
        x = ops.linear(x, l.weight, l.bias)
        if i < len(layers) - 1 or relu_last:
            x = torch.relu(x)
    return x


def shard_tables(table_sizes: Sequence[int], world: int) -> List[Tuple[int, int]]:
    """Contiguous [lo, hi) table blocks per rank, balancing total rows greedily."""
    T = len(table_sizes)
    if world > T:
        raise ValueError(f"{world} ranks but only {T} tables")
    total = sum(table_sizes)
    bounds, lo, acc = [], 0, 0
    for r in range(world):
        if r == world - 1:
            hi = T
        else:
            target = total * (r + 1) / world
            hi, acc = lo + 1, acc + table_sizes[lo]          # at least one table each
            while hi < T - (world - 1 - r) and acc + table_sizes[hi] / 2 <= target:
                acc += table_sizes[hi]
                hi += 1
        bounds.append((lo, hi))
        lo = hi
    return bounds


class _AllToAll(torch.autograd.Function):
    """[B_global, T_r, E] (this rank's tables, all samples) -> [B_local, T_all, E]."""

    @staticmethod
    def forward(ctx, local_emb, t_counts, group):
        world = len(t_counts)
        Bg, Tr, E = local_emb.shape
        Bl = Bg // world
        send = local_emb.contiguous().view(-1)
        send_splits = [Bl * Tr * E] * world
        recv_splits = [Bl * t * E for t in t_counts]
        recv = torch.empty(sum(recv_splits), dtype=local_emb.dtype, device=local_emb.device)
        dist.all_to_all_single(recv, send, recv_splits, send_splits, group=group)
        parts = torch.split(recv, recv_splits)
        out = torch.cat([p.view(Bl, t, E) for p, t in zip(parts, t_counts)], dim=1)
        ctx.meta = (t_counts, group, Tr, Bl, E)
        return out

    @staticmethod
    def backward(ctx, g):
        t_counts, group, Tr, Bl, E = ctx.meta
        world = len(t_counts)
        g = g.contiguous()
        send = torch.cat([c.reshape(-1) for c in torch.split(g, t_counts, dim=1)])
        send_splits = [Bl * t * E for t in t_counts]
        recv_splits = [Bl * Tr * E] * world
        recv = torch.empty(sum(recv_splits), dtype=g.dtype, device=g.device)
        dist.all_to_all_single(recv, send, recv_splits, send_splits, group=group)
        return recv.view(world * Bl, Tr, E), None, None


class DLRM(nn.Module):
    def __init__(self, cfg: DLRMConfig, device=None, rank: int = 0, world: int = 1, group=None):
        super().__init__()
        from cloudtik_amd.ops.embedding import EmbeddingBagCollection
        self.cfg, self.rank, self.world, self.group = cfg, rank, world, group
        E = cfg.embedding_dim
        if cfg.bottom_mlp[-1] != E:
            raise ValueError("bottom MLP output must equal the embedding dim")
        self.bounds = shard_tables(cfg.table_sizes, world)
        lo, hi = self.bounds[rank]
        self.t_counts = [b - a for a, b in self.bounds]
        self.local_tables = list(range(lo, hi))
        self.bottom = _mlp([cfg.dense_features] + cfg.bottom_mlp, device)
        F = len(cfg.table_sizes) + 1
        # dense layers first: their init must not depend on how many table rows this rank owns
        self.top = _mlp([E + F * (F - 1) // 2] + cfg.top_mlp, device)
        # MLP weight gradients in line, not on the side stream: the GEMMs are small and the
        # step is launch-bound, so the cross-stream events cost more than the overlap returns
        # (1.20-1.32 vs 1.56-1.90 ms per 2048-sample step, 3 interleaved rounds;
        # profiles/r6/SUMMARY.md)
        from cloudtik_amd.ops.linear import use_wgrad_side_stream
        use_wgrad_side_stream(list(self.bottom.parameters()) + list(self.top.parameters()), False)
        # tables are seeded per table so any sharding produces identical weights
        self.emb = EmbeddingBagCollection([cfg.table_sizes[t] for t in self.local_tables], E, device=device,
                                          sparse_lr=cfg.sparse_lr)
        with torch.no_grad():
            base = 0
            for t in self.local_tables:
                n = cfg.table_sizes[t]
                g = torch.Generator().manual_seed(1000 + t)
                b = (1.0 / n) ** 0.5
                self.emb.weight[base:base + n].copy_((torch.rand(n, E, generator=g) * 2 - 1) * b)
                base += n

    def dense_parameters(self):
        return [p for n, p in self.named_parameters() if not n.startswith("emb.")]

    def forward(self, dense: torch.Tensor, idx: torch.Tensor, offs: torch.Tensor, batch_global: int):
        """dense: [B_local, 13]; (idx, offs): CSR bags of this rank's tables over the global
        batch (table-major, offsets length T_r * B_global + 1)."""
        from cloudtik_amd import ops
        x = _run_mlp(self.bottom, dense, relu_last=True)
        ly = self.emb(idx, offs, batch_global)                        # [B_global, T_r, E]
        if self.world > 1:
            ly = _AllToAll.apply(ly, self.t_counts, self.group)        # [B_local, T_all, E]
        z = ops.dot_interaction(x, ly.to(x.dtype))
        return _run_mlp(self.top, z, relu_last=False).squeeze(-1)


def synthetic_batch(cfg: DLRMConfig, batch_global: int, step: int, tables: Sequence[int], device=None,
                    pooling: int = 1):
    """Deterministic global batch: every rank can build the sparse inputs of its own tables
    and the dense slice of its own samples without communication."""
    g = torch.Generator().manual_seed(7919 * step + 17)
    dense = torch.rand(batch_global, cfg.dense_features, generator=g)
    labels = torch.randint(0, 2, (batch_global,), generator=g).float()
    idxs, offs = [], []
    for t in range(len(cfg.table_sizes)):
        gt = torch.Generator().manual_seed(104729 * step + 31 * t + 5)
        ind = torch.randint(0, cfg.table_sizes[t], (batch_global * pooling,), generator=gt)
        if t in tables:
            idxs.append(ind)
            offs.append(torch.arange(batch_global, dtype=torch.int64) * pooling)
    from cloudtik_amd.ops.embedding import pack_bags
    idx, off = pack_bags(idxs, offs, batch_global)
    return dense.to(device), labels.to(device), idx.to(device), off.to(device)
