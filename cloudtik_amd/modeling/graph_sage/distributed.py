"""Partitioned (distributed) GraphSAGE: graph partitions, cross-partition neighbour
sampling and sharded node embeddings over ``torch.distributed`` (reference
graph_sage/modeling/launch.py:632 -- partition the graph, start DGL graph servers and
samplers -- and model/homogeneous/distributed/trainer.py:54-57 -- DistGraph, DistEmbedding,
distributed neighbour sampler).

No graph-server processes: every training rank owns one partition and answers the other
ranks' requests inside collective calls (``all_to_all_single`` over RCCL/xGMI on GPUs, gloo
on CPU), so sampling and embedding traffic ride the same fabric as the gradients.

* ``partition_graph``: node -> part assignment by linear deterministic greedy streaming
  (LDG: place a node where most of its already-placed neighbours are, weighted by the
  part's remaining capacity) or hashing; each part file keeps the in-edges of the nodes it
  owns (global ids, edge ids, split) plus the global node -> part map.
* ``DistGraph``: one partition with a CSR of its owned nodes' in-edges.
* ``dist_sample_blocks``: multi-hop sampling where the frontier may contain any node: the
  owner of each frontier node samples its neighbours (requests and answers exchanged with
  two all-to-alls per hop) -- the same ``Block`` structures the single-graph model uses.
* ``DistEmbedding``: learnable node embeddings sharded by owner; lookups gather rows from
  their owners, gradients flow back to the owners, which apply a sparse Adagrad step (the
  dense SAGE layers are data-parallel as usual).
* ``DistLinkPredictionTrainer``: each rank trains on the edges whose destination it owns.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from cloudtik_amd.ops.graph import CSR
from .graph import Block, Graph


# ------------------------------------------------------------------------------ partitioning
def _ldg_assign(src: np.ndarray, dst: np.ndarray, num_nodes: int, parts: int, seed: int) -> np.ndarray:
    """Linear deterministic greedy streaming partition (Stanton & Kliot): nodes arrive in a
    random order; a node joins the part holding most of its already-placed neighbours,
    scaled by (1 - size / capacity), ties to the smallest part."""
    order = np.argsort(np.concatenate([src, dst]), kind="stable")
    both = np.concatenate([dst, src])[order]                 # neighbours grouped by node
    starts = np.searchsorted(np.concatenate([src, dst])[order], np.arange(num_nodes + 1))
    cap = num_nodes / parts * 1.05 + 1
    part = np.full(num_nodes, -1, np.int64)
    size = np.zeros(parts, np.float64)
    rng = np.random.default_rng(seed)
    for v in rng.permutation(num_nodes):
        nb = both[starts[v]:starts[v + 1]]
        placed = part[nb]
        placed = placed[placed >= 0]
        score = np.bincount(placed, minlength=parts).astype(np.float64) * (1.0 - size / cap)
        best = np.flatnonzero(score == score.max())
        p = best[np.argmin(size[best])]
        part[v] = p
        size[p] += 1
    return part


def partition_graph(g: Graph, num_parts: int, out_dir: str, method: str = "ldg", seed: int = 0) -> Dict:
    """Write ``num_parts`` partitions of ``g`` under ``out_dir``; returns the metadata."""
    os.makedirs(out_dir, exist_ok=True)
    src, dst = g.src.cpu().numpy(), g.dst.cpu().numpy()
    if method == "ldg":
        part = _ldg_assign(src, dst, g.num_nodes, num_parts, seed)
    elif method == "hash":
        part = (np.arange(g.num_nodes) * 2654435761 % (2 ** 32)) % num_parts
    else:
        raise ValueError("method must be ldg or hash")
    part_t = torch.from_numpy(part.astype(np.int32))
    eid = np.arange(len(src))
    cut = int((part[src] != part[dst]).sum())
    for p in range(num_parts):
        own = np.flatnonzero(part == p)
        sel = part[dst] == p                                  # in-edges of owned nodes
        rec = {"owned": torch.from_numpy(own), "src": torch.from_numpy(src[sel]), "dst": torch.from_numpy(dst[sel]),
               "eid": torch.from_numpy(eid[sel]), "node_part": part_t,
               "edge_split": None if g.edge_split is None else g.edge_split.cpu()[torch.from_numpy(sel)],
               "reverse_eid": None if g.reverse_eid is None else g.reverse_eid.cpu()[torch.from_numpy(sel)]}
        torch.save(rec, os.path.join(out_dir, f"part{p}.pt"))
    meta = {"num_parts": num_parts, "num_nodes": g.num_nodes, "num_edges": g.num_edges, "method": method,
            "edge_cut": cut, "part_sizes": np.bincount(part, minlength=num_parts).tolist()}
    with open(os.path.join(out_dir, "partition.json"), "w") as f:
        json.dump(meta, f, indent=2)
    return meta


# ------------------------------------------------------------------------------ partition view
class DistGraph:
    def __init__(self, part_dir: str, rank: int, world: int, device=None):
        with open(os.path.join(part_dir, "partition.json")) as f:
            self.meta = json.load(f)
        if self.meta["num_parts"] != world:
            raise ValueError(f"{self.meta['num_parts']} partitions for {world} ranks")
        self.rank, self.world = rank, world
        self.device = torch.device(device or "cpu")
        rec = torch.load(os.path.join(part_dir, f"part{rank}.pt"), weights_only=True)
        dev = self.device
        self.num_nodes = int(self.meta["num_nodes"])
        self.node_part = rec["node_part"].to(dev).long()
        self.owned = rec["owned"].to(dev).long()
        self.local_of = torch.full((self.num_nodes,), -1, dtype=torch.long, device=dev)
        self.local_of[self.owned] = torch.arange(self.owned.numel(), device=dev)
        src, dst = rec["src"].to(dev).long(), rec["dst"].to(dev).long()
        self.src, self.dst, self.eid = src, dst, rec["eid"].to(dev).long()
        self.edge_split = None if rec["edge_split"] is None else rec["edge_split"].to(dev)
        self.reverse_eid = None if rec["reverse_eid"] is None else rec["reverse_eid"].to(dev)
        rows = self.local_of[dst]
        order = torch.argsort(rows * self.num_nodes + src)
        counts = torch.bincount(rows, minlength=self.owned.numel())
        rowptr = torch.zeros(self.owned.numel() + 1, dtype=torch.long, device=dev)
        rowptr[1:] = torch.cumsum(counts, 0)
        self.csr = CSR(rowptr, src[order].contiguous(), self.owned.numel())
        self.csr_eid = self.eid[order]

    def sample_local(self, nodes: torch.Tensor, fanout: int, gen: torch.Generator,
                     exclude_eids: Optional[torch.Tensor]) -> Tuple[torch.Tensor, torch.Tensor]:
        """(row index into ``nodes``, neighbour global id) for owned ``nodes``."""
        dev = self.device
        loc = self.local_of[nodes]
        start = self.csr.rowptr[loc]
        deg = self.csr.rowptr[loc + 1] - start
        k = deg if fanout <= 0 else torch.clamp(deg, max=fanout)
        rows = torch.repeat_interleave(torch.arange(nodes.numel(), device=dev), k)
        if not rows.numel():
            return rows, rows
        pos = torch.arange(rows.numel(), device=dev) - torch.repeat_interleave(torch.cumsum(k, 0) - k, k)
        full = deg[rows] <= fanout if fanout > 0 else torch.ones_like(rows, dtype=torch.bool)
        rnd = torch.rand(rows.numel(), generator=gen).to(dev)
        pick = torch.where(full, pos, (rnd * deg[rows]).long().clamp(max=deg[rows] - 1))
        eidx = start[rows] + pick
        nbr = self.csr.col[eidx]
        if exclude_eids is not None and exclude_eids.numel():
            keep = ~torch.isin(self.csr_eid[eidx], exclude_eids)
            rows, nbr = rows[keep], nbr[keep]
        return rows, nbr


# ------------------------------------------------------------------------------ collectives
def _exchange(send: List[torch.Tensor], device) -> List[torch.Tensor]:
    """Variable-size all-to-all of 1-D int64 tensors (one per destination rank)."""
    world = len(send)
    sizes = torch.tensor([t.numel() for t in send], dtype=torch.long, device=device)
    recv_sizes = torch.empty_like(sizes)
    dist.all_to_all_single(recv_sizes, sizes)
    flat = torch.cat(send) if send else torch.empty(0, dtype=torch.long, device=device)
    out = torch.empty(int(recv_sizes.sum()), dtype=flat.dtype, device=device)
    dist.all_to_all_single(out, flat, output_split_sizes=recv_sizes.tolist(), input_split_sizes=sizes.tolist())
    return list(out.split(recv_sizes.tolist())) if world else []


def _exchange_rows(send: List[torch.Tensor], dim: int, device, dtype) -> List[torch.Tensor]:
    """Variable-size all-to-all of [n_i, dim] float tensors."""
    sizes = torch.tensor([t.shape[0] for t in send], dtype=torch.long, device=device)
    recv_sizes = torch.empty_like(sizes)
    dist.all_to_all_single(recv_sizes, sizes)
    flat = torch.cat(send).reshape(-1)
    out = torch.empty(int(recv_sizes.sum()) * dim, dtype=dtype, device=device)
    dist.all_to_all_single(out, flat, output_split_sizes=(recv_sizes * dim).tolist(),
                           input_split_sizes=(sizes * dim).tolist())
    return list(out.view(-1, dim).split(recv_sizes.tolist()))


def dist_sample_neighbors(dg: DistGraph, dst_nodes: torch.Tensor, fanout: int, gen: torch.Generator,
                          exclude_eids: Optional[torch.Tensor] = None) -> Block:
    """Collective: every rank calls it once per hop.  Requests for non-owned frontier nodes
    go to their owners, which sample and send back (row, neighbour) pairs."""
    dev = dg.device
    owner = dg.node_part[dst_nodes]
    req_idx = [torch.nonzero(owner == r).flatten() for r in range(dg.world)]
    asked = _exchange([dst_nodes[i] for i in req_idx], dev)          # nodes others ask me about
    if exclude_eids is None:
        exclude_eids = torch.empty(0, dtype=torch.long, device=dev)
    all_excl = torch.cat(_exchange([exclude_eids] * dg.world, dev))  # exclusions are global edge ids
    ans_rows, ans_nbr = [], []
    for r in range(dg.world):
        rows, nbr = dg.sample_local(asked[r], fanout, gen, all_excl)
        ans_rows.append(rows)
        ans_nbr.append(nbr)
    got_rows = _exchange(ans_rows, dev)
    got_nbr = _exchange(ans_nbr, dev)
    rows = torch.cat([req_idx[r][got_rows[r]] for r in range(dg.world)])
    nbr = torch.cat(got_nbr)
    all_nodes = torch.cat([dst_nodes, nbr])
    uniq, inv = torch.unique(all_nodes, return_inverse=True)
    first = torch.full((uniq.numel(),), all_nodes.numel(), dtype=torch.long, device=dev)
    first.scatter_reduce_(0, inv, torch.arange(all_nodes.numel(), device=dev), "amin")
    order = torch.argsort(first)
    local_of = torch.empty_like(order)
    local_of[order] = torch.arange(order.numel(), device=dev)
    src_nodes = uniq[order]
    col = local_of[inv[dst_nodes.numel():]]
    return Block(src_nodes, int(dst_nodes.numel()), CSR.from_edges(rows, col, dst_nodes.numel(), src_nodes.numel()))


def dist_sample_blocks(dg: DistGraph, seeds: torch.Tensor, fanouts: List[int], gen: torch.Generator,
                       exclude_eids: Optional[torch.Tensor] = None):
    blocks: List[Block] = []
    nodes = seeds
    for f in reversed(fanouts):
        b = dist_sample_neighbors(dg, nodes, f, gen, exclude_eids)
        blocks.insert(0, b)
        nodes = b.src_nodes
    return nodes, blocks


# ------------------------------------------------------------------------------ sharded embeddings
def sharded_gather(dg: DistGraph, local_rows: torch.Tensor, nodes: torch.Tensor) -> torch.Tensor:
    """Collective: rows of a node-sharded matrix (``local_rows[i]`` belongs to
    ``dg.owned[i]``) for arbitrary global ``nodes``, fetched from their owners."""
    owner = dg.node_part[nodes]
    idx = [torch.nonzero(owner == r).flatten() for r in range(dg.world)]
    asked = _exchange([nodes[i] for i in idx], dg.device)
    dim = local_rows.shape[1]
    got = _exchange_rows([local_rows[dg.local_of[a]] for a in asked], dim, dg.device, local_rows.dtype)
    out = torch.empty(nodes.numel(), dim, dtype=local_rows.dtype, device=dg.device)
    for r in range(dg.world):
        out[idx[r]] = got[r]
    return out


class _DistEmbFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, emb: "DistEmbedding", nodes: torch.Tensor):
        ctx.emb, ctx.nodes = emb, nodes
        return emb.gather(nodes)

    @staticmethod
    def backward(ctx, grad):
        ctx.emb.push_grad(ctx.nodes, grad)
        return None, None, None


class DistEmbedding(nn.Module):
    """Node embeddings sharded by owner partition, with an owner-side sparse Adagrad step
    (reference DGL DistEmbedding + SparseAdagrad in the distributed GraphSAGE trainer)."""

    def __init__(self, dg: DistGraph, dim: int, lr: float = 0.05, eps: float = 1e-10, init_std: float = 0.1,
                 seed: int = 0):
        super().__init__()
        self.dg, self.dim, self.lr, self.eps = dg, dim, lr, eps
        gen = torch.Generator().manual_seed(seed)
        full = torch.randn(dg.num_nodes, dim, generator=gen) * init_std     # same init on every rank
        self.table = full[dg.owned.cpu()].to(dg.device)                     # keep only owned rows
        self.state = torch.zeros_like(self.table)
        self.anchor = nn.Parameter(torch.zeros(()))                          # lets autograd reach push_grad
        self._pending: List[Tuple[torch.Tensor, torch.Tensor]] = []

    def _route(self, nodes):
        owner = self.dg.node_part[nodes]
        return [torch.nonzero(owner == r).flatten() for r in range(self.dg.world)]

    def gather(self, nodes: torch.Tensor) -> torch.Tensor:
        return sharded_gather(self.dg, self.table, nodes)

    def push_grad(self, nodes: torch.Tensor, grad: torch.Tensor):
        idx = self._route(nodes)
        ids = _exchange([nodes[i] for i in idx], self.dg.device)
        grads = _exchange_rows([grad[i].contiguous().to(self.table.dtype) for i in idx], self.dim, self.dg.device,
                               self.table.dtype)
        self._pending.append((torch.cat(ids), torch.cat(grads)))

    @torch.no_grad()
    def step(self):
        """Apply the accumulated sparse gradients to the owned rows (Adagrad)."""
        if not self._pending:
            return
        ids = torch.cat([p[0] for p in self._pending])
        g = torch.cat([p[1] for p in self._pending])
        self._pending.clear()
        loc = self.dg.local_of[ids]
        acc = torch.zeros_like(self.table).index_add_(0, loc, g)
        touched = torch.unique(loc)
        self.state[touched] += acc[touched] ** 2
        self.table[touched] -= self.lr * acc[touched] / (self.state[touched].sqrt() + self.eps)

    def forward(self, nodes: torch.Tensor) -> torch.Tensor:
        return _DistEmbFn.apply(self.anchor, self, nodes)


# ------------------------------------------------------------------------------ training
@dataclass
class DistTrainConfig:
    num_hidden: int = 32
    num_layers: int = 2
    fan_out: Tuple[int, ...] = (10, 5)
    batch_size: int = 256
    num_epochs: int = 1
    lr: float = 0.01
    emb_lr: float = 0.05
    seed: int = 0


class DistLinkPredictionTrainer:
    """Link prediction on a partitioned graph: a rank trains on the training edges whose
    destination it owns; SAGE layers are data-parallel (all-reduced), node embeddings are
    sharded (DistEmbedding)."""

    def __init__(self, dg: DistGraph, cfg: DistTrainConfig):
        from .model import EdgeDecoder, SAGEConv
        self.dg, self.cfg = dg, cfg
        torch.manual_seed(cfg.seed)
        h = cfg.num_hidden
        self.emb = DistEmbedding(dg, h, lr=cfg.emb_lr, seed=cfg.seed)
        self.layers = nn.ModuleList([SAGEConv(h, h) for _ in range(cfg.num_layers)]).to(dg.device)
        self.decoder = EdgeDecoder(h).to(dg.device)
        self.dense = list(self.layers.parameters()) + list(self.decoder.parameters())
        for p in self.dense:                               # identical dense init on every rank
            dist.broadcast(p.data, 0)
        self.opt = torch.optim.Adam(self.dense, lr=cfg.lr)
        split = dg.edge_split
        mask = torch.ones_like(dg.eid, dtype=torch.bool) if split is None else split == 0
        self.train_idx = torch.nonzero(mask).flatten()
        self.gen = torch.Generator().manual_seed(cfg.seed + 1000 * dg.rank)

    def _encode(self, seeds, exclude=None):
        input_nodes, blocks = dist_sample_blocks(self.dg, seeds, list(self.cfg.fan_out), self.gen, exclude)
        x = self.emb(input_nodes)
        for i, (blk, layer) in enumerate(zip(blocks, self.layers)):
            x = layer(blk, x)
            if i < len(self.layers) - 1:
                x = F.relu(x)
        return x

    def step(self, idx: torch.Tensor) -> float:
        dg = self.dg
        ps, pd = dg.src[idx], dg.dst[idx]
        nd = torch.randint(0, dg.num_nodes, (idx.numel(),), generator=self.gen).to(dg.device)
        seeds, inv = torch.unique(torch.cat([ps, pd, nd]), return_inverse=True)
        n = idx.numel()
        excl = dg.eid[idx]                                   # hide the positives (and reverses)
        if dg.reverse_eid is not None:
            rev = dg.reverse_eid[idx]
            excl = torch.cat([excl, rev[rev >= 0]])
        h = self._encode(seeds, excl)
        pos = self.decoder(h[inv[:n]], h[inv[n:2 * n]])
        neg = self.decoder(h[inv[:n]], h[inv[2 * n:]])
        loss = F.binary_cross_entropy_with_logits(pos, torch.ones_like(pos)) + \
            F.binary_cross_entropy_with_logits(neg, torch.zeros_like(neg))
        self.opt.zero_grad(set_to_none=True)
        loss.backward()
        for p in self.dense:
            if p.grad is not None:
                dist.all_reduce(p.grad)
                p.grad.div_(dg.world)
        self.opt.step()
        self.emb.step()
        return float(loss.detach())

    @torch.no_grad()
    def embeddings(self, chunk: int = 65536) -> torch.Tensor:
        """Layer-wise inference with full neighbourhoods: each rank computes the layer
        outputs of the nodes it owns, reading its inputs' previous-layer rows from their
        owners.  Returns the owned rows (``dg.owned`` order)."""
        dg = self.dg
        h = self.emb.table
        n_chunks = torch.tensor([(dg.owned.numel() + chunk - 1) // chunk], device=dg.device)
        dist.all_reduce(n_chunks, op=dist.ReduceOp.MAX)        # same number of collectives everywhere
        for i, layer in enumerate(self.layers):
            outs = []
            for c in range(int(n_chunks)):
                nodes = dg.owned[c * chunk:(c + 1) * chunk]
                blk = dist_sample_neighbors(dg, nodes, 0, self.gen)
                y = layer(blk, sharded_gather(dg, h, blk.src_nodes))
                outs.append(F.relu(y) if i < len(self.layers) - 1 else y)
            h = torch.cat(outs)
        return h

    def gather_embeddings(self) -> Optional[torch.Tensor]:
        """All node embeddings on rank 0 ([num_nodes, hidden], global id order); None elsewhere."""
        h = self.embeddings().float().cpu()
        parts = [None] * self.dg.world
        dist.all_gather_object(parts, (self.dg.owned.cpu(), h))
        if self.dg.rank != 0:
            return None
        out = torch.empty(self.dg.num_nodes, h.shape[1])
        for ids, rows in parts:
            out[ids] = rows
        return out

    def save(self, path: str):
        torch.save({"state_dict": {"layers": self.layers.state_dict(), "decoder": self.decoder.state_dict()},
                    "config": dict(self.cfg.__dict__)}, path)

    @torch.no_grad()
    def evaluate(self, split: int = 2, max_edges: int = 4096) -> float:
        """Global AUC over the ``split`` edges (each rank scores the ones it owns)."""
        from .trainer import _auc
        dg = self.dg
        idx = torch.nonzero(dg.edge_split == split).flatten()[:max_edges] if dg.edge_split is not None else \
            torch.arange(min(max_edges, dg.eid.numel()), device=dg.device)
        ps, pd = dg.src[idx], dg.dst[idx]
        nd = torch.randint(0, dg.num_nodes, (idx.numel(),), generator=self.gen).to(dg.device)
        seeds, inv = torch.unique(torch.cat([ps, pd, nd]), return_inverse=True)
        n = idx.numel()
        h = self._encode(seeds)
        pos = self.decoder(h[inv[:n]], h[inv[n:2 * n]]).float().cpu()
        neg = self.decoder(h[inv[:n]], h[inv[2 * n:]]).float().cpu()
        self.emb._pending.clear()
        parts = [None] * dg.world
        dist.all_gather_object(parts, (pos, neg))
        return _auc(torch.cat([p[0] for p in parts]), torch.cat([p[1] for p in parts]))

    def train(self) -> Dict[str, float]:
        cfg, dg = self.cfg, self.dg
        steps = torch.tensor([max(1, self.train_idx.numel() // cfg.batch_size)], device=dg.device)
        dist.all_reduce(steps, op=dist.ReduceOp.MIN)          # collectives stay in lockstep
        hist = {"losses": []}
        for _ in range(cfg.num_epochs):
            perm = self.train_idx[torch.randperm(self.train_idx.numel(), generator=self.gen).to(dg.device)]
            tot = 0.0
            for i in range(int(steps)):
                tot += self.step(perm[i * cfg.batch_size:(i + 1) * cfg.batch_size])
            hist["losses"].append(tot / int(steps))
        return hist
