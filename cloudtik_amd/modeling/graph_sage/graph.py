"""Tabular -> graph construction and GPU neighbour sampling for GraphSAGE (reference
graph_sage/modeling/build_graph.py:27-200, tokenizer.py, and DGL's NeighborSampler /
edge-prediction sampler used by model/homogeneous/trainer.py:87-140).

The graph is homogeneous: every node type (e.g. card, merchant) gets a contiguous id range
(``type_offset``) after renumbering its id column; each tabular row becomes an edge and,
with ``reverse_edges``, its reverse.  The whole graph stays resident on the GPU (a 288 GB
HBM3E device holds billion-edge graphs), so sampling is a few batched tensor ops on device
instead of a CPU sampler process pool or a partitioned graph server.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch

from cloudtik_amd.ops.graph import CSR


@dataclass
class Graph:
    num_nodes: int
    src: torch.Tensor                 # int64 [E]
    dst: torch.Tensor                 # int64 [E]
    node_type: torch.Tensor           # int64 [N]
    type_names: List[str]
    type_offset: Dict[str, int]
    edge_split: Optional[torch.Tensor] = None      # int64 [E] 0 train / 1 val / 2 test
    edge_label: Optional[torch.Tensor] = None
    reverse_eid: Optional[torch.Tensor] = None     # int64 [E] id of the reverse edge (or -1)
    node_index: Dict[str, Any] = field(default_factory=dict)   # type -> pandas Index of raw ids
    _in_csr: Optional[CSR] = None

    @property
    def num_edges(self) -> int:
        return int(self.src.numel())

    def to(self, device) -> "Graph":
        mv = lambda t: None if t is None else t.to(device)
        return Graph(self.num_nodes, mv(self.src), mv(self.dst), mv(self.node_type), self.type_names,
                     self.type_offset, mv(self.edge_split), mv(self.edge_label), mv(self.reverse_eid),
                     self.node_index)

    def in_csr(self) -> CSR:
        """Rows = destination nodes, columns = their in-neighbours (message sources);
        also keeps the edge id of every CSR entry for edge exclusion."""
        if self._in_csr is None:
            order = torch.argsort(self.dst * self.num_nodes + self.src)
            counts = torch.bincount(self.dst, minlength=self.num_nodes)
            rowptr = torch.zeros(self.num_nodes + 1, dtype=torch.long, device=self.src.device)
            rowptr[1:] = torch.cumsum(counts, 0)
            self._in_csr = CSR(rowptr, self.src[order].contiguous(), self.num_nodes)
            self._in_eid = order               # CSR position -> edge id
        return self._in_csr

    def save(self, path: str):
        torch.save({k: getattr(self, k) for k in ("num_nodes", "src", "dst", "node_type", "type_names",
                                                  "type_offset", "edge_split", "edge_label", "reverse_eid")}, path)

    @classmethod
    def load(cls, path: str) -> "Graph":
        return cls(**torch.load(path, weights_only=True))


def build_graph(df, config: Dict[str, Any]) -> Graph:
    """tabular2graph config: node_columns {column: type}, edge_types [[src_col, rel, dst_col]],
    optional reverse_edges, edge_label column, edge_split column (0/1/2)."""
    node_columns: Dict[str, str] = config["node_columns"]
    types: List[str] = list(config.get("node_types") or dict.fromkeys(node_columns.values()))
    index: Dict[str, Any] = {}
    import pandas as pd
    for t in types:
        cols = [c for c, ty in node_columns.items() if ty == t]
        vals = pd.concat([df[c] for c in cols], ignore_index=True)
        index[t] = pd.Index(pd.unique(vals))
    offset, n = {}, 0
    for t in types:
        offset[t] = n
        n += len(index[t])
    node_type = torch.cat([torch.full((len(index[t]),), i, dtype=torch.long) for i, t in enumerate(types)])

    def ids(col):
        t = node_columns[col]
        return torch.from_numpy(index[t].get_indexer(df[col]).astype(np.int64)) + offset[t]

    rels = {r[1]: (r[0], r[2]) for r in config["edge_types"]}
    reverse = config.get("reverse_edges") or {}
    srcs, dsts, splits, labels, rev = [], [], [], [], []
    seen = set()
    split_col = config.get("edge_split")
    label_col = config.get("edge_label")
    R = len(df)
    base = 0
    rel_base = {}
    for rel, (sc, dc) in rels.items():
        if rel in seen:
            continue
        pair = [rel] + ([reverse[rel]] if rel in reverse and reverse[rel] in rels else [])
        for r in pair:
            seen.add(r)
            s, d = rels[r]
            srcs.append(ids(s))
            dsts.append(ids(d))
            rel_base[r] = base
            base += R
            if split_col:
                splits.append(torch.from_numpy(df[split_col].to_numpy().astype(np.int64)))
            if label_col:
                labels.append(torch.from_numpy(df[label_col].to_numpy().astype(np.float32)))
        if len(pair) == 2:
            a, b = rel_base[pair[0]], rel_base[pair[1]]
            rev.append((a, b))
    src, dst = torch.cat(srcs), torch.cat(dsts)
    reid = torch.full((src.numel(),), -1, dtype=torch.long)
    for a, b in rev:
        ar = torch.arange(R)
        reid[a + ar] = b + ar
        reid[b + ar] = a + ar
    return Graph(n, src, dst, node_type, types, offset, torch.cat(splits) if splits else None,
                 torch.cat(labels) if labels else None, reid, index)


# ---------------------------------------------------------------------- sampling
@dataclass
class Block:
    """One message-passing layer: dst nodes are the first ``num_dst`` of ``src_nodes``."""
    src_nodes: torch.Tensor        # global ids [S]
    num_dst: int
    csr: CSR                       # rows = dst (local), cols = local src index


def sample_neighbors(g: Graph, dst_nodes: torch.Tensor, fanout: int, gen: Optional[torch.Generator] = None,
                     exclude_eids: Optional[torch.Tensor] = None) -> Block:
    """Up to ``fanout`` in-neighbours per dst (all of them if the degree is smaller; with
    replacement otherwise).  ``exclude_eids`` removes those edges (the positive training
    edges and their reverses, so a model cannot read the answer off the graph)."""
    csr = g.in_csr()
    dev = dst_nodes.device
    start = csr.rowptr[dst_nodes]
    deg = csr.rowptr[dst_nodes + 1] - start
    if fanout <= 0:
        k = deg
    else:
        k = torch.clamp(deg, max=fanout)
    rows = torch.repeat_interleave(torch.arange(dst_nodes.numel(), device=dev), k)
    if rows.numel():
        pos_in_row = torch.arange(rows.numel(), device=dev) - torch.repeat_interleave(torch.cumsum(k, 0) - k, k)
        full = deg[rows] <= fanout if fanout > 0 else torch.ones_like(rows, dtype=torch.bool)
        rnd = torch.rand(rows.numel(), device=dev, generator=gen) if gen is None or gen.device == dev else \
            torch.rand(rows.numel(), generator=gen).to(dev)
        pick = torch.where(full, pos_in_row, (rnd * deg[rows]).long().clamp(max=deg[rows] - 1))
        eidx = start[rows] + pick
    else:
        eidx = rows
    nbr = csr.col[eidx]
    if exclude_eids is not None and exclude_eids.numel() and eidx.numel():
        eid = g._in_eid[eidx]
        keep = ~torch.isin(eid, exclude_eids)
        rows, nbr = rows[keep], nbr[keep]
    # local numbering: dst nodes first, then new sources in order of first appearance
    all_nodes = torch.cat([dst_nodes, nbr])
    uniq, inv = torch.unique(all_nodes, return_inverse=True)
    first = torch.full((uniq.numel(),), all_nodes.numel(), dtype=torch.long, device=dev)
    first.scatter_reduce_(0, inv, torch.arange(all_nodes.numel(), device=dev), "amin")
    order = torch.argsort(first)
    local_of = torch.empty_like(order)
    local_of[order] = torch.arange(order.numel(), device=dev)
    src_nodes = uniq[order]
    col = local_of[inv[dst_nodes.numel():]]
    block_csr = CSR.from_edges(rows, col, dst_nodes.numel(), src_nodes.numel())
    return Block(src_nodes, int(dst_nodes.numel()), block_csr)


def sample_blocks(g: Graph, seeds: torch.Tensor, fanouts: List[int], gen=None,
                  exclude_eids: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, List[Block]]:
    """Multi-layer sampling from the output layer down; returns (input nodes, blocks in
    forward order)."""
    blocks: List[Block] = []
    nodes = seeds
    for f in reversed(fanouts):
        b = sample_neighbors(g, nodes, f, gen, exclude_eids)
        blocks.insert(0, b)
        nodes = b.src_nodes
    return nodes, blocks


def full_blocks(g: Graph, num_layers: int) -> List[Block]:
    """Whole-graph message passing (layer-wise inference)."""
    nodes = torch.arange(g.num_nodes, device=g.src.device)
    return [Block(nodes, g.num_nodes, g.in_csr())] * num_layers
