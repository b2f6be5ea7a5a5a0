"""GraphSAGE encoder + edge decoder for link prediction (reference
graph_sage/modeling/model/homogeneous/model.py:29-160: DGL SAGEConv 'mean' layers, a 3-layer
MLP decoder over h_src * h_dst, layer-wise full-graph inference).

``SAGEConv`` computes ``fc_self(h_dst) + fc_neigh(mean_{u in N(v)} h_u)``; the mean
aggregation is the HIP CSR SpMM kernel (ops.SpMM, with its transpose for backward), the two
projections are plain GEMMs.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from cloudtik_amd.ops.graph import SpMM

from .graph import Block, Graph


class SAGEConv(nn.Module):
    def __init__(self, in_feats: int, out_feats: int, bias: bool = True):
        super().__init__()
        self.fc_self = nn.Linear(in_feats, out_feats, bias=bias)
        self.fc_neigh = nn.Linear(in_feats, out_feats, bias=False)
        nn.init.xavier_uniform_(self.fc_self.weight, gain=nn.init.calculate_gain("relu"))
        nn.init.xavier_uniform_(self.fc_neigh.weight, gain=nn.init.calculate_gain("relu"))

    def forward(self, block: Block, h: torch.Tensor, agg: Optional[SpMM] = None) -> torch.Tensor:
        agg = agg or SpMM(block.csr, mean=True)
        # project first when it shrinks the rows the aggregation has to move
        if self.fc_neigh.out_features < self.fc_neigh.in_features:
            neigh = agg(self.fc_neigh(h))
        else:
            neigh = self.fc_neigh(agg(h))
        return self.fc_self(h[:block.num_dst]) + neigh


class GraphSAGE(nn.Module):
    def __init__(self, in_feats: int, hidden: int, out_feats: int, num_layers: int):
        super().__init__()
        dims = [in_feats] + [hidden] * (num_layers - 1) + [out_feats]
        self.layers = nn.ModuleList(SAGEConv(dims[i], dims[i + 1]) for i in range(num_layers))

    def forward(self, blocks: List[Block], x: torch.Tensor) -> torch.Tensor:
        h = x
        for i, (layer, b) in enumerate(zip(self.layers, blocks)):
            h = layer(b, h)
            if i != len(self.layers) - 1:
                h = F.relu(h)
        return h


class EdgeDecoder(nn.Module):
    def __init__(self, hidden: int):
        super().__init__()
        self.mlp = nn.Sequential(nn.Linear(hidden, hidden), nn.ReLU(), nn.Linear(hidden, hidden), nn.ReLU(),
                                 nn.Linear(hidden, 1))

    def forward(self, h_src: torch.Tensor, h_dst: torch.Tensor) -> torch.Tensor:
        return self.mlp(h_src * h_dst).squeeze(-1)


class GraphSAGEModel(nn.Module):
    """Node-id embeddings (transductive; or a projection of node features) -> GraphSAGE ->
    edge scores."""

    def __init__(self, num_nodes: int, hidden: int, num_layers: int, in_feats: Optional[int] = None,
                 node_features: Optional[torch.Tensor] = None):
        super().__init__()
        self.hidden = hidden
        if node_features is None:
            self.emb = nn.Embedding(num_nodes, in_feats or hidden)
            nn.init.normal_(self.emb.weight, std=0.1)
            self.register_buffer("node_features", None, persistent=False)
            d_in = in_feats or hidden
        else:
            self.emb = None
            self.register_buffer("node_features", node_features.float(), persistent=False)
            d_in = node_features.shape[1]
        self.encoder = GraphSAGE(d_in, hidden, hidden, num_layers)
        self.decoder = EdgeDecoder(hidden)

    def inputs(self, nodes: torch.Tensor) -> torch.Tensor:
        return self.emb(nodes) if self.emb is not None else self.node_features[nodes]

    def encode(self, input_nodes: torch.Tensor, blocks: List[Block]) -> torch.Tensor:
        return self.encoder(blocks, self.inputs(input_nodes))

    def forward(self, input_nodes, blocks, pos_src, pos_dst, neg_src, neg_dst):
        """pos_/neg_ endpoints are indices into the seed set (the output rows)."""
        h = self.encode(input_nodes, blocks)
        return self.decoder(h[pos_src], h[pos_dst]), self.decoder(h[neg_src], h[neg_dst])

    @torch.no_grad()
    def inference(self, g: Graph, batch_rows: int = 1 << 20) -> torch.Tensor:
        """Layer-wise full-neighbour inference for every node (no sampling)."""
        dev = g.src.device
        nodes = torch.arange(g.num_nodes, device=dev)
        h = torch.cat([self.inputs(nodes[i:i + batch_rows]) for i in range(0, g.num_nodes, batch_rows)])
        block = Block(nodes, g.num_nodes, g.in_csr())
        agg = SpMM(block.csr, mean=True)
        for i, layer in enumerate(self.encoder.layers):
            h = layer(block, h, agg)
            if i != len(self.encoder.layers) - 1:
                h = F.relu(h)
        return h
