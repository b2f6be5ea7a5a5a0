"""Link-prediction training of GraphSAGE node embeddings (reference
graph_sage/modeling/model/homogeneous/trainer.py:40-230 and distributed/trainer.py:54-176:
DGL edge DataLoader with negative sampling, DDP over gloo).

MI355X path: the graph, node embeddings and sampler state live on the GPU; each step samples
a batch of training edges, uniform negative destinations, and a multi-hop neighbourhood
with the training edges (and their reverses) excluded; aggregation runs through the HIP
SpMM kernel.  With several ranks (cloudtik-run, one per GPU) every rank takes its own
shard of the training edges and DistributedDataParallel all-reduces the gradients over RCCL.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch
import torch.distributed as dist
import torch.nn.functional as F

from .graph import Graph, sample_blocks
from .model import GraphSAGEModel


@dataclass
class TrainConfig:
    num_epochs: int = 2
    num_hidden: int = 64
    num_layers: int = 2
    fan_out: List[int] = field(default_factory=lambda: [10, 15])
    batch_size: int = 1024
    batch_size_eval: int = 100_000
    eval_every: int = 1
    lr: float = 5e-3
    log_every: int = 20
    exclude_reverse_edges: bool = True
    seed: int = 0


def _auc(pos: torch.Tensor, neg: torch.Tensor) -> float:
    s = torch.cat([pos, neg]).double()
    y = torch.cat([torch.ones_like(pos), torch.zeros_like(neg)]).double()
    order = torch.argsort(s)
    ranks = torch.empty_like(s)
    ranks[order] = torch.arange(1, s.numel() + 1, device=s.device, dtype=torch.double)
    # average ranks of ties
    uniq, inv = torch.unique(s, return_inverse=True)
    mean_rank = torch.zeros_like(uniq).index_add_(0, inv, ranks) / torch.bincount(inv).double()
    r = mean_rank[inv]
    npos, nneg = float(y.sum()), float((1 - y).sum())
    return float((r[y == 1].sum() - npos * (npos + 1) / 2) / (npos * nneg))


class LinkPredictionTrainer:
    def __init__(self, graph: Graph, config: TrainConfig, device=None, node_features: Optional[torch.Tensor] = None):
        self.cfg = config
        self.device = torch.device(device) if device else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        self.g = graph.to(self.device)
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        torch.manual_seed(config.seed)
        if len(config.fan_out) != config.num_layers:
            raise ValueError("fan_out needs one entry per layer")
        self.model = GraphSAGEModel(self.g.num_nodes, config.num_hidden, config.num_layers,
                                    node_features=None if node_features is None else node_features.to(self.device)
                                    ).to(self.device)
        self.ddp = None
        if self.world > 1:
            self.ddp = torch.nn.parallel.DistributedDataParallel(
                self.model, device_ids=[self.device.index] if self.device.type == "cuda" else None)
        self.opt = torch.optim.Adam(self.model.parameters(), lr=config.lr)
        split = self.g.edge_split
        E = self.g.num_edges
        all_e = torch.arange(E, device=self.device)
        self.train_eids = all_e if split is None else all_e[split == 0]
        self.val_eids = all_e[:0] if split is None else all_e[split == 1]
        self.test_eids = all_e[:0] if split is None else all_e[split == 2]
        self.gen = torch.Generator(device=self.device).manual_seed(config.seed + 1000 * self.rank)

    def _step(self, eids: torch.Tensor) -> float:
        g, cfg = self.g, self.cfg
        ps, pd = g.src[eids], g.dst[eids]
        nd = torch.randint(0, g.num_nodes, (eids.numel(),), device=self.device, generator=self.gen)
        seeds, inv = torch.unique(torch.cat([ps, pd, nd]), return_inverse=True)
        n = eids.numel()
        excl = None
        if cfg.exclude_reverse_edges:
            excl = eids
            if g.reverse_eid is not None:
                r = g.reverse_eid[eids]
                excl = torch.cat([eids, r[r >= 0]])
        input_nodes, blocks = sample_blocks(g, seeds, cfg.fan_out, self.gen, excl)
        model = self.ddp or self.model
        pos, neg = model(input_nodes, blocks, inv[:n], inv[n:2 * n], inv[:n], inv[2 * n:])
        loss = F.binary_cross_entropy_with_logits(pos, torch.ones_like(pos)) + \
            F.binary_cross_entropy_with_logits(neg, torch.zeros_like(neg))
        self.opt.zero_grad(set_to_none=True)
        loss.backward()
        self.opt.step()
        return float(loss.detach())

    @torch.no_grad()
    def evaluate(self, eids: torch.Tensor) -> Optional[float]:
        if eids.numel() == 0:
            return None
        self.model.eval()
        h = self.model.inference(self.g)
        g = self.g
        gen = torch.Generator(device=self.device).manual_seed(self.cfg.seed + 7)
        nd = torch.randint(0, g.num_nodes, (eids.numel(),), device=self.device, generator=gen)
        dec = self.model.decoder
        pos = torch.cat([dec(h[g.src[c]], h[g.dst[c]]) for c in eids.split(self.cfg.batch_size_eval)])
        neg = torch.cat([dec(h[g.src[c]], h[n]) for c, n in zip(eids.split(self.cfg.batch_size_eval),
                                                                nd.split(self.cfg.batch_size_eval))])
        self.model.train()
        return _auc(pos.float(), neg.float())

    def train(self) -> Dict[str, float]:
        cfg = self.cfg
        shard = self.train_eids[self.rank::self.world]
        # equal step counts on every rank keep DDP's collectives in lockstep
        steps = shard.numel() // cfg.batch_size if self.world > 1 else -(-shard.numel() // cfg.batch_size)
        if self.world > 1:
            t = torch.tensor([steps], device=self.device)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            steps = int(t)
        hist: Dict[str, float] = {}
        for epoch in range(cfg.num_epochs):
            t0 = time.time()
            perm = shard[torch.randperm(shard.numel(), device=self.device, generator=self.gen)]
            tot = 0.0
            for i in range(max(steps, 1)):
                tot += self._step(perm[i * cfg.batch_size:(i + 1) * cfg.batch_size])
                if cfg.log_every and i % cfg.log_every == 0 and self.rank == 0:
                    print(f"epoch {epoch} step {i}/{steps} loss {tot / (i + 1):.4f}", flush=True)
            hist["loss"] = tot / max(steps, 1)
            hist["epoch_seconds"] = time.time() - t0
            if cfg.eval_every and (epoch + 1) % cfg.eval_every == 0 and self.rank == 0:
                auc = self.evaluate(self.val_eids)
                if auc is not None:
                    hist["val_auc"] = auc
                    print(f"epoch {epoch} val auc {auc:.4f}", flush=True)
        test_auc = self.evaluate(self.test_eids) if self.rank == 0 else None
        if test_auc is not None:
            hist["test_auc"] = test_auc
        return hist

    @torch.no_grad()
    def embeddings(self) -> torch.Tensor:
        self.model.eval()
        return self.model.inference(self.g)

    def save(self, path: str):
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        torch.save({"state_dict": self.model.state_dict(), "config": vars(self.cfg)}, path)
