"""Partitioned GraphSAGE over gloo with 2 ranks: partition quality and bookkeeping,
cross-partition sampling returns only real (non-excluded) edges and the same neighbourhoods
as the single-graph sampler when fanout covers every neighbour, sharded embeddings match a
dense table (values, gradients, sparse Adagrad step), and distributed link prediction learns
(reference graph_sage/modeling/model/homogeneous/distributed/trainer.py, launch.py:632)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from cloudtik_amd.modeling.graph_sage.graph import Graph, sample_neighbors
from cloudtik_amd.modeling.graph_sage.distributed import partition_graph


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def community_graph(n=200, comms=4, deg=6, p_in=0.9, seed=0) -> Graph:
    """Undirected community graph (edges stored both ways with reverse ids); 80/10/10 split."""
    g = torch.Generator().manual_seed(seed)
    size = n // comms
    src = torch.randint(0, n, (n * deg // 2,), generator=g)
    same = torch.rand(src.numel(), generator=g) < p_in
    base = (src // size) * size
    dst = torch.where(same, base + torch.randint(0, size, src.shape, generator=g), torch.randint(0, n, src.shape,
                                                                                                  generator=g))
    keep = src != dst
    src, dst = src[keep], dst[keep]
    m = src.numel()
    split = torch.zeros(m, dtype=torch.long)
    r = torch.rand(m, generator=g)
    split[r > 0.8] = 1
    split[r > 0.9] = 2
    ar = torch.arange(m)
    return Graph(n, torch.cat([src, dst]), torch.cat([dst, src]), torch.zeros(n, dtype=torch.long), ["node"],
                 {"node": 0}, torch.cat([split, split]), None, torch.cat([ar + m, ar]))


def test_partition_ldg_beats_hash(tmp_path):
    g = community_graph()
    ldg = partition_graph(g, 2, str(tmp_path / "ldg"), "ldg")
    hsh = partition_graph(g, 2, str(tmp_path / "hash"), "hash")
    assert sum(ldg["part_sizes"]) == g.num_nodes and max(ldg["part_sizes"]) <= g.num_nodes * 0.55
    assert ldg["edge_cut"] < 0.6 * hsh["edge_cut"]
    # every edge lands in exactly one part (its destination's owner)
    eids = []
    for p in range(2):
        rec = torch.load(str(tmp_path / "ldg" / f"part{p}.pt"), weights_only=True)
        assert (rec["node_part"][rec["dst"]] == p).all()
        eids.append(rec["eid"])
    assert torch.equal(torch.sort(torch.cat(eids)).values, torch.arange(g.num_edges))


def _worker(rank, world, port, part_dir, out):
    import torch.distributed as dist
    from cloudtik_amd.modeling.graph_sage.distributed import (DistEmbedding, DistGraph, DistLinkPredictionTrainer,
                                                              DistTrainConfig, dist_sample_blocks,
                                                              dist_sample_neighbors)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = community_graph()
        edges = set(zip(g.src.tolist(), g.dst.tolist()))
        dg = DistGraph(part_dir, rank, world)
        res = {}
        # 1. full-fanout sampling == single-graph sampling, whatever the owner of each seed
        seeds = torch.arange(rank, g.num_nodes, 7)
        blk = dist_sample_neighbors(dg, seeds, 0, torch.Generator().manual_seed(rank))
        ref = sample_neighbors(g, seeds, 0)
        def adj(b):
            out = set()
            for r in range(b.num_dst):
                for c in b.csr.col[b.csr.rowptr[r]:b.csr.rowptr[r + 1]].tolist():
                    out.add((int(b.src_nodes[c]), int(b.src_nodes[r])))
            return out
        res["full_equal"] = adj(blk) == adj(ref) and torch.equal(blk.src_nodes[:blk.num_dst], seeds)
        # 2. fanout-limited multi-hop sampling with exclusions: only real, non-excluded edges
        excl = torch.arange(0, g.num_edges, 3)
        keep = torch.ones(g.num_edges, dtype=torch.bool)
        keep[excl] = False
        kept_pairs = set(zip(g.src[keep].tolist(), g.dst[keep].tolist()))   # a multi-edge may survive
        inputs, blocks = dist_sample_blocks(dg, seeds, [4, 3], torch.Generator().manual_seed(10 + rank), excl)
        res["sample_real"] = all(adj(b) <= kept_pairs for b in blocks)
        res["sample_deg"] = all(bool((b.csr.degrees() <= f).all()) for b, f in zip(blocks, [4, 3]))
        res["sample_inputs"] = torch.equal(inputs, blocks[0].src_nodes) and \
            torch.equal(blocks[1].src_nodes[:blocks[1].num_dst], seeds)
        res["sample_ok"] = res["sample_real"] and res["sample_deg"] and res["sample_inputs"]
        # 3. sharded embeddings == dense table: lookup, gradient and sparse Adagrad step
        emb = DistEmbedding(dg, 8, lr=0.1, seed=3)
        dense = torch.randn(g.num_nodes, 8, generator=torch.Generator().manual_seed(3)) * 0.1
        nodes = torch.randint(0, g.num_nodes, (50,), generator=torch.Generator().manual_seed(20 + rank))
        x = emb(nodes)
        res["lookup"] = torch.allclose(x, dense[nodes])
        w = torch.randn(8, generator=torch.Generator().manual_seed(30 + rank))
        (x * w).sum().backward()
        emb.step()
        # expected: every rank's gradient rows summed per node, then Adagrad from zero state
        allg = torch.zeros_like(dense)
        for r in range(world):
            nr = torch.randint(0, g.num_nodes, (50,), generator=torch.Generator().manual_seed(20 + r))
            wr = torch.randn(8, generator=torch.Generator().manual_seed(30 + r))
            allg.index_add_(0, nr, wr.expand(50, 8))
        upd = dense - 0.1 * allg / (allg.pow(2).sqrt() + 1e-10)
        res["adagrad"] = torch.allclose(emb.table, upd[dg.owned], atol=1e-6)
        # 4. distributed link prediction learns
        tr = DistLinkPredictionTrainer(dg, DistTrainConfig(num_hidden=16, fan_out=(5, 5), batch_size=64,
                                                           num_epochs=6, lr=0.01, emb_lr=0.1))
        hist = tr.train()
        res["losses"] = hist["losses"]
        res["auc"] = tr.evaluate(2)
        # 5. distributed layer-wise inference == full-graph inference with the same weights
        table = tr.emb.gather(torch.arange(g.num_nodes))
        got = tr.gather_embeddings()
        if rank == 0:
            from cloudtik_amd.modeling.graph_sage.graph import full_blocks
            with torch.no_grad():
                h = table
                for i, (b, layer) in enumerate(zip(full_blocks(g, len(tr.layers)), tr.layers)):
                    h = layer(b, h)
                    h = torch.relu(h) if i < len(tr.layers) - 1 else h
            res["infer"] = torch.allclose(got, h, atol=1e-5)
        else:
            res["infer"] = got is None
        dense_sum = sum(float(p.detach().sum()) for p in tr.dense)
        t = torch.tensor([dense_sum])
        dist.all_reduce(t)
        res["dense_in_sync"] = abs(float(t) / world - dense_sum) < 1e-4
        out[rank] = res
    finally:
        dist.destroy_process_group()


def test_distributed_graphsage_gloo(tmp_path):
    g = community_graph()
    partition_graph(g, 2, str(tmp_path), "ldg")
    out = mp.Manager().dict()
    mp.spawn(_worker, args=(2, _port(), str(tmp_path), out), nprocs=2, join=True)
    for r in range(2):
        res = out[r]
        assert res["full_equal"], r
        assert res["sample_ok"], (r, res["sample_real"], res["sample_deg"], res["sample_inputs"])
        assert res["lookup"] and res["adagrad"], r
        assert res["dense_in_sync"] and res["infer"], r
        assert res["losses"][-1] < res["losses"][0] * 0.9, res["losses"]
        assert res["auc"] > 0.7, res["auc"]
