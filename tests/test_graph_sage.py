"""GraphSAGE (ai.modeling.graph_sage) on CPU: SpMM reference + autograd, graph building,
neighbour sampling invariants, link-prediction quality, the run.py workflow and 2-rank DDP.
DGL is not installed, so parity with the reference's DGL numbers is unpinned; the checks
are against dense PyTorch math and a planted-community graph."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from cloudtik_amd.ops.graph import CSR, SpMM, spmm_reference
from cloudtik_amd.modeling.graph_sage import LinkPredictionTrainer, TrainConfig, build_graph, sample_blocks


def _dense(csr: CSR):
    A = torch.zeros(csr.n_rows, csr.n_cols)
    dst = torch.repeat_interleave(torch.arange(csr.n_rows), csr.degrees())
    A.index_put_((dst, csr.col), csr.weight if csr.weight is not None else torch.ones(csr.col.numel()),
                 accumulate=True)
    return A


def test_spmm_mean_forward_backward_matches_dense():
    torch.manual_seed(0)
    dst = torch.randint(0, 30, (200,))
    src = torch.randint(0, 40, (200,))
    csr = CSR.from_edges(dst, src, 30, 40)
    A = _dense(csr)
    deg = A.sum(1, keepdim=True).clamp(min=1)
    x = torch.randn(40, 16, requires_grad=True)
    y = SpMM(csr, mean=True)(x)
    torch.testing.assert_close(y, (A / deg) @ x.detach(), rtol=1e-5, atol=1e-5)
    g = torch.randn_like(y)
    y.backward(g)
    torch.testing.assert_close(x.grad, (A / deg).t() @ g, rtol=1e-5, atol=1e-5)
    w = torch.rand(200)
    csr_w = CSR.from_edges(dst, src, 30, 40, w)
    torch.testing.assert_close(spmm_reference(csr_w, x.detach()), _dense(csr_w) @ x.detach(), rtol=1e-5, atol=1e-5)


def _table(n=6000, seed=0):
    import pandas as pd
    rng = np.random.default_rng(seed)
    C = 8
    card = rng.integers(0, 400, n)
    comm = card % C
    merch = np.where(rng.random(n) < 0.9, comm * 25 + rng.integers(0, 25, n), rng.integers(0, 200, n))
    return pd.DataFrame({"card_id": card, "merchant_id": merch, "amount": rng.random(n),
                         "split": rng.choice([0, 1, 2], n, p=[.8, .1, .1]), "is_fraud?": (rng.random(n) < .05) * 1})


CFG = {"node_types": ["card", "merchant"], "node_columns": {"card_id": "card", "merchant_id": "merchant"},
       "edge_types": [["card_id", "pay", "merchant_id"], ["merchant_id", "charge", "card_id"]],
       "reverse_edges": {"pay": "charge", "charge": "pay"}, "edge_split": "split", "edge_label": "is_fraud?"}


def test_build_graph_and_sampling():
    df = _table(2000).drop_duplicates(["card_id", "merchant_id"]).reset_index(drop=True)   # no multi-edges
    g = build_graph(df, CFG)
    n_card, n_merch = df.card_id.nunique(), df.merchant_id.nunique()
    R = len(df)
    assert g.num_nodes == n_card + n_merch and g.num_edges == 2 * R
    e = torch.arange(R)
    assert torch.equal(g.src[g.reverse_eid[e]], g.dst[e]) and torch.equal(g.dst[g.reverse_eid[e]], g.src[e])
    assert bool((g.node_type[g.src[:R]] == 0).all()) and bool((g.node_type[g.dst[:R]] == 1).all())
    seeds = torch.unique(g.src[:50])
    excl = torch.cat([e[:50], g.reverse_eid[:50]])
    inputs, blocks = sample_blocks(g, seeds, [3, 4], torch.Generator().manual_seed(0), excl)
    last = blocks[-1]
    assert torch.equal(last.src_nodes[:last.num_dst], seeds)
    assert int(last.csr.degrees().max()) <= 4
    assert torch.equal(blocks[0].src_nodes, inputs)
    assert torch.equal(blocks[0].src_nodes[:blocks[0].num_dst], blocks[1].src_nodes)
    # excluded edges never appear as (dst <- src) messages of the output layer
    banned = set(zip(g.dst[excl].tolist(), g.src[excl].tolist()))
    dsts = torch.repeat_interleave(torch.arange(last.num_dst), last.csr.degrees())
    got = set(zip(last.src_nodes[dsts].tolist(), last.src_nodes[last.csr.col].tolist()))
    assert not (got & banned)


def test_link_prediction_learns_communities():
    g = build_graph(_table(), CFG)
    tr = LinkPredictionTrainer(g, TrainConfig(num_epochs=3, num_hidden=32, batch_size=512, log_every=0), device="cpu")
    h = tr.train()
    assert h["test_auc"] > 0.85, h
    emb = tr.embeddings()
    assert emb.shape == (g.num_nodes, 32) and torch.isfinite(emb).all()


def test_graph_sage_run_workflow(tmp_path):
    import yaml
    df = _table(3000)
    raw = tmp_path / "tx.csv"
    df.to_csv(raw, index=False)
    (tmp_path / "t2g.yaml").write_text(yaml.safe_dump(CFG))
    from cloudtik_amd.modeling.graph_sage import run as gs_run
    out = gs_run.main(["--raw-data-path", str(raw), "--tabular2graph", str(tmp_path / "t2g.yaml"),
                       "--output-dir", str(tmp_path / "out"), "--num-epochs", "1", "--num-hidden", "16",
                       "--fan-out", "5,5", "--batch-size", "512", "--log-every", "0", "--device", "cpu"])
    import pandas as pd
    d = pd.read_csv(out["data_with_embeddings"])
    assert "card_id" not in d.columns and "n0_c0_e0" in d.columns and "n1_c0_e15" in d.columns
    assert len(d) == 3000 and np.load(out["embeddings"]).shape[1] == 16


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("num_parts", [1, 2])
def test_graph_sage_ddp_gloo(tmp_path, num_parts):
    df = _table(3000)
    raw = tmp_path / "tx.csv"
    df.to_csv(raw, index=False)
    import yaml
    (tmp_path / "t2g.yaml").write_text(yaml.safe_dump(CFG))
    env = dict(os.environ, PYTHONPATH=os.getcwd(), OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                        "-m", "cloudtik_amd.modeling.graph_sage.run", "--raw-data-path", str(raw),
                        "--tabular2graph", str(tmp_path / "t2g.yaml"), "--output-dir", str(tmp_path / "out"),
                        "--num-epochs", "2", "--num-hidden", "16", "--fan-out", "5,5", "--batch-size", "256",
                        "--log-every", "0", "--device", "cpu", "--num-parts", str(num_parts),
                        "--temp-dir", str(tmp_path)],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    import json
    res = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert res["test_auc"] > 0.75, res
    if num_parts > 1:        # partitioned graph + sharded embeddings, cut edges sampled remotely
        assert res["partition"]["edge_cut"] > 0 and os.path.exists(res["embeddings"])
