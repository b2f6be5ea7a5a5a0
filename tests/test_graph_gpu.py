"""GPU numerics of the graph / boosted-tree kernels (csrc/graph_ml.hip) against the fp32
PyTorch references, plus the modeling workloads end to end on the MI355X."""
import numpy as np
import pytest
import torch

from cloudtik_amd import ops
from cloudtik_amd.ops import graph as G

pytestmark = pytest.mark.gpu
dev = torch.device("cuda", 0)


@pytest.mark.parametrize("F,N,S,B", [(13, 10001, 1, 256), (5, 4099, 7, 64), (3, 2050, 40, 256), (8, 65536, 16, 256)])
def test_gbdt_hist_kernel(F, N, S, B):
    g = torch.Generator().manual_seed(F * N)
    ldb = (N + 3) // 4 * 4
    bins = torch.zeros(F, ldb, dtype=torch.uint8)
    bins[:, :N] = torch.randint(0, B, (F, N), generator=g).to(torch.uint8)
    node = torch.randint(-1, S, (N,), generator=g, dtype=torch.int32)
    gh = torch.randn(N, 2, generator=g)
    want = G.gbdt_histogram_reference(bins, N, node, gh, S, B)
    got = ops.gbdt_histogram(bins.to(dev), N, node.to(dev), gh.to(dev), S, B)
    torch.testing.assert_close(got.cpu(), want, rtol=1e-4, atol=1e-3)


def _random_trees(T, depth, F, B, g):
    M = 2 ** (depth + 1) - 1
    feat = torch.randint(0, F, (T, M), generator=g, dtype=torch.int32)
    leafmask = torch.rand(T, M, generator=g) < 0.2
    feat[leafmask] = -1
    feat[:, M // 2:] = -1
    thr = torch.randint(1, B - 1, (T, M), generator=g, dtype=torch.int32)
    dleft = torch.randint(0, 2, (T, M), generator=g).to(torch.uint8)
    leaf = torch.randn(T, M, generator=g)
    return feat, thr, dleft, leaf


@pytest.mark.parametrize("K", [1, 3])
def test_gbdt_predict_kernel(K):
    g = torch.Generator().manual_seed(K)
    F, N, B = 9, 5003, 256
    ldb = (N + 3) // 4 * 4
    bins = torch.zeros(F, ldb, dtype=torch.uint8)
    bins[:, :N] = torch.randint(0, B, (F, N), generator=g).to(torch.uint8)
    trees = _random_trees(12 * K, 5, F, B, g)
    want = G.gbdt_predict_reference(bins, N, *trees, K)
    got = ops.gbdt_predict(bins.to(dev), N, *[t.to(dev) for t in trees], K)
    torch.testing.assert_close(got.cpu(), want, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("D", [8, 64, 256, 1024])
def test_csr_spmm_kernel(dtype, D):
    g = torch.Generator().manual_seed(D)
    n_dst, n_src, E = 3001, 2000, 40000
    dst = torch.randint(0, n_dst - 10, (E,), generator=g)          # the last rows stay empty
    src = torch.randint(0, n_src, (E,), generator=g)
    w = torch.rand(E, generator=g)
    x = torch.randn(n_src, D, generator=g).to(dtype)
    for weight in (None, w):
        for mean in (False, True):
            csr = G.CSR.from_edges(dst, src, n_dst, n_src, weight)
            want = G.spmm_reference(csr, x.float(), mean)
            got = G._spmm_raw(csr.to(dev), x.to(dev), mean)
            tol = 1e-4 if dtype == torch.float32 else 2e-2
            torch.testing.assert_close(got.float().cpu(), want, rtol=tol, atol=tol)


def test_spmm_autograd_gpu_matches_cpu():
    g = torch.Generator().manual_seed(0)
    dst = torch.randint(0, 500, (6000,), generator=g)
    src = torch.randint(0, 700, (6000,), generator=g)
    csr = G.CSR.from_edges(dst, src, 500, 700)
    x = torch.randn(700, 32, generator=g)
    gy = torch.randn(500, 32, generator=g)
    xc = x.clone().requires_grad_()
    G.SpMM(csr, mean=True)(xc).backward(gy)
    xg = x.to(dev).requires_grad_()
    G.SpMM(csr.to(dev), mean=True)(xg).backward(gy.to(dev))
    torch.testing.assert_close(xg.grad.cpu(), xc.grad, rtol=1e-4, atol=1e-5)


def test_native_check_rejects_bad_columns():
    csr = G.CSR(torch.tensor([0, 2]), torch.tensor([0, 9]), 4)
    x = torch.randn(4, 8, device=dev)
    out = torch.empty(1, 8, device=dev)
    with pytest.raises(RuntimeError):
        ops.require_native().csr_spmm(csr.rowptr.to(dev), csr.col.to(dev), None, None, False, x, out, True)


def test_gbdt_booster_gpu_quality_and_native():
    from sklearn.metrics import roc_auc_score
    from cloudtik_amd.modeling.gbdt import DMatrix, train
    rng = np.random.default_rng(0)
    N, F = 200_000, 20
    X = rng.normal(size=(N, F)).astype(np.float32)
    X[rng.random((N, F)) < 0.03] = np.nan
    z = np.nan_to_num(X)
    y = (rng.random(N) < 1 / (1 + np.exp(-(2 * z[:, 0] - z[:, 1] ** 2 + z[:, 2] * z[:, 3])))).astype(np.float32)
    params = {"objective": "binary:logistic", "max_depth": 6, "eta": 0.2}
    bg = train(params, DMatrix(X[:160_000], y[:160_000]), 40, device=dev)
    auc_g = roc_auc_score(y[160_000:], bg.predict(X[160_000:]))
    bc = train(params, DMatrix(X[:160_000:8], y[:160_000:8]), 40, device="cpu")   # small CPU run as a bar
    auc_c = roc_auc_score(y[160_000:], bc.predict(X[160_000:]))
    assert auc_g > 0.85 and auc_g > auc_c - 0.01, (auc_g, auc_c)


def test_graph_sage_trains_on_gpu():
    import pandas as pd
    from cloudtik_amd.modeling.graph_sage import LinkPredictionTrainer, TrainConfig, build_graph
    rng = np.random.default_rng(0)
    n = 20000
    card = rng.integers(0, 1000, n)
    merch = np.where(rng.random(n) < 0.9, (card % 8) * 60 + rng.integers(0, 60, n), rng.integers(0, 480, n))
    df = pd.DataFrame({"card_id": card, "merchant_id": merch, "split": rng.choice([0, 1, 2], n, p=[.8, .1, .1])})
    cfg = {"node_columns": {"card_id": "card", "merchant_id": "merchant"},
           "edge_types": [["card_id", "pay", "merchant_id"], ["merchant_id", "charge", "card_id"]],
           "reverse_edges": {"pay": "charge", "charge": "pay"}, "edge_split": "split"}
    tr = LinkPredictionTrainer(build_graph(df, cfg), TrainConfig(num_epochs=2, num_hidden=64, batch_size=1024,
                                                                 log_every=0), device=dev)
    h = tr.train()
    assert h["test_auc"] > 0.85, h


def test_transfer_learning_gpu_bf16():
    from cloudtik_amd.modeling.transfer_learning import get_model, synthetic_image_dataset
    m = get_model("resnet50", use_case="image_classification", num_classes=4, freeze_backbone=True, device=dev)
    assert m.dtype == torch.bfloat16
    hist = m.train(synthetic_image_dataset(128, 4, image_size=64), epochs=1, batch_size=32, log_every=0)
    assert np.isfinite(hist[-1]["loss"])


def test_gbdt_native_level_kernels_match_cpu_growth():
    """The fused GPU level kernels grow the same trees as the tensor-op CPU path."""
    from cloudtik_amd.modeling.gbdt import DMatrix, train
    rng = np.random.default_rng(3)
    N, F = 20000, 10
    X = rng.normal(size=(N, F)).astype(np.float32)
    X[rng.random((N, F)) < 0.05] = np.nan
    z = np.nan_to_num(X)
    y = (z[:, 0] + 0.5 * z[:, 1] ** 2 - z[:, 2] + rng.normal(size=N) * 0.3).astype(np.float32)
    for params in ({"objective": "reg:squarederror", "max_depth": 5, "eta": 0.3, "max_bin": 64},
                   {"objective": "reg:squarederror", "max_depth": 4, "eta": 0.3, "max_bin": 256, "lambda": 2.0,
                    "alpha": 0.5, "gamma": 0.1, "min_child_weight": 5, "colsample_bytree": 0.7}):
        bg = train(params, DMatrix(X, y), 8, device=dev)
        bc = train(params, DMatrix(X, y), 8, device="cpu")
        assert torch.equal(bg.trees.feat[0].cpu(), bc.trees.feat[0]) and torch.equal(bg.trees.thr[0].cpu()[bc.trees.feat[0] >= 0], bc.trees.thr[0][bc.trees.feat[0] >= 0])
        pg, pc = bg.predict(X), bc.predict(X)
        assert np.corrcoef(pg, pc)[0, 1] > 0.999 and np.abs(pg - pc).mean() < 1e-2 * y.std()
