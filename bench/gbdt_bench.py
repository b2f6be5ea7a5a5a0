"""GBDT (hist) training/inference throughput on one GPU: synthetic HIGGS-shaped problem
(N rows x 28 float features, binary:logistic, depth 8, 256 bins).  Reports seconds per
boosting round, histogram-kernel share, and ensemble prediction rows/s."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--features", type=int, default=28)
    ap.add_argument("--rounds", type=int, default=100)
    ap.add_argument("--depth", type=int, default=8)
    a = ap.parse_args()
    from cloudtik_amd.modeling.gbdt import BinMapper, Booster, DMatrix, train
    from sklearn.metrics import roc_auc_score
    rng = np.random.default_rng(0)
    X = rng.normal(size=(a.rows, a.features)).astype(np.float32)
    w = rng.normal(size=a.features)
    logit = X @ w * 0.5 + np.sin(X[:, 0] * 2) + X[:, 1] * X[:, 2]
    y = (rng.random(a.rows) < 1 / (1 + np.exp(-logit))).astype(np.float32)
    n_tr = int(a.rows * 0.9)
    dtr, dte = DMatrix(X[:n_tr], y[:n_tr]), DMatrix(X[n_tr:], y[n_tr:])
    params = {"objective": "binary:logistic", "max_depth": a.depth, "eta": 0.1, "max_bin": 256}
    train(params, dtr, 3)                         # warm-up: kernels, allocator
    torch.cuda.synchronize()
    # quantisation (quantile sketch + binning to uint8 on the GPU) timed on its own
    t0 = time.time()
    b = Booster(params)
    b.mapper = BinMapper(256).fit(dtr.X.to(b.device))
    dtr.binned(b.mapper, b.device)
    torch.cuda.synchronize()
    t_prep = time.time() - t0
    t0 = time.time()
    b.train(dtr, a.rounds)
    torch.cuda.synchronize()
    t_train = time.time() - t0
    b.predict(dte)
    torch.cuda.synchronize()
    t0 = time.time()
    p = b.predict(dte)
    t_pred = time.time() - t0
    print(json.dumps({"rows": n_tr, "features": a.features, "depth": a.depth, "rounds": a.rounds,
                      "quantize_seconds": round(t_prep, 3), "train_seconds": round(t_train, 3), "ms_per_round": round(1000 * t_train / a.rounds, 3),
                      "predict_rows_per_sec": round(len(p) / t_pred), "test_auc": round(roc_auc_score(y[n_tr:], p), 4)}),
          flush=True)


if __name__ == "__main__":
    main()
