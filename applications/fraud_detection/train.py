#!/usr/bin/env python3
"""Fraud detection application (reference applications/ai/fraud_detection/src/train.py:
XGBoost baseline + GraphSAGE card/merchant embeddings -> XGBoost on the enriched table).

Pipeline on the MI355X modeling library:
  1. tabular preprocessing (config-driven transforms, time split) -- ``modeling.gbdt.data``
  2. GBDT baseline on the transaction features                   -- ``modeling.gbdt``
  3. card <-> merchant graph, GraphSAGE link prediction          -- ``modeling.graph_sage``
  4. node embeddings joined back to every transaction, GBDT again
Reports test AUC-PR for both models.  Without ``--data`` it generates a synthetic
credit-card table in the shape of the reference's TabFormer input (fraudsters use
compromised cards at a ring of merchants, so graph structure carries signal the per-row
features do not).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import numpy as np  # noqa: E402


def synthetic_transactions(n=200_000, cards=20_000, merchants=3_000, seed=0):
    import pandas as pd
    rng = np.random.default_rng(seed)
    card = rng.integers(0, cards, n)
    home = card % merchants
    local = np.minimum(merchants - 1, home + rng.integers(0, 40, n))
    merch = np.where(rng.random(n) < 0.8, local, rng.integers(0, merchants, n))
    compromised = rng.random(cards) < 0.02
    ring = rng.choice(merchants, 60, replace=False)
    is_c = compromised[card]
    at_ring = is_c & (rng.random(n) < 0.5)
    merch = np.where(at_ring, rng.choice(ring, n), merch)
    fraud = (at_ring & (rng.random(n) < 0.7)) | (rng.random(n) < 0.002)
    amount = np.round(rng.lognormal(3.5, 1.0, n) * np.where(fraud, 1.6, 1.0), 2)
    year = rng.choice([2016, 2017, 2018, 2019], n, p=[.3, .3, .2, .2])
    return pd.DataFrame({"user": card // 3, "card": card % 3, "year": year, "month": rng.integers(1, 13, n),
                         "day": rng.integers(1, 29, n),
                         "time": [f"{h:02d}:{m:02d}" for h, m in zip(rng.integers(0, 24, n), rng.integers(0, 60, n))],
                         "amount": [f"${a:.2f}" for a in amount], "use_chip": rng.choice(["Swipe", "Chip", "Online"], n),
                         "merchant_name": merch, "mcc": (merch * 7) % 90 + 5000,
                         "errors?": rng.choice(["", "Bad PIN", "Insufficient Balance"], n, p=[.97, .02, .01]),
                         "is_fraud?": np.where(fraud, "Yes", "No")})


PROCESSING = {
    "data_transform": [
        {"categorify": {"merchant_name": "merchant_id", "is_fraud?": "is_fraud?"}},
        {"strip_chars": {"amount": {"amount": "$"}}},
        {"combine_cols": {"card_id": {"concatenate_strings": ["user", "card"]}}},
        {"time_to_seconds": {"time": "time"}},
        {"change_datatype": {"amount": "float32", "card_id": "float32"}},
        {"min_max_normalization": {"time": "time"}},
        {"one_hot_encoding": {"use_chip": True}},
        {"string_to_list": {"errors?": {"errors?": ","}}},
        {"multi_hot_encoding": {"errors?": True}},
        {"add_constant_feature": {"split": 0}},
        {"modify_on_conditions": {"split": {"df.year == 2018": 1, "df.year > 2018": 2}}}],
}
GRAPH = {"node_types": ["card", "merchant"], "node_columns": {"card_id": "card", "merchant_id": "merchant"},
         "edge_types": [["card_id", "pay", "merchant_id"], ["merchant_id", "charge", "card_id"]],
         "reverse_edges": {"pay": "charge", "charge": "pay"}, "edge_split": "split", "edge_label": "is_fraud?"}
IGNORE = ["merchant_name", "user", "card", "split", "card_id", "merchant_id"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--data", help="CSV in the TabFormer column layout (default: synthetic)")
    ap.add_argument("--rows", type=int, default=200_000)
    ap.add_argument("--rounds", type=int, default=200)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--hidden", type=int, default=32)
    ap.add_argument("--device", default=None)
    a = ap.parse_args()
    import pandas as pd
    import torch
    from cloudtik_amd.modeling.gbdt import Booster, DMatrix, evaluate_metric
    from cloudtik_amd.modeling.gbdt.data import DataTransformer, feature_frame
    from cloudtik_amd.modeling.graph_sage import LinkPredictionTrainer, TrainConfig, build_graph
    from cloudtik_amd.modeling.graph_sage.run import apply_embeddings

    df = pd.read_csv(a.data) if a.data else synthetic_transactions(a.rows)
    df = DataTransformer(df).apply(PROCESSING["data_transform"])
    target = "is_fraud?"
    params = {"objective": "binary:logistic", "eta": 0.1, "max_depth": 6, "eval_metric": "aucpr"}

    def fit_eval(frame, ignore):
        tr, te = frame[frame["split"] == 0], frame[frame["split"] != 0]
        Xtr, ytr = feature_frame(tr, target, [c for c in ignore if c in tr.columns])
        Xte, yte = feature_frame(te, target, [c for c in ignore if c in te.columns])
        b = Booster(params, device=a.device).train(DMatrix(Xtr, ytr), a.rounds)
        p = torch.tensor(b.predict(DMatrix(Xte)))[:, None]
        return evaluate_metric("aucpr", p, torch.tensor(yte.to_numpy()), torch.ones(len(yte)))

    base = fit_eval(df, IGNORE)
    graph = build_graph(df, GRAPH)
    tr = LinkPredictionTrainer(graph, TrainConfig(num_epochs=a.epochs, num_hidden=a.hidden, batch_size=2048,
                                                  log_every=0), device=a.device)
    hist = tr.train()
    emb = tr.embeddings().float().cpu().numpy()
    enriched = apply_embeddings(df.copy(), graph, emb, GRAPH["node_columns"])
    with_emb = fit_eval(enriched, IGNORE)
    print(json.dumps({"rows": len(df), "baseline_test_aucpr": round(base, 4),
                      "with_graph_embeddings_test_aucpr": round(with_emb, 4),
                      "graph_sage_test_auc": round(hist.get("test_auc", float("nan")), 4),
                      "graph": {"nodes": graph.num_nodes, "edges": graph.num_edges}}), flush=True)


if __name__ == "__main__":
    main()
