#!/usr/bin/env python3
"""Hyperparameter search over an MLP on the scikit-learn digits images with concurrent trials
(one GPU per trial when GPUs are visible) and every trial logged to the cluster's MLflow
tracking server (reference examples/runtime/ai/basics/pytorch/
mnist-pytorch-single-node-hyperopt-mlflow.py; the 8x8 digits ship with scikit-learn, so the
example needs no download).

    python examples/ai/basics/digits_hyperopt_tracking.py --trials 8
    cloudtik submit cluster.yaml examples/ai/basics/digits_hyperopt_tracking.py
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", ".."))


def load_digits_split(seed=0):
    import numpy as np
    from sklearn.datasets import load_digits
    d = load_digits()
    x = (d.data / 16.0).astype("float32")
    y = d.target.astype("int64")
    idx = np.random.default_rng(seed).permutation(len(x))
    cut = int(0.8 * len(x))
    return x[idx[:cut]], y[idx[:cut]], x[idx[cut:]], y[idx[cut:]]


def objective(params):
    """One trial: train, evaluate, log the run; runs in its own process (one GPU)."""
    import torch
    import torch.nn.functional as F
    from cloudtik_amd.models.mlp import MLP
    from cloudtik_amd.runtime.ai.tracking import start_run
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    xtr, ytr, xva, yva = (torch.from_numpy(a).to(dev) for a in load_digits_split())
    torch.manual_seed(0)
    model = MLP(64, (params["hidden"], params["hidden"] // 2), 10, dropout=params["dropout"], device=dev)
    opt = torch.optim.AdamW(model.parameters(), lr=params["lr"], weight_decay=params["weight_decay"])
    name = f"lr{params['lr']:.1e}-h{params['hidden']}-pid{os.getpid()}"
    with start_run(params.get("experiment", "digits-hyperopt"), run_name=name) as run:
        run.log_params({k: v for k, v in params.items() if k != "experiment"})
        for epoch in range(params["epochs"]):
            model.train()
            perm = torch.randperm(len(xtr), device=dev)
            for i in range(0, len(xtr), 64):
                b = perm[i:i + 64]
                loss = F.cross_entropy(model(xtr[b]), ytr[b])
                opt.zero_grad()
                loss.backward()
                opt.step()
            model.eval()
            with torch.no_grad():
                logits = model(xva)
                val_loss = float(F.cross_entropy(logits, yva))
                acc = float((logits.argmax(1) == yva).float().mean())
            run.log_metrics({"val_loss": val_loss, "val_accuracy": acc}, step=epoch)
    return {"loss": val_loss, "accuracy": acc}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=8)
    ap.add_argument("--concurrent", type=int, default=None)
    ap.add_argument("--epochs", type=int, default=8)
    ap.add_argument("--experiment", default="digits-hyperopt")
    a = ap.parse_args(argv)
    from cloudtik_amd.runtime.ai.tune import choice, loguniform, tune, uniform
    space = {"lr": loguniform(1e-4, 3e-2), "weight_decay": loguniform(1e-5, 1e-2), "dropout": uniform(0.0, 0.4),
             "hidden": choice([64, 128, 256]), "epochs": choice([a.epochs]), "experiment": choice([a.experiment])}
    res = tune(objective, space, num_trials=a.trials, max_concurrent=a.concurrent)
    best = res.best
    out = {"best_params": {k: v for k, v in best.params.items() if k not in ("experiment",)},
           "best": best.result, "trials": len(res.trials), "failed": sum(t.error is not None for t in res.trials)}
    print(json.dumps(out), flush=True)
    return out


if __name__ == "__main__":
    main()
