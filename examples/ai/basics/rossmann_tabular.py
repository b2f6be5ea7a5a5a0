#!/usr/bin/env python3
"""Tabular sales forecasting with categorical embeddings (reference examples/runtime/ai/
basics/keras/rossmann-keras-spark-horovod-hyperopt-mlflow.py: Spark feature engineering ->
Parquet -> distributed training -> RMSPE; the Keras model is rebuilt in PyTorch and trained
with the flat-parameter Trainer).

Without ``--data`` a Rossmann-shaped synthetic table is generated (stores x days with
store / day-of-week / promo / holiday effects), so the example runs offline.

    python examples/ai/basics/rossmann_tabular.py --epochs 5
    cloudtik-run -np 2 examples/ai/basics/rossmann_tabular.py --data /path/to/prepared.parquet
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", ".."))

CATEGORICAL = ["Store", "DayOfWeek", "Promo", "StateHoliday", "SchoolHoliday", "Month"]
CONTINUOUS = ["CompetitionDistance", "Day"]


def synthetic_rossmann(stores=200, days=240, seed=0):
    import numpy as np
    import pandas as pd
    rng = np.random.default_rng(seed)
    s = np.repeat(np.arange(stores), days)
    d = np.tile(np.arange(days), stores)
    dow = d % 7
    promo = (rng.random(len(s)) < 0.4).astype(int)
    hol = (rng.random(len(s)) < 0.03).astype(int)
    school = (rng.random(len(s)) < 0.15).astype(int)
    base = rng.lognormal(8.5, 0.3, stores)[s]
    dist = rng.lognormal(7.0, 1.0, stores)[s]
    sales = base * (1 + 0.25 * promo) * (1 - 0.8 * hol) * np.array([1.1, 1.0, 0.95, 0.95, 1.05, 1.2, 0.3])[dow] \
        * (1 + 0.05 * np.sin(d / 30.0)) * rng.lognormal(0, 0.05, len(s))
    return pd.DataFrame({"Store": s, "DayOfWeek": dow, "Promo": promo, "StateHoliday": hol, "SchoolHoliday": school,
                         "Month": (d // 30) % 12, "CompetitionDistance": dist, "Day": d, "Sales": sales})


def rmspe(pred, y):
    import numpy as np
    return float(np.sqrt(np.mean(((y - pred) / y) ** 2)))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--data", default=None)
    ap.add_argument("--epochs", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--lr", type=float, default=3e-3)
    a = ap.parse_args(argv)
    import numpy as np
    import pandas as pd
    import torch
    import torch.nn as nn
    from cloudtik_amd.runtime.ai.tracking import start_run
    from cloudtik_amd.train.trainer import setup_distributed
    from cloudtik_amd.parallel import GradBucketer
    from cloudtik_amd.train.optim import FlatParamSpace, FusedAdam

    rank, world, dev = setup_distributed()
    df = pd.read_parquet(a.data) if a.data else synthetic_rossmann()
    df = df[df.Sales > 0]
    cards = {c: int(df[c].max()) + 1 for c in CATEGORICAL}
    valid = df.Day >= df.Day.max() - 30          # last month held out
    mu = df[CONTINUOUS].mean()
    sd = df[CONTINUOUS].std() + 1e-6
    logy = np.log(df.Sales.to_numpy(np.float64))
    ymu, ysd = float(logy.mean()), float(logy.std() + 1e-6)     # the model predicts standardised log sales

    def tensors(part):
        cat = torch.tensor(part[CATEGORICAL].to_numpy(np.int64))
        con = torch.tensor(((part[CONTINUOUS] - mu) / sd).to_numpy(np.float32))
        y = torch.tensor(((np.log(part.Sales.to_numpy(np.float64)) - ymu) / ysd).astype(np.float32))
        return cat.to(dev), con.to(dev), y.to(dev)

    tr, va = tensors(df[~valid].iloc[rank::world]), tensors(df[valid])

    class Net(nn.Module):
        def __init__(self):
            super().__init__()
            self.emb = nn.ModuleList(nn.Embedding(cards[c], min(16, (cards[c] + 1) // 2)) for c in CATEGORICAL)
            width = sum(e.embedding_dim for e in self.emb) + len(CONTINUOUS)
            self.mlp = nn.Sequential(nn.Linear(width, 256), nn.ReLU(), nn.Linear(256, 128), nn.ReLU(),
                                     nn.Linear(128, 1))

        def forward(self, cat, con):
            h = torch.cat([e(cat[:, i]) for i, e in enumerate(self.emb)] + [con], 1)
            return self.mlp(h).squeeze(1)

    torch.manual_seed(0)
    model = Net().to(dev)
    named = list(model.named_parameters())
    space = FlatParamSpace([p for _, p in named], names=[n for n, _ in named])
    opt = FusedAdam(space, lr=a.lr)
    ddp = GradBucketer(space) if world > 1 else None
    with start_run("rossmann") as run:
        run.log_params({"epochs": a.epochs, "batch": a.batch, "lr": a.lr, "world": world})
        for epoch in range(a.epochs):
            model.train()
            perm = torch.randperm(len(tr[2]), device=dev)
            steps = len(perm) // a.batch
            if world > 1:                        # equal step counts on every rank
                t = torch.tensor([steps], device=dev)
                torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MIN)
                steps = int(t)
            for i in range(steps):
                b = perm[i * a.batch:(i + 1) * a.batch]
                loss = nn.functional.mse_loss(model(tr[0][b], tr[1][b]), tr[2][b])
                loss.backward()
                if ddp is not None:
                    ddp.finish()
                opt.step()
                opt.zero_grad()
            model.eval()
            with torch.no_grad():
                pred = np.exp(model(va[0], va[1]).double().cpu().numpy() * ysd + ymu)
            score = rmspe(pred, np.exp(va[2].double().cpu().numpy() * ysd + ymu))
            run.log_metric("val_rmspe", score, step=epoch)
    if ddp is not None:
        ddp.remove()
    if rank == 0:
        print(json.dumps({"val_rmspe": score, "world": world}), flush=True)
    return score


if __name__ == "__main__":
    main()
