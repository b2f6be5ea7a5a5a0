"""Spark/pandas -> Parquet store -> distributed training estimator (SURVEY.md §2.14 Horovod
Spark estimators): 1 rank and 2 gloo ranks learn a separable problem; transform() scores."""
import numpy as np
import pandas as pd
import pytest
import torch


def _df(n=2048, seed=0):
    rng = np.random.default_rng(seed)
    x = rng.normal(size=(n, 8)).astype(np.float32)
    w = rng.normal(size=(8,)).astype(np.float32)
    y = (x @ w > 0).astype(np.int64)
    return pd.DataFrame({"features": list(x), "label": y})


@pytest.mark.parametrize("num_proc", [1, 2])
def test_torch_estimator_fit_transform(tmp_path, num_proc):
    from cloudtik_amd.runtime.ai.estimator import Store, TorchEstimator
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(8, 32), torch.nn.ReLU(), torch.nn.Linear(32, 2))
    est = TorchEstimator(net, loss="cross_entropy", optimizer="adamw", lr=1e-2, batch_size=64, epochs=4,
                         num_proc=num_proc, store=Store.create(str(tmp_path)), master_port=29700 + num_proc)
    df = _df()
    model = est.fit(df)
    assert model.history and model.history[-1]["loss"] < model.history[0]["loss"]
    out = model.transform(df)
    pred = np.stack(out["label__output"].to_list()).argmax(1)
    assert (pred == df["label"].to_numpy()).mean() > 0.9
    assert (tmp_path / "intermediate_train_data").exists() and (tmp_path / "runs" / model.run_id).exists()
