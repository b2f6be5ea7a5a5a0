"""Spark-to-training estimators (reference: the Horovod-on-Spark estimator examples,
``hvd.spark.torch.TorchEstimator`` + ``Store`` -> Parquet -> Petastorm readers,
examples/runtime/ai/basics/pytorch/mnist-pytorch-spark-horovod-hyperopt-mlflow.py:159-214;
SURVEY.md §2.14 "Spark data parallelism").

    store = Store.create("/data/estimator")          # local path, hdfs://..., s3://...
    est = TorchEstimator(model=net, loss="cross_entropy", optimizer="adamw", lr=1e-3,
                         feature_cols=["features"], label_cols=["label"], batch_size=128,
                         epochs=5, num_proc=8, store=store)
    trained = est.fit(df)                            # Spark or pandas DataFrame
    scored = trained.transform(df)                   # adds "label__output"

``fit`` materialises the DataFrame once as Parquet in the store (Spark writes it directly in
parallel; pandas goes through pyarrow), launches ``num_proc`` ranks with ``cloudtik-run``'s
function API (one rank per GPU, RCCL data parallelism through the framework Trainer: flat
parameter space, bucketed all-reduce overlapped with backward, fused optimizers), each rank
taking its shard of one global per-epoch permutation through the native pinned-memory
loader (equal batch counts on every rank), and returns a
``TorchModel`` with the rank-0 weights.  Checkpoints go to the store's run directory.
"""
from __future__ import annotations

import copy
import os
import uuid
from typing import Any, Callable, Dict, List, Optional, Sequence, Union

import numpy as np
import torch


class Store:
    """Where an estimator keeps its materialised data, checkpoints and run outputs."""

    def __init__(self, prefix: str):
        self.prefix = prefix.rstrip("/")

    @staticmethod
    def create(prefix: str) -> "Store":
        return Store(prefix)

    @property
    def is_local(self) -> bool:
        return "://" not in self.prefix or self.prefix.startswith("file://")

    def _path(self, *parts) -> str:
        p = "/".join([self.prefix, *parts])
        return p[len("file://"):] if p.startswith("file://") else p

    def train_data_path(self, dataset_id: str) -> str:
        return self._path("intermediate_train_data", dataset_id)

    def val_data_path(self, dataset_id: str) -> str:
        return self._path("intermediate_val_data", dataset_id)

    def run_path(self, run_id: str) -> str:
        return self._path("runs", run_id)

    def checkpoint_path(self, run_id: str) -> str:
        return self._path("runs", run_id, "checkpoints")


def _is_spark_df(df) -> bool:
    return type(df).__module__.startswith("pyspark")


def _to_columns(pdf, cols: Sequence[str]) -> Dict[str, np.ndarray]:
    out = {}
    for c in cols:
        v = pdf[c].to_numpy()
        if v.dtype == object:                         # array-valued cells (vectors, lists)
            v = np.stack([np.asarray(x) for x in v])
        out[c] = v
    return out


def write_dataframe(df, path: str, cols: Sequence[str], num_files: int) -> List[str]:
    """Materialise ``cols`` of a Spark or pandas DataFrame as ``num_files`` Parquet files."""
    from cloudtik_amd.data.parquet import write_parquet
    if _is_spark_df(df):
        df.select(*cols).repartition(num_files).write.mode("overwrite").parquet(path)
        return [path]
    os.makedirs(path, exist_ok=True)
    cols_np = _to_columns(df, cols)
    n = len(df)
    files = []
    bounds = np.linspace(0, n, num_files + 1).astype(int)
    for i in range(num_files):
        lo, hi = bounds[i], bounds[i + 1]
        f = os.path.join(path, f"part-{i:05d}.parquet")
        write_parquet(f, {c: a[lo:hi] for c, a in cols_np.items()})
        files.append(f)
    return files


def _loss_fn(loss: Union[str, Callable]) -> Callable:
    if callable(loss):
        return loss
    import torch.nn.functional as F
    return {"cross_entropy": lambda o, y: F.cross_entropy(o.float(), y.long()),
            "mse": lambda o, y: F.mse_loss(o.float().reshape(y.shape), y.float()),
            "bce": lambda o, y: F.binary_cross_entropy_with_logits(o.float().reshape(y.shape), y.float())}[loss]


def _train_rank(state: Dict[str, Any]):
    """Runs on every rank (cloudtik-run function API)."""
    import glob
    from cloudtik_amd.data.parquet import ParquetDataLoader
    from cloudtik_amd.train.trainer import Trainer
    model = copy.deepcopy(state["model"])                 # shipped with the function (cloudpickle)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    files = sorted(glob.glob(os.path.join(state["train_path"], "*.parquet")) +
                   glob.glob(os.path.join(state["train_path"], "*", "*.parquet")))
    feat, lab = state["feature_cols"], state["label_cols"]
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    # every rank gets the same number of batches (a data-parallel step count mismatch would
    # deadlock the collectives): the loader shards one global permutation by rank
    loader = ParquetDataLoader(files, state["batch_size"], columns=list(feat) + list(lab), seed=state["seed"],
                               device=dev, drop_last=True, rank=rank, world=world)
    loss_fn = _loss_fn(state["loss"])

    def step(m, batch):
        x = batch[feat[0]] if len(feat) == 1 else torch.cat([batch[c].reshape(len(batch[c]), -1).float()
                                                             for c in feat], 1)
        y = batch[lab[0]]
        out = m(x.float() if x.dtype == torch.float64 else x)
        loss = loss_fn(out, y)
        return loss, {"loss": loss.detach()}

    trainer = Trainer(model, optimizer=state["optimizer"], lr=state["lr"], train_loader=loader, step_fn=step,
                      epochs=state["epochs"], log_every=0, checkpoint_dir=state["checkpoint_dir"])
    hist = trainer.fit()
    trainer.close()
    if rank != 0:
        return {"history": hist}
    return {"history": hist, "state_dict": {k: v.detach().cpu() for k, v in trainer.model.state_dict().items()}}


class TorchModel:
    """Trained model returned by ``TorchEstimator.fit`` (a Spark Transformer equivalent)."""

    def __init__(self, model: torch.nn.Module, feature_cols, label_cols, history=None, run_id: str = ""):
        self.model, self.feature_cols, self.label_cols = model, list(feature_cols), list(label_cols)
        self.history, self.run_id = history or [], run_id

    def getModel(self) -> torch.nn.Module:          # reference API name
        return self.model

    @torch.no_grad()
    def predict(self, features: np.ndarray, batch_size: int = 4096) -> np.ndarray:
        self.model.eval()
        dev = next(self.model.parameters()).device
        outs = []
        for s in range(0, len(features), batch_size):
            x = torch.as_tensor(np.asarray(features[s:s + batch_size])).to(dev)
            outs.append(self.model(x.float() if x.dtype == torch.float64 else x).float().cpu().numpy())
        return np.concatenate(outs) if outs else np.zeros((0,))

    def transform(self, df):
        """Adds ``<label>__output`` with the model outputs (pandas in, pandas out; a Spark
        DataFrame is converted through Arrow)."""
        spark = _is_spark_df(df)
        pdf = df.toPandas() if spark else df.copy()
        feats = _to_columns(pdf, self.feature_cols)
        x = feats[self.feature_cols[0]] if len(self.feature_cols) == 1 else np.concatenate(
            [feats[c].reshape(len(pdf), -1) for c in self.feature_cols], 1)
        out = self.predict(x)
        pdf[f"{self.label_cols[0]}__output"] = list(out) if out.ndim > 1 else out
        if spark:
            return df.sparkSession.createDataFrame(pdf)
        return pdf


class TorchEstimator:
    def __init__(self, model: torch.nn.Module, loss: Union[str, Callable] = "cross_entropy",
                 optimizer: str = "adamw", lr: float = 1e-3, feature_cols: Sequence[str] = ("features",),
                 label_cols: Sequence[str] = ("label",), batch_size: int = 32, epochs: int = 1,
                 num_proc: int = 1, store: Optional[Store] = None, run_id: Optional[str] = None,
                 seed: int = 0, master_port: int = 29600):
        self.model, self.loss, self.optimizer, self.lr = model, loss, optimizer, lr
        self.feature_cols, self.label_cols = list(feature_cols), list(label_cols)
        self.batch_size, self.epochs, self.num_proc = batch_size, epochs, num_proc
        self.store = store or Store.create(os.path.join(os.getcwd(), ".cloudtik_estimator"))
        self.run_id = run_id or f"run_{uuid.uuid4().hex[:8]}"
        self.seed, self.master_port = seed, master_port

    def fit(self, df) -> TorchModel:
        dataset_id = uuid.uuid4().hex[:8]
        path = self.store.train_data_path(dataset_id)
        write_dataframe(df, path, self.feature_cols + self.label_cols, max(1, self.num_proc))
        state = {"model": copy.deepcopy(self.model).cpu(), "train_path": path, "feature_cols": self.feature_cols,
                 "label_cols": self.label_cols, "batch_size": self.batch_size, "epochs": self.epochs,
                 "optimizer": self.optimizer, "lr": self.lr, "loss": self.loss, "seed": self.seed,
                 "checkpoint_dir": self.store.checkpoint_path(self.run_id)}
        if self.num_proc <= 1:
            results = [_train_rank(state)]
        else:
            from cloudtik_amd.runner import run
            results = run(_train_rank, (state,), num_proc=self.num_proc, master_port=self.master_port,
                          bind_cpus=False)
        trained = copy.deepcopy(self.model).cpu()
        trained.load_state_dict(results[0]["state_dict"])
        return TorchModel(trained, self.feature_cols, self.label_cols, results[0]["history"], self.run_id)
