"""Spark -> Parquet -> GPU training pipeline pieces (north-star config 5; reference flow:
examples/runtime/ai/basics/pytorch/mnist-pytorch-spark-horovod-hyperopt-mlflow.py:159-214 --
Spark prepares data, writes Parquet to the Store (HDFS / cloud storage), Horovod trainers
read it back through Petastorm).

* ``write_image_shards``  -- the ETL side: image rows (uint8 HWC + label) written as Parquet
  part files, by Spark when pyspark is installed (one task per part) and by a process pool
  of pyarrow writers otherwise; paths may be local or ``hdfs://`` / object-store URLs.
* ``ParquetImageLoader``  -- the training side: each rank streams its own part files row
  group by row group with bounded host memory (data/streaming.py), stages uint8 batches in
  pinned host slots and copies them on a side stream, and one HIP pass
  (``ops.images_to_tensor``) turns them into normalised, optionally flipped bf16
  channels-last tensors on the GPU.
"""
from __future__ import annotations

import glob
import os
from concurrent.futures import ProcessPoolExecutor
from typing import Dict, Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch


def _part_path(root: str, i: int) -> str:
    return os.path.join(root, f"part-{i:05d}.parquet")


def _write_part(args) -> str:
    root, i, rows, size, classes, seed = args
    from cloudtik_amd.data.parquet import write_parquet
    rng = np.random.default_rng(seed + i)
    labels = rng.integers(0, classes, rows).astype(np.int64)
    # class-dependent colour so a model can learn from the synthetic images
    base = (rng.random((classes, 1, 1, 3)) * 200).astype(np.uint8)
    img = (base[labels] + rng.integers(0, 56, (rows, size, size, 3), dtype=np.uint8)).astype(np.uint8)
    path = _part_path(root, i)
    write_parquet(path, {"image": img.reshape(rows, -1), "label": labels}, row_group_size=max(1, min(rows, 1024)))
    return path


def write_image_shards(root: str, total_rows: int, num_parts: int, image_size: int = 224, num_classes: int = 1000,
                       seed: int = 0, engine: str = "auto", workers: int = 4) -> List[str]:
    """Synthetic ImageNet-shaped ETL output: ``num_parts`` Parquet files under ``root``."""
    os.makedirs(root, exist_ok=True)
    per = [total_rows // num_parts + (1 if i < total_rows % num_parts else 0) for i in range(num_parts)]
    tasks = [(root, i, per[i], image_size, num_classes, seed) for i in range(num_parts)]
    use_spark = engine == "spark"
    if engine == "auto":
        from cloudtik_amd.runtime.ai.data import get_data_api
        use_spark = get_data_api("spark").available()
    if use_spark:
        from pyspark.sql import SparkSession
        spark = SparkSession.builder.appName("cloudtik-amd-etl").getOrCreate()
        return spark.sparkContext.parallelize(tasks, num_parts).map(_write_part).collect()
    if workers <= 1 or num_parts == 1:
        return [_write_part(t) for t in tasks]
    with ProcessPoolExecutor(min(workers, num_parts)) as ex:
        return list(ex.map(_write_part, tasks))


def rank_parts(root: str, rank: int, world: int) -> List[str]:
    parts = sorted(glob.glob(os.path.join(root, "*.parquet")))
    if len(parts) < world:
        raise ValueError(f"{len(parts)} part files for {world} ranks")
    return parts[rank::world]


class ParquetImageLoader:
    """Batches of (normalised bf16 NHWC images, labels) from a rank's Parquet part files.

    ``streaming=True`` (default): row groups are decoded on the fly with bounded host memory
    (data/streaming.py), staged through pinned slots and copied on a side stream.
    ``streaming=False``: the rank's parts are loaded once into host memory and served by the
    native prefetching loader (small datasets, repeated epochs without re-reading)."""

    def __init__(self, paths: Sequence[str], batch_size: int, image_size: int = 224, shuffle: bool = True,
                 seed: int = 0, flip_prob: float = 0.5, num_workers: int = 4, prefetch: int = 4,
                 mean=None, std=None, device=None, streaming: bool = True, window: int = 4, read_ahead: int = 2):
        from cloudtik_amd.ops.vision import IMAGENET_MEAN, IMAGENET_STD
        self.streaming = streaming
        shapes = {"image": (image_size, image_size, 3)}
        if streaming:
            from cloudtik_amd.data.streaming import ParquetRowGroupStream, PinnedBatchLoader, agree_min_batches
            self.stream = ParquetRowGroupStream(paths, batch_size, ["image", "label"], shapes, shuffle=shuffle,
                                                seed=seed, window=window, read_ahead=read_ahead,
                                                num_workers=num_workers, drop_last=True)
            self.stream.max_batches = agree_min_batches(len(self.stream))
            self.num_rows = self.stream.num_rows
            dev = torch.device(device) if device is not None else (
                torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
            self.pinned = PinnedBatchLoader(self.stream, dev, prefetch)
        else:
            from cloudtik_amd.data.loader import NativeLoader
            from cloudtik_amd.data.parquet import read_parquet_columns
            cols = read_parquet_columns(list(paths), ["image", "label"], shapes=shapes)
            self.num_rows = len(cols["label"])
            # equal-size batches on every rank keep the collectives in lockstep
            self.loader = NativeLoader(cols, batch_size, shuffle=shuffle, seed=seed, drop_last=True,
                                       num_workers=num_workers, prefetch=prefetch, device=device)
        self.flip_prob = flip_prob
        self.mean, self.std = mean or IMAGENET_MEAN, std or IMAGENET_STD
        self.gen = torch.Generator(device="cpu").manual_seed(seed + 17)

    def __len__(self) -> int:
        return len(self.stream) if self.streaming else len(self.loader)

    def set_epoch(self, epoch: int):
        (self.stream if self.streaming else self.loader).set_epoch(epoch)

    def _batches(self):
        if not self.streaming:
            yield from self.loader
            return
        yield from self.pinned

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        from cloudtik_amd import ops
        for b in self._batches():
            imgs = b["image"]
            flip = None
            if self.flip_prob > 0:
                flip = (torch.rand(imgs.shape[0], generator=self.gen) < self.flip_prob).to(torch.uint8)
                flip = flip.to(imgs.device, non_blocking=True)
            yield ops.images_to_tensor(imgs, flip, self.mean, self.std), b["label"]

    def close(self):
        if not self.streaming:
            self.loader.close()
