"""Dataset factory (reference modeling/transfer_learning/dataset_factory.py:100 ``load_dataset``
and ``get_dataset``): a (category, framework, source) key selects the dataset class.

* ``load_dataset(dataset_dir, category, framework, dataset_name=None, **kw)`` -- a user dataset:
  image classification = a folder of class sub-folders (optionally under train / validation /
  test split folders); text classification = csv / tsv files (label, text) in a directory, or
  any local ``datasets`` files (source ``hugging_face``); image anomaly detection = the
  good / bad folder layout of ``AnomalyImageFolder``;
* ``get_dataset(dataset_dir, category, framework, dataset_name, source)`` -- a catalogue
  dataset: ``hugging_face`` reads the local HF cache / files (no download on this platform).
Only the ``pytorch`` framework exists here (TensorFlow is not part of the MI355X stack).
"""
from __future__ import annotations

import csv
import os
from typing import Any, Dict, List, Optional

import numpy as np

_REGISTRY: Dict[str, Dict[str, str]] = {
    "image_classification": {"user": "image_folder"},
    "text_classification": {"user": "text_csv", "hugging_face": "hf_text"},
    "image_anomaly_detection": {"user": "anomaly_folder"},
}


def _check(category: str, framework: str, source: Optional[str]) -> str:
    if not category:
        raise ValueError("Category parameter must be specified.")
    if not framework:
        raise ValueError("Framework parameter must be specified.")
    if framework.lower() != "pytorch":
        raise NotImplementedError(f"framework {framework!r} is not supported (pytorch only)")
    cat = category.lower()
    src = (source or "user").lower()
    if cat not in _REGISTRY or src not in _REGISTRY[cat]:
        raise NotImplementedError(f"no {src} dataset for {category!r}; supported: {_REGISTRY}")
    return _REGISTRY[cat][src]


class ImageFolderSplits:
    """Folder-of-class-folders image dataset with optional train / validation / test splits."""

    SPLITS = ("train", "validation", "test")

    def __init__(self, dataset_dir: str, dataset_name: Optional[str] = None, image_size: int = 224):
        from .datasets import ImageFolderDataset
        self.dataset_dir, self.dataset_name = dataset_dir, dataset_name or os.path.basename(dataset_dir.rstrip("/"))
        present = [s for s in self.SPLITS if os.path.isdir(os.path.join(dataset_dir, s))]
        roots = {s: os.path.join(dataset_dir, s) for s in present} or {"train": dataset_dir}
        first = ImageFolderDataset(next(iter(roots.values())), image_size)
        self.class_names: List[str] = list(first.classes)
        self.splits = {s: (first if i == 0 else ImageFolderDataset(r, image_size, classes=self.class_names))
                       for i, (s, r) in enumerate(roots.items())}

    @property
    def train_subset(self):
        return self.splits.get("train")

    @property
    def validation_subset(self):
        return self.splits.get("validation")

    @property
    def test_subset(self):
        return self.splits.get("test")

    def __len__(self):
        return sum(len(d) for d in self.splits.values())


class TextCSVDataset:
    """Text classification from delimited files: each row ``label<delimiter>text`` (reference
    PyTorchTextClassificationDataset / TFCustomTextClassificationDataset conventions:
    ``class_names``, ``label_map_func``, ``delimiter``, ``header``, ``select_cols``,
    ``exclude_cols``)."""

    def __init__(self, dataset_dir: str, dataset_name: Optional[str] = None, csv_file_name: Optional[str] = None,
                 class_names: Optional[List[str]] = None, label_map_func=None, delimiter: str = ",",
                 header: bool = False, select_cols: Optional[List[int]] = None,
                 exclude_cols: Optional[List[int]] = None, max_length: int = 128, vocab_size: int = 30522):
        from .datasets import HashTokenizer, TextClassificationDataset
        files = [csv_file_name] if csv_file_name else sorted(
            f for f in os.listdir(dataset_dir) if f.endswith((".csv", ".tsv", ".txt")))
        if not files:
            raise ValueError(f"no csv / tsv / txt files in {dataset_dir}")
        rows: List[List[str]] = []
        for f in files:
            with open(os.path.join(dataset_dir, f), newline="") as fh:
                r = csv.reader(fh, delimiter=delimiter)
                if header:
                    next(r, None)
                rows += [row for row in r if row]
        cols = list(range(len(rows[0])))
        if select_cols:
            cols = [c for c in cols if c in select_cols]
        if exclude_cols:
            cols = [c for c in cols if c not in exclude_cols]
        labels_raw = [row[cols[0]] for row in rows]
        texts = [" ".join(row[c] for c in cols[1:]) for row in rows]
        if label_map_func is not None:
            labels = [int(label_map_func(v)) for v in labels_raw]
            self.class_names = class_names or [str(i) for i in range(max(labels) + 1)]
        else:
            self.class_names = class_names or sorted(set(labels_raw))
            idx = {c: i for i, c in enumerate(self.class_names)}
            labels = [idx[v] for v in labels_raw]
        self.dataset_dir, self.dataset_name = dataset_dir, dataset_name
        self.dataset = TextClassificationDataset(texts, labels, HashTokenizer(vocab_size, max_length), self.class_names)
        self._split = None

    def __len__(self):
        return len(self.dataset)

    def shuffle_split(self, train_pct: float = 0.75, val_pct: float = 0.25, test_pct: float = 0.0,
                      seed: Optional[int] = None):
        import torch
        n = len(self.dataset)
        idx = np.random.default_rng(seed).permutation(n)
        a, b = int(n * train_pct), int(n * (train_pct + val_pct))
        self._split = [torch.utils.data.Subset(self.dataset, idx[s].tolist()) for s in
                       (slice(0, a), slice(a, b), slice(b, n))]
        return self

    @property
    def train_subset(self):
        return self._split[0] if self._split else self.dataset

    @property
    def validation_subset(self):
        return self._split[1] if self._split else None

    @property
    def test_subset(self):
        return self._split[2] if self._split else None


def _construct(kind: str, dataset_dir: str, dataset_name: Optional[str], **kwargs: Any):
    if kind == "image_folder":
        return ImageFolderSplits(dataset_dir, dataset_name, **kwargs)
    if kind == "text_csv":
        return TextCSVDataset(dataset_dir, dataset_name, **kwargs)
    if kind == "hf_text":
        from .hugging_face import HuggingFaceTextClassificationDataset
        return HuggingFaceTextClassificationDataset(dataset_dir, dataset_name, **kwargs)
    if kind == "anomaly_folder":
        from .anomaly_detection import AnomalyImageFolder
        return AnomalyImageFolder(dataset_dir, **kwargs)
    raise NotImplementedError(kind)


def load_dataset(dataset_dir: str, category: str, framework: str, dataset_name: Optional[str] = None,
                 source: Optional[str] = None, **kwargs):
    """A user dataset from ``dataset_dir`` (see the module docstring for the layouts)."""
    if not os.path.isdir(dataset_dir):
        raise FileNotFoundError(dataset_dir)
    return _construct(_check(category, framework, source), dataset_dir, dataset_name, **kwargs)


def get_dataset(dataset_dir: str, category: str, framework: str, dataset_name: Optional[str] = None,
                source: Optional[str] = None, **kwargs):
    """A catalogue dataset; the source defaults to hugging_face for PyTorch text datasets
    (reference dataset_factory.py get_dataset)."""
    if dataset_name and not source and category == "text_classification":
        source = "hugging_face"
    return _construct(_check(category, framework, source), dataset_dir, dataset_name, **kwargs)
