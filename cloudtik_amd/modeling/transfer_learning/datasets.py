"""Datasets for transfer learning (reference modeling/transfer_learning/*/datasets: torchvision
ImageFolder, HF / TFDS text datasets).

* ``ImageFolderDataset`` -- ``root/<class>/<image>`` files decoded with Pillow, resized and
  centre-cropped to ``image_size``, ImageNet-normalised, CHW float32.
* ``ArrayImageDataset`` / ``synthetic_image_dataset`` -- in-memory arrays (e.g. columns read
  from Parquet by the Spark -> AI pipeline).
* ``TextClassificationDataset`` with ``HashTokenizer`` -- no pretrained vocabulary can be
  fetched here, so words map to ids by a stable hash into the model's vocabulary (a
  ``tokenizers`` JSON file can be passed instead when one is available locally).
"""
from __future__ import annotations

import os
import zlib
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch
from torch.utils.data import Dataset

MEAN = np.array([0.485, 0.456, 0.406], np.float32)[:, None, None]
STD = np.array([0.229, 0.224, 0.225], np.float32)[:, None, None]
IMG_EXT = (".jpg", ".jpeg", ".png", ".bmp", ".webp")


class ImageFolderDataset(Dataset):
    def __init__(self, root: str, image_size: int = 224, classes: Optional[List[str]] = None):
        self.root = root
        self.classes = classes or sorted(d for d in os.listdir(root) if os.path.isdir(os.path.join(root, d)))
        self.samples: List[Tuple[str, int]] = []
        for i, c in enumerate(self.classes):
            d = os.path.join(root, c)
            for f in sorted(os.listdir(d)):
                if f.lower().endswith(IMG_EXT):
                    self.samples.append((os.path.join(d, f), i))
        self.image_size = image_size

    def __len__(self):
        return len(self.samples)

    def load(self, path: str) -> np.ndarray:
        from PIL import Image
        s = self.image_size
        with Image.open(path) as im:
            im = im.convert("RGB")
            w, h = im.size
            scale = (s * 256 // 224) / min(w, h)
            im = im.resize((max(s, round(w * scale)), max(s, round(h * scale))), Image.BILINEAR)
            w, h = im.size
            l, t = (w - s) // 2, (h - s) // 2
            im = im.crop((l, t, l + s, t + s))
            a = np.asarray(im, dtype=np.float32).transpose(2, 0, 1) / 255.0
        return (a - MEAN) / STD

    def __getitem__(self, i):
        path, y = self.samples[i]
        return torch.from_numpy(self.load(path)), torch.tensor(y)


class ArrayImageDataset(Dataset):
    def __init__(self, images: np.ndarray, labels: np.ndarray, classes: Optional[List[str]] = None,
                 normalize: bool = False):
        self.x = images
        self.y = labels.astype(np.int64)
        self.classes = classes or [str(c) for c in range(int(self.y.max()) + 1)]
        self.normalize = normalize

    def __len__(self):
        return len(self.y)

    def __getitem__(self, i):
        x = self.x[i].astype(np.float32)
        if self.normalize:
            x = (x / 255.0 - MEAN) / STD
        return torch.from_numpy(np.ascontiguousarray(x)), torch.tensor(self.y[i])


def synthetic_image_dataset(n: int, num_classes: int, image_size: int = 224, seed: int = 0) -> ArrayImageDataset:
    """Class-dependent mean colour + noise: learnable, so fine-tuning runs can be checked."""
    rng = np.random.default_rng(seed)
    y = rng.integers(0, num_classes, n)
    centers = rng.normal(size=(num_classes, 3, 1, 1)).astype(np.float32)
    x = centers[y] + 0.8 * rng.normal(size=(n, 3, image_size, image_size)).astype(np.float32)
    return ArrayImageDataset(x, y)


class HashTokenizer:
    """Lower-case whitespace/punctuation split; word -> R + crc32(word) % (vocab - R) with
    R = min(1000, vocab // 4) reserved ids.  Ids 0 / 101 / 102 are [PAD] / [CLS] / [SEP] as
    in BERT vocabularies."""

    PAD, CLS, SEP = 0, 101, 102

    def __init__(self, vocab_size: int = 30522, max_length: int = 128, tokenizer_file: Optional[str] = None):
        if vocab_size < 512:
            raise ValueError("HashTokenizer needs a vocabulary of at least 512 ids")
        self.vocab_size, self.max_length = vocab_size, max_length
        self.reserved = min(1000, vocab_size // 4)
        self.tok = None
        if tokenizer_file:
            from tokenizers import Tokenizer
            self.tok = Tokenizer.from_file(tokenizer_file)

    def ids(self, text: str) -> List[int]:
        if self.tok is not None:
            return self.tok.encode(text).ids[1:-1]
        import re
        r = self.reserved
        return [r + zlib.crc32(w.encode()) % (self.vocab_size - r) for w in re.findall(r"\w+|[^\w\s]", text.lower())]

    def __call__(self, texts: Sequence[str]) -> Tuple[torch.Tensor, torch.Tensor]:
        L = self.max_length
        out = torch.zeros(len(texts), L, dtype=torch.long)
        mask = torch.zeros(len(texts), L, dtype=torch.long)
        for i, t in enumerate(texts):
            ids = [self.CLS] + self.ids(t)[:L - 2] + [self.SEP]
            out[i, :len(ids)] = torch.tensor(ids)
            mask[i, :len(ids)] = 1
        return out, mask


class TextClassificationDataset(Dataset):
    def __init__(self, texts: Sequence[str], labels: Sequence[int], tokenizer: HashTokenizer,
                 classes: Optional[List[str]] = None):
        self.ids, self.mask = tokenizer(list(texts))
        self.y = torch.as_tensor(np.asarray(labels, dtype=np.int64))
        self.classes = classes or [str(c) for c in range(int(self.y.max()) + 1)]

    def __len__(self):
        return len(self.y)

    def __getitem__(self, i):
        return {"input_ids": self.ids[i], "attention_mask": self.mask[i], "label": self.y[i]}

    @classmethod
    def from_csv(cls, path: str, text_col: str, label_col: str, tokenizer: HashTokenizer):
        import pandas as pd
        df = pd.read_csv(path)
        classes = sorted(df[label_col].astype(str).unique())
        labels = df[label_col].astype(str).map({c: i for i, c in enumerate(classes)}).to_numpy()
        return cls(df[text_col].astype(str).tolist(), labels, tokenizer, classes)
