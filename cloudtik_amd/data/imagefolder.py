"""ImageNet-style image folders (``root/<class>/<image>.jpg``) -> GPU batches: the data path
of the reference's ResNet-50 training (models/image_recognition/pytorch/common/main.py:
torchvision ``ImageFolder`` + ``RandomResizedCrop`` / ``RandomHorizontalFlip`` train and
``Resize(256)`` + ``CenterCrop(224)`` eval transforms, DataLoader workers).

torchvision is not part of this stack, so decoding and the geometric transforms are done
here with PIL in a process pool (one batch per task, ``forkserver`` workers so the parent's
HIP context is never forked).  Each batch arrives as uint8 HWC, is pinned, copied to the GPU
asynchronously and turned into normalised bf16 channels-last by the fused ingest kernel
(``ops.images_to_tensor``: /255, mean/std, optional per-image horizontal flip -- the flip
is done there, not on the CPU).  Ranks take disjoint slices of one per-epoch permutation
with the same number of batches each (collectives stay in lockstep).
"""
from __future__ import annotations

import math
import multiprocessing as mp
import os
import random
from typing import Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch

IMG_EXTS = (".jpg", ".jpeg", ".png", ".bmp", ".ppm", ".webp", ".tif", ".tiff")


def scan_image_folder(root: str) -> Tuple[List[Tuple[str, int]], List[str]]:
    """(path, class index) pairs and the sorted class names, torchvision ImageFolder order."""
    classes = sorted(d.name for d in os.scandir(root) if d.is_dir())
    samples = []
    for ci, c in enumerate(classes):
        for dirpath, _, files in sorted(os.walk(os.path.join(root, c))):
            for f in sorted(files):
                if f.lower().endswith(IMG_EXTS):
                    samples.append((os.path.join(dirpath, f), ci))
    return samples, classes


def random_resized_crop_box(w: int, h: int, rng: random.Random, scale=(0.08, 1.0), ratio=(3 / 4, 4 / 3)):
    """(left, top, width, height) of a RandomResizedCrop (10 tries, then a centre crop)."""
    area = w * h
    for _ in range(10):
        target = area * rng.uniform(*scale)
        ar = math.exp(rng.uniform(math.log(ratio[0]), math.log(ratio[1])))
        cw, ch = int(round(math.sqrt(target * ar))), int(round(math.sqrt(target / ar)))
        if 0 < cw <= w and 0 < ch <= h:
            return rng.randint(0, w - cw), rng.randint(0, h - ch), cw, ch
    in_ratio = w / h
    if in_ratio < ratio[0]:
        cw, ch = w, int(round(w / ratio[0]))
    elif in_ratio > ratio[1]:
        ch, cw = h, int(round(h * ratio[1]))
    else:
        cw, ch = w, h
    return (w - cw) // 2, (h - ch) // 2, cw, ch


def _decode_batch(task):
    """Worker: decode + crop + resize one batch -> uint8 [n, size, size, 3]."""
    from PIL import Image
    paths, seeds, size, train, resize = task
    out = np.empty((len(paths), size, size, 3), np.uint8)
    for i, (p, s) in enumerate(zip(paths, seeds)):
        with Image.open(p) as im:
            im = im.convert("RGB")
            w, h = im.size
            if train:
                l, t, cw, ch = random_resized_crop_box(w, h, random.Random(s))
                im = im.resize((size, size), Image.BILINEAR, box=(l, t, l + cw, t + ch))
            else:
                sc = resize / min(w, h)
                nw, nh = max(size, int(round(w * sc))), max(size, int(round(h * sc)))
                im = im.resize((nw, nh), Image.BILINEAR)
                l, t = (nw - size) // 2, (nh - size) // 2
                im = im.crop((l, t, l + size, t + size))
            out[i] = np.asarray(im, dtype=np.uint8)
    return out


class ImageFolderLoader:
    """Yields ``(images bf16 [B, 3, S, S] channels_last, labels int64 [B])`` on ``device``."""

    def __init__(self, root: str, batch_size: int, train: bool = True, image_size: int = 224,
                 resize: Optional[int] = None, rank: int = 0, world: int = 1, seed: int = 0, workers: int = 8,
                 prefetch: int = 4, flip_prob: float = 0.5, device=None, drop_last: bool = True,
                 samples: Optional[Sequence[Tuple[str, int]]] = None):
        if samples is None:
            samples, self.classes = scan_image_folder(root)
        else:
            self.classes = sorted({c for _, c in samples})
        if not samples:
            raise FileNotFoundError(f"no images under {root}")
        self.samples = list(samples)
        self.batch_size, self.train, self.size = batch_size, train, image_size
        self.resize = resize or int(round(image_size / 0.875))
        self.rank, self.world, self.seed = rank, world, seed
        self.workers, self.prefetch = max(0, workers), max(1, prefetch)
        self.flip_prob = flip_prob if train else 0.0
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.drop_last = drop_last
        self.epoch = 0
        self._pool = None

    def __len__(self) -> int:
        per_rank = len(self.samples) // self.world
        return per_rank // self.batch_size if self.drop_last else -(-per_rank // self.batch_size)

    def set_epoch(self, epoch: int):
        self.epoch = epoch

    def _indices(self) -> np.ndarray:
        n = len(self.samples)
        idx = np.random.default_rng(self.seed + self.epoch).permutation(n) if self.train else np.arange(n)
        per_rank = n // self.world
        return idx[self.rank * per_rank:(self.rank + 1) * per_rank]

    def _tasks(self):
        idx = self._indices()
        nb = len(self)
        base = (self.seed * 1000003 + self.epoch) * 1000003
        for b in range(nb):
            sel = idx[b * self.batch_size:(b + 1) * self.batch_size]
            yield ([self.samples[i][0] for i in sel], [base + int(i) for i in sel], self.size, self.train,
                   self.resize), np.array([self.samples[i][1] for i in sel], np.int64)

    def _ensure_pool(self):
        if self._pool is None and self.workers > 0:
            ctx = mp.get_context("forkserver")
            self._pool = ctx.Pool(self.workers)
        return self._pool

    def _emit(self, u8: np.ndarray, labels: np.ndarray, gen: torch.Generator):
        from cloudtik_amd import ops
        x = torch.from_numpy(u8)
        y = torch.from_numpy(labels)
        flip = None
        if self.flip_prob > 0:
            flip = (torch.rand(x.shape[0], generator=gen) < self.flip_prob).to(torch.uint8)
        if self.device.type == "cuda":
            x = x.pin_memory().to(self.device, non_blocking=True)
            y = y.pin_memory().to(self.device, non_blocking=True)
            if flip is not None:
                flip = flip.to(self.device, non_blocking=True)
        return ops.images_to_tensor(x, flip), y

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        gen = torch.Generator().manual_seed(self.seed * 7919 + self.epoch)
        tasks = list(self._tasks())
        pool = self._ensure_pool()
        if pool is None:
            for t, labels in tasks:
                yield self._emit(_decode_batch(t), labels, gen)
            return
        # bounded run-ahead: at most `prefetch` decoded batches outstanding
        pending = []
        it = iter(tasks)
        for t, labels in it:
            pending.append((pool.apply_async(_decode_batch, (t,)), labels))
            if len(pending) >= self.prefetch:
                break
        while pending:
            res, labels = pending.pop(0)
            nxt = next(it, None)
            if nxt is not None:
                pending.append((pool.apply_async(_decode_batch, (nxt[0],)), nxt[1]))
            yield self._emit(res.get(), labels, gen)

    def close(self):
        if self._pool is not None:
            self._pool.terminate()
            self._pool.join()
            self._pool = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass
