"""COCO-format detection / instance-segmentation data -> GPU batches for the R-CNN family
(reference: the quickstart Mask R-CNN's maskrcnn_benchmark ``data/datasets/coco.py`` +
``data/transforms`` + ``structures/segmentation_mask.py``, and the COCO evaluation it runs;
SURVEY.md §2.12).

* ``CocoDetection``: instances JSON -> per-image boxes (xyxy), contiguous labels (1..K in
  category-id order), instance masks decoded from polygons (PIL rasterisation) or RLE
  (uncompressed counts or the compressed string form); crowd boxes are dropped for training.
* transforms: shorter side to ``min_size`` with the longer side capped at ``max_size``,
  random horizontal flip (train), ImageNet normalisation -- done in a ``forkserver`` process
  pool, one image per task.
* collation: images padded to a multiple of 32 into one [N, 3, H, W] batch, masks padded
  to the same canvas, per-image sizes kept for the RPN / box clipping.
* ``evaluate_bbox``: COCO-style box AP (IoU 0.50:0.05:0.95, 101-point interpolation,
  max 100 detections, all areas) -- pycocotools is not in this stack.
"""
from __future__ import annotations

import json
import multiprocessing as mp
import os
import random
from typing import Any, Dict, Iterator, List, Sequence

import numpy as np
import torch

MEAN = np.array([0.485, 0.456, 0.406], np.float32) * 255
STD = np.array([0.229, 0.224, 0.225], np.float32) * 255


# ---------------------------------------------------------------------------- masks
def rle_decode(rle: Dict[str, Any], h: int, w: int) -> np.ndarray:
    """COCO RLE (column-major run lengths, starting with zeros) -> [h, w] uint8."""
    counts = rle["counts"]
    if isinstance(counts, (str, bytes)):
        counts = _rle_string_to_counts(counts.decode() if isinstance(counts, bytes) else counts)
    flat = np.zeros(h * w, np.uint8)
    pos, val = 0, 0
    for c in counts:
        if val:
            flat[pos:pos + c] = 1
        pos += c
        val ^= 1
    return flat.reshape(w, h).T.copy()


def _rle_string_to_counts(s: str) -> List[int]:
    """The compressed RLE string form: 5-bit groups with a continuation bit (0x20) and a
    sign bit on the last group; counts after the second are deltas to the count two back."""
    counts, p = [], 0
    while p < len(s):
        x, k, more = 0, 0, True
        while more:
            c = ord(s[p]) - 48
            x |= (c & 0x1F) << (5 * k)
            more = bool(c & 0x20)
            p += 1
            k += 1
            if not more and (c & 0x10):
                x |= -1 << (5 * k)
        if len(counts) > 2:
            x += counts[-2]
        counts.append(x)
    return counts


def polygons_to_mask(polys: Sequence[Sequence[float]], h: int, w: int) -> np.ndarray:
    from PIL import Image, ImageDraw
    im = Image.new("L", (w, h), 0)
    d = ImageDraw.Draw(im)
    for p in polys:
        if len(p) >= 6:
            d.polygon([(float(p[i]), float(p[i + 1])) for i in range(0, len(p) - 1, 2)], outline=1, fill=1)
    return np.asarray(im, np.uint8)


def segmentation_to_mask(seg, h: int, w: int) -> np.ndarray:
    if isinstance(seg, list):
        return polygons_to_mask(seg, h, w)
    return rle_decode(seg, h, w)


# ---------------------------------------------------------------------------- dataset
class CocoDetection:
    def __init__(self, img_dir: str, ann_file: str, train: bool = True, with_masks: bool = True,
                 remove_empty: bool = True):
        with open(ann_file) as f:
            d = json.load(f)
        self.img_dir, self.train, self.with_masks = img_dir, train, with_masks
        self.cat_ids = sorted(c["id"] for c in d.get("categories", []))
        self.cat_to_label = {c: i + 1 for i, c in enumerate(self.cat_ids)}
        self.label_to_cat = {v: k for k, v in self.cat_to_label.items()}
        anns: Dict[int, List[dict]] = {}
        for a in d.get("annotations", []):
            anns.setdefault(a["image_id"], []).append(a)
        self.images = []
        for im in sorted(d["images"], key=lambda x: x["id"]):
            a = [x for x in anns.get(im["id"], []) if not (train and x.get("iscrowd", 0))]
            a = [x for x in a if x["bbox"][2] > 1 and x["bbox"][3] > 1]
            if train and remove_empty and not a:
                continue
            self.images.append((im, a))

    @property
    def num_classes(self) -> int:
        return len(self.cat_ids) + 1

    def __len__(self):
        return len(self.images)

    def ground_truth(self) -> Dict[int, Dict[str, np.ndarray]]:
        """Per-image boxes (xyxy) / labels / crowd flags in original coordinates (evaluation)."""
        out = {}
        for im, anns in self.images:
            b = np.array([[a["bbox"][0], a["bbox"][1], a["bbox"][0] + a["bbox"][2], a["bbox"][1] + a["bbox"][3]]
                          for a in anns], np.float32).reshape(-1, 4)
            out[im["id"]] = {"boxes": b, "labels": np.array([self.cat_to_label[a["category_id"]] for a in anns]),
                             "crowd": np.array([bool(a.get("iscrowd", 0)) for a in anns], bool)}
        return out


def _load_sample(task):
    """Worker: decode + resize (+ flip) one image and its instances."""
    from PIL import Image
    path, anns, min_size, max_size, flip, with_masks, cat_to_label = task
    with Image.open(path) as im:
        im = im.convert("RGB")
        w0, h0 = im.size
        s = min_size / min(h0, w0)
        if max(h0, w0) * s > max_size:
            s = max_size / max(h0, w0)
        w, h = int(round(w0 * s)), int(round(h0 * s))
        img = np.asarray(im.resize((w, h), Image.BILINEAR), np.float32)
    boxes = np.array([[a["bbox"][0], a["bbox"][1], a["bbox"][0] + a["bbox"][2], a["bbox"][1] + a["bbox"][3]]
                      for a in anns], np.float32).reshape(-1, 4) * s
    labels = np.array([cat_to_label[a["category_id"]] for a in anns], np.int64)
    masks = None
    if with_masks:
        masks = np.zeros((len(anns), h, w), np.uint8)
        for i, a in enumerate(anns):
            if a.get("segmentation"):
                m = segmentation_to_mask(a["segmentation"], h0, w0)
            else:                                      # no outline: the box is the mask
                x1, y1, x2, y2 = (boxes[i] / s).round().astype(int)
                m = np.zeros((h0, w0), np.uint8)
                m[y1:y2, x1:x2] = 1
            masks[i] = np.asarray(Image.fromarray(m * 255).resize((w, h), Image.NEAREST)) > 127
    if flip:
        img = img[:, ::-1]
        boxes = boxes.copy()
        boxes[:, [0, 2]] = w - boxes[:, [2, 0]]
        if masks is not None:
            masks = masks[:, :, ::-1]
    img = ((img - MEAN) / STD).transpose(2, 0, 1)
    return (np.ascontiguousarray(img), boxes, labels, None if masks is None else np.ascontiguousarray(masks),
            (h, w), s)


class CocoLoader:
    """Yields ``(images [N,3,H,W], targets, image_sizes, image_ids, scales)`` batches."""

    def __init__(self, ds: CocoDetection, batch_size: int, min_size: int = 800, max_size: int = 1333,
                 rank: int = 0, world: int = 1, seed: int = 0, workers: int = 8, prefetch: int = 2,
                 flip_prob: float = 0.5, device=None, size_divisibility: int = 32, drop_last: bool = True,
                 fixed_canvas: bool = False):
        self.ds, self.batch_size = ds, batch_size
        self.min_size, self.max_size = min_size, max_size
        self.rank, self.world, self.seed = rank, world, seed
        self.workers, self.prefetch = workers, max(1, prefetch)
        self.flip_prob = flip_prob if ds.train else 0.0
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.div, self.drop_last, self.epoch = size_divisibility, drop_last, 0
        # fixed_canvas: batches are grouped by orientation (reference AspectRatioGroupedBatchSampler)
        # and padded to one canvas per orientation, so the conv / GEMM shapes take two values
        # for the whole run -- MIOpen solver lookups and kernel selection happen once, not per batch
        self.fixed_canvas = fixed_canvas
        self._pool = None

    def __len__(self):
        if self.fixed_canvas:
            if self.drop_last:
                # every rank yields the minimum number of full same-orientation batches over
                # all ranks (each rank can compute every rank's split: same permutation seed)
                return min(sum(1 for g in self._groups(r) if len(g) == self.batch_size) for r in range(self.world))
            return len(self._groups(self.rank))
        per = len(self.ds) // self.world if self.drop_last else -(-len(self.ds) // self.world)
        return per // self.batch_size if self.drop_last else -(-per // self.batch_size)

    def set_epoch(self, epoch: int):
        self.epoch = epoch

    def _rank_indices(self, rank):
        n = len(self.ds)
        idx = np.random.default_rng(self.seed + self.epoch).permutation(n) if self.ds.train else np.arange(n)
        per = n // self.world if self.drop_last else -(-n // self.world)
        return idx[rank * per:(rank + 1) * per]

    def _groups(self, rank):
        """Same-orientation batches (landscape / portrait canvases) of ``rank``'s images."""
        idx = self._rank_indices(rank)
        land = [i for i in idx if self.ds.images[int(i)][0]["width"] >= self.ds.images[int(i)][0]["height"]]
        port = [i for i in idx if self.ds.images[int(i)][0]["width"] < self.ds.images[int(i)][0]["height"]]
        return [g[b:b + self.batch_size] for g in (land, port) for b in range(0, len(g), self.batch_size)]

    def _batches(self):
        idx = self._rank_indices(self.rank)
        rng = random.Random(self.seed * 7919 + self.epoch)
        if self.fixed_canvas:
            groups = self._groups(self.rank)
            if self.ds.train:
                rng.shuffle(groups)
            if self.drop_last:
                # full batches only, no image twice; ranks with more full batches drop the
                # surplus so every rank yields len(self) batches (collectives stay matched)
                groups = [g for g in groups if len(g) == self.batch_size][:len(self)]
        else:
            groups = [idx[b * self.batch_size:(b + 1) * self.batch_size] for b in range(len(self))]
        for sel in groups:
            if len(sel) == 0:
                break
            tasks = []
            for i in sel:
                im, anns = self.ds.images[int(i)]
                tasks.append((os.path.join(self.ds.img_dir, im["file_name"]), anns, self.min_size, self.max_size,
                              rng.random() < self.flip_prob, self.ds.with_masks, self.ds.cat_to_label))
            yield tasks, [self.ds.images[int(i)][0]["id"] for i in sel]

    def _collate(self, samples, ids):
        H = max(s[4][0] for s in samples)
        W = max(s[4][1] for s in samples)
        if self.fixed_canvas:
            lo, hi = -(-self.min_size // self.div) * self.div, -(-self.max_size // self.div) * self.div
            H, W = (lo, hi) if W >= H and H <= lo else (hi, lo) if H > W and W <= lo else (hi, hi)
        H, W = -(-H // self.div) * self.div, -(-W // self.div) * self.div
        imgs = torch.zeros(len(samples), 3, H, W)
        targets, sizes, scales = [], [], []
        for i, (img, boxes, labels, masks, (h, w), s) in enumerate(samples):
            imgs[i, :, :h, :w] = torch.from_numpy(img)
            t = {"boxes": torch.from_numpy(boxes), "labels": torch.from_numpy(labels)}
            if masks is not None:
                m = torch.zeros(masks.shape[0], H, W, dtype=torch.uint8)
                m[:, :h, :w] = torch.from_numpy(masks)
                t["masks"] = m
            targets.append(t)
            sizes.append((h, w))
            scales.append(s)
        if self.device.type == "cuda":
            imgs = imgs.pin_memory().to(self.device, non_blocking=True)
            targets = [{k: v.pin_memory().to(self.device, non_blocking=True) for k, v in t.items()} for t in targets]
        return imgs, targets, sizes, ids, scales

    def __iter__(self) -> Iterator:
        batches = list(self._batches())
        if self.workers <= 0:
            for tasks, ids in batches:
                yield self._collate([_load_sample(t) for t in tasks], ids)
            return
        if self._pool is None:
            self._pool = mp.get_context("forkserver").Pool(self.workers)
        pending = []
        it = iter(batches)
        for tasks, ids in it:
            pending.append(([self._pool.apply_async(_load_sample, (t,)) for t in tasks], ids))
            if len(pending) >= self.prefetch:
                break
        while pending:
            futs, ids = pending.pop(0)
            nxt = next(it, None)
            if nxt is not None:
                pending.append(([self._pool.apply_async(_load_sample, (t,)) for t in nxt[0]], nxt[1]))
            yield self._collate([f.get() for f in futs], ids)

    def close(self):
        if self._pool is not None:
            self._pool.terminate()
            self._pool.join()
            self._pool = None


# ---------------------------------------------------------------------------- evaluation
def _iou_xyxy(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    lt = np.maximum(a[:, None, :2], b[None, :, :2])
    rb = np.minimum(a[:, None, 2:], b[None, :, 2:])
    wh = np.clip(rb - lt, 0, None)
    inter = wh[..., 0] * wh[..., 1]
    area = lambda x: (x[:, 2] - x[:, 0]) * (x[:, 3] - x[:, 1])  # noqa: E731
    return inter / np.maximum(area(a)[:, None] + area(b)[None, :] - inter, 1e-12)


def evaluate_bbox(dets: Dict[int, Dict[str, np.ndarray]], gts: Dict[int, Dict[str, np.ndarray]],
                  max_dets: int = 100) -> Dict[str, float]:
    """COCO-style box AP.  dets / gts: image id -> {"boxes" [n,4] xyxy, "labels" [n],
    "scores" [n] (dets only), "crowd" [n] bool (gts, optional)}.  Greedy matching by score
    per image and class; detections matched to crowd regions are ignored.  Returns AP
    (IoU .50:.95), AP50 and AP75."""
    thrs = np.linspace(0.5, 0.95, 10)
    rec_pts = np.linspace(0, 1, 101)
    labels = sorted({int(v) for g in gts.values() for v in g["labels"]})
    aps = np.full((len(thrs), len(labels)), np.nan)
    empty = {"boxes": np.zeros((0, 4)), "labels": np.zeros(0), "scores": np.zeros(0)}
    for li, lab in enumerate(labels):
        scores, tp, npos = [], [[] for _ in thrs], 0
        for img in sorted(set(gts) | set(dets)):
            g = gts.get(img, empty)
            gm = np.asarray(g["labels"]) == lab
            gb = np.asarray(g["boxes"], np.float64).reshape(-1, 4)[gm]
            crowd = np.asarray(g.get("crowd", np.zeros(len(g["labels"]), bool)), bool)[gm]
            npos += int((~crowd).sum())
            d = dets.get(img, empty)
            dm = np.asarray(d["labels"]) == lab
            db = np.asarray(d["boxes"], np.float64).reshape(-1, 4)[dm]
            ds = np.asarray(d["scores"], np.float64)[dm]
            order = np.argsort(-ds, kind="stable")[:max_dets]
            db, ds = db[order], ds[order]
            iou = _iou_xyxy(db, gb) if len(gb) and len(db) else np.zeros((len(db), len(gb)))
            for ti, t in enumerate(thrs):
                used = np.zeros(len(gb), bool)
                for k in range(len(db)):
                    bj, best = -1, t
                    for j in range(len(gb)):            # real objects first, then crowd regions
                        if not crowd[j] and not used[j] and iou[k, j] >= best:
                            bj, best = j, iou[k, j]
                    if bj < 0:
                        for j in range(len(gb)):
                            if crowd[j] and iou[k, j] >= t:
                                bj = j
                                break
                    if bj >= 0 and crowd[bj]:
                        tp[ti].append(-1)
                    elif bj >= 0:
                        used[bj] = True
                        tp[ti].append(1)
                    else:
                        tp[ti].append(0)
            scores += list(ds)
        if npos == 0:
            continue
        order = np.argsort(-np.array(scores), kind="stable")
        for ti in range(len(thrs)):
            t = np.array(tp[ti], np.int64)[order] if scores else np.zeros(0, np.int64)
            t = t[t >= 0]
            ctp, cfp = np.cumsum(t == 1), np.cumsum(t == 0)
            rec = ctp / npos
            prec = ctp / np.maximum(ctp + cfp, 1e-12)
            for i in range(len(prec) - 2, -1, -1):
                prec[i] = max(prec[i], prec[i + 1])
            inds = np.searchsorted(rec, rec_pts, side="left")
            q = np.array([prec[i] if i < len(prec) else 0.0 for i in inds])
            aps[ti, li] = q.mean()
    m = lambda a: float(np.nanmean(a)) if np.isfinite(a).any() else 0.0  # noqa: E731
    return {"AP": m(aps), "AP50": m(aps[0]), "AP75": m(aps[5])}
