"""Box utilities shared by the detection models: IoU, box coding, anchor matching, sampling,
anchor generation.

These are what maskrcnn_benchmark's ``structures/boxlist_ops.py``, ``modeling/box_coder.py``,
``modeling/matcher.py``, ``modeling/balanced_positive_negative_sampler.py`` and
``modeling/rpn/anchor_generator.py`` provide to the reference's Mask R-CNN
(applications/ai/quickstart/models/object_detection/pytorch/maskrcnn/maskrcnn-benchmark).
Here they are plain batched tensor code: every op runs on the device the boxes live on, with
no per-box Python loops, so an MI355X step issues a handful of large elementwise / reduction
kernels instead of thousands of tiny ones.  Boxes are ``(x1, y1, x2, y2)`` in pixels with the
continuous (no +1) area convention.
"""
from __future__ import annotations

import math
from typing import List, Sequence, Tuple

import torch

BBOX_XFORM_CLIP = math.log(1000.0 / 16)


def box_area(b: torch.Tensor) -> torch.Tensor:
    return (b[:, 2] - b[:, 0]).clamp(min=0) * (b[:, 3] - b[:, 1]).clamp(min=0)


def box_iou(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """[Na, Nb] IoU matrix."""
    area_a, area_b = box_area(a), box_area(b)
    lt = torch.max(a[:, None, :2], b[None, :, :2])
    rb = torch.min(a[:, None, 2:], b[None, :, 2:])
    wh = (rb - lt).clamp(min=0)
    inter = wh[..., 0] * wh[..., 1]
    return inter / (area_a[:, None] + area_b[None, :] - inter).clamp(min=1e-9)


def clip_boxes(b: torch.Tensor, size: Tuple[int, int]) -> torch.Tensor:
    h, w = size
    return torch.stack([b[:, 0].clamp(0, w), b[:, 1].clamp(0, h), b[:, 2].clamp(0, w), b[:, 3].clamp(0, h)], 1)


def remove_small(b: torch.Tensor, min_size: float) -> torch.Tensor:
    ws, hs = b[:, 2] - b[:, 0], b[:, 3] - b[:, 1]
    return torch.nonzero((ws >= min_size) & (hs >= min_size)).squeeze(1)


def cxcywh_to_xyxy(b):
    cx, cy, w, h = b.unbind(-1)
    return torch.stack([cx - w / 2, cy - h / 2, cx + w / 2, cy + h / 2], -1)


def xyxy_to_cxcywh(b):
    x1, y1, x2, y2 = b.unbind(-1)
    return torch.stack([(x1 + x2) / 2, (y1 + y2) / 2, x2 - x1, y2 - y1], -1)


class BoxCoder:
    """(dx, dy, dw, dh) regression targets scaled by ``weights``."""

    def __init__(self, weights=(1.0, 1.0, 1.0, 1.0), clip=BBOX_XFORM_CLIP):
        self.weights = weights
        self.clip = clip

    def encode(self, gt: torch.Tensor, ref: torch.Tensor) -> torch.Tensor:
        wx, wy, ww, wh = self.weights
        rw, rh = ref[:, 2] - ref[:, 0], ref[:, 3] - ref[:, 1]
        rx, ry = ref[:, 0] + 0.5 * rw, ref[:, 1] + 0.5 * rh
        gw, gh = gt[:, 2] - gt[:, 0], gt[:, 3] - gt[:, 1]
        gx, gy = gt[:, 0] + 0.5 * gw, gt[:, 1] + 0.5 * gh
        return torch.stack([wx * (gx - rx) / rw, wy * (gy - ry) / rh,
                            ww * torch.log(gw / rw), wh * torch.log(gh / rh)], 1)

    def decode(self, codes: torch.Tensor, ref: torch.Tensor) -> torch.Tensor:
        """codes [K, 4*C] (class-specific) or [K, 4]; ref [K, 4] -> boxes of codes' shape."""
        ref = ref.to(codes.dtype)
        wx, wy, ww, wh = self.weights
        rw, rh = ref[:, 2] - ref[:, 0], ref[:, 3] - ref[:, 1]
        rx, ry = ref[:, 0] + 0.5 * rw, ref[:, 1] + 0.5 * rh
        c = codes.reshape(codes.shape[0], codes.shape[-1] // 4, 4)
        dx, dy = c[..., 0] / wx, c[..., 1] / wy
        dw, dh = (c[..., 2] / ww).clamp(max=self.clip), (c[..., 3] / wh).clamp(max=self.clip)
        px, py = dx * rw[:, None] + rx[:, None], dy * rh[:, None] + ry[:, None]
        pw, ph = torch.exp(dw) * rw[:, None], torch.exp(dh) * rh[:, None]
        out = torch.stack([px - 0.5 * pw, py - 0.5 * ph, px + 0.5 * pw, py + 0.5 * ph], -1)
        return out.reshape(codes.shape)


class Matcher:
    """Assign each anchor / proposal (column) to its best ground-truth box (row).

    Result per column: gt index, ``BELOW_LOW`` (-1, background) or ``BETWEEN`` (-2, ignored).
    ``allow_low_quality`` also keeps, for every gt, the columns with its highest IoU."""

    BELOW_LOW = -1
    BETWEEN = -2

    def __init__(self, high: float, low: float, allow_low_quality: bool = False):
        assert low <= high
        self.high, self.low, self.allow_low_quality = high, low, allow_low_quality

    def __call__(self, iou: torch.Tensor) -> torch.Tensor:
        if iou.numel() == 0:
            return torch.full((iou.shape[1],), self.BELOW_LOW, dtype=torch.long, device=iou.device)
        # elementwise selects only: boolean-mask assignment would go through nonzero() and
        # stall the host on the GPU once per call
        vals, idx = iou.max(0)
        out = torch.where(vals < self.low, torch.full_like(idx, self.BELOW_LOW),
                          torch.where(vals < self.high, torch.full_like(idx, self.BETWEEN), idx))
        if self.allow_low_quality:
            best = iou.max(1, keepdim=True).values
            out = torch.where(((iou == best) & (best > 0)).any(0), idx, out)
        return out


def sample_pos_neg(labels: torch.Tensor, batch_size: int, positive_fraction: float,
                   generator: torch.Generator = None):
    """Balanced sampling of one image's matched labels (>=1 positive, 0 negative, -1 ignore):
    returns boolean masks (pos, neg)."""
    pos = torch.nonzero(labels >= 1).squeeze(1)
    neg = torch.nonzero(labels == 0).squeeze(1)
    n_pos = min(pos.numel(), int(batch_size * positive_fraction))
    n_neg = min(neg.numel(), batch_size - n_pos)
    dev = labels.device
    pp = pos[torch.randperm(pos.numel(), device=dev)[:n_pos]]
    nn_ = neg[torch.randperm(neg.numel(), device=dev)[:n_neg]]
    pm = torch.zeros_like(labels, dtype=torch.bool)
    nm = torch.zeros_like(labels, dtype=torch.bool)
    pm[pp] = True
    nm[nn_] = True
    return pm, nm


def sample_pos_neg_batched(labels: torch.Tensor, batch_size: int, positive_fraction: float,
                           generator: torch.Generator = None):
    """``sample_pos_neg`` for a batch of images at once, with no host synchronisation:
    labels [N, A] -> boolean masks (pos, neg) [N, A].

    Each candidate draws a uniform key; the positives with the ``batch_size *
    positive_fraction`` smallest keys are taken (a uniform random subset), then the negatives
    with the smallest keys fill the rest of the row's ``batch_size``.  Counts stay on the
    device (top-k + comparisons), so the caller never waits for the GPU."""
    N, A = labels.shape
    dev = labels.device
    P = int(batch_size * positive_fraction)
    r = torch.rand(labels.shape, device=dev, generator=generator)
    never = torch.full_like(r, 2.0)
    pm = torch.zeros_like(labels, dtype=torch.bool)
    nm = torch.zeros_like(labels, dtype=torch.bool)
    n_pos = torch.zeros(N, 1, dtype=torch.long, device=dev)
    if P > 0:
        pk, pi = torch.where(labels >= 1, r, never).topk(min(P, A), dim=1, largest=False)
        pos_ok = pk < 2
        pm = pm.scatter(1, pi, pos_ok)
        n_pos = pos_ok.sum(1, keepdim=True)
    kn = min(batch_size, A)
    nk, ni = torch.where(labels == 0, r, never).topk(kn, dim=1, largest=False)
    neg_ok = (nk < 2) & (torch.arange(kn, device=dev)[None, :] < batch_size - n_pos)
    nm = nm.scatter(1, ni, neg_ok)
    return pm, nm


def smooth_l1(x: torch.Tensor, y: torch.Tensor, beta: float = 1.0 / 9, reduction: str = "sum") -> torch.Tensor:
    d = (x - y).abs()
    loss = torch.where(d < beta, 0.5 * d * d / beta, d - 0.5 * beta) if beta > 0 else d
    return loss.sum() if reduction == "sum" else loss.mean() if reduction == "mean" else loss


class AnchorGenerator:
    """Anchors for every feature level: ``sizes[l]`` x ``aspect_ratios`` centred on a stride
    grid.  Cell anchors are computed once; grids are cached per (level, H, W, device)."""

    def __init__(self, sizes: Sequence[Sequence[float]], aspect_ratios: Sequence[float] = (0.5, 1.0, 2.0),
                 strides: Sequence[int] = (4, 8, 16, 32, 64), offset: float = 0.0):
        self.strides = list(strides)
        self.offset = offset
        self.cell = []
        for sz in sizes:
            cells = []
            for ar in aspect_ratios:          # ratio = h / w
                for s in sz:
                    w = s / math.sqrt(ar)
                    h = s * math.sqrt(ar)
                    cells.append([-w / 2, -h / 2, w / 2, h / 2])
            self.cell.append(torch.tensor(cells, dtype=torch.float32))
        self._cache = {}

    def num_anchors_per_location(self) -> List[int]:
        return [c.shape[0] for c in self.cell]

    def grid_anchors(self, level: int, h: int, w: int, device) -> torch.Tensor:
        key = (level, h, w, str(device))
        a = self._cache.get(key)
        if a is None:
            st = self.strides[level]
            ys = (torch.arange(h, device=device, dtype=torch.float32) + self.offset) * st
            xs = (torch.arange(w, device=device, dtype=torch.float32) + self.offset) * st
            yy, xx = torch.meshgrid(ys, xs, indexing="ij")
            shifts = torch.stack([xx, yy, xx, yy], -1).reshape(-1, 1, 4)
            a = (shifts + self.cell[level].to(device)[None]).reshape(-1, 4)   # (H, W, A) order
            self._cache[key] = a
        return a

    def __call__(self, feats: List[torch.Tensor]) -> List[torch.Tensor]:
        return [self.grid_anchors(i, f.shape[-2], f.shape[-1], f.device) for i, f in enumerate(feats)]


def permute_flatten(x: torch.Tensor, n_per_anchor: int) -> torch.Tensor:
    """[N, A*K, H, W] head output -> [N, H*W*A, K] (matches AnchorGenerator order)."""
    N, AK, H, W = x.shape
    A = AK // n_per_anchor
    return x.reshape(N, A, n_per_anchor, H, W).permute(0, 3, 4, 1, 2).reshape(N, -1, n_per_anchor)
