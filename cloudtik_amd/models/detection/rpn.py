"""Region Proposal Network (reference: maskrcnn_benchmark ``modeling/rpn/{rpn,inference,loss}.py``
of the quickstart Mask R-CNN).

Per image and pyramid level the top ``pre_nms_top_n`` objectness scores are decoded against
their anchors, clipped, filtered by size and suppressed with the HIP bitmask NMS
(``ops.batched_nms``, one launch for all levels of an image: the level id keeps levels apart);
the best ``post_nms_top_n`` survive.  Training samples 256 anchors per image (half positive)
from an IoU matcher (0.7 / 0.3, low-quality matches kept) for the objectness BCE and the
smooth-L1 box loss.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from cloudtik_amd import ops
from cloudtik_amd.models.detection import box_ops as B


class RPNHead(nn.Module):
    def __init__(self, channels: int, num_anchors: int, device=None, dtype=None):
        super().__init__()
        mk = lambda ci, co, k: nn.Conv2d(ci, co, k, 1, k // 2, device=device, dtype=torch.float32)  # noqa: E731
        self.conv, self.cls, self.bbox = mk(channels, channels, 3), mk(channels, num_anchors, 1), \
            mk(channels, num_anchors * 4, 1)
        for c in (self.conv, self.cls, self.bbox):
            nn.init.normal_(c.weight, std=0.01)
            nn.init.zeros_(c.bias)
        if dtype is not None:
            self.to(dtype)

    def forward(self, feats):
        logits, deltas = [], []
        for f in feats:
            t = F.relu(self.conv(f))
            logits.append(self.cls(t))
            deltas.append(self.bbox(t))
        return logits, deltas


class RPN(nn.Module):
    def __init__(self, channels: int, anchor_generator: B.AnchorGenerator, pre_nms_top_n=(2000, 1000),
                 post_nms_top_n=(2000, 1000), nms_thresh: float = 0.7, fg_iou: float = 0.7, bg_iou: float = 0.3,
                 batch_size_per_image: int = 256, positive_fraction: float = 0.5, min_size: float = 0.0,
                 device=None, dtype=None):
        super().__init__()
        self.anchor_generator = anchor_generator
        self.head = RPNHead(channels, anchor_generator.num_anchors_per_location()[0], device, dtype)
        self.pre_nms_top_n, self.post_nms_top_n = pre_nms_top_n, post_nms_top_n
        self.nms_thresh, self.min_size = nms_thresh, min_size
        self.matcher = B.Matcher(fg_iou, bg_iou, allow_low_quality=True)
        self.coder = B.BoxCoder((1.0, 1.0, 1.0, 1.0))
        self.batch_size_per_image, self.positive_fraction = batch_size_per_image, positive_fraction

    def _select(self, obj: List[torch.Tensor], boxes: List[torch.Tensor], size: Tuple[int, int]) -> torch.Tensor:
        """One image: obj[l] [HWA], boxes[l] [HWA, 4] (decoded) -> proposals [K, 4]."""
        pre = self.pre_nms_top_n[0 if self.training else 1]
        post = self.post_nms_top_n[0 if self.training else 1]
        sc, bx, lv = [], [], []
        for l, (o, b) in enumerate(zip(obj, boxes)):
            k = min(pre, o.numel())
            s, i = o.topk(k)
            sc.append(s)
            bx.append(b[i])
            lv.append(torch.full((k,), l, dtype=torch.long, device=o.device))
        s, b, lvl = torch.cat(sc), B.clip_boxes(torch.cat(bx), size), torch.cat(lv)
        keep = B.remove_small(b, self.min_size)
        s, b, lvl = s[keep], b[keep], lvl[keep]
        keep = ops.batched_nms(b, s, lvl, self.nms_thresh)[:post]
        return b[keep]

    def _select_batched(self, obj: List[torch.Tensor], reg: List[torch.Tensor], anchors: List[torch.Tensor],
                        image_sizes: List[Tuple[int, int]]) -> List[torch.Tensor]:
        """All images at once: obj[l] [N, HWA], reg[l] [N, HWA, 4] -> proposals per image.

        Same result as ``_select`` per image, but boxes are decoded only where the top-k
        selected them, and every (image, level) pair is one segment of a single segmented-NMS
        launch (static segment offsets: no host sync until the final per-image counts).
        Boxes failing the size filter are parked as empty boxes far outside the image, so
        they suppress nothing, and are dropped afterwards."""
        pre = self.pre_nms_top_n[0 if self.training else 1]
        post = self.post_nms_top_n[0 if self.training else 1]
        N = obj[0].shape[0]
        sc, bx, ks = [], [], []
        for o, r, a in zip(obj, reg, anchors):
            k = min(pre, o.shape[1])
            s, i = o.topk(k, dim=1)                                              # sorted, [N, k]
            codes = r.gather(1, i[..., None].expand(-1, -1, 4)).reshape(-1, 4)
            bx.append(self.coder.decode(codes, a[i.reshape(-1)]).reshape(N, k, 4))
            sc.append(s)
            ks.append(k)
        s, b = torch.cat(sc, 1), torch.cat(bx, 1)                              # [N, K], [N, K, 4]
        K = s.shape[1]
        hw = torch.tensor([[w, h, w, h] for h, w in image_sizes], dtype=b.dtype, device=b.device)
        b = torch.minimum(b.clamp(min=0), hw[:, None, :])
        ws, hs = b[..., 2] - b[..., 0], b[..., 3] - b[..., 1]
        valid = (ws >= self.min_size) & (hs >= self.min_size)
        b = torch.where(valid[..., None], b, torch.full_like(b, -1e4))
        off = [0]
        for _ in range(N):
            for k in ks:
                off.append(off[-1] + k)
        keep = ops.nms_segments(b.reshape(-1, 4), off, self.nms_thresh).reshape(N, K) & valid
        s = torch.where(keep, s, torch.full_like(s, float("-inf")))
        top, idx = s.topk(min(post, K), dim=1)
        counts = torch.isfinite(top).sum(1).tolist()
        sel = b.gather(1, idx[..., None].expand(-1, -1, 4))
        return [sel[n, :c] for n, c in enumerate(counts)]

    def forward(self, feats: List[torch.Tensor], image_sizes: List[Tuple[int, int]],
                targets: Optional[List[Dict[str, torch.Tensor]]] = None):
        logits, deltas = self.head(feats)
        anchors = self.anchor_generator(feats)
        N = feats[0].shape[0]
        obj = [B.permute_flatten(l, 1).squeeze(-1).float() for l in logits]          # [N, HWA] per level
        reg = [B.permute_flatten(d, 4).float() for d in deltas]                      # [N, HWA, 4]
        with torch.no_grad():
            proposals = self._select_batched([o.detach() for o in obj], [r.detach() for r in reg], anchors,
                                             image_sizes)
        losses = {}
        if self.training and targets is not None:
            losses = self.loss(torch.cat(obj, 1), torch.cat(reg, 1), torch.cat(anchors), targets)
        return proposals, losses

    def loss(self, obj, reg, anchors, targets):
        """Sync-free: matching by selects, batched top-k sampling, and losses as masked sums
        over all anchors (no boolean indexing, whose nonzero() would stall the host)."""
        labels, tgts = [], []
        for t in targets:
            gt = t["boxes"].to(anchors)
            if gt.numel():
                m = self.matcher(B.box_iou(gt, anchors))
                lab = torch.where(m >= 0, 1.0, torch.where(m == B.Matcher.BETWEEN, -1.0, 0.0))
                tgts.append(self.coder.encode(gt[m.clamp(min=0)], anchors))
            else:
                lab = torch.zeros(anchors.shape[0], device=anchors.device)
                tgts.append(torch.zeros_like(anchors))
            labels.append(lab)
        labels, tgts = torch.stack(labels), torch.stack(tgts)
        pos, neg = B.sample_pos_neg_batched(labels, self.batch_size_per_image, self.positive_fraction)
        sampled = (pos | neg).float()
        n_s = sampled.sum().clamp(min=1)
        # non-positive anchors regress onto themselves: zero loss and zero, finite gradient
        tgts = torch.where(pos[..., None], tgts, reg.detach())
        box = B.smooth_l1(reg, tgts, beta=1.0 / 9, reduction="none").sum() / n_s
        cls = (F.binary_cross_entropy_with_logits(obj, labels.clamp(min=0), reduction="none") * sampled).sum() / n_s
        return {"loss_objectness": cls, "loss_rpn_box_reg": box}
