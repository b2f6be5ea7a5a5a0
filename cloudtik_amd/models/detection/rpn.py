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

    def forward(self, feats: List[torch.Tensor], image_sizes: List[Tuple[int, int]],
                targets: Optional[List[Dict[str, torch.Tensor]]] = None):
        logits, deltas = self.head(feats)
        anchors = self.anchor_generator(feats)
        N = feats[0].shape[0]
        obj = [B.permute_flatten(l, 1).squeeze(-1).float() for l in logits]          # [N, HWA] per level
        reg = [B.permute_flatten(d, 4).float() for d in deltas]                      # [N, HWA, 4]
        proposals = []
        with torch.no_grad():
            for n in range(N):
                dec = [self.coder.decode(r[n].detach(), a) for r, a in zip(reg, anchors)]
                proposals.append(self._select([o[n].detach() for o in obj], dec, image_sizes[n]))
        losses = {}
        if self.training and targets is not None:
            losses = self.loss(torch.cat(obj, 1), torch.cat(reg, 1), torch.cat(anchors), targets)
        return proposals, losses

    def loss(self, obj, reg, anchors, targets):
        labels, tgts = [], []
        for n, t in enumerate(targets):
            gt = t["boxes"].to(anchors)
            m = self.matcher(B.box_iou(gt, anchors))
            lab = (m >= 0).float()
            lab[m == B.Matcher.BETWEEN] = -1
            labels.append(lab)
            tgts.append(self.coder.encode(gt[m.clamp(min=0)], anchors) if gt.numel() else torch.zeros_like(anchors))
        pos, neg = [], []
        for lab in labels:
            p, q = B.sample_pos_neg(lab, self.batch_size_per_image, self.positive_fraction)
            pos.append(p)
            neg.append(q)
        pos, neg = torch.stack(pos), torch.stack(neg)
        labels, tgts = torch.stack(labels), torch.stack(tgts)
        sampled = pos | neg
        n_s = max(int(sampled.sum()), 1)
        box = B.smooth_l1(reg[pos], tgts[pos], beta=1.0 / 9) / n_s
        cls = F.binary_cross_entropy_with_logits(obj[sampled], labels[sampled])
        return {"loss_objectness": cls, "loss_rpn_box_reg": box}
