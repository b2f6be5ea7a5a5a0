"""RetinaNet (ResNet-FPN P3-P7, focal loss).

Reference: the torchvision RetinaNet inference run by the quickstart scripts and
maskrcnn_benchmark's RetinaNet head whose loss is the ``SigmoidFocalLoss`` C++/CUDA op of
csrc/vision.cpp.  The classification loss here is the HIP focal-loss
kernel (``ops.sigmoid_focal_loss``: fused sigmoid / log / pow over [anchors, classes] in one
pass, fwd + bwd), normalised by the number of foreground anchors.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from cloudtik_amd import ops
from cloudtik_amd.models.detection import box_ops as B
from cloudtik_amd.models.detection.backbone import ResNetFPN


class RetinaHead(nn.Module):
    def __init__(self, channels: int, num_anchors: int, num_classes: int, convs: int = 4,
                 prior: float = 0.01, device=None, dtype=None):
        super().__init__()

        def tower():
            layers = []
            for _ in range(convs):
                c = nn.Conv2d(channels, channels, 3, 1, 1, device=device, dtype=torch.float32)
                nn.init.normal_(c.weight, std=0.01)
                nn.init.zeros_(c.bias)
                layers += [c, nn.ReLU(inplace=True)]
            return nn.Sequential(*layers)
        self.cls_tower, self.box_tower = tower(), tower()
        self.cls = nn.Conv2d(channels, num_anchors * num_classes, 3, 1, 1, device=device, dtype=torch.float32)
        self.box = nn.Conv2d(channels, num_anchors * 4, 3, 1, 1, device=device, dtype=torch.float32)
        for c in (self.cls, self.box):
            nn.init.normal_(c.weight, std=0.01)
        nn.init.constant_(self.cls.bias, -math.log((1 - prior) / prior))
        nn.init.zeros_(self.box.bias)
        self.num_classes = num_classes
        if dtype is not None:
            self.to(dtype)

    def forward(self, feats):
        return ([B.permute_flatten(self.cls(self.cls_tower(f)), self.num_classes) for f in feats],
                [B.permute_flatten(self.box(self.box_tower(f)), 4) for f in feats])


class RetinaNet(nn.Module):
    """``num_classes`` excludes background (focal loss: one sigmoid per foreground class);
    target and output labels are 1..num_classes."""

    def __init__(self, num_classes: int = 80, depth: int = 50, fpn_channels: int = 256,
                 anchor_sizes=(32, 64, 128, 256, 512), aspect_ratios=(0.5, 1.0, 2.0),
                 scales=(1.0, 2 ** (1 / 3), 2 ** (2 / 3)), fg_iou: float = 0.5, bg_iou: float = 0.4,
                 gamma: float = 2.0, alpha: float = 0.25, score_thresh: float = 0.05, topk_candidates: int = 1000,
                 nms_thresh: float = 0.5, detections_per_img: int = 100, frozen_bn: bool = True,
                 device=None, dtype=torch.bfloat16):
        super().__init__()
        self.backbone = ResNetFPN(depth, 1, 64, fpn_channels, (3, 4, 5), "p6p7", frozen_bn=frozen_bn,
                                  device=device, dtype=dtype)
        sizes = [[s * k for k in scales] for s in anchor_sizes]
        self.anchors = B.AnchorGenerator(sizes, aspect_ratios, self.backbone.strides)
        A = self.anchors.num_anchors_per_location()[0]
        self.head = RetinaHead(fpn_channels, A, num_classes, device=device, dtype=dtype)
        self.matcher = B.Matcher(fg_iou, bg_iou, allow_low_quality=True)
        self.coder = B.BoxCoder((1.0, 1.0, 1.0, 1.0))
        self.num_classes, self.gamma, self.alpha = num_classes, gamma, alpha
        self.score_thresh, self.topk, self.nms_thresh = score_thresh, topk_candidates, nms_thresh
        self.detections_per_img = detections_per_img
        self.dtype = dtype
        if device is not None and torch.device(device).type == "cuda":
            self.to(memory_format=torch.channels_last)     # every conv weight NHWC, like the activations

    def forward(self, images: torch.Tensor, targets: Optional[List[Dict[str, torch.Tensor]]] = None,
                image_sizes: Optional[List[Tuple[int, int]]] = None):
        sizes = image_sizes or [tuple(images.shape[-2:])] * images.shape[0]
        x = images.to(self.dtype)
        if x.is_cuda:
            x = x.contiguous(memory_format=torch.channels_last)
        feats = self.backbone(x)
        cls, reg = self.head(feats)
        anchors = self.anchors(feats)
        if self.training:
            return self.loss(torch.cat(cls, 1).float(), torch.cat(reg, 1).float(), torch.cat(anchors), targets)
        return self.postprocess([c.float() for c in cls], [r.float() for r in reg], anchors, sizes)

    def loss(self, cls, reg, anchors, targets):
        N = cls.shape[0]
        labels, tg = [], []
        for t in targets:
            gt = t["boxes"].to(anchors)
            m = self.matcher(B.box_iou(gt, anchors))
            lab = t["labels"].to(anchors.device)[m.clamp(min=0)].long()      # 1..K foreground
            lab[m == B.Matcher.BELOW_LOW] = 0
            lab[m == B.Matcher.BETWEEN] = -1
            labels.append(lab)
            tg.append(self.coder.encode(gt[m.clamp(min=0)], anchors))
        labels, tg = torch.stack(labels), torch.stack(tg)
        pos = labels > 0
        n_pos = max(float(pos.sum()), 1.0)
        # target labels are 1..K (0 = background), exactly the focal kernel's convention
        loss_cls = ops.sigmoid_focal_loss(cls.reshape(-1, self.num_classes), labels.reshape(-1), self.gamma,
                                          self.alpha, reduction="sum") / n_pos
        loss_box = F.l1_loss(reg[pos], tg[pos], reduction="sum") / n_pos
        return {"loss_classifier": loss_cls, "loss_box_reg": loss_box}

    @torch.no_grad()
    def postprocess(self, cls, reg, anchors, sizes):
        N = cls[0].shape[0]
        out = []
        for n in range(N):
            bs, ss, ls = [], [], []
            for c, r, a in zip(cls, reg, anchors):
                sc = torch.sigmoid(c[n]).reshape(-1)
                keep = torch.nonzero(sc > self.score_thresh).squeeze(1)
                sc = sc[keep]
                k = min(self.topk, sc.numel())
                sc, i = sc.topk(k)
                idx = keep[i]
                ai, lab = idx // self.num_classes, idx % self.num_classes + 1
                bs.append(B.clip_boxes(self.coder.decode(r[n][ai], a[ai]), sizes[n]))
                ss.append(sc)
                ls.append(lab)
            b, s, l = torch.cat(bs), torch.cat(ss), torch.cat(ls)
            keep = ops.batched_nms(b, s, l, self.nms_thresh)[:self.detections_per_img]
            out.append({"boxes": b[keep], "scores": s[keep], "labels": l[keep]})
        return out


def retinanet_resnet50_fpn(num_classes: int = 80, **kw) -> RetinaNet:
    return RetinaNet(num_classes, 50, **kw)
