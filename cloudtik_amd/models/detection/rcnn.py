"""Faster R-CNN / Mask R-CNN with a ResNet(-X)-FPN backbone.

Reference workload: the quickstart Mask R-CNN training/inference
(applications/ai/quickstart/bin/maskrcnn/*, models/object_detection/pytorch/maskrcnn/
maskrcnn-benchmark: ``GeneralizedRCNN`` = backbone + RPN + ROI heads, R-50-FPN, custom C++
NMS / ROIAlign ops listed in csrc/vision.cpp:11-24) and the torchvision Faster/Mask R-CNN
inference scripts.  Here the C++ ops are the HIP kernels of
``cloudtik_amd.ops`` (bitmask NMS, ROIAlign fwd/bwd) and the backbone runs NHWC bf16.

    model = mask_rcnn_resnet50_fpn(num_classes=81, device="cuda")
    losses = model(images, targets)          # training: dict of 5 losses
    dets = model.eval()(images)              # inference: list of {boxes, scores, labels, masks}

``images`` is a normalised [N, 3, H, W] batch (padded to a multiple of 32); ``targets`` is a
list of ``{"boxes": [G, 4] xyxy, "labels": [G] in 1..num_classes-1, "masks": [G, H, W]}``.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn

from cloudtik_amd.models.detection import box_ops as B
from cloudtik_amd.models.detection.backbone import ResNetFPN
from cloudtik_amd.models.detection.roi_heads import RoIHeads
from cloudtik_amd.models.detection.rpn import RPN


class GeneralizedRCNN(nn.Module):
    def __init__(self, num_classes: int = 81, depth: int = 50, groups: int = 1, width_per_group: int = 64,
                 with_mask: bool = True, fpn_channels: int = 256, anchor_sizes=(32, 64, 128, 256, 512),
                 aspect_ratios=(0.5, 1.0, 2.0), rpn_pre_nms=(2000, 1000), rpn_post_nms=(2000, 1000),
                 box_batch_per_image: int = 512, representation: int = 1024, frozen_bn: bool = True,
                 device=None, dtype=torch.bfloat16):
        super().__init__()
        self.backbone = ResNetFPN(depth, groups, width_per_group, fpn_channels, (2, 3, 4, 5), "maxpool",
                                  frozen_bn=frozen_bn, device=device, dtype=dtype)
        anchors = B.AnchorGenerator([[s] for s in anchor_sizes], aspect_ratios, self.backbone.strides)
        self.rpn = RPN(fpn_channels, anchors, rpn_pre_nms, rpn_post_nms, device=device, dtype=dtype)
        self.roi_heads = RoIHeads(fpn_channels, self.backbone.strides, num_classes, with_mask,
                                  hidden=representation, batch_size_per_image=box_batch_per_image,
                                  device=device, dtype=dtype)
        self.dtype = dtype
        if device is not None and torch.device(device).type == "cuda":
            self.to(memory_format=torch.channels_last)     # every conv weight NHWC, like the activations

    def forward(self, images: torch.Tensor, targets: Optional[List[Dict[str, torch.Tensor]]] = None,
                image_sizes: Optional[List[Tuple[int, int]]] = None):
        if self.training and targets is None:
            raise ValueError("training needs targets")
        sizes = image_sizes or [tuple(images.shape[-2:])] * images.shape[0]
        x = images.to(self.dtype)
        if x.is_cuda:
            x = x.contiguous(memory_format=torch.channels_last)
        feats = self.backbone(x)
        proposals, rpn_losses = self.rpn(feats, sizes, targets)
        dets, roi_losses = self.roi_heads(feats, proposals, sizes, targets)
        if self.training:
            return {**rpn_losses, **roi_losses}
        return dets


def mask_rcnn_resnet50_fpn(num_classes: int = 81, **kw) -> GeneralizedRCNN:
    return GeneralizedRCNN(num_classes, 50, with_mask=True, **kw)


def faster_rcnn_resnet50_fpn(num_classes: int = 81, **kw) -> GeneralizedRCNN:
    return GeneralizedRCNN(num_classes, 50, with_mask=False, **kw)


def mask_rcnn_resnext101_32x8d_fpn(num_classes: int = 81, **kw) -> GeneralizedRCNN:
    return GeneralizedRCNN(num_classes, 101, 32, 8, with_mask=True, **kw)


def synthetic_detection_batch(n: int, size: int = 800, num_classes: int = 81, max_objects: int = 8,
                              with_masks: bool = True, device=None, generator: torch.Generator = None):
    """Random normalised images with random boxes / labels / box-shaped masks."""
    g = generator or torch.Generator().manual_seed(0)
    images = torch.randn(n, 3, size, size, generator=g)
    targets = []
    for _ in range(n):
        k = int(torch.randint(1, max_objects + 1, (1,), generator=g))
        xy = torch.rand(k, 2, generator=g) * size * 0.7
        wh = (torch.rand(k, 2, generator=g) * 0.25 + 0.05) * size
        boxes = torch.cat([xy, (xy + wh).clamp(max=size - 1)], 1)
        t = {"boxes": boxes, "labels": torch.randint(1, num_classes, (k,), generator=g)}
        if with_masks:
            m = torch.zeros(k, size, size, dtype=torch.uint8)
            for i, (x1, y1, x2, y2) in enumerate(boxes.round().long().tolist()):
                m[i, y1:y2, x1:x2] = 1
            t["masks"] = m
        targets.append(t)
    if device is not None:
        images = images.to(device)
        targets = [{k: v.to(device) for k, v in t.items()} for t in targets]
    return images, targets
