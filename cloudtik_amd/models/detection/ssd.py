"""Single-Shot Detectors: SSD-ResNet34 (training) and SSD-MobileNet (inference).

Reference workloads: the quickstart SSD-ResNet34 training
(models/object_detection/pytorch/ssd-resnet34/training/cpu: the MLPerf SSD with a
ResNet-34 trunk whose conv4 stage keeps stride 1, six feature maps 38/19/10/5/3/1, 8732
default boxes, smooth-L1 + hard-negative-mined cross entropy, hand-rolled bucketed DDP
``distributed.py:13-48``) and SSD-MobileNet inference.  Data parallelism is the framework's
``GradBucketer`` (one flat gradient buffer, bucketed RCCL all-reduce overlapped with
backward), which is the same flatten -> all-reduce -> scale pattern without the copies.

Default boxes are ``(cx, cy, w, h)`` relative to the image; box regression uses the SSD
variances (0.1 centre, 0.2 size).  Post-processing decodes all boxes of a batch in one pass
and runs per-class HIP NMS (``ops.batched_nms``).
"""
from __future__ import annotations

import itertools
import math
from typing import Dict, List, Optional, Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F

from cloudtik_amd import ops
from cloudtik_amd.models import resnet as R
from cloudtik_amd.models.detection import box_ops as B


class DefaultBoxes:
    def __init__(self, fig_size: int, feat_size: Sequence[int], steps: Sequence[float], scales: Sequence[float],
                 aspect_ratios: Sequence[Sequence[float]], scale_xy: float = 0.1, scale_wh: float = 0.2,
                 reduce_first: bool = False):
        boxes = []
        self.num_per_loc = []
        for i, fs in enumerate(feat_size):
            sk1, sk2 = scales[i] / fig_size, scales[i + 1] / fig_size
            sizes = [(sk1, sk1)]
            if not (reduce_first and i == 0):     # TF SSD-MobileNet: 3 boxes on the first map
                sizes.append((math.sqrt(sk1 * sk2),) * 2)
            for a in aspect_ratios[i]:
                w, h = sk1 * math.sqrt(a), sk1 / math.sqrt(a)
                sizes += [(w, h), (h, w)]
            self.num_per_loc.append(len(sizes))
            fk = fig_size / steps[i]
            for (w, h), (y, x) in itertools.product(sizes, itertools.product(range(fs), repeat=2)):
                boxes.append(((x + 0.5) / fk, (y + 0.5) / fk, w, h))
        # order: level-major, then (size, y, x) -- matched by SSDHead.flatten
        self.cxcywh = torch.tensor(boxes, dtype=torch.float32).clamp(0, 1)
        self.xyxy = B.cxcywh_to_xyxy(self.cxcywh)
        self.scale_xy, self.scale_wh = scale_xy, scale_wh

    def __len__(self):
        return self.cxcywh.shape[0]

    def encode(self, boxes_xyxy: torch.Tensor, db: torch.Tensor) -> torch.Tensor:
        g = B.xyxy_to_cxcywh(boxes_xyxy)
        return torch.cat([(g[..., :2] - db[..., :2]) / (self.scale_xy * db[..., 2:]),
                          torch.log(g[..., 2:] / db[..., 2:]) / self.scale_wh], -1)

    def decode(self, loc: torch.Tensor, db: torch.Tensor) -> torch.Tensor:
        cxy = loc[..., :2] * self.scale_xy * db[..., 2:] + db[..., :2]
        wh = torch.exp(loc[..., 2:] * self.scale_wh) * db[..., 2:]
        return B.cxcywh_to_xyxy(torch.cat([cxy, wh], -1))


def ssd300_default_boxes() -> DefaultBoxes:
    return DefaultBoxes(300, [38, 19, 10, 5, 3, 1], [8, 16, 32, 64, 100, 300], [21, 45, 99, 153, 207, 261, 315],
                        [[2], [2, 3], [2, 3], [2, 3], [2], [2]])


def ssd_mobilenet_default_boxes() -> DefaultBoxes:
    return DefaultBoxes(300, [19, 10, 5, 3, 2, 1], [16, 32, 64, 100, 150, 300], [60, 105, 150, 195, 240, 285, 330],
                        [[2], [2, 3], [2, 3], [2, 3], [2, 3], [2, 3]], reduce_first=True)


def _cbr(cin, cout, k, stride=1, padding=None, groups=1, device=None, dtype=None, act=True):
    conv = nn.Conv2d(cin, cout, k, stride, k // 2 if padding is None else padding, groups=groups, bias=False,
                     device=device, dtype=torch.float32)
    nn.init.kaiming_normal_(conv.weight, mode="fan_out", nonlinearity="relu")
    return nn.Sequential(conv.to(dtype) if dtype is not None else conv,
                         R.BatchNormAct(cout, relu=act, device=device, dtype=dtype))


class ResNet34Trunk(nn.Module):
    """ResNet-34 conv1..conv4 with conv4's stride set to 1 (38x38x256 at 300x300 input)."""

    def __init__(self, device=None, dtype=None):
        super().__init__()
        r = R.ResNet((3, 4, 6, 3), 1, device=device, dtype=dtype, block=R.BasicBlock)
        first = r.layer3[0]
        first.conv1.stride = (1, 1)
        first.down.stride = (1, 1)
        self.conv1, self.bn1, self.layer1, self.layer2, self.layer3 = r.conv1, r.bn1, r.layer1, r.layer2, r.layer3
        self.out_channels = 256

    def forward(self, x):
        x = F.max_pool2d(self.bn1(self.conv1(x)), 3, 2, 1)
        return [self.layer3(self.layer2(self.layer1(x)))]


class MobileNetV1Trunk(nn.Module):
    """MobileNet-v1 (depthwise separable) returning conv11 (19x19x512) and conv13 (10x10x1024)."""

    CFG = [(64, 1), (128, 2), (128, 1), (256, 2), (256, 1), (512, 2), (512, 1), (512, 1), (512, 1), (512, 1),
           (512, 1), (1024, 2), (1024, 1)]

    def __init__(self, width: float = 1.0, device=None, dtype=None):
        super().__init__()
        kw = dict(device=device, dtype=dtype)
        c = int(32 * width)
        layers = [_cbr(3, c, 3, 2, **kw)]
        for cout, s in self.CFG:
            cout = int(cout * width)
            layers.append(nn.Sequential(_cbr(c, c, 3, s, groups=c, **kw), _cbr(c, cout, 1, **kw)))
            c = cout
        self.layers = nn.ModuleList(layers)
        self.tap = 11                     # layers[11] = conv11 (layers[0] is the stem)
        self.channels = (int(512 * width), c)

    def forward(self, x):
        out = []
        for i, l in enumerate(self.layers):
            x = l(x)
            if i == self.tap:
                out.append(x)
        out.append(x)
        return out


class SSD(nn.Module):
    def __init__(self, trunk: nn.Module, trunk_channels: Sequence[int], extra_channels: Sequence[int],
                 extra_mid: Sequence[int], extra_strides: Sequence[int], extra_pads: Sequence[int],
                 dboxes: DefaultBoxes, num_classes: int = 81, device=None, dtype=torch.bfloat16):
        super().__init__()
        kw = dict(device=device, dtype=dtype)
        self.trunk = trunk
        extras, cin = [], trunk_channels[-1]
        for cout, mid, s, p in zip(extra_channels, extra_mid, extra_strides, extra_pads):
            extras.append(nn.Sequential(_cbr(cin, mid, 1, **kw), _cbr(mid, cout, 3, s, p, **kw)))
            cin = cout
        self.extras = nn.ModuleList(extras)
        chans = list(trunk_channels) + list(extra_channels)
        self.loc, self.conf = nn.ModuleList(), nn.ModuleList()
        for c, nd in zip(chans, dboxes.num_per_loc):
            for lst, k in ((self.loc, 4), (self.conf, num_classes)):
                conv = nn.Conv2d(c, nd * k, 3, 1, 1, device=device, dtype=torch.float32)
                nn.init.xavier_uniform_(conv.weight)
                nn.init.zeros_(conv.bias)
                lst.append(conv.to(dtype) if dtype is not None else conv)
        self.dboxes = dboxes
        self.num_classes = num_classes
        self.dtype = dtype
        if device is not None and torch.device(device).type == "cuda":
            self.to(memory_format=torch.channels_last)

    def features(self, x):
        feats = self.trunk(x)
        y = feats[-1]
        for e in self.extras:
            y = e(y)
            feats.append(y)
        return feats

    @staticmethod
    def _flatten(t, k):
        # [N, nd*k, H, W] -> [N, nd*H*W, k] in (size, y, x) order (DefaultBoxes order)
        N, C, H, W = t.shape
        return t.reshape(N, C // k, k, H, W).permute(0, 1, 3, 4, 2).reshape(N, -1, k)

    def forward(self, images: torch.Tensor, targets: Optional[List[Dict[str, torch.Tensor]]] = None):
        x = images.to(self.dtype)
        if x.is_cuda:
            x = x.contiguous(memory_format=torch.channels_last)
        feats = self.features(x)
        loc = torch.cat([self._flatten(l(f), 4) for l, f in zip(self.loc, feats)], 1).float()
        conf = torch.cat([self._flatten(c(f), self.num_classes) for c, f in zip(self.conf, feats)], 1).float()
        if self.training:
            return self.loss(loc, conf, targets, images.shape[-1])
        return loc, conf

    def match(self, targets, size: int):
        """Per image: label [D] and encoded box target [D, 4] for every default box (IoU >= 0.5,
        plus the best default of every object)."""
        db = self.dboxes.xyxy.to(targets[0]["boxes"].device)
        labels, locs = [], []
        for t in targets:
            gt = t["boxes"].float() / size
            iou = B.box_iou(gt, db)
            best_iou, best_gt = iou.max(0)
            best_db = iou.argmax(1)
            best_iou[best_db] = 2.0
            best_gt[best_db] = torch.arange(gt.shape[0], device=gt.device)
            lab = t["labels"].long()[best_gt]
            lab[best_iou < 0.5] = 0
            labels.append(lab)
            locs.append(self.dboxes.encode(gt[best_gt], self.dboxes.cxcywh.to(gt.device)))
        return torch.stack(labels), torch.stack(locs)

    def loss(self, loc, conf, targets, size: int):
        labels, tloc = self.match(targets, size)
        pos = labels > 0
        n_pos = pos.sum(1)
        l_loc = (F.smooth_l1_loss(loc, tloc, reduction="none", beta=1.0).sum(-1) * pos).sum(1)
        ce = F.cross_entropy(conf.reshape(-1, self.num_classes), labels.reshape(-1), reduction="none").view_as(labels)
        # hard negative mining: the 3*n_pos highest-loss negatives of each image
        neg_ce = ce.detach().masked_fill(pos, 0.0)
        rank = neg_ce.argsort(1, descending=True).argsort(1)
        neg = rank < (3 * n_pos).clamp(max=labels.shape[1])[:, None]
        l_conf = (ce * (pos | neg)).sum(1)
        denom = n_pos.float().clamp(min=1e-6)
        total = ((l_loc + l_conf) * (n_pos > 0).float() / denom).mean()
        return {"loss": total}

    @torch.no_grad()
    def postprocess(self, loc, conf, size: int, score_thresh: float = 0.05, nms_thresh: float = 0.5,
                    max_det: int = 200):
        db = self.dboxes.cxcywh.to(loc.device)
        boxes = self.dboxes.decode(loc, db).clamp(0, 1) * size          # [N, D, 4]
        probs = F.softmax(conf, -1)[..., 1:]                             # [N, D, K-1]
        out = []
        for n in range(loc.shape[0]):
            sc = probs[n].reshape(-1)
            keep = torch.nonzero(sc > score_thresh).squeeze(1)
            d, lab = keep // (self.num_classes - 1), keep % (self.num_classes - 1) + 1
            b, s = boxes[n][d], sc[keep]
            k = ops.batched_nms(b, s, lab, nms_thresh)[:max_det]
            out.append({"boxes": b[k], "scores": s[k], "labels": lab[k]})
        return out


def ssd300_resnet34(num_classes: int = 81, device=None, dtype=torch.bfloat16) -> SSD:
    return SSD(ResNet34Trunk(device, dtype), [256], [512, 512, 256, 256, 256], [256, 256, 128, 128, 128],
               [2, 2, 2, 1, 1], [1, 1, 1, 0, 0], ssd300_default_boxes(), num_classes, device, dtype)


def ssd300_mobilenet_v1(num_classes: int = 91, device=None, dtype=torch.bfloat16) -> SSD:
    trunk = MobileNetV1Trunk(device=device, dtype=dtype)
    return SSD(trunk, list(trunk.channels), [512, 256, 256, 128], [256, 128, 128, 64], [2, 2, 2, 2], [1, 1, 1, 1],
               ssd_mobilenet_default_boxes(), num_classes, device, dtype)
