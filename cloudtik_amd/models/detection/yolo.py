"""YOLOv4 (CSPDarknet53 + SPP + PANet, three YOLO heads) for inference.

Reference workload: the quickstart YOLOv4 inference (applications/ai/quickstart, GPU/XPU
inference scripts).  Random-init weights (no checkpoints here); the model
has the published YOLOv4 topology (608x608 input, strides 8/16/32, 3 anchors per scale).

Decoding is vectorised over all three scales at once and the final per-class suppression
is the HIP bitmask NMS (``ops.batched_nms``).
"""
from __future__ import annotations

from typing import List, Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F

from cloudtik_amd import ops
from cloudtik_amd.models import resnet as R
from cloudtik_amd.models.detection import box_ops as B

YOLOV4_ANCHORS = [[(12, 16), (19, 36), (40, 28)], [(36, 75), (76, 55), (72, 146)],
                  [(142, 110), (192, 243), (459, 401)]]


class ConvBNAct(nn.Module):
    def __init__(self, cin, cout, k, stride=1, act="mish", device=None, dtype=None):
        super().__init__()
        conv = nn.Conv2d(cin, cout, k, stride, k // 2, bias=False, device=device, dtype=torch.float32)
        nn.init.kaiming_normal_(conv.weight, mode="fan_out", nonlinearity="leaky_relu", a=0.1)
        self.conv = conv.to(dtype) if dtype is not None else conv
        self.bn = R.BatchNormAct(cout, relu=False, device=device, dtype=dtype)
        self.act = act

    def forward(self, x):
        x = self.bn(self.conv(x))
        return F.mish(x) if self.act == "mish" else F.leaky_relu(x, 0.1)


class ResUnit(nn.Module):
    def __init__(self, c, hidden, device=None, dtype=None):
        super().__init__()
        self.a = ConvBNAct(c, hidden, 1, device=device, dtype=dtype)
        self.b = ConvBNAct(hidden, c, 3, device=device, dtype=dtype)

    def forward(self, x):
        return x + self.b(self.a(x))


class CSPStage(nn.Module):
    def __init__(self, cin, cout, n, first=False, device=None, dtype=None):
        super().__init__()
        kw = dict(device=device, dtype=dtype)
        hid = cout if first else cout // 2
        self.down = ConvBNAct(cin, cout, 3, 2, **kw)
        self.split1 = ConvBNAct(cout, hid, 1, **kw)
        self.split2 = ConvBNAct(cout, hid, 1, **kw)
        self.blocks = nn.Sequential(*[ResUnit(hid, cout // 2 if first else hid, **kw) for _ in range(n)])
        self.post = ConvBNAct(hid, hid, 1, **kw)
        self.fuse = ConvBNAct(2 * hid, cout, 1, **kw)

    def forward(self, x):
        x = self.down(x)
        return self.fuse(torch.cat([self.post(self.blocks(self.split2(x))), self.split1(x)], 1))


class CSPDarknet53(nn.Module):
    def __init__(self, width: float = 1.0, depth=(1, 2, 8, 8, 4), device=None, dtype=None):
        super().__init__()
        ch = [int(c * width) for c in (32, 64, 128, 256, 512, 1024)]
        self.stem = ConvBNAct(3, ch[0], 3, device=device, dtype=dtype)
        self.stages = nn.ModuleList([CSPStage(ch[i], ch[i + 1], depth[i], first=(i == 0), device=device, dtype=dtype)
                                     for i in range(5)])
        self.channels = ch[3:]

    def forward(self, x):
        x = self.stem(x)
        outs = []
        for i, s in enumerate(self.stages):
            x = s(x)
            if i >= 2:
                outs.append(x)
        return outs                       # strides 8, 16, 32


def _conv_set(cin, cout, n, device, dtype):
    """Alternating 1x1 (cout) / 3x3 (2*cout) leaky convs, n layers, ending on 1x1."""
    layers, c = [], cin
    for i in range(n):
        k, co = (1, cout) if i % 2 == 0 else (3, 2 * cout)
        layers.append(ConvBNAct(c, co, k, act="leaky", device=device, dtype=dtype))
        c = co
    return nn.Sequential(*layers)


class YOLOv4(nn.Module):
    def __init__(self, num_classes: int = 80, width: float = 1.0, depth=(1, 2, 8, 8, 4),
                 anchors: Sequence = YOLOV4_ANCHORS, device=None, dtype=torch.bfloat16):
        super().__init__()
        kw = dict(device=device, dtype=dtype)
        self.backbone = CSPDarknet53(width, depth, **kw)
        c3, c4, c5 = self.backbone.channels
        h3, h4, h5 = c3 // 2, c4 // 2, c5 // 2
        self.pre_spp = _conv_set(c5, h5, 3, device, dtype)
        self.post_spp = _conv_set(4 * h5, h5, 3, device, dtype)
        self.lat5 = ConvBNAct(h5, h4, 1, act="leaky", **kw)
        self.lat4 = ConvBNAct(c4, h4, 1, act="leaky", **kw)
        self.td4 = _conv_set(2 * h4, h4, 5, device, dtype)
        self.lat4b = ConvBNAct(h4, h3, 1, act="leaky", **kw)
        self.lat3 = ConvBNAct(c3, h3, 1, act="leaky", **kw)
        self.td3 = _conv_set(2 * h3, h3, 5, device, dtype)
        self.down3 = ConvBNAct(h3, h4, 3, 2, act="leaky", **kw)
        self.bu4 = _conv_set(2 * h4, h4, 5, device, dtype)
        self.down4 = ConvBNAct(h4, h5, 3, 2, act="leaky", **kw)
        self.bu5 = _conv_set(2 * h5, h5, 5, device, dtype)
        self.num_classes = num_classes
        self.anchors = [torch.tensor(a, dtype=torch.float32) for a in anchors]
        self.strides = (8, 16, 32)
        no = 3 * (5 + num_classes)
        self.heads = nn.ModuleList()
        for c in (h3, h4, h5):
            out = nn.Conv2d(2 * c, no, 1, device=device, dtype=torch.float32)
            nn.init.normal_(out.weight, std=0.01)
            nn.init.constant_(out.bias, 0.0)
            self.heads.append(nn.Sequential(ConvBNAct(c, 2 * c, 3, act="leaky", **kw),
                                            out.to(dtype) if dtype is not None else out))
        self.dtype = dtype
        if device is not None and torch.device(device).type == "cuda":
            self.to(memory_format=torch.channels_last)

    def forward(self, images: torch.Tensor) -> List[torch.Tensor]:
        x = images.to(self.dtype)
        if x.is_cuda:
            x = x.contiguous(memory_format=torch.channels_last)
        c3, c4, c5 = self.backbone(x)
        p5 = self.pre_spp(c5)
        p5 = self.post_spp(torch.cat([F.max_pool2d(p5, k, 1, k // 2) for k in (13, 9, 5)] + [p5], 1))
        up = F.interpolate(self.lat5(p5), size=c4.shape[-2:], mode="nearest")
        p4 = self.td4(torch.cat([self.lat4(c4), up], 1))
        up = F.interpolate(self.lat4b(p4), size=c3.shape[-2:], mode="nearest")
        p3 = self.td3(torch.cat([self.lat3(c3), up], 1))
        n4 = self.bu4(torch.cat([self.down3(p3), p4], 1))
        n5 = self.bu5(torch.cat([self.down4(n4), p5], 1))
        return [h(f) for h, f in zip(self.heads, (p3, n4, n5))]

    @torch.no_grad()
    def decode(self, outs: List[torch.Tensor], scale_xy: float = 1.05) -> torch.Tensor:
        """-> [N, total_anchors, 5 + C] with boxes xyxy in pixels, objectness, class probs."""
        res = []
        for o, a, s in zip(outs, self.anchors, self.strides):
            N, _, H, W = o.shape
            p = o.float().reshape(N, 3, 5 + self.num_classes, H, W).permute(0, 1, 3, 4, 2)
            gy, gx = torch.meshgrid(torch.arange(H, device=o.device), torch.arange(W, device=o.device), indexing="ij")
            grid = torch.stack([gx, gy], -1).float()
            xy = (torch.sigmoid(p[..., :2]) * scale_xy - 0.5 * (scale_xy - 1) + grid) * s
            wh = torch.exp(p[..., 2:4].clamp(max=10)) * a.to(o.device).view(1, 3, 1, 1, 2)
            box = B.cxcywh_to_xyxy(torch.cat([xy, wh], -1))
            res.append(torch.cat([box, torch.sigmoid(p[..., 4:])], -1).reshape(N, -1, 5 + self.num_classes))
        return torch.cat(res, 1)

    @torch.no_grad()
    def postprocess(self, outs, size, conf_thresh: float = 0.25, nms_thresh: float = 0.45, max_det: int = 300,
                    max_candidates: int = 30000):
        det = self.decode(outs)
        results = []
        for d in det:
            scores = d[:, 4:5] * d[:, 5:]
            keep = torch.nonzero(scores > conf_thresh)
            i, c = keep[:, 0], keep[:, 1]
            s = scores[i, c]
            if s.numel() > max_candidates:      # bound the NMS bitmask (n^2 / 64 words)
                s, top = s.topk(max_candidates)
                i, c = i[top], c[top]
            b = B.clip_boxes(d[i, :4], size)
            k = ops.batched_nms(b, s, c, nms_thresh)[:max_det]
            results.append({"boxes": b[k], "scores": s[k], "labels": c[k]})
        return results


def yolov4(num_classes: int = 80, **kw) -> YOLOv4:
    return YOLOv4(num_classes, **kw)
