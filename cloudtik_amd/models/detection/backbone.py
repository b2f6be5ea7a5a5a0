"""Detection backbones: ResNet / ResNeXt bodies with a Feature Pyramid Network.

Reference: maskrcnn_benchmark ``modeling/backbone/{resnet,fpn,backbone}.py`` as used by the
quickstart Mask R-CNN (R-50-FPN) and the torchvision detection models the quickstart runs for
inference (Faster / Mask R-CNN, RetinaNet).

MI355X layout: the body is ``models.resnet.ResNet`` (NHWC bf16, fused BN+ReLU(+add) HIP
kernels, MIOpen convolutions).  Detection fine-tuning freezes the BatchNorm statistics
(``freeze_bn``), which turns every BN into a per-channel affine applied by the same kernel
family.  FPN lateral/output convolutions stay NHWC so no layout transposes appear between
the body, the pyramid and the heads.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from cloudtik_amd.models import resnet as R


def freeze_bn(module: nn.Module, freeze_params: bool = True) -> nn.Module:
    """BatchNormAct layers use their running statistics in training too (FrozenBatchNorm)."""
    for m in module.modules():
        if isinstance(m, R.BatchNormAct):
            m.frozen = True
            if freeze_params:
                m.weight.requires_grad_(False)
                m.bias.requires_grad_(False)
    return module


def _conv(cin, cout, k, stride=1, device=None, dtype=None, bias=True, init="kaiming_uniform"):
    c = nn.Conv2d(cin, cout, k, stride, k // 2, bias=bias, device=device, dtype=torch.float32)
    if init == "kaiming_uniform":
        nn.init.kaiming_uniform_(c.weight, a=1)
    else:
        nn.init.normal_(c.weight, std=0.01)
    if bias:
        nn.init.zeros_(c.bias)
    return c.to(dtype) if dtype is not None else c


class FPN(nn.Module):
    """Top-down pyramid: P_l = conv3x3(lateral(C_l) + upsample(P_{l+1})).

    ``extra``: ``"maxpool"`` adds P6 = maxpool(P5) (Mask/Faster R-CNN); ``"p6p7"`` adds
    P6 = conv(C5 or P5, stride 2), P7 = conv(relu(P6), stride 2) (RetinaNet); ``None`` none."""

    def __init__(self, in_channels: List[int], out_channels: int = 256, extra: Optional[str] = "maxpool",
                 extra_from_p5: bool = True, device=None, dtype=None):
        super().__init__()
        kw = dict(device=device, dtype=dtype)
        self.lateral = nn.ModuleList([_conv(c, out_channels, 1, **kw) for c in in_channels])
        self.output = nn.ModuleList([_conv(out_channels, out_channels, 3, **kw) for _ in in_channels])
        self.extra = extra
        self.extra_from_p5 = extra_from_p5
        if extra == "p6p7":
            cin = out_channels if extra_from_p5 else in_channels[-1]
            self.p6 = _conv(cin, out_channels, 3, 2, **kw)
            self.p7 = _conv(out_channels, out_channels, 3, 2, **kw)

    def forward(self, feats: List[torch.Tensor]) -> List[torch.Tensor]:
        last = self.lateral[-1](feats[-1])
        outs = [self.output[-1](last)]
        for i in range(len(feats) - 2, -1, -1):
            lat = self.lateral[i](feats[i])
            last = lat + F.interpolate(last, size=lat.shape[-2:], mode="nearest")
            outs.insert(0, self.output[i](last))
        if self.extra == "maxpool":
            outs.append(F.max_pool2d(outs[-1], 1, 2, 0))
        elif self.extra == "p6p7":
            p6 = self.p6(outs[-1] if self.extra_from_p5 else feats[-1])
            outs += [p6, self.p7(F.relu(p6))]
        return outs


class ResNetFPN(nn.Module):
    """ResNet/ResNeXt body + FPN.  ``levels`` picks the body outputs fed to the FPN
    (2..5 = C2..C5 for R-CNN, 3..5 for RetinaNet)."""

    def __init__(self, depth: int = 50, groups: int = 1, width_per_group: int = 64, out_channels: int = 256,
                 levels=(2, 3, 4, 5), extra: Optional[str] = "maxpool", frozen_bn: bool = True,
                 freeze_stem: bool = True, device=None, dtype=torch.bfloat16):
        super().__init__()
        layers = {18: (2, 2, 2, 2), 34: (3, 4, 6, 3), 50: (3, 4, 6, 3), 101: (3, 4, 23, 3), 152: (3, 8, 36, 3)}[depth]
        block = R.BasicBlock if depth < 50 else R.Bottleneck
        self.body = R.ResNet(layers, num_classes=1, device=device, dtype=dtype, block=block, groups=groups,
                             width_per_group=width_per_group)
        del self.body.fc
        self.levels = tuple(levels)
        self.fpn = FPN([self.body.stage_channels[l - 2] for l in self.levels], out_channels, extra,
                       device=device, dtype=dtype)
        if device is not None and torch.device(device).type == "cuda":
            self.fpn.to(memory_format=torch.channels_last)
        self.out_channels = out_channels
        self.strides = [2 ** l for l in self.levels] + ([2 ** (self.levels[-1] + 1)] if extra == "maxpool" else
                                                        [2 ** (self.levels[-1] + 1), 2 ** (self.levels[-1] + 2)]
                                                        if extra == "p6p7" else [])
        if frozen_bn:
            freeze_bn(self.body)
        if freeze_stem:
            for p in list(self.body.conv1.parameters()) + list(self.body.bn1.parameters()):
                p.requires_grad_(False)

    def forward(self, x: torch.Tensor) -> List[torch.Tensor]:
        c = self.body.features(x)
        return self.fpn([c[l - 2] for l in self.levels])
