"""ResNet-50 (v1.5) for the reference's image-recognition workloads.

Parity targets: torchvision ``resnet50`` trained with SGD + DDP, channels_last + bf16
(applications/ai/quickstart/models/image_recognition/pytorch/common/main.py:276-296,317,
585-586) and the synthetic benchmark
(examples/runtime/ai/basics/pytorch/imagenet-resnet50-synthetic-pytorch-distributed.py).

MI355X layout: NHWC (channels_last) bf16 activations and weights; convolutions go to
MIOpen; every BatchNorm is fused with its ReLU -- and, at the end of a bottleneck, with the
residual add -- in ONE HIP kernel pair (csrc/batchnorm.hip: per-channel statistics with a
Chan-merged parallel variance, then normalise+add+ReLU), instead of BN / add / ReLU as
three separate memory passes.
"""
from __future__ import annotations

import math

import os
import sys
import time

import torch
import torch.nn as nn
import torch.nn.functional as F

from cloudtik_amd.ops.linear import use_wgrad_side_stream
from cloudtik_amd import ops
from cloudtik_amd.ops import conv as igemm
from cloudtik_amd.ops.conv1x1 import conv1x1, conv3x3

import os

# the downsample branch's conv on its own stream, concurrent with conv1 -> conv2 -> conv3 of the
# block (its autograd backward then runs on that stream too, beside the main branch's)
_DOWN_STREAM = os.environ.get("CLOUDTIK_AMD_RESNET_DOWN_STREAM", "0") == "1"
_DOWN_STREAMS = {}


def _down_stream(device):
    s = _DOWN_STREAMS.get(device)
    if s is None:
        s = _DOWN_STREAMS[device] = torch.cuda.Stream(device=device)
    return s


class BatchNormAct(nn.Module):
    """BatchNorm2d (+ optional residual add) (+ optional ReLU), NHWC, fused on GPU."""

    def __init__(self, C, relu=True, eps=1e-5, momentum=0.1, zero_init=False, device=None,
                 dtype=None):
        super().__init__()
        self.weight = nn.Parameter(torch.full((C,), 0.0 if zero_init else 1.0, device=device, dtype=dtype))
        self.bias = nn.Parameter(torch.zeros(C, device=device, dtype=dtype))
        self.register_buffer("running_mean", torch.zeros(C, device=device))
        self.register_buffer("running_var", torch.ones(C, device=device))
        self.relu, self.eps, self.momentum = relu, eps, momentum
        self.frozen = False        # detection fine-tuning: running statistics only (FrozenBatchNorm)

    def forward(self, x, residual=None):
        return ops.batch_norm_act(x, self.weight, self.bias, self.running_mean, self.running_var,
                                  residual=residual, relu=self.relu, training=self.training and not self.frozen,
                                  momentum=self.momentum, eps=self.eps)


def _conv(cin, cout, k, stride=1, device=None, dtype=None, groups=1, dilation=1):
    c = nn.Conv2d(cin, cout, k, stride=stride, padding=dilation * (k // 2), bias=False, device=device,
                  dtype=torch.float32, groups=groups, dilation=dilation)
    nn.init.kaiming_normal_(c.weight, mode="fan_out", nonlinearity="relu")
    return c.to(dtype) if dtype is not None else c


class BasicBlock(nn.Module):
    """Two 3x3 convolutions (ResNet-18/34; the SSD-ResNet34 backbone)."""
    expansion = 1

    def __init__(self, cin, width, stride=1, downsample=False, device=None, dtype=None, groups=1,
                 base_width=64, dilation=1):
        super().__init__()
        kw = dict(device=device, dtype=dtype)
        self.conv1 = _conv(cin, width, 3, stride, dilation=dilation, **kw)
        self.bn1 = BatchNormAct(width, **kw)
        self.conv2 = _conv(width, width, 3, dilation=dilation, **kw)
        self.bn2 = BatchNormAct(width, relu=True, zero_init=True, **kw)   # fused add + ReLU
        self.down = None
        if downsample:
            self.down = _conv(cin, width, 1, stride, **kw)
            self.down_bn = BatchNormAct(width, relu=False, **kw)

    def forward(self, x):
        idt = self.down_bn(self.down(x)) if self.down is not None else x
        return self.bn2(conv3x3(self.bn1(conv3x3(x, self.conv1)), self.conv2), residual=idt)


class Bottleneck(nn.Module):
    """1x1 -> 3x3 (grouped for ResNeXt: ``groups`` x ``base_width``) -> 1x1, v1.5 stride."""
    expansion = 4

    def __init__(self, cin, width, stride=1, downsample=False, device=None, dtype=None, groups=1,
                 base_width=64, dilation=1):
        super().__init__()
        kw = dict(device=device, dtype=dtype)
        cout = width * self.expansion
        inner = int(width * (base_width / 64.0)) * groups
        self.conv1 = _conv(cin, inner, 1, **kw)
        self.bn1 = BatchNormAct(inner, **kw)
        self.conv2 = _conv(inner, inner, 3, stride, groups=groups, dilation=dilation, **kw)  # v1.5
        self.bn2 = BatchNormAct(inner, **kw)
        self.conv3 = _conv(inner, cout, 1, **kw)
        self.bn3 = BatchNormAct(cout, relu=True, zero_init=True, **kw)  # fused add + ReLU
        self.down = None
        if downsample:
            self.down = _conv(cin, cout, 1, stride, **kw)
            self.down_bn = BatchNormAct(cout, relu=False, **kw)

    def forward(self, x):
        if igemm.ENABLED and igemm.eligible(x, self.conv1.weight, (1, 1), (0, 0)):
            # every conv on the in-tree implicit-GEMM MFMA kernels (ops/conv.py); conv1 hands
            # out an alias of x for the residual / downsample branch so its data-gradient
            # epilogue absorbs that branch's gradient
            st = self.training and not self.bn1.frozen      # BatchNorm statistics from the conv epilogues
            out, x = igemm.conv2d(x, self.conv1, keep_input=True, bn_stats=st)
            side = None
            if self.down is not None and _DOWN_STREAM and x.is_cuda:
                cur = torch.cuda.current_stream(x.device)
                side = _down_stream(x.device)
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    d = igemm.conv2d(x, self.down, bn_stats=st)
                x.record_stream(side)
            else:
                d = igemm.conv2d(x, self.down, bn_stats=st) if self.down is not None else None
            out = self.bn2(igemm.conv2d(self.bn1(out), self.conv2, bn_stats=st))
            c3 = igemm.conv2d(out, self.conv3, bn_stats=st)
            if side is not None:
                cur.wait_stream(side)
                d.record_stream(cur)
                part = getattr(d, "_ct_bn_part", None)
                if part is not None:
                    part[0].record_stream(cur)
            b3, bd = self.bn3, getattr(self, "down_bn", None)
            if (d is not None and st and b3.relu and not bd.relu and not bd.frozen and not b3.frozen
                    and b3.momentum is not None and (b3.eps, b3.momentum) == (bd.eps, bd.momentum)):
                # bn3(conv3) + down_bn(down) + ReLU in one apply pass: the downsample branch's
                # BatchNorm output is never written (ops.functional._BNAddBNActFn)
                return ops.batch_norm_add_bn_act(c3, b3.weight, b3.bias, b3.running_mean, b3.running_var,
                                                 d, bd.weight, bd.bias, bd.running_mean, bd.running_var,
                                                 momentum=b3.momentum, eps=b3.eps)
            idt = bd(d) if d is not None else x
            return b3(c3, residual=idt)
        # MIOpen path (CLOUDTIK_AMD_CONV_IGEMM=0, CPU): 1x1 convs as NHWC GEMMs, conv1's dgrad
        # GEMM absorbs the residual branch's gradient (ops/conv1x1.py)
        out, x = conv1x1(x, self.conv1, keep_input=True)
        idt = self.down_bn(conv1x1(x, self.down)) if self.down is not None else x
        out = self.bn2(conv3x3(self.bn1(out), self.conv2))
        return self.bn3(conv1x1(out, self.conv3), residual=idt)


class ResNet(nn.Module):
    """ResNet / ResNeXt family (torchvision-equivalent topology; ``features()`` returns the
    C2..C5 maps for detection backbones)."""

    def __init__(self, layers=(3, 4, 6, 3), num_classes=1000, device=None, dtype=torch.bfloat16,
                 block=None, groups=1, width_per_group=64):
        super().__init__()
        block = block or Bottleneck
        kw = dict(device=device, dtype=dtype)
        self.conv1 = _conv(3, 64, 7, 2, **kw)
        self.bn1 = BatchNormAct(64, **kw)
        cin = 64
        stages = []
        self.stage_channels = []
        for i, (n, w) in enumerate(zip(layers, (64, 128, 256, 512))):
            blocks = []
            for j in range(n):
                stride = 2 if (j == 0 and i > 0) else 1
                down = j == 0 and (stride != 1 or cin != w * block.expansion)
                blocks.append(block(cin, w, stride, downsample=down, groups=groups, base_width=width_per_group, **kw))
                cin = w * block.expansion
            stages.append(nn.Sequential(*blocks))
            self.stage_channels.append(cin)
        self.layer1, self.layer2, self.layer3, self.layer4 = stages
        fc = nn.Linear(cin, num_classes, device=device)
        bound = 1.0 / math.sqrt(cin)
        nn.init.uniform_(fc.weight, -bound, bound)
        nn.init.uniform_(fc.bias, -bound, bound)
        self.fc = fc.to(dtype)
        if device is not None and torch.device(device).type == "cuda":
            self.to(memory_format=torch.channels_last)
        # memory-bound backward (BatchNorm passes): weight gradients on the side stream beside
        # it (ops/linear.py use_wgrad_side_stream)
        use_wgrad_side_stream(self, True)

    def stem(self, x):
        bn = self.bn1
        if bn.relu and self.training and not bn.frozen:
            # conv + BN + ReLU + max-pool with the BN backward folded into the conv weight gradient
            out = ops.stem_block(x, self.conv1, bn)
            if out is not None:
                return out
        y = igemm.stem_conv(x, self.conv1)
        if bn.relu and self.training and not bn.frozen:
            # BN + ReLU + 3x3/2 max-pool in one pass (the full-resolution activation is never
            # written; ops/functional.py batch_norm_relu_maxpool)
            return ops.batch_norm_relu_maxpool(y, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                                               training=True, momentum=bn.momentum, eps=bn.eps)
        return F.max_pool2d(bn(y), 3, 2, 1)

    def features(self, x):
        """[C2, C3, C4, C5] (strides 4, 8, 16, 32)."""
        c2 = self.layer1(self.stem(x))
        c3 = self.layer2(c2)
        c4 = self.layer3(c3)
        return [c2, c3, c4, self.layer4(c4)]

    def forward(self, x):
        x = self.layer4(self.layer3(self.layer2(self.layer1(self.stem(x)))))
        x = torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
        return self.fc(x)


def resnet50(num_classes=1000, device=None, dtype=torch.bfloat16):
    return ResNet((3, 4, 6, 3), num_classes, device=device, dtype=dtype)


def resnet34(num_classes=1000, device=None, dtype=torch.bfloat16):
    return ResNet((3, 4, 6, 3), num_classes, device=device, dtype=dtype, block=BasicBlock)


def resnet101(num_classes=1000, device=None, dtype=torch.bfloat16):
    return ResNet((3, 4, 23, 3), num_classes, device=device, dtype=dtype)


def resnext50_32x4d(num_classes=1000, device=None, dtype=torch.bfloat16):
    return ResNet((3, 4, 6, 3), num_classes, device=device, dtype=dtype, groups=32, width_per_group=4)


def resnext101_32x16d(num_classes=1000, device=None, dtype=torch.bfloat16):
    """ResNeXt101-32x16d (the reference's quickstart inference model,
    applications/ai/quickstart/bin/resnext-32x16d*)."""
    return ResNet((3, 4, 23, 3), num_classes, device=device, dtype=dtype, groups=32, width_per_group=16)


def resnet18_like_small(num_classes=10, device=None, dtype=torch.float32):
    """Tiny bottleneck ResNet for CPU tests."""
    return ResNet((1, 1, 1, 1), num_classes, device=device, dtype=dtype)


class ResNetTrainStep:
    """forward -> CE loss -> backward (overlapped bucketed all-reduce) -> fused SGD."""

    def __init__(self, model, optimizer, bucketer=None, scheduler=None):
        self.model, self.opt, self.ddp, self.sched = model, optimizer, bucketer, scheduler

    # CLOUDTIK_AMD_STEP_PHASES=<ms>: print the host time of each phase of any step slower than
    # that (a diagnostic for host-side stalls, e.g. in collective waits)
    _PHASES = float(os.environ.get("CLOUDTIK_AMD_STEP_PHASES", "0") or 0)

    def __call__(self, x, y):
        t = [time.perf_counter()] if self._PHASES else None
        logits = self.model(x)
        loss = F.cross_entropy(logits.float(), y)
        t and t.append(time.perf_counter())
        loss.backward()
        t and t.append(time.perf_counter())
        if self.ddp is not None:
            self.ddp.finish()
        t and t.append(time.perf_counter())
        self.opt.step()
        if self.sched is not None:
            self.sched.step()
        self.opt.zero_grad()
        if t:
            t.append(time.perf_counter())
            if (t[-1] - t[0]) * 1e3 > self._PHASES:
                ph = ", ".join(f"{n} {(b - a) * 1e3:.1f}" for n, a, b in
                               zip(("forward", "backward", "finish", "optimizer"), t, t[1:]))
                print(f"[step phases ms] {ph}", file=sys.stderr, flush=True)
        return loss
