"""Stem block gradients vs fp32 PyTorch: the folded BatchNorm backward (ops.stem_block) and the
composed path (stem conv + batch_norm_relu_maxpool); prints relative errors.

    python bench/stem_fold_check.py
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cloudtik_amd import ops  # noqa: E402
from cloudtik_amd.models.resnet import BatchNormAct  # noqa: E402
from cloudtik_amd.ops import conv as CV  # noqa: E402


def rel(a, b):
    return round(((a.float() - b.float()).norm() / b.float().norm()).item(), 5)


def run(folded, N=2, HW=64, seed=1):
    dev = torch.device("cuda")
    torch.manual_seed(seed)
    x = torch.randn(N, 3, HW, HW, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    conv = torch.nn.Conv2d(3, 64, 7, 2, 3, bias=False).to(dev, torch.bfloat16)
    bn = BatchNormAct(64, device=dev, dtype=torch.bfloat16)
    with torch.no_grad():
        conv.weight.copy_(torch.randn_like(conv.weight) * 0.1)
        bn.weight.copy_(torch.rand(64, device=dev) + 0.5)
        bn.bias.copy_(torch.randn(64, device=dev) * 0.1)
    conv.weight.data = conv.weight.data.contiguous(memory_format=torch.channels_last)
    if folded:
        out = ops.stem_block(x, conv, bn)
    else:
        y = CV.stem_conv(x, conv)
        out = ops.batch_norm_relu_maxpool(y, bn.weight, bn.bias, bn.running_mean, bn.running_var, training=True)
    r = torch.randn(out.shape, device=dev)
    (out.float() * r).sum().backward()
    w = conv.weight.detach().float().requires_grad_()
    g = bn.weight.detach().float().requires_grad_()
    b = bn.bias.detach().float().requires_grad_()
    rm, rv = torch.zeros(64, device=dev), torch.ones(64, device=dev)
    yr = F.conv2d(x.float(), w, stride=2, padding=3)
    ref = F.max_pool2d(F.relu(F.batch_norm(yr, rm, rv, g, b, training=True, momentum=0.1, eps=1e-5)), 3, 2, 1)
    (ref * r).sum().backward()
    return {"folded": folded, "out": rel(out, ref), "dw": rel(conv.weight.grad, w.grad),
            "dgamma": rel(bn.weight.grad, g.grad), "dbeta": rel(bn.bias.grad, b.grad)}


if __name__ == "__main__":
    for f in (False, True):
        for hw in (64, 112):
            print(json.dumps(dict(run(f, HW=hw), HW=hw)), flush=True)
