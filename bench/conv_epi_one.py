"""Tiny driver for hardware-counter runs of one conv shape: `--iters` forward launches plain
(EPI 0) and with the BatchNorm statistics epilogue (EPI 1), or data gradients plain and with
the fused BatchNorm backward (EPI 2).  No timing of its own -- run it under rocprofv3.

    rocprofv3 --pmc ... -- python bench/conv_epi_one.py --shape 64,256,56,1,1
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cloudtik_amd import ops  # noqa: E402
from cloudtik_amd.ops import conv as CV  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="64,256,56,1,1", help="ci,co,H,k,stride")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--dgrad", action="store_true")
    a = ap.parse_args()
    ci, co, H, k, s = (int(v) for v in a.shape.split(","))
    pad = k // 2
    C = ops.require_native()
    dev = torch.device("cuda")
    cl = torch.channels_last
    x = torch.randn(a.batch, ci, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    w = (torch.randn(co, ci, k, k, device=dev) * 0.05).to(torch.bfloat16).contiguous(memory_format=cl)
    if not a.dgrad:
        for _ in range(a.iters):
            CV.conv_fwd(x, w, (s, s), (pad, pad))
            CV.conv_fwd(x, w, (s, s), (pad, pad), partials=True)
    else:
        Ho = (H + 2 * pad - k) // s + 1
        dy = torch.randn(a.batch, co, Ho, Ho, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
        g = torch.ones(ci, device=dev, dtype=torch.bfloat16)
        _, stat = C.bn_fwd_train(x, None, g, torch.zeros_like(g), torch.zeros(ci, device=dev),
                                 torch.ones(ci, device=dev), 1e-5, 0.1, True)
        link = CV.BnBwdLink(x, stat, 2)
        for _ in range(a.iters):
            CV.conv_dgrad(dy, w, x.shape, (s, s), (pad, pad))
            CV.conv_dgrad(dy, w, x.shape, (s, s), (pad, pad), bn=link)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
