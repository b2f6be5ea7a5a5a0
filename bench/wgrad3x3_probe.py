"""Conv weight-gradient kernels on ResNet-50 shapes (3x3 stride 1 / 2, narrow 1x1; batch 256): total time of
``ops.conv.conv_wgrad`` (kernel + split-K reduce) per configuration.  Run under
``rocprofv3 --kernel-trace --stats`` for the kernel / reduce split.

    python bench/wgrad3x3_probe.py [--cfgs=-1,12,13] [--shapes l1,l2,l1c3] [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cloudtik_amd.ops import conv as CV  # noqa: E402

# name: (ci, co, input H, kernel, stride)
SHAPES = {"l1": (64, 64, 56, 3, 1), "l2": (128, 128, 28, 3, 1), "l3": (256, 256, 14, 3, 1), "l4": (512, 512, 7, 3, 1),
          "l2s2": (128, 128, 56, 3, 2), "l3s2": (256, 256, 28, 3, 2), "l4s2": (512, 512, 14, 3, 2),
          "l1c3": (64, 256, 56, 1, 1), "l1c1": (256, 64, 56, 1, 1), "l1c1a": (64, 64, 56, 1, 1),
          "l2c3": (128, 512, 28, 1, 1), "l2c1": (512, 128, 28, 1, 1), "l3c1a": (512, 256, 28, 1, 1),
          "l3c3": (256, 1024, 14, 1, 1), "l3c1": (1024, 256, 14, 1, 1), "l4c1a": (1024, 512, 14, 1, 1),
          "l4c3": (512, 2048, 7, 1, 1), "l4c1": (2048, 512, 7, 1, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfgs", default="-1,13")
    ap.add_argument("--shapes", default="l1,l2,l3,l4,l2s2,l3s2,l4s2")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda")
    for name in a.shapes.split(","):
        ci, co, H, k, st = SHAPES[name]
        pad = k // 2
        Ho = (H + 2 * pad - k) // st + 1
        x = torch.randn(a.batch, ci, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dy = torch.randn(a.batch, co, Ho, Ho, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        shape = (co, ci, k, k)
        row = {"shape": name, "gflop": round(2 * a.batch * Ho * Ho * co * ci * k * k / 1e9, 1)}
        for cfg in [int(v) for v in a.cfgs.split(",")]:
            CV._WG_CFG = cfg
            fn = lambda: CV.conv_wgrad(dy, x, shape, (st, st), (pad, pad))  # noqa: E731
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            row[f"c{cfg}_us"] = round(e0.elapsed_time(e1) / a.iters * 1e3, 1)
        CV._WG_CFG = -1
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
