"""3x3 weight-gradient kernels on the ResNet-50 3x3 shapes (stride 1 and 2) (batch 256): total time of
``ops.conv.conv_wgrad`` (kernel + split-K reduce) per configuration.  Run under
``rocprofv3 --kernel-trace --stats`` for the kernel / reduce split.

    python bench/wgrad3x3_probe.py [--cfgs -1,13,15] [--shapes l1,l2] [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cloudtik_amd.ops import conv as CV  # noqa: E402

SHAPES = {"l1": (64, 56, 1), "l2": (128, 28, 1), "l3": (256, 14, 1), "l4": (512, 7, 1),
          "l2s2": (128, 56, 2), "l3s2": (256, 28, 2), "l4s2": (512, 14, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfgs", default="-1,13")
    ap.add_argument("--shapes", default="l1,l2,l3,l4,l2s2,l3s2,l4s2")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda")
    for name in a.shapes.split(","):
        c, H, st = SHAPES[name]
        Ho = (H - 1) // st + 1
        x = torch.randn(a.batch, c, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dy = torch.randn(a.batch, c, Ho, Ho, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        shape = (c, c, 3, 3)
        row = {"shape": name, "gflop": round(2 * a.batch * Ho * Ho * c * c * 9 / 1e9, 1)}
        for cfg in [int(v) for v in a.cfgs.split(",")]:
            CV._WG_CFG = cfg
            fn = lambda: CV.conv_wgrad(dy, x, shape, (st, st), (1, 1))  # noqa: E731
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
