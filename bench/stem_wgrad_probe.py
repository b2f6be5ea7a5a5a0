"""ResNet-50 stem weight gradient (7x7 / 2 over the NHWC4 / NHWC8 image batch, 64 outputs) per
wgrad tile configuration and split-K workgroup target: it is the last kernel of the backward,
alone on the chip.

    python bench/stem_wgrad_probe.py [--cfgs 5,1,4,0] [--blocks 256,512,1024]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cloudtik_amd.ops import conv as CV  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfgs", default="5,1,4,0")
    ap.add_argument("--blocks", default="256,512,1024")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--cp", type=int, default=4)
    a = ap.parse_args()
    dev = torch.device("cuda")
    x = torch.randn(a.batch, 3, 224, 224, device=dev).to(torch.bfloat16)
    x4 = CV.to_nhwc8(x, a.cp)
    dy = torch.randn(a.batch, 64, 112, 112, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    for cfg in [int(c) for c in a.cfgs.split(",")]:
        for b in [int(v) for v in a.blocks.split(",")]:
            CV._WG_CFG, CV.STEM_WGRAD_CFG, CV.STEM_WGRAD_BLOCKS = -1, cfg, b
            fn = lambda: CV.stem_wgrad(dy, x4, (64, 3, 7, 7), (2, 2), (3, 3))  # noqa: E731
            try:
                for _ in range(3):
                    fn()
            except RuntimeError as e:
                print(json.dumps({"cfg": cfg, "blocks": b, "error": str(e)[:80]}), flush=True)
                continue
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                fn()
            e1.record()
            torch.cuda.synchronize()
            print(json.dumps({"cfg": cfg, "blocks": b, "us": round(e0.elapsed_time(e1) / 10 * 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
