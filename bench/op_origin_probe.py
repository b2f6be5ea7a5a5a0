"""Which aten ops launch the generic PyTorch elementwise / copy kernels inside a ResNet-50 (or
BERT-large) training step: one profiled step after warm-up, kernels grouped by the aten op that
launched them (torch.profiler CPU-op -> kernel correlation).

    python bench/op_origin_probe.py [--model resnet50] [--match elementwise]"""
import argparse
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--match", default="at::native")
    a = ap.parse_args()
    args = bench.parse(["--model", a.model, "--steps", "1", "--warmup", "1"])
    dev = torch.device("cuda")
    build = bench.build_resnet if a.model == "resnet50" else bench.build_bert
    step, close, info = build(args, 0, 1, dev, a.model)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        step()
        torch.cuda.synchronize()
    agg = defaultdict(lambda: [0, 0.0])
    for ev in prof.events():
        if ev.device_type.name != "CUDA" and not getattr(ev, "kernels", None):
            continue
        for k in getattr(ev, "kernels", []) or []:
            if a.match in k.name:
                key = (ev.name, str(ev.input_shapes)[:120], k.name[:70])
                agg[key][0] += 1
                agg[key][1] += k.duration / 1e3 if hasattr(k, "duration") else 0.0
    for (op, shp, kn), (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"{us:9.1f} us  x{n:3d}  {op:40s} {shp:60s} {kn}")
    close()


if __name__ == "__main__":
    main()
