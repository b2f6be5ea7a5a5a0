"""ResNet-50 stem BatchNorm + ReLU + 3x3/2 max-pool (bn_apply_pool_kernel) and its backward
(maxpool3s2_bwd_kernel) at batch 256 x 64 x 112 x 112: HIP-event time per call and effective
bandwidth (bytes the kernel must move).

    python bench/stem_pool_probe.py [--N 256]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cloudtik_amd import ops  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=256)
    a = ap.parse_args()
    C, H = 64, 112
    OH = (H - 1) // 2 + 1
    dev = torch.device("cuda")
    Cn = ops.require_native()
    x = torch.randn(a.N, C, H, H, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    g = torch.ones(C, device=dev, dtype=torch.bfloat16)
    b = torch.zeros(C, device=dev, dtype=torch.bfloat16)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    y = ops.batch_norm_relu_maxpool(x.requires_grad_(), g, b, rm, rv, training=True)
    dy = torch.randn_like(y)
    t_fb = timeit(lambda: y.backward(dy, retain_graph=True))
    t_all = timeit(lambda: ops.batch_norm_relu_maxpool(x, g, b, rm, rv, training=True))
    xb = x.numel() * 2
    yb = a.N * C * OH * OH * 2
    print(json.dumps({"N": a.N, "fwd_us_incl_stats": round(t_all, 1), "bwd_us_incl_bn_bwd": round(t_fb, 1),
                      "pool_fwd_bytes_mb": round((xb + yb + yb // 2) / 1e6), "pool_bwd_bytes_mb":
                      round((yb + yb // 2 + xb) / 1e6)}))


if __name__ == "__main__":
    main()
