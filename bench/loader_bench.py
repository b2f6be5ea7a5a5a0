#!/usr/bin/env python3
"""Native loader throughput: ImageNet-shaped uint8 batches (256 x 3 x 224 x 224) from host
memory to the GPU, with a compute-stream consumer.  Prints GB/s and batches/s."""
import argparse
import json
import time

import numpy as np
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=8192)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--epochs", type=int, default=2)
    a = ap.parse_args()
    from cloudtik_amd.data import NativeLoader
    x = np.random.randint(0, 255, (a.rows, 3, 224, 224), dtype=np.uint8)
    y = np.arange(a.rows, dtype=np.int64)
    L = NativeLoader({"image": x, "label": y}, a.batch, num_workers=a.workers, prefetch=6, device="cuda")
    for b in L:       # warm epoch
        pass
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    nb = 0
    for e in range(a.epochs):
        L.set_epoch(e + 1)
        for b in L:
            b["image"].float().mean()      # a consumer kernel on the compute stream
            nb += 1
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    gb = nb * a.batch * 3 * 224 * 224 / 1e9
    print(json.dumps({"batches_per_s": round(nb / dt, 1), "images_per_s": round(nb * a.batch / dt),
                      "GB_per_s": round(gb / dt, 2), "workers": a.workers}))


if __name__ == "__main__":
    main()
