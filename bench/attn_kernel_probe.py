"""Attention kernels in isolation on the BERT-large shape (B 256, S 128, 16 heads x 64, packed
qkv as the transformer block passes it, key-padding bias, dropout 0.1): forward and backward
times (HIP events, 20 back-to-back calls) and the HBM-traffic floor of each.

    python bench/attn_kernel_probe.py [--B 256] [--S 128] [--p 0.1]"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


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
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--S", type=int, default=128)
    ap.add_argument("--H", type=int, default=16)
    ap.add_argument("--p", type=float, default=0.1)
    a = ap.parse_args()
    from cloudtik_amd import ops
    C = ops.require_native()
    B, S, H, D = a.B, a.S, a.H, 64
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = (torch.randn(B, S, 3, H, D, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
    kb = torch.zeros(B, S, device="cuda")
    kb[:, S - S // 8:] = -10000.0
    o = torch.empty(B, S, H, D, device="cuda", dtype=torch.bfloat16)
    do = torch.randn(B, S, H, D, device="cuda", generator=g).to(torch.bfloat16)
    dqkv = torch.empty_like(qkv)
    scale = 1.0 / math.sqrt(D)
    fwd = lambda: C.attn_fwd(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], o, kb, scale, a.p, 1, 0, False)
    lse = fwd()
    bwd = lambda: C.attn_bwd(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], o, do, dqkv[:, :, 0], dqkv[:, :, 1],
                             dqkv[:, :, 2], kb, lse, scale, a.p, 1, 0, False)
    t_f, t_b = timeit(fwd), timeit(bwd)
    mb = B * S * H * D * 2 / 1e6
    fl = 4 * B * H * S * S * D
    print(json.dumps({"B": B, "S": S, "p": a.p, "fwd_us": round(t_f, 1), "bwd_us": round(t_b, 1),
                      "fwd_hbm_mb": round(4 * mb), "bwd_hbm_mb": round(8 * mb),
                      "fwd_tb_s": round(4 * mb / t_f, 2), "bwd_tb_s": round(8 * mb / t_b, 2),
                      "fwd_tflops": round(fl / t_f / 1e6), "bwd_tflops": round(2.5 * fl / t_b / 1e6)}), flush=True)


if __name__ == "__main__":
    main()
