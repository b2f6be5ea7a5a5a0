"""What the conv epilogues cost in the training step: implicit-GEMM conv forward plain (EPI 0)
vs with the BatchNorm tile statistics (EPI 1), and data gradient plain vs with the fused
BatchNorm + ReLU backward reduction (EPI 2), on ResNet-50 shapes at batch 256.

Each variant is timed cache-hot (the same operands every call, as bench/conv_igemm_probe.py
does) and cache-cold (rotating over enough operand copies that the 256 MiB Infinity Cache
cannot hold them, as in the training step, where every conv reads a tensor another kernel
wrote long before).  HIP-event timing of back-to-back calls; one markdown table.

    python bench/conv_epi_probe.py [--iters 12]
"""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cloudtik_amd import ops  # noqa: E402
from cloudtik_amd.ops import conv as CV  # noqa: E402

SHAPES = [("l1.c3", 64, 256, 56, 1, 1), ("l1.c1", 256, 64, 56, 1, 1), ("l2.c1a", 256, 128, 56, 1, 1),
          ("l2.c2", 128, 128, 28, 3, 1), ("l2.c3", 128, 512, 28, 1, 1), ("l3.c2", 256, 256, 14, 3, 1),
          ("l3.c3", 256, 1024, 14, 1, 1)]


def timeit(fns, iters):
    """mean us per call of fns[i % len(fns)] over `iters` calls (after one warm pass)"""
    for f in fns:
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(iters):
        fns[i % len(fns)]()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def nhwc(t):
    return t.contiguous(memory_format=torch.channels_last)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--cfgs", default="-1", help="conv configurations to time (comma list; -1 = auto)")
    ap.add_argument("--shapes", default="", help="comma list of shape names (default: all)")
    a = ap.parse_args()
    cfgs = [int(c) for c in a.cfgs.split(",")]
    want = set(a.shapes.split(",")) if a.shapes else None
    C = ops.require_native()
    dev = torch.device("cuda")
    print("| conv | cfg | fwd EPI0 hot / cold us | fwd EPI1 (stats) hot / cold us | dgrad EPI0 hot / cold us | "
          "dgrad EPI2 (BN bwd) hot / cold us | dgrad EPI2 bitmask + accumulate (the residual input) hot / cold us |")
    print("|---|---|---:|---:|---:|---:|---:|")
    for name, ci, co, H, k, s in SHAPES:
        if want and name not in want:
            continue
        pad = k // 2
        xbytes = a.batch * ci * H * H * 2
        ncopy = max(2, math.ceil(600e6 / xbytes))
        xs = [nhwc(torch.randn(a.batch, ci, H, H, device=dev).to(torch.bfloat16)) for _ in range(ncopy)]
        w = nhwc((torch.randn(co, ci, k, k, device=dev) * (2.0 / (ci * k * k)) ** 0.5).to(torch.bfloat16))
        Ho = (H + 2 * pad - k) // s + 1
        dys = [nhwc(torch.randn(a.batch, co, Ho, Ho, device=dev).to(torch.bfloat16)) for _ in range(ncopy)]
        gamma = torch.ones(ci, device=dev, dtype=torch.bfloat16)
        beta = torch.zeros(ci, device=dev, dtype=torch.bfloat16)
        rm, rv = torch.zeros(ci, device=dev), torch.ones(ci, device=dev)
        links, links3, outs = [], [], []
        for x in xs:                       # x = the output of a BN + ReLU whose input is xb
            xb = x
            _, stat = C.bn_fwd_train(xb, None, gamma, beta, rm, rv, 1e-5, 0.1, True)
            links.append(CV.BnBwdLink(xb, stat, 2))
            # the residual BN + ReLU of the ResNet block input: bitmask (mode 3), and the data
            # gradient accumulates into the residual branch's gradient
            mask = torch.empty(xb.numel() // 8, device=dev, dtype=torch.uint8)
            _, stat3 = C.bn_fwd_train(xb, None, gamma, beta, rm, rv, 1e-5, 0.1, True, mask)
            links3.append(CV.BnBwdLink(xb, stat3, 3, mask))
            outs.append(torch.zeros_like(xb))
        for cfg in cfgs:
            CV._CFG = cfg
            r = {}
            for tag, sel in (("hot", lambda L: L[:1]), ("cold", lambda L: L)):
              try:
                r[("f0", tag)] = timeit([lambda x=x: CV.conv_fwd(x, w, (s, s), (pad, pad)) for x in sel(xs)], a.iters)
                r[("f1", tag)] = timeit([lambda x=x: CV.conv_fwd(x, w, (s, s), (pad, pad), partials=True)
                                         for x in sel(xs)], a.iters)
                r[("d0", tag)] = timeit([lambda dy=dy: CV.conv_dgrad(dy, w, xs[0].shape, (s, s), (pad, pad))
                                         for dy in sel(dys)], a.iters)
                pairs = list(zip(sel(dys), sel(links)))
                r[("d2", tag)] = timeit([lambda dy=dy, L=L: CV.conv_dgrad(dy, w, xs[0].shape, (s, s), (pad, pad),
                                                                          bn=L)
                                         for dy, L in pairs], a.iters)
                trip = list(zip(sel(dys), sel(links3), sel(outs)))
                r[("d3", tag)] = timeit([lambda dy=dy, L=L, o=o: CV.conv_dgrad(dy, w, xs[0].shape, (s, s), (pad, pad),
                                                                               out=o, accumulate=True, bn=L,
                                                                               bn_y=o)
                                         for dy, L, o in trip], a.iters)
              except RuntimeError:          # a configuration this shape's fwd or dgrad rejects
                pass
            cell = lambda k: (f"{r[(k, 'hot')]:.1f} / {r[(k, 'cold')]:.1f}" if (k, 'cold') in r else "-")
            print(f"| {name} {ci}->{co} {H}x{H} k{k} | {cfg} | {cell('f0')} | {cell('f1')} | {cell('d0')} | "
                  f"{cell('d2')} | {cell('d3')} |", flush=True)
        CV._CFG = -1
        del xs, dys, links, links3, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
