#!/usr/bin/env python3
"""BERT-large GEMM microbench: forward / dgrad / wgrad shapes at 32768 tokens, and split-K
alternatives for the weight-gradient GEMMs (dW = dY^T X has K = tokens = 32768 but only
N*K/(256*256) = 16..192 output tiles, too few to fill 256 CUs)."""
import argparse
import json

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def timeit(fn, iters=20, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--tunableop", default="off", choices=["off", "use"])
    args = ap.parse_args()
    if args.tunableop == "use":
        import os
        import torch.cuda.tunable as tn
        tn.enable(True)
        tn.tuning_enable(False)
        tn.set_filename(os.path.join(os.path.dirname(__file__), "..", "cloudtik_amd", "ops", "tunableop",
                                     "gfx950_tunableop.csv"))
    T = args.tokens
    dev = "cuda"
    bf = torch.bfloat16
    shapes = {"qkv": (1024, 3072), "proj": (1024, 1024), "ffn1": (1024, 4096), "ffn2": (4096, 1024)}
    res = {}
    for name, (din, dout) in shapes.items():
        x = torch.randn(T, din, device=dev, dtype=bf)
        w = torch.randn(dout, din, device=dev, dtype=bf)
        dy = torch.randn(T, dout, device=dev, dtype=bf)
        g = torch.zeros(dout, din, device=dev, dtype=bf)
        fl = 2.0 * T * din * dout
        r = {}
        r["fwd"] = timeit(lambda: torch.nn.functional.linear(x, w))
        r["dgrad"] = timeit(lambda: torch.mm(dy, w))
        r["wgrad_addmm"] = timeit(lambda: g.addmm_(dy.t(), x))
        r["wgrad_mm"] = timeit(lambda: torch.mm(dy.t(), x))
        ref = torch.mm(dy.t().float(), x.float())
        for S in (2, 4, 8):
            dyb = dy.view(S, T // S, dout).transpose(1, 2)
            xb = x.view(S, T // S, din)
            r[f"wgrad_sk{S}_bf16"] = timeit(lambda: g.add_(torch.bmm(dyb, xb).sum(0)))
            try:
                r[f"wgrad_sk{S}_fp32"] = timeit(lambda: g.add_(torch.bmm(dyb, xb, out_dtype=torch.float32).sum(0)))
                err = (torch.bmm(dyb, xb, out_dtype=torch.float32).sum(0) - ref).abs().max().item()
                r[f"wgrad_sk{S}_fp32_maxerr"] = err
            except Exception as e:  # noqa: BLE001
                r[f"wgrad_sk{S}_fp32"] = str(e)[:80]
        try:
            r["wgrad_mm_fp32out"] = timeit(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32))
        except Exception as e:  # noqa: BLE001
            r["wgrad_mm_fp32out"] = str(e)[:80]
        r["wgrad_mm_maxerr"] = (torch.mm(dy.t(), x).float() - ref).abs().max().item()
        r["TFLOPs"] = {k: round(fl / v / 1e9, 1) for k, v in r.items() if isinstance(v, float) and "err" not in k}
        res[name] = r
        print(name, json.dumps(r["TFLOPs"]), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
