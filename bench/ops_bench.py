#!/usr/bin/env python3
"""Microbench of the BERT-large elementwise / normalisation kernels at 32768 tokens:
LayerNorm fwd/bwd (hidden 1024, fused bias+dropout+residual) and bias+GELU fwd/bwd (4096).
Prints us per call and effective HBM bandwidth."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def timeit(fn, iters=50, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0


def main():
    from cloudtik_amd import ops
    C = ops.require_native()
    M, H, I = 32768, 1024, 4096
    bf = torch.bfloat16
    dev = "cuda"
    x = torch.randn(M, H, device=dev, dtype=bf)
    res = torch.randn_like(x)
    bias = torch.randn(H, device=dev, dtype=bf)
    g = torch.ones(H, device=dev, dtype=bf)
    b = torch.zeros(H, device=dev, dtype=bf)
    out = {}
    y, s, mean, rstd = C.layernorm_fwd(x, bias, res, g, b, 1e-12, False, 0.1, 1, 0)
    out["ln_fwd_us"] = timeit(lambda: C.layernorm_fwd(x, bias, res, g, b, 1e-12, False, 0.1, 1, 0))
    out["ln_fwd_TBps"] = 4 * M * H * 2 / out["ln_fwd_us"] / 1e6
    dy = torch.randn_like(x)
    dg = torch.zeros(H, device=dev, dtype=bf)
    db = torch.zeros(H, device=dev, dtype=bf)
    dbias = torch.zeros(H, device=dev, dtype=bf)
    f = lambda: C.layernorm_bwd_into(dy, s, g, mean, rstd, False, dg, db, dbias, True, 0.1, 1, 0)
    out["ln_bwd_us"] = timeit(f)
    out["ln_bwd_TBps"] = 4 * M * H * 2 / out["ln_bwd_us"] / 1e6
    # the same kernels without dropout: the difference is the cost of regenerating the mask
    out["ln_fwd_p0_us"] = timeit(lambda: C.layernorm_fwd(x, bias, res, g, b, 1e-12, False, 0.0, 1, 0))
    y0, s0, mean0, rstd0 = C.layernorm_fwd(x, bias, res, g, b, 1e-12, False, 0.0, 1, 0)
    out["ln_bwd_p0_us"] = timeit(lambda: C.layernorm_bwd_into(dy, s0, g, mean0, rstd0, False, dg, db, dbias, True,
                                                              0.0, 1, 0))
    z = torch.randn(M, I, device=dev, dtype=bf)
    bi = torch.randn(I, device=dev, dtype=bf)
    out["bias_gelu_fwd_us"] = timeit(lambda: C.bias_act_fwd(z, bi, 1))
    out["bias_gelu_fwd_TBps"] = 2 * M * I * 2 / out["bias_gelu_fwd_us"] / 1e6
    dyi = torch.randn_like(z)
    out["bias_gelu_bwd_us"] = timeit(lambda: C.bias_act_bwd(dyi, z, bi, 1, True))
    out["bias_gelu_bwd_TBps"] = 3 * M * I * 2 / out["bias_gelu_bwd_us"] / 1e6
    print(json.dumps({k: round(v, 2) for k, v in out.items()}))


if __name__ == "__main__":
    main()
