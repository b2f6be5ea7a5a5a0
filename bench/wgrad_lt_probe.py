#!/usr/bin/env python3
"""Split-K weight-gradient GEMM on the BERT-large shapes (tokens 32768): torch.bmm (heuristic
algorithm) vs the binding's strided-batched hipBLASLt call tuned over every solution
(ops/csrc/bindings_lt.cpp lt_bmm_tuned), with a numerics check against fp32."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from cloudtik_amd import ops
from cloudtik_amd.ops.linear import splitk_factor


def timeit(fn, iters=20, warmup=3):
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
    C = ops.require_native()
    T = 32768
    res = {}
    for name, (N, K) in {"qkv": (3072, 1024), "proj": (1024, 1024), "ffn1": (4096, 1024), "ffn2": (1024, 4096)}.items():
        dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * T * N * K
        r = {}
        for S in sorted({splitk_factor(T, N, K), 2, 4, 8}):
            Ts = T // S
            P = torch.empty(S, N, K, device="cuda", dtype=torch.float32)
            t_bmm = timeit(lambda: torch.bmm(dy.view(S, Ts, N).transpose(1, 2), x.view(S, Ts, K),
                                             out_dtype=torch.float32))
            tuned = C.lt_bmm_tuned(dy[:Ts], x[:Ts], P[0], True, False, S, Ts * N, Ts * K, N * K, 0)
            t_lt = timeit(lambda: C.lt_bmm_tuned(dy[:Ts], x[:Ts], P[0], True, False, S, Ts * N, Ts * K, N * K, 0))
            ref = torch.bmm(dy.view(S, Ts, N).transpose(1, 2).float(), x.view(S, Ts, K).float())
            err = ((P - ref).abs().max() / ref.abs().max()).item()
            r[f"S{S}"] = {"bmm_ms": round(t_bmm, 4), "lt_ms": round(t_lt, 4), "tune_ms": round(tuned, 4),
                          "bmm_TF": round(fl / t_bmm / 1e9, 1), "lt_TF": round(fl / t_lt / 1e9, 1),
                          "rel_err": err, "chosen_S": S == splitk_factor(T, N, K)}
        res[name] = r
        print(name, json.dumps(r), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
