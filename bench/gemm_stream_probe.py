"""Streamed persistent MFMA GEMM (csrc/gemm_nt.hip gemm_nt_stream_kernel) vs the one-tile kernel
vs hipBLASLt on the BERT-large forward (+ bias) and data-gradient GEMMs, tokens 32768.

Correctness first (relative error vs an fp32 reference on the same random operands), then
timing in interleaved rounds within one process (HIP events over ``--iters`` back-to-back
calls per round; the median and min over ``--rounds`` rounds are reported, cdna_hip_programming
§5.4 rule 24).  Prints one JSON line per shape and a markdown table on stderr.

    python bench/gemm_stream_probe.py [--tokens 32768] [--rounds 5] [--iters 20]
"""
import argparse
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters):
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--wgs", type=int, default=0, help="persistent workgroups (0: one per CU)")
    a = ap.parse_args()
    from cloudtik_amd import ops
    C = ops.require_native()
    T = a.tokens
    bf = torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(0)

    def rnd(*s, sc=1.0):
        return (torch.randn(*s, device="cuda", generator=g) * sc).to(bf)

    # (name, kind, M, N, K): fwd = x[M,K] W[N,K]^T + b; dgrad = dy[M,K] W[K,N]
    cases = [("qkv_fwd", "fwd", T, 3072, 1024), ("wo_fwd", "fwd", T, 1024, 1024), ("ffn2_fwd", "fwd", T, 1024, 4096),
             ("ffn1_fwd_plain", "fwd", T, 4096, 1024),
             ("qkv_dgrad_dx", "dgrad", T, 1024, 3072), ("wo_dgrad_dx", "dgrad", T, 1024, 1024),
             ("ffn1_dgrad_dx", "dgrad", T, 1024, 4096), ("ffn2_dgrad_dh", "dgrad", T, 4096, 1024)]
    rows = []
    for name, kind, M, N, K in cases:
        A = rnd(M, K)
        if kind == "fwd":
            W = rnd(N, K, sc=K ** -0.5)
            b = rnd(N, sc=0.1)
            ref = (A.float() @ W.float().t() + b.float())
            fns = {"hipblaslt": lambda: F.linear(A, W, b),
                   "one_tile": lambda D=torch.empty(M, N, device="cuda", dtype=bf): (C.gemm_nt(A, W, D, 5, False, b, None,
                                                                                                None), D)[1],
                   "stream": lambda D=torch.empty(M, N, device="cuda", dtype=bf): (C.gemm_nt_stream(A, W, D, b, False,
                                                                                                    a.wgs), D)[1]}
        else:
            W = rnd(K, N, sc=K ** -0.5)
            ref = A.float() @ W.float()
            fns = {"hipblaslt": lambda: torch.matmul(A, W),
                   "one_tile": lambda D=torch.empty(M, N, device="cuda", dtype=bf): (C.gemm_nn(A, W, D, 0, False, None,
                                                                                                None, None), D)[1],
                   "stream": lambda D=torch.empty(M, N, device="cuda", dtype=bf): (C.gemm_nt_stream(A, W, D, None, True,
                                                                                                    a.wgs), D)[1]}
        err = {}
        for k, fn in fns.items():
            out = fn()
            torch.cuda.synchronize()
            err[k] = ((out.float() - ref).norm() / ref.norm()).item()
        for fn in fns.values():                    # warm every variant
            for _ in range(3):
                fn()
        torch.cuda.synchronize()
        times = {k: [] for k in fns}
        for _ in range(a.rounds):
            for k, fn in fns.items():
                times[k].append(timeit(fn, a.iters))
        fl = 2.0 * M * N * K
        row = {"case": name, "M": M, "N": N, "K": K, "rel_err": {k: round(v, 5) for k, v in err.items()}}
        for k, ts in times.items():
            med = statistics.median(ts)
            row[f"{k}_us"] = round(med, 1)
            row[f"{k}_min_us"] = round(min(ts), 1)
            row[f"{k}_tflops"] = round(fl / med / 1e6)
        rows.append(row)
        print(json.dumps(row), flush=True)
        del A, W, ref
        torch.cuda.empty_cache()
    print("| case | M x N x K | hipBLASLt us | one-tile us | stream us | stream TF/s | stream vs hipBLASLt |",
          file=sys.stderr)
    print("|---|---|---:|---:|---:|---:|---:|", file=sys.stderr)
    for r in rows:
        print(f"| {r['case']} | {r['M']}x{r['N']}x{r['K']} | {r['hipblaslt_us']} | {r['one_tile_us']} | "
              f"{r['stream_us']} | {r['stream_tflops']} | {r['hipblaslt_us'] / r['stream_us']:.3f}x |", file=sys.stderr)


if __name__ == "__main__":
    main()
