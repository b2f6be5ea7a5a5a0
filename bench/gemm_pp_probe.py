"""Paired-tile GEMM (csrc/gemm_pp.hip) vs the one-tile MFMA GEMM (csrc/gemm_nt.hip) vs hipBLASLt on
the BERT-large forward projection shapes (tokens 32768), random bf16 operands.

Numerics first (small shapes with few workgroups, uneven tiles per group, every epilogue), then
median time of interleaved rounds.  Prints one JSON line per shape.

    python bench/gemm_pp_probe.py [--rounds 5] [--iters 10] [--eslots 1,2,4,8]
"""
import argparse
import json
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def ref_epi(A, B, bias, epi):
    z = A.float() @ B.float().t()
    if epi == 0:
        return z, None
    z = z + bias.float()
    if epi == 5:
        return z, None
    phi = 0.5 * (1.0 + torch.erf(z / math.sqrt(2.0)))
    pdf = torch.exp(-0.5 * z * z) / math.sqrt(2.0 * math.pi)
    return z * phi, phi + z * pdf


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def check(C, dev):
    out = []
    g = torch.Generator(device="cpu").manual_seed(0)
    for (M, N, K, wgs) in [(2048, 512, 256, 8), (2176, 768, 192, 8), (4096, 1024, 1024, 16), (32768, 4096, 1024, 0)]:
        A = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)
        B = (torch.randn(N, K, generator=g) * K ** -0.5).to(dev, torch.bfloat16)
        bias = (torch.randn(N, generator=g) * 0.5).to(dev, torch.bfloat16)
        for epi in (0, 5, 6):
            for es in (1, 4):
                D = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                aux = torch.empty_like(D) if epi == 6 else None
                ok = C.gemm_pp(A, B, D, epi, bias if epi else None, aux, wgs, es)
                torch.cuda.synchronize()
                zr, dr = ref_epi(A, B, bias, epi)
                r = {"M": M, "N": N, "K": K, "wgs": wgs, "epi": epi, "eslots": es, "ok": bool(ok),
                     "err": rel(D, zr) if ok else None}
                if epi == 6 and ok:
                    r["err_aux"] = rel(aux, dr)
                out.append(r)
                if M >= 32768:
                    break
    return out


def timeit(fn, iters):
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
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--eslots", default="1,2,4,8")
    ap.add_argument("--skip-check", action="store_true")
    ap.add_argument("--shapes", default="ffn1,ffn1_plain,qkv,wo,ffn2")
    a = ap.parse_args()
    from cloudtik_amd import ops
    C = ops.require_native()
    dev = torch.device("cuda")
    if not a.skip_check:
        res = check(C, dev)
        bad = [r for r in res if not r["ok"] or r["err"] > 1e-2 or r.get("err_aux", 0) > 1e-2]
        print(json.dumps({"check": res, "bad": len(bad)}), flush=True)
        if bad:
            sys.exit(1)
    eslots = [int(x) for x in a.eslots.split(",")]
    g = torch.Generator(device="cpu").manual_seed(1)
    for name, M, N, K, epi in [("ffn1", 32768, 4096, 1024, 6), ("ffn1_plain", 32768, 4096, 1024, 0),
                               ("qkv", 32768, 3072, 1024, 5), ("wo", 32768, 1024, 1024, 0),
                               ("ffn2", 32768, 1024, 4096, 0)]:
        if name not in a.shapes.split(","):
            continue
        A = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)
        B = (torch.randn(N, K, generator=g) * K ** -0.5).to(dev, torch.bfloat16)
        bias = (torch.randn(N, generator=g) * 0.5).to(dev, torch.bfloat16)
        D = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        aux = torch.empty_like(D)
        fns = {}
        for es in eslots:
            fns[f"pp_e{es}"] = (lambda es=es: C.gemm_pp(A, B, D, epi, bias if epi else None,
                                                        aux if epi == 6 else None, 0, es))
        # the one-tile kernel with the same epilogue (gemm_nt epi 6 = bias + GELU + gelu', 5 = bias)
        fns["onetile"] = lambda: C.gemm_nt(A, B, D, epi, False, bias if epi else None, aux if epi == 6 else None, None)
        if epi == 0:
            fns["hipblaslt"] = lambda: torch.mm(A, B.t(), out=D)
        elif epi == 5:
            fns["hipblaslt"] = lambda: torch.addmm(bias, A, B.t(), out=D)
        for f in fns.values():
            f()
        times = {k: [] for k in fns}
        for _ in range(a.rounds):
            for k, f in fns.items():
                times[k].append(timeit(f, a.iters))
        med = {k: round(statistics.median(v), 1) for k, v in times.items()}
        flops = 2.0 * M * N * K
        print(json.dumps({"shape": name, "dma": os.environ.get("CLOUDTIK_AMD_PP_DMA", "0"), "M": M, "N": N, "K": K, "epi": epi, "us": med,
                          "tflops": {k: round(flops / t / 1e6) for k, t in med.items()}}), flush=True)


if __name__ == "__main__":
    main()
