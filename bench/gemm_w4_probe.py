"""Four-wave GEMM (gemm_nt.hip gemm_w4_kernel) vs the 8-wave one-tile kernel vs hipBLASLt on the
BERT-large forward projection shapes (tokens 32768), random bf16 operands.  Numerics first, then
median time of interleaved rounds; one JSON line per shape.

    python bench/gemm_w4_probe.py [--rounds 5] [--iters 10]
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
    return z * phi, phi + z * torch.exp(-0.5 * z * z) / math.sqrt(2.0 * math.pi)


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


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
    ap.add_argument("--skip-check", action="store_true")
    a = ap.parse_args()
    from cloudtik_amd import ops
    C = ops.require_native()
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(0)
    if not a.skip_check:
        out, bad = [], 0
        for (M, N, K) in [(256, 256, 64), (512, 768, 128), (2048, 1024, 1024), (32768, 4096, 1024)]:
            A = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)
            B = (torch.randn(N, K, generator=g) * K ** -0.5).to(dev, torch.bfloat16)
            bias = (torch.randn(N, generator=g) * 0.5).to(dev, torch.bfloat16)
            for epi in (0, 5, 6):
                D = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
                aux = torch.full_like(D, float("nan")) if epi == 6 else None
                ok = C.gemm_w4(A, B, D, epi, bias if epi else None, aux)
                torch.cuda.synchronize()
                zr, dr = ref_epi(A, B, bias, epi)
                r = {"M": M, "N": N, "K": K, "epi": epi, "ok": bool(ok), "nan": bool(torch.isnan(D).any()),
                     "err": rel(D, zr)}
                if epi == 6:
                    r["err_aux"] = rel(aux, dr)
                bad += (not ok) or r["nan"] or r["err"] > 1e-2 or r.get("err_aux", 0) > 1e-2
                out.append(r)
        print(json.dumps({"check": out, "bad": bad}), flush=True)
        if bad:
            sys.exit(1)
    for name, M, N, K, epi in [("ffn1_plain", 32768, 4096, 1024, 0), ("ffn1", 32768, 4096, 1024, 6),
                               ("ffn2", 32768, 1024, 4096, 0), ("qkv", 32768, 3072, 1024, 5),
                               ("wo", 32768, 1024, 1024, 0)]:
        A = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)
        B = (torch.randn(N, K, generator=g) * K ** -0.5).to(dev, torch.bfloat16)
        bias = (torch.randn(N, generator=g) * 0.5).to(dev, torch.bfloat16)
        D = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        aux = torch.empty_like(D)
        fns = {"w4": lambda: C.gemm_w4(A, B, D, epi, bias if epi else None, aux if epi == 6 else None),
               "onetile": lambda: C.gemm_nt(A, B, D, epi, False, bias if epi else None, aux if epi == 6 else None,
                                            None)}
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
        print(json.dumps({"shape": name, "diag": os.environ.get("CLOUDTIK_AMD_GEMM_W4_DIAG", "0"), "us": med,
                          "tflops": {k: round(flops / t / 1e6) for k, t in med.items()}}), flush=True)


if __name__ == "__main__":
    main()
