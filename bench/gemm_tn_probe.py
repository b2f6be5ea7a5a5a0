"""Weight-gradient GEMM probe: the HIP gemm_tn kernel (csrc/gemm.hip) vs the hipBLASLt path
(ops.linear.wgrad_accumulate) on the BERT-large dW shapes, plus a numerics check.

    python bench/gemm_tn_probe.py [--tokens 32768]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
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
    ap.add_argument("--only", type=int, nargs=3, metavar=("M", "N", "S"),
                    help="time one shape / split only (for counter runs)")
    a = ap.parse_args()
    from cloudtik_amd import ops
    from cloudtik_amd.ops.linear import wgrad_accumulate
    C = ops.require_native()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    # numerics: small exact-ish check of every mode
    T, M, N = 512, 512, 768
    A = torch.randn(T, M, device=dev).bfloat16()
    B = torch.randn(T, N, device=dev).bfloat16()
    ref = A.float().t() @ B.float()
    out = torch.empty(2, M, N, device=dev)
    assert C.gemm_tn(A, B, out, 2, 0)
    err = (out.sum(0) - ref).abs().max().item()
    g = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
    assert C.gemm_tn(A, B, g, 1, 2)
    err2 = (g.float() - ref).abs().max().item()
    print(f"numerics: split2 fp32 max err {err:.3e}, bf16 out max err {err2:.3e} (|ref| max {ref.abs().max().item():.1f})",
          flush=True)
    T = a.tokens
    shapes = [(a.only[0], a.only[1])] if a.only else [(1024, 1024), (3072, 1024), (4096, 1024), (1024, 4096)]
    for (M, N) in shapes:
        dy = torch.randn(T, M, device=dev).bfloat16()
        x = torch.randn(T, N, device=dev).bfloat16()
        flops = 2.0 * T * M * N
        g = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
        t_blas = timeit(lambda: wgrad_accumulate(g, dy, x))
        res = [f"hipBLASLt path {t_blas * 1e3:7.1f} us ({flops / t_blas / 1e9:6.0f} TF)"]
        for S in ((a.only[2],) if a.only else (1, 2, 4, 8, 16)):
            if T % (64 * S):
                continue
            P = torch.empty(S, M, N, device=dev)

            def run():
                if S == 1:
                    C.gemm_tn(dy, x, g, 1, 1)
                else:
                    C.gemm_tn(dy, x, P, S, 0)
                    C.splitk_reduce(P, g, True)
            t = timeit(run)
            res.append(f"S={S} {t * 1e3:7.1f} us ({flops / t / 1e9:6.0f} TF)")
        print(f"M={M} N={N} T={T}: " + " | ".join(res), flush=True)


if __name__ == "__main__":
    main()
