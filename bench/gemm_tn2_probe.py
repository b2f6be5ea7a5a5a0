"""Weight-gradient GEMM dW = dY^T X on the BERT-large shapes (tokens 32768): the MFMA kernel's
TN layout (ct_gemm_tn2, split-K into fp32 slabs) vs hipBLASLt's batched split-K GEMM (the
current wgrad path), each followed by the same splitk_reduce into a bf16 gradient.

    python bench/gemm_tn2_probe.py [--tokens 32768]"""
import argparse
import json
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
    ap.add_argument("--tokens", type=int, default=32768)
    a = ap.parse_args()
    from cloudtik_amd import ops
    from cloudtik_amd.ops.linear import splitk_factor, tn2_splits
    C = ops.require_native()
    T = a.tokens
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, N, K in [("qkv", 3072, 1024), ("proj", 1024, 1024), ("ffn1", 4096, 1024), ("ffn2", 1024, 4096)]:
        dy = torch.randn(T, N, device="cuda", generator=g).to(torch.bfloat16)
        x = torch.randn(T, K, device="cuda", generator=g).to(torch.bfloat16)
        ref = dy.float().t() @ x.float()
        fl = 2 * T * N * K
        row = {"case": name, "N": N, "K": K}
        row["tn2_splits_chosen"] = tn2_splits(T, N, K)
        for S in sorted({splitk_factor(T, N, K), tn2_splits(T, N, K), 2, 4, 5, 6, 8, 16}):
            if T // 64 < S:
                continue
            P = torch.empty(S, N, K, device="cuda")
            t_gemm = timeit(lambda: C.gemm_tn2(dy, x, P, S, False))
            gr = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
            C.gemm_tn2(dy, x, P, S, False)
            C.splitk_reduce(P, gr, True)
            err = ((gr.float() - ref).norm() / ref.norm()).item()
            t_red = timeit(lambda: C.splitk_reduce(P, gr, True))
            row[f"tn2_S{S}_us"] = round(t_gemm, 1)
            row[f"tn2_S{S}_tflops"] = round(fl / t_gemm / 1e6)
            row[f"reduce_S{S}_us"] = round(t_red, 1)
            row[f"tn2_S{S}_relerr"] = float(f"{err:.1e}")
        S = splitk_factor(T, N, K)
        t_bmm = timeit(lambda: torch.bmm(dy.view(S, T // S, N).transpose(1, 2), x.view(S, T // S, K),
                                         out_dtype=torch.float32))
        row["hipblaslt_bmm_S"] = S
        row["hipblaslt_bmm_us"] = round(t_bmm, 1)
        row["hipblaslt_bmm_tflops"] = round(fl / t_bmm / 1e6)
        gr = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
        t_acc = timeit(lambda: gr.addmm_(dy.t(), x))
        row["hipblaslt_addmm_us"] = round(t_acc, 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
