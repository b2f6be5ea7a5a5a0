"""Hand-written MFMA GEMM (csrc/gemm_nt.hip) vs hipBLASLt (torch.mm) on the BERT-large GEMM
shapes (tokens 32768), and the fused FFN epilogues vs GEMM + separate elementwise kernel.

    python bench/gemm_nt_probe.py [--tokens 32768]"""
import argparse
import json

import torch


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
    C = ops.require_native()
    T = a.tokens
    bf = torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(0)
    rnd = lambda *s, sc=1.0: (torch.randn(*s, device="cuda", generator=g) * sc).to(bf)
    # (name, M, N, K): D[M,N] = A[M,K] B[N,K]^T
    for name, M, N, K in [("qkv_fwd", T, 3072, 1024), ("wo_fwd", T, 1024, 1024), ("ffn1_fwd", T, 4096, 1024),
                          ("ffn2_fwd", T, 1024, 4096), ("ffn_dgrad_dh", T, 4096, 1024),
                          ("ffn_dgrad_dx", T, 1024, 4096), ("qkv_dgrad_dx", T, 1024, 3072)]:
        A, B = rnd(M, K), rnd(N, K, sc=K ** -0.5)
        D = torch.empty(M, N, device="cuda", dtype=bf)
        t_blas = timeit(lambda: torch.mm(A, B.t(), out=D))
        ok = C.gemm_nt(A, B, D, 0, False, None, None, None)
        t_hip = timeit(lambda: C.gemm_nt(A, B, D, 0, False, None, None, None)) if ok else None
        err = ((D.float() - (A.float() @ B.float().t())).abs().max().item()) if ok else None
        fl = 2 * M * N * K
        print(json.dumps({"case": name, "M": M, "N": N, "K": K, "hipblaslt_us": round(t_blas, 1),
                          "hip_us": t_hip and round(t_hip, 1), "hipblaslt_tflops": round(fl / t_blas / 1e6),
                          "hip_tflops": t_hip and round(fl / t_hip / 1e6), "max_abs_err": err}), flush=True)
    # fused FFN epilogues
    H, F = 1024, 4096
    x2, W1, b1 = rnd(T, H), rnd(F, H, sc=0.03), rnd(F, sc=0.1)
    W2, df = rnd(H, F, sc=0.03), rnd(T, H)
    t_unf = timeit(lambda: C.bias_act_fwd(torch.mm(x2, W1.t()), b1, 1))
    h, aux = torch.empty(T, F, device="cuda", dtype=bf), torch.empty(T, F, device="cuda", dtype=bf)
    t_fus = timeit(lambda: C.gemm_nt(x2, W1, h, 1, False, b1, aux, None))
    print(json.dumps({"case": "ffn1_fwd_bias_gelu", "unfused_us": round(t_unf, 1), "fused_us": round(t_fus, 1)}),
          flush=True)
    z = torch.mm(x2, W1.t())
    db = torch.zeros(F, device="cuda", dtype=torch.float32)
    t_unf = timeit(lambda: C.bias_act_bwd_into(torch.mm(df, W2), z, b1, 1, db, True))
    W2t = W2.t().contiguous()
    dz = torch.empty(T, F, device="cuda", dtype=bf)
    t_fus = timeit(lambda: C.gemm_nt(df, W2t, dz, 2, False, None, aux, db))
    t_tr = timeit(lambda: W2.t().contiguous())
    t_nn = timeit(lambda: C.gemm_nn(df, W2, dz, 2, False, b1, z, db))
    t_nn0 = timeit(lambda: C.gemm_nn(df, W2, dz, 0, False, None, None, None))
    print(json.dumps({"case": "ffn_dgrad_dgelu_bgrad", "unfused_us": round(t_unf, 1), "fused_us": round(t_fus, 1),
                      "w2_transpose_us": round(t_tr, 1), "nn_fused_us": round(t_nn, 1),
                      "nn_plain_us": round(t_nn0, 1)}), flush=True)


if __name__ == "__main__":
    main()
