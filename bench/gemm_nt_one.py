"""Run one GEMM shape repeatedly through the HIP gemm_nt kernel and hipBLASLt (for rocprofv3).

    python bench/gemm_nt_one.py M N K [iters]"""
import sys

import torch


def main():
    M, N, K = (int(x) for x in sys.argv[1:4])
    it = int(sys.argv[4]) if len(sys.argv) > 4 else 10
    from cloudtik_amd import ops
    C = ops.require_native()
    g = torch.Generator(device="cuda").manual_seed(0)
    A = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    B = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).to(torch.bfloat16)
    D = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    for _ in range(it):
        assert C.gemm_nt(A, B, D, 0, False, None, None, None)
        torch.mm(A, B.t(), out=D)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
