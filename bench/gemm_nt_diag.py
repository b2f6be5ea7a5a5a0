"""Time gemm_nt (and hipBLASLt) on a few shapes; run under CLOUDTIK_AMD_GEMM_DIAG=0/1/2 to get
the full kernel / no-DMA / no-barrier timings (diagnostic variants compute wrong results)."""
import json
import os

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
    from cloudtik_amd import ops
    C = ops.require_native()
    g = torch.Generator(device="cuda").manual_seed(0)
    out = {"diag": os.environ.get("CLOUDTIK_AMD_GEMM_DIAG", "0")}
    for M, N, K in [(32768, 1024, 4096), (32768, 4096, 1024), (8192, 8192, 8192)]:
        A = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
        B = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).to(torch.bfloat16)
        D = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        t = timeit(lambda: C.gemm_nt(A, B, D, 0, False, None, None, None))
        tb = timeit(lambda: torch.mm(A, B.t(), out=D))
        out[f"{M}x{N}x{K}"] = {"hip_tflops": round(2 * M * N * K / t / 1e6), "blas_tflops": round(2 * M * N * K / tb / 1e6)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
