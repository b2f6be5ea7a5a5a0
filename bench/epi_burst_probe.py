"""Is the fused-epilogue cost of the one-tile MFMA GEMM a chip-wide HBM burst (every CU
storing its tile at once) or per-CU work?  Time the FFN1 (EPI 6) and FFN data-gradient (EPI 7)
kernels per tile-round at full occupancy (2048 / 256 tiles: every CU) and with only half of the
CUs busy (128 tiles), each with and without its epilogue (the no-epilogue diagnostic build is
the CLOUDTIK_AMD_GEMM_DIAG=4 process)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from cloudtik_amd import ops  # noqa: E402

C = ops.require_native()
dev = torch.device("cuda")


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


out = {"diag": os.environ.get("CLOUDTIK_AMD_GEMM_DIAG", "0")}
K = 1024
for M, N in ((32768, 4096), (4096, 4096), (2048, 4096)):
    tiles = (M // 256) * (N // 256)
    x = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) * K ** -0.5).bfloat16()
    b = torch.randn(N, device=dev).bfloat16()
    h, g = torch.empty(M, N, device=dev, dtype=torch.bfloat16), torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    t6 = timeit(lambda: C.gemm_nt(x, w, h, 6, False, b, g, None))
    # data gradient: [M, K] x [K, N] (W2 read in place as [K, N]) * g, bias-gradient sums
    w2 = (torch.randn(K, N, device=dev) * K ** -0.5).bfloat16()
    dz = torch.empty_like(h)
    db = torch.zeros(N, device=dev)
    t7 = timeit(lambda: C.gemm_nn(x, w2, dz, 7, False, None, g, db))
    t7n = timeit(lambda: C.gemm_nn(x, w2, dz, 7, False, None, g, None))     # no bias-gradient sums
    db16 = torch.zeros(16, N, device=x.device, dtype=torch.float32)
    t7r = timeit(lambda: C.gemm_nn(x, w2, dz, 7, False, None, g, db16))     # sums spread over 16 rows
    t0 = timeit(lambda: C.gemm_nt(x, w, h, 0, False, None, None, None))
    # data gradient accumulated into the residual gradient (the NN dgrad sites): D += A . B
    tacc = timeit(lambda: C.gemm_nn(x, w2, dz, 0, True, None, None, None))
    rounds = max(1, -(-tiles // 256))
    out[f"{M}x{N}"] = {"tiles": tiles, "rounds": rounds, "epi6_us": round(t6, 1), "epi7_us": round(t7, 1), "epi7_nobgrad_us": round(t7n, 1), "epi7_rows16_us": round(t7r, 1),
                       "plain_us": round(t0, 1), "acc_nn_us": round(tacc, 1),
                       "acc_nn_per_round": round(tacc / rounds, 2), "epi6_per_round": round(t6 / rounds, 2),
                       "epi7_per_round": round(t7 / rounds, 2), "plain_per_round": round(t0 / rounds, 2)}
print(json.dumps(out))
