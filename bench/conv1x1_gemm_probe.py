"""ResNet-50's stride-1 1x1 convolutions: MIOpen vs plain GEMMs over the NHWC activations.

In channels_last a stride-1 1x1 conv is a GEMM over [N*H*W, C] rows: fwd Y = X W^T, dgrad
dX = dY W, wgrad dW = dY^T X.  This times each of the three passes both ways (HIP events,
median of 20) for every 1x1 shape of ResNet-50 at batch 256 and prints the weighted total
per training step.  MIOpen's wgrad time includes its workspace zero-fill and fp32->bf16 cast
kernels (they run on the same stream)."""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from cloudtik_amd.ops.linear import wgrad_accumulate  # noqa: E402

dev = torch.device("cuda")
N = 256
# (H, Cin, Cout, occurrences per ResNet-50 step)
SHAPES = [(56, 64, 64, 1), (56, 256, 64, 2), (56, 64, 256, 4), (56, 256, 128, 1),
          (28, 128, 512, 4), (28, 512, 128, 3), (28, 512, 256, 1), (14, 256, 1024, 6),
          (14, 1024, 256, 5), (14, 1024, 512, 1), (7, 512, 2048, 3), (7, 2048, 512, 2)]


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


tot = {k: 0.0 for k in ("mi_f", "mi_d", "mi_w", "g_f", "g_d", "g_w", "g_wsk")}
print(f"{'H':>3} {'Cin':>5} {'Cout':>5} | {'MIOpen fwd':>10} {'dgrad':>8} {'wgrad':>8} | "
      f"{'GEMM fwd':>9} {'dgrad':>8} {'wgrad':>8} {'wgrad-sk':>9}", flush=True)
for H, ci, co, n in SHAPES:
    x = torch.randn(N, ci, H, H, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(co, ci, 1, 1, device=dev, dtype=torch.bfloat16) * 0.05).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(N, co, H, H, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    M = N * H * H
    x2 = x.permute(0, 2, 3, 1).reshape(M, ci)
    dy2 = dy.permute(0, 2, 3, 1).reshape(M, co)
    w2 = w.reshape(co, ci)
    g = torch.zeros(co, ci, device=dev, dtype=torch.bfloat16)
    r = {
        "mi_f": timeit(lambda: F.conv2d(x, w)),
        "mi_d": timeit(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [True, False, False])),
        "mi_w": timeit(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [False, True, False])),
        "g_f": timeit(lambda: torch.mm(x2, w2.t())),
        "g_d": timeit(lambda: torch.mm(dy2, w2)),
        "g_w": timeit(lambda: g.addmm_(dy2.t(), x2)),
        "g_wsk": timeit(lambda: wgrad_accumulate(g, dy2, x2)),
    }
    # numerics: GEMM vs MIOpen
    y_ref = F.conv2d(x, w).permute(0, 2, 3, 1).reshape(M, co).float()
    err = (torch.mm(x2, w2.t()).float() - y_ref).abs().max().item()
    for k, v in r.items():
        tot[k] += n * v
    print(f"{H:3d} {ci:5d} {co:5d} | {r['mi_f']:10.3f} {r['mi_d']:8.3f} {r['mi_w']:8.3f} | "
          f"{r['g_f']:9.3f} {r['g_d']:8.3f} {r['g_w']:8.3f} {r['g_wsk']:9.3f}   (x{n}, fwd max err {err:.3g})",
          flush=True)
print(f"per step (weighted) MIOpen fwd {tot['mi_f']:.3f} dgrad {tot['mi_d']:.3f} wgrad {tot['mi_w']:.3f} "
      f"= {tot['mi_f'] + tot['mi_d'] + tot['mi_w']:.3f} ms", flush=True)
print(f"per step (weighted) GEMM   fwd {tot['g_f']:.3f} dgrad {tot['g_d']:.3f} wgrad {tot['g_w']:.3f} "
      f"(split-K {tot['g_wsk']:.3f}) = {tot['g_f'] + tot['g_d'] + min(tot['g_w'], tot['g_wsk']):.3f} ms", flush=True)
