"""ResNet-50's stride-1 3x3 convolutions: MIOpen backward-data vs the same dgrad issued as a
forward convolution (dX = conv2d(dY, flip(W)^T, pad 1)), NHWC bf16, batch 256; HIP-event
medians of 20, ms.  Also times the forward and wgrad for reference."""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
import cloudtik_amd.ops  # noqa: E402,F401  (installs the shipped MIOpen solver db)

dev = torch.device("cuda")
N = 256
SHAPES = [(56, 64, 3), (28, 128, 3), (14, 256, 5), (7, 512, 2)]   # (H, C, stride-1 occurrences)


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


tot = [0.0, 0.0, 0.0, 0.0]
for H, C, n in SHAPES:
    x = torch.randn(N, C, H, H, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(C, C, 3, 3, device=dev, dtype=torch.bfloat16) * 0.05).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(N, C, H, H, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)

    def mi_dgrad():
        return torch.ops.aten.convolution_backward(dy, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                                   [True, False, False])[0]

    def fwd_dgrad():
        wt = w.flip(2, 3).transpose(0, 1).contiguous(memory_format=torch.channels_last)
        return F.conv2d(dy, wt, padding=1)

    err = (mi_dgrad().float() - fwd_dgrad().float()).abs().max().item()
    r = [timeit(lambda: F.conv2d(x, w, padding=1)), timeit(mi_dgrad), timeit(fwd_dgrad),
         timeit(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0],
                                                            1, [False, True, False]))]
    for i in range(4):
        tot[i] += n * r[i]
    print(f"H {H:3d} C {C:4d} | fwd {r[0]:.3f} | dgrad MIOpen {r[1]:.3f}  as-fwd {r[2]:.3f} | wgrad {r[3]:.3f}"
          f"   (x{n}, max diff {err:.3g})", flush=True)
print(f"per step: fwd {tot[0]:.3f}  dgrad MIOpen {tot[1]:.3f}  as-fwd {tot[2]:.3f}  wgrad {tot[3]:.3f} ms", flush=True)
