"""One conv shape through ops/conv.py fwd + dgrad (and the equivalent-GEMM forward), for
rocprofv3 --kernel-trace: separates kernel time from host overhead.
    python bench/conv_igemm_one.py CI CO H K S [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cloudtik_amd.ops import conv as CV  # noqa: E402

ci, co, H, k, s = (int(v) for v in sys.argv[1:6])
iters = int(sys.argv[6]) if len(sys.argv) > 6 else 10
pad = k // 2
dev = torch.device("cuda")
x = torch.randn(256, ci, H, H, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
w = (torch.randn(co, ci, k, k, device=dev) * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
y = CV.conv_fwd(x, w, (s, s), (pad, pad))
dy = torch.randn_like(y).contiguous(memory_format=torch.channels_last)
for _ in range(iters):
    CV.conv_fwd(x, w, (s, s), (pad, pad))
torch.cuda.synchronize()
for _ in range(iters):
    CV.conv_dgrad(dy, w, x.shape, (s, s), (pad, pad))
torch.cuda.synchronize()
print("done")
