"""Probe MIOpen solver speed for the Mask R-CNN conv shapes (NHWC bf16 fwd+bwd)."""
import os
import time
import torch

dev = torch.device("cuda")
CASES = [  # (name, N, Cin, Cout, H, k, stride, bias, transpose)
    ("fpn_out_p2", 4, 256, 256, 200, 3, 1, True, False),
    ("fpn_lat_c2", 4, 256, 256, 200, 1, 1, True, False),
    ("fpn_lat_c5", 4, 2048, 256, 25, 1, 1, True, False),
    ("rpn_conv_p2", 4, 256, 256, 200, 3, 1, True, False),
    ("rpn_cls_p2", 4, 256, 3, 200, 1, 1, True, False),
    ("rpn_box_p2", 4, 256, 12, 200, 1, 1, True, False),
    ("mask_conv", 512, 256, 256, 14, 3, 1, True, False),
    ("mask_deconv", 512, 256, 256, 14, 2, 2, True, True),
    ("mask_logits", 512, 256, 81, 28, 1, 1, True, False),
    ("backbone_3x3", 4, 64, 64, 200, 3, 1, False, False),
]
print("env naive wrw/bwd disabled:", os.environ.get("MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_WRW"), flush=True)
for name, N, ci, co, H, k, s, bias, tr in CASES:
    if tr:
        conv = torch.nn.ConvTranspose2d(ci, co, k, s, bias=bias, device=dev, dtype=torch.bfloat16)
    else:
        conv = torch.nn.Conv2d(ci, co, k, s, k // 2, bias=bias, device=dev, dtype=torch.bfloat16)
    conv = conv.to(memory_format=torch.channels_last)
    x = torch.randn(N, ci, H, H, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_()
    ts = []
    for i in range(5):
        torch.cuda.synchronize()
        t = time.perf_counter()
        y = conv(x)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        y.backward(torch.ones_like(y))
        torch.cuda.synchronize()
        ts.append(((t1 - t) * 1000, (time.perf_counter() - t1) * 1000))
    f = min(a for a, _ in ts[1:]); b = min(b for _, b in ts[1:])
    print(f"{name:14s} fwd {f:8.3f} ms  bwd {b:8.3f} ms", flush=True)
