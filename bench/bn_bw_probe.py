"""BatchNorm apply pass vs plain copies on the largest ResNet-50 activation shapes: achieved
bandwidth from the nominal bytes (each operand read once, the output written once).

    python bench/bn_bw_probe.py"""
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
    from cloudtik_amd import ops
    C_ = ops.require_native()
    for (N, C, H, W) in [(256, 256, 56, 56), (256, 64, 56, 56), (256, 512, 28, 28), (256, 1024, 14, 14)]:
        x = torch.randn(N, C, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        r = torch.randn_like(x)
        a = torch.rand(C, device="cuda") + 0.5
        b = torch.randn(C, device="cuda")
        y = torch.empty_like(x)
        nb = x.numel() * 2
        row = {"shape": [N, C, H, W], "MB": round(nb / 1e6, 1)}
        t = timeit(lambda: C_.bn_apply(x, None, a, b, True))
        row["bn_apply_us"], row["bn_apply_TBs"] = round(t, 1), round(2 * nb / t / 1e6, 2)
        t = timeit(lambda: C_.bn_apply(x, r, a, b, True))
        row["bn_apply_res_us"], row["bn_apply_res_TBs"] = round(t, 1), round(3 * nb / t / 1e6, 2)
        t = timeit(lambda: y.copy_(x))
        row["copy_us"], row["copy_TBs"] = round(t, 1), round(2 * nb / t / 1e6, 2)
        t = timeit(lambda: torch.add(x, r, out=y))
        row["add_us"], row["add_TBs"] = round(t, 1), round(3 * nb / t / 1e6, 2)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
