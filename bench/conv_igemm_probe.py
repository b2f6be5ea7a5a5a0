"""Implicit-GEMM conv kernels (ops/conv.py) vs MIOpen on every ResNet-50 conv shape, batch 256.

Checks numerics (fwd, dgrad, BN tile statistics) against an fp32 reference on a slice of the
batch, then times fwd and dgrad for each tile configuration and for MIOpen (F.conv2d /
convolution_backward with the shipped solver db).  Prints a markdown table.

    python bench/conv_igemm_probe.py [--batch 256] [--quick]
"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cloudtik_amd.ops import conv as CV  # noqa: E402

# (name, ci, co, H, k, stride, calls per ResNet-50 step)
SHAPES = [
    ("l1.c1a", 64, 64, 56, 1, 1, 1), ("l1.c2", 64, 64, 56, 3, 1, 3), ("l1.c3", 64, 256, 56, 1, 1, 3),
    ("l1.c1", 256, 64, 56, 1, 1, 2),
    ("l2.c1a", 256, 128, 56, 1, 1, 1), ("l2.c2s2", 128, 128, 56, 3, 2, 1), ("l2.c2", 128, 128, 28, 3, 1, 3),
    ("l2.c3", 128, 512, 28, 1, 1, 4), ("l2.down", 256, 512, 56, 1, 2, 1), ("l2.c1", 512, 128, 28, 1, 1, 3),
    ("l3.c1a", 512, 256, 28, 1, 1, 1), ("l3.c2s2", 256, 256, 28, 3, 2, 1), ("l3.c2", 256, 256, 14, 3, 1, 5),
    ("l3.c3", 256, 1024, 14, 1, 1, 6), ("l3.down", 512, 1024, 28, 1, 2, 1), ("l3.c1", 1024, 256, 14, 1, 1, 5),
    ("l4.c1a", 1024, 512, 14, 1, 1, 1), ("l4.c2s2", 512, 512, 14, 3, 2, 1), ("l4.c2", 512, 512, 7, 3, 1, 2),
    ("l4.c3", 512, 2048, 7, 1, 1, 3), ("l4.down", 1024, 2048, 14, 1, 2, 1), ("l4.c1", 2048, 512, 7, 1, 1, 2),
]


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3   # us


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def check(ci, co, H, k, s, dev):
    pad = k // 2
    g = torch.Generator(device="cpu").manual_seed(ci * 7 + co + H)
    x = torch.randn(4, ci, H, H, generator=g).to(dev, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(co, ci, k, k, generator=g) * (2.0 / (ci * k * k)) ** 0.5).to(dev, torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    ref = F.conv2d(x.float(), w.float(), stride=s, padding=pad)
    y, mean, var = CV.conv_fwd(x, w, (s, s), (pad, pad), stats=True)
    e_fwd = rel(y, ref)
    yb = y.float()
    e_mean = (mean - yb.mean((0, 2, 3))).abs().max().item()
    e_var = rel(var, yb.var((0, 2, 3), unbiased=False))
    dy = torch.randn(ref.shape, generator=g).to(dev, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xr = x.float().requires_grad_()
    F.conv2d(xr, w.float(), stride=s, padding=pad).backward(dy.float())
    dx = CV.conv_dgrad(dy, w, x.shape, (s, s), (pad, pad))
    e_dx = rel(dx, xr.grad)
    wr = w.float().requires_grad_()
    F.conv2d(x.float(), wr, stride=s, padding=pad).backward(dy.float())
    dw = CV.conv_wgrad(dy, x, w.shape, (s, s), (pad, pad))
    e_dw = rel(dw, wr.grad)
    return e_fwd, e_dx, e_mean, e_var, e_dw


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--cfgs", default="-1,1,4,5,7,8,9")
    ap.add_argument("--shapes", default="", help="comma list of shape names (default: all)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.backends.cudnn.benchmark = False
    cfgs = [int(c) for c in a.cfgs.split(",")]
    print("| conv | shape | err fwd / dx / mean / var | MIOpen fwd us | igemm fwd us (cfg) | MIOpen dgrad us | "
          "igemm dgrad us | calls |")
    print("|---|---|---|---:|---:|---:|---:|---:|")
    tot = {"mi_f": 0.0, "ig_f": 0.0, "mi_d": 0.0, "ig_d": 0.0}
    roofs = []
    want = set(a.shapes.split(",")) if a.shapes else None
    for name, ci, co, H, k, s, calls in SHAPES:
        if want and name not in want:
            continue
        errs = check(ci, co, H, k, s, dev)
        pad = k // 2
        x = torch.randn(a.batch, ci, H, H, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(co, ci, k, k, device=dev) * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        y = F.conv2d(x, w, stride=s, padding=pad)
        dy = torch.randn_like(y).contiguous(memory_format=torch.channels_last)
        mi_f = timeit(lambda: F.conv2d(x, w, stride=s, padding=pad))
        mi_d = timeit(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [pad, pad], [1, 1], False,
                                                                  [0, 0], 1, [True, False, False]))
        mi_w = timeit(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [pad, pad], [1, 1], False,
                                                                  [0, 0], 1, [False, True, False]))
        wper = []
        for c in [int(v) for v in os.environ.get("WCFGS", "-1,2,3,9,11").split(",")]:
            CV._WG_CFG = c
            try:
                wper.append((timeit(lambda: CV.conv_wgrad(dy, x, w.shape, (s, s), (pad, pad))), c))
            except RuntimeError:
                pass
        CV._WG_CFG = -1
        ig_w = wper[0][0]
        tot["mi_w"] = tot.get("mi_w", 0.0) + mi_w * calls
        tot["ig_w"] = tot.get("ig_w", 0.0) + ig_w * calls
        best_f, best_d = None, None
        per = []
        for c in cfgs:
            CV._CFG = c
            # forward (Co = co) and data gradient (Co = ci) are timed independently: a
            # configuration may fit one and not the other
            try:
                tf = timeit(lambda: CV.conv_fwd(x, w, (s, s), (pad, pad)))
            except RuntimeError:
                tf = None
            try:
                td = timeit(lambda: CV.conv_dgrad(dy, w, x.shape, (s, s), (pad, pad)))
            except RuntimeError:
                td = None
            if tf is None and td is None:
                continue
            per.append(f"c{c}:{'-' if tf is None else f'{tf:.0f}'}/{'-' if td is None else f'{td:.0f}'}")
            if tf is not None and (best_f is None or tf < best_f[0]):
                best_f = (tf, c)
            if td is not None and (best_d is None or td < best_d[0]):
                best_d = (td, c)
            if c == -1:
                auto_f, auto_d = tf, td
        CV._CFG = -1
        tot["mi_f"] += mi_f * calls
        tot["mi_d"] += mi_d * calls
        tot["ig_f"] += auto_f * calls
        tot["ig_d"] += auto_d * calls
        # roofline: minimum HBM bytes (read X, W once, write Y) at 6 TB/s vs bf16 MFMA at 2.5 PF
        Ho = (H + 2 * pad - k) // s + 1
        fl = 2.0 * a.batch * Ho * Ho * co * ci * k * k
        by = 2.0 * (a.batch * H * H * ci + co * ci * k * k + a.batch * Ho * Ho * co)
        roof = max(by / 6e12, fl / 2.5e15) * 1e6
        roofs.append({"conv": name, "roofline_us": round(roof, 1), "fwd_us": round(auto_f, 1),
                      "dgrad_us": round(auto_d, 1), "wgrad_us": round(ig_w, 1), "fwd_tflops": round(fl / auto_f / 1e6),
                      "fwd_TBs": round(by / auto_f / 1e6, 2), "fwd_pct_roofline": round(100 * roof / auto_f),
                      "dgrad_pct_roofline": round(100 * roof / auto_d), "wgrad_pct_roofline": round(100 * roof / ig_w),
                      "calls": calls})
        print(f"| {name} | {ci}->{co} {H}x{H} k{k} s{s} | {errs[0]:.1e} / {errs[1]:.1e} / {errs[2]:.1e} / "
              f"{errs[3]:.1e} | {mi_f:.1f} | {auto_f:.1f} (best {best_f[0]:.1f} c{best_f[1]}) | {mi_d:.1f} | "
              f"{auto_d:.1f} (best {best_d[0]:.1f} c{best_d[1]}) | {calls} |", flush=True)
        print("    cfg fwd/dgrad us: " + " ".join(per) + f" | wgrad MIOpen {mi_w:.0f} igemm "
              + " ".join(f"c{c}:{t:.0f}" for t, c in wper) + f" err {errs[4]:.1e}", file=sys.stderr, flush=True)
    print(f"\nper ResNet-50 step (auto cfg): MIOpen fwd {tot['mi_f'] / 1e3:.2f} ms, igemm fwd {tot['ig_f'] / 1e3:.2f} ms; "
          f"MIOpen dgrad {tot['mi_d'] / 1e3:.2f} ms, igemm dgrad {tot['ig_d'] / 1e3:.2f} ms; "
          f"MIOpen wgrad {tot['mi_w'] / 1e3:.2f} ms, igemm wgrad {tot['ig_w'] / 1e3:.2f} ms")
    print("\n| conv | roofline us | fwd us (% roof, TF/s, TB/s) | dgrad us (% roof) | wgrad us (% roof) | calls |")
    print("|---|---:|---:|---:|---:|---:|")
    for r in roofs:
        print(f"| {r['conv']} | {r['roofline_us']} | {r['fwd_us']} ({r['fwd_pct_roofline']}%, {r['fwd_tflops']}, "
              f"{r['fwd_TBs']}) | {r['dgrad_us']} ({r['dgrad_pct_roofline']}%) | {r['wgrad_us']} "
              f"({r['wgrad_pct_roofline']}%) | {r['calls']} |")
    w = sum(r["calls"] * r["roofline_us"] for r in roofs)
    print(f"\nper step: roofline {3 * w / 1e3:.2f} ms for fwd+dgrad+wgrad vs igemm "
          f"{(tot['ig_f'] + tot['ig_d'] + tot['ig_w']) / 1e3:.2f} ms")


if __name__ == "__main__":
    main()
