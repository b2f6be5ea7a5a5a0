"""Host-side (Python) cost of one training step of a bench model: cProfile over K steps issued
WITHOUT waiting for the GPU in between (the host time that decides whether the GPU queue stays
full), plus the wall time of the issue loop itself.

    python bench/host_profile.py --model resnet50 --steps 5 [--top 40]"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--sort", default="tottime")
    a = ap.parse_args()
    import torch
    import bench
    args = bench.parse(["--model", a.model, "--graph", "off"])
    dev = torch.device("cuda", 0)
    if a.model == "resnet50":
        step, _close, _info = bench.build_resnet(args, 0, 1, dev, "resnet50")
    else:
        step, _close, _info = bench.build_bert(args, 0, 1, dev, a.model)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for _ in range(a.steps):
        step()
    pr.disable()
    t_issue = (time.perf_counter() - t0) / a.steps
    torch.cuda.synchronize()
    t_all = (time.perf_counter() - t0) / a.steps
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats(a.sort).print_stats(a.top)
    print(f"host issue {t_issue * 1e3:.2f} ms/step under cProfile; issue + drain {t_all * 1e3:.2f} ms/step")
    print(s.getvalue())


if __name__ == "__main__":
    main()
